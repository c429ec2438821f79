"""Host enqueue time per world tick vs device time on C1 (132 bodies, rigid only)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
lpe = bench._load("lpe", os.path.join(bench.PKG, "lpe.py")); scenes = bench._load("scenes", os.path.join(bench.PKG, "scenes.py"))
s = scenes.rigid_scene("C1"); b, v = scenes.to_bodies(s["bodies"])
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=s["U"], pgs_iterations=s["pgs_iterations"]))
ctx.rigid_upload(b, v)
ctx.world_tick(1 / 120, 60); ctx.sync()
for rep in range(3):
    ctx.sync(); t0 = time.perf_counter()
    for i in range(200): ctx.world_tick(1 / 120, 1)
    t1 = time.perf_counter(); ctx.sync(); t2 = time.perf_counter()
    print(f"C1 200 calls: host {1e6 * (t1 - t0) / 200:.1f} us/tick, wall {1e6 * (t2 - t0) / 200:.1f} us/tick", flush=True)
hs = []
for rep in range(7):
    ctx.sync(); t0 = time.perf_counter(); ctx.world_tick(1 / 120, 1); hs.append(1e6 * (time.perf_counter() - t0))
ctx.sync()
print("C1 one call after a sync: host", round(sorted(hs)[3], 1), "us")
ctx.timing(1); ctx.timing_reset(); ctx.world_tick(1 / 120, 20); t = ctx.timing_read(); ctx.timing(0)
tot = sum(vv[0] for vv in t.values()) / 20 * 1e3
print("C1 sum of kernel times per tick (HIP events, all streams):", round(tot, 1), "us;", len(t), "kernels")
ctx.close()
