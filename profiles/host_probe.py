"""Host enqueue time per world tick vs device time (settled snapshot): whether the host keeps ahead of the GPU."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe, scenes
import numpy as np
z = np.load("/tmp/lpe_snap.npz")
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_upload(z["bodies"], z["verts"])
ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
ctx.world_set_coupling(None)
ctx.world_tick(1 / 120, 20); ctx.sync()
for k in (1, 10):
    for rep in range(3):
        ctx.sync()
        t0 = time.perf_counter()
        for i in range(20 // k):
            ctx.world_tick(1 / 120, k)
        t1 = time.perf_counter()
        ctx.sync()
        t2 = time.perf_counter()
        print(f"calls of {k} tick(s): host enqueue {1e6 * (t1 - t0) / 20:.1f} us/tick, wall {1e6 * (t2 - t0) / 20:.1f} us/tick", flush=True)
ctx.close()
# one call right after a sync: the host's own enqueue cost (nothing to wait for)
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_upload(z["bodies"], z["verts"])
ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
ctx.world_set_coupling(None)
ctx.world_tick(1 / 120, 20); ctx.sync()
for k in (1, 2, 4):
    hs = []
    for rep in range(5):
        ctx.sync()
        t0 = time.perf_counter(); ctx.world_tick(1 / 120, k); t1 = time.perf_counter()
        hs.append(1e6 * (t1 - t0) / k)
    ctx.sync()
    print(f"after a sync, one call of {k} tick(s): host {sorted(hs)[2]:.1f} us/tick (median of 5)", flush=True)
ctx.close()
