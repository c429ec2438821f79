"""Round 4: where a small config's tick goes (the launch
tax).  Runs one of BASELINE.json's small configs (C1 rigid stack, C2 dam
break) after its settle, and prints one JSON line: the tick rate over a
window, the library's per-kernel HIP-event times over a second window (avg
us per launch, launches per tick) and their sum per tick against the wall
time per tick -- a sum well below the wall time means the tick is bound by
launch issue, not by the kernels."""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "little-physics-engine_amd")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


lpe = _load("lpe", os.path.join(PKG, "lpe.py"))
scenes = _load("scenes", os.path.join(PKG, "scenes.py"))

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="C1", choices=("C1", "C2", "C3", "C4"))
ap.add_argument("--ticks", type=int, default=500)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
DT = 1.0 / 120.0

c = lpe.Context(0)
if a.scene in ("C1", "C3"):
    s = scenes.rigid_scene(a.scene)
    b, v = scenes.to_bodies(s["bodies"])
    c.rigid_set_config(lpe.rigid_config(universe=s["U"], pgs_iterations=s["pgs_iterations"]))
    c.rigid_upload(b, v)
    prep = 240 if a.scene == "C3" else 60
else:
    s = scenes.scene(a.scene)
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    c.rigid_set_config(lpe.rigid_config(universe=s["U"]))
    c.rigid_upload(b, v)
    c.sph_set_config(lpe.default_fluid_config())
    c.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    c.world_set_coupling(None)
    prep = 90 if a.scene == "C4" else 30
c.world_tick(DT, prep)
c.sync()
rates = []
for _ in range(a.rounds):
    t0 = time.perf_counter()
    c.world_tick(DT, a.ticks)
    c.sync()
    rates.append(a.ticks / (time.perf_counter() - t0))
rates.sort()
# one tick per call (the drop-in's host loop)
t0 = time.perf_counter()
for _ in range(a.ticks):
    c.world_tick(DT, 1)
c.sync()
one = a.ticks / (time.perf_counter() - t0)
c.timing(True)
c.timing_reset()
nt = min(a.ticks, 200)
c.world_tick(DT, nt)
c.sync()
tm = c.timing_read()
c.timing(False)
c.close()
per_tick = {k: dict(us_per_launch=round(1e3 * ms / max(calls, 1), 2), launches_per_tick=round(calls / nt, 2),
                    us_per_tick=round(1e3 * ms / nt, 2)) for k, (ms, calls) in sorted(tm.items(), key=lambda kv: -kv[1][0])}
ksum = sum(1e3 * ms / nt for ms, _ in tm.values())
print(json.dumps(dict(probe="small_config", scene=a.scene, ticks=a.ticks, ticks_per_s=round(rates[len(rates) // 2], 1),
                      rates=[round(r, 1) for r in rates], one_tick_calls_per_s=round(one, 1),
                      wall_us_per_tick=round(1e6 / rates[len(rates) // 2], 1), timing_ticks=nt,
                      kernel_sum_us_per_tick=round(ksum, 1),
                      launches_per_tick=round(sum(c_ for _, c_ in tm.values()) / nt, 1), kernels=per_tick)))
