"""Round 4: what the slab path costs one GPU.  Scene M (or --scene) as the
single domain and as ONE slab rank (nranks = 1 over RCCL: the slab kernels,
capacity-sized grids and the per-sub-step bbox record / unpack / exchange
call, with no neighbour traffic), the same ticks, interleaved windows.
Prints one JSON line."""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

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
slab = _load("slab", os.path.join(PKG, "slab.py"))

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="M")
ap.add_argument("--prep", type=int, default=300)
ap.add_argument("--ticks", type=int, default=100)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--timing", action="store_true", help="per-kernel HIP-event times of one window each")
ap.add_argument("--loop", action="store_true", help="also a 1-rank slab through the in-process transport")
ap.add_argument("--only", choices=("single", "slab1", "slab1_loopback"), default=None,
                help="build and time only this configuration (for a profiler run)")
a = ap.parse_args()
s = scenes.scene(a.scene)
fl = s["fluid"]
b, v = scenes.to_bodies(s["bodies"])
cfg = lpe.default_fluid_config()
DT = 1.0 / 120.0


def make(slabbed, rccl=True):
    c = lpe.Context(0)
    c.rigid_set_config(lpe.rigid_config(universe=s["U"]))
    c.rigid_upload(b, v)
    if slabbed:
        slab.setup_rank(c, 0, 1, fl, np.array([-np.inf, np.inf], np.float32), cfg)
        if rccl:
            c.mg_init_rccl(1, 0, lpe.mg_unique_id())
    else:
        c.sph_set_config(cfg)
        c.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    c.world_set_coupling(None)
    if slabbed and not rccl:
        lpe.mg_loopback_run([c], a.prep, world=lpe.WorldConfig(DT, 1.0, 1.0, 1.0))
    else:
        c.world_tick(DT, a.prep)
    c.sync()
    return c


if a.only:
    ctxs = {a.only: make(a.only != "single", rccl=a.only == "slab1")}
else:
    ctxs = {"single": make(False), "slab1": make(True)}
    if a.loop:
        ctxs["slab1_loopback"] = make(True, rccl=False)
rates = {k: [] for k in ctxs}
for _ in range(a.rounds):
    for k, c in ctxs.items():
        c.sync()
        t0 = time.perf_counter()
        if k == "slab1_loopback":
            lpe.mg_loopback_run([c], a.ticks, world=lpe.WorldConfig(DT, 1.0, 1.0, 1.0))
        else:
            c.world_tick(DT, a.ticks)
        c.sync()
        rates[k].append(a.ticks / (time.perf_counter() - t0))
out = {"scene": a.scene, "prep": a.prep, "ticks": a.ticks,
       "ticks_per_s": {k: [round(r, 1) for r in v] for k, v in rates.items()},
       "median": {k: round(float(np.median(v)), 1) for k, v in rates.items()}}
if a.timing:
    for k, c in ctxs.items():
        if k == "slab1_loopback":
            continue
        c.timing(1)
        c.timing_reset()
        c.world_tick(DT, 20)
        t = c.timing_read()
        c.timing(0)
        out[f"kernels_us_{k}"] = {n: round(ms / max(cl, 1) * 1e3, 2) for n, (ms, cl) in sorted(t.items())}
        out[f"tick_kernel_ms_{k}"] = round(sum(ms for ms, _ in t.values()) / 20, 3)
if "slab1" in ctxs:
    out["slab1_owned"] = ctxs["slab1"].sph_stats()["slabOwned"]
for c in ctxs.values():
    c.close()
print(json.dumps(out))
