"""Tick rates of the small configurations (C1 box stack, C3 random polygons,
C2 64k dam break) and of scene M from its settled snapshot, for A/B runs of
library variants:

    LPE_LIB=profiles/_var/liblpe_X.so python profiles/config_ab.py [--m]

One JSON line: ticks/s (median of 3 windows of >= 1 s) per configuration,
multi-tick calls and one-tick calls (the drop-in path)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

DT = 1.0 / 120.0


def windows(ctx, one_tick, n=3, min_s=1.0):
    rates = []
    per = 50
    for _ in range(n + 1):
        ctx.sync()
        t0 = time.perf_counter()
        if one_tick:
            for _ in range(per):
                ctx.world_tick(DT, 1)
        else:
            ctx.world_tick(DT, per)
        ctx.sync()
        el = time.perf_counter() - t0
        rates.append(per / el)
        per = max(50, int(per * min_s / el) + 1)
    return round(float(np.median(rates[1:])), 1)


def main():
    lpe = bench._load("lpe", os.path.join(bench.PKG, "lpe.py"))
    scenes = bench._load("scenes", os.path.join(bench.PKG, "scenes.py"))
    out = {"lib": os.environ.get("LPE_LIB", "default")}
    for name in ("C1", "C3"):
        s = scenes.rigid_scene(name)
        b, v = scenes.to_bodies(s["bodies"])
        ctx = lpe.Context(0)
        try:
            ctx.rigid_set_config(lpe.rigid_config(universe=s["U"], pgs_iterations=s["pgs_iterations"]))
            ctx.rigid_upload(b, v)
            ctx.world_tick(DT, 240 if name == "C3" else 60)
            out[name] = windows(ctx, False)
            out[name + "_1tick"] = windows(ctx, True)
        finally:
            ctx.close()
    s = scenes.scene("C2")
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    ctx = lpe.Context(0)
    try:
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        ctx.rigid_upload(b, v)
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.world_set_coupling(None)
        ctx.world_tick(DT, 30)
        out["C2"] = windows(ctx, False)
        out["C2_1tick"] = windows(ctx, True)
    finally:
        ctx.close()
    if "--m" in sys.argv and os.path.exists("/tmp/lpe_snap.npz"):
        z = np.load("/tmp/lpe_snap.npz")
        ctx = lpe.Context(0)
        try:
            ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
            ctx.sph_set_config(lpe.default_fluid_config())
            ctx.rigid_upload(z["bodies"], z["verts"])
            ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
            ctx.world_set_coupling(None)
            ctx.world_tick(DT, 20)
            out["M_snap"] = windows(ctx, False, n=3, min_s=2.0)
            out["M_snap_1tick"] = windows(ctx, True, n=3, min_s=2.0)
        finally:
            ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
