"""Round 5: tick rates of the settled metric scene (profiles/snapshot.py state)
in multi-tick calls and one-tick calls, alternating, three windows each --
for the heavy-tile A/B (LPE_NO_HEAVY=1 turns them off); PGS_MODE=1: the
opt-in Jacobi contact solver."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe  # noqa: E402
DT = 1.0 / 120.0
z = np.load("/tmp/lpe_snap.npz")
ctx = lpe.Context(0)
MODE = int(os.environ.get("PGS_MODE", "0"))
ctx.rigid_set_config(lpe.rigid_config(universe=32.0, pgsMode=MODE))
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_upload(z["bodies"], z["verts"])
ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
ctx.world_set_coupling(None)
ctx.world_tick(DT, 30)
ctx.sync()
out = {"heavy": os.environ.get("LPE_NO_HEAVY") is None, "pgsMode": MODE, "multi": [], "one": []}
for rep in range(3):
    for mode in ("multi", "one"):
        n = 400
        ctx.sync()
        t0 = time.perf_counter()
        if mode == "multi":
            ctx.world_tick(DT, n)
        else:
            for _ in range(n):
                ctx.world_tick(DT, 1)
        ctx.sync()
        out[mode].append(round(n / (time.perf_counter() - t0), 1))
ctx.close()
print(json.dumps(out), flush=True)
