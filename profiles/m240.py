"""Scene M advanced N device ticks in the world tick (test_configs_gpu's _advanced), then the status."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe, scenes
import numpy as np
n = int(sys.argv[1]) if len(sys.argv) > 1 else 240
s = scenes.scene("M"); fl = s["fluid"]; b, v = scenes.to_bodies(s["bodies"])
ctx = lpe.Context(0)
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
ctx.rigid_upload(b, v)
ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
t0 = time.perf_counter()
for k in range(0, n, 20):
    ctx.world_tick(1 / 120, min(20, n - k)); ctx.sync()
    st = ctx.sph_stats()
    print(os.environ.get("LPE_LIB", "default"), "tick", k + 20, "maxOcc", st["maxCellOccupancy"], flush=True)
out = ctx.sph_download()
print("ok", n, "ticks", round(time.perf_counter() - t0, 2), "s", np.isfinite(out["x"]).all(), flush=True)
ctx.close()
