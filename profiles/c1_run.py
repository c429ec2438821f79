"""C1 (8x16 box stack) world ticks for kernel traces: python profiles/c1_run.py [TICKS] [SCENE]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe, scenes
name = sys.argv[2] if len(sys.argv) > 2 else "C1"
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
if name in ("C1", "C3"):
    s = scenes.rigid_scene(name)
    b, v = scenes.to_bodies(s["bodies"])
    ctx = lpe.Context(0)
    ctx.rigid_set_config(lpe.rigid_config(universe=s["U"], pgs_iterations=s["pgs_iterations"]))
    ctx.rigid_upload(b, v)
else:
    s = scenes.scene(name)
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    ctx = lpe.Context(0)
    ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
    ctx.rigid_upload(b, v)
    ctx.sph_set_config(lpe.default_fluid_config())
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    ctx.world_set_coupling(None)
ctx.world_tick(1 / 120, n)
ctx.sync()
ctx.close()
print("done", name, n)
