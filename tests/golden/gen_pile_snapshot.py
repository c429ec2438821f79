"""Settled pile of the metric scene M (tick 250 of the resident device tick:
the 4,096 pentagons resting in and on the SPH pool) for the rigid-path parity
test at scale and the bench's rigid microbench.  Generated on the MI355X with
this repository's own HIP path (not the reference):
    python tests/golden/gen_pile_snapshot.py   ->   gpurun_out/pile_M_t250.npz
then copied to tests/golden/."""
import importlib.util, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(ROOT, "little-physics-engine_amd")
def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path); mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod; spec.loader.exec_module(mod); return mod
lpe = _load("lpe", os.path.join(PKG, "lpe.py")); scenes = _load("scenes", os.path.join(PKG, "scenes.py"))
s = scenes.scene("M"); fl = s["fluid"]; bodies, verts = scenes.to_bodies(s["bodies"])
ctx = lpe.Context(0)
ctx.sph_set_config(lpe.default_fluid_config()); ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
ctx.rigid_upload(bodies, verts)
ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
ctx.world_set_coupling(None)
ctx.world_tick(1/120, 250); ctx.sync()
b = ctx.rigid_download()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "pile_M_t250.npz"), bodies=b, verts=np.asarray(verts))
print(len(b), b.dtype)
