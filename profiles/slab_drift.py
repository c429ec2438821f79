# Per-tick fluid displacement diagnostic behind profiles/r01/slab_drift.json:
# python profiles/slab_drift.py MW2 350 (single-domain world ticks, one GPU).
import os, sys, json, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import importlib.util
def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path); m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m; spec.loader.exec_module(m); return m
PKG = os.path.join(os.path.dirname(__file__), "..", "little-physics-engine_amd")
lpe = _load("lpe", os.path.join(PKG, "lpe.py")); scenes = _load("scenes", os.path.join(PKG, "scenes.py"))
name = sys.argv[1]; T = int(sys.argv[2])
s = scenes.scene(name); fl = s["fluid"]; bodies, verts = scenes.to_bodies(s["bodies"])
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=s["U"])); ctx.rigid_upload(bodies, verts)
ctx.sph_set_config(lpe.default_fluid_config())
ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
ctx.world_set_coupling(None)
prev = ctx.sph_download()
out = []
for t in range(T):
    ctx.world_tick(1.0 / 120.0, 1)
    cur = ctx.sph_download()
    dx = np.abs(cur["x"] - prev["x"]); sp = np.hypot(cur["vx"], cur["vy"])
    rec = dict(t=t, maxdx=float(dx.max()), n03=int((dx > 0.3).sum()), n01=int((dx > 0.1).sum()),
               maxv=float(sp.max()), xmin=float(cur["x"].min()), xmax=float(cur["x"].max()))
    if dx.max() > 0.1:
        i = int(dx.argmax()); rec.update(i=i, x0=float(prev["x"][i]), x1=float(cur["x"][i]), y1=float(cur["y"][i]))
    out.append(rec); prev = cur
    if t % 25 == 0 or dx.max() > 0.2: print(json.dumps(rec), flush=True)
ctx.close()
