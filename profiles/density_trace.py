"""Round 5: per-tile phase times of the tick's density pass (k_density<true>)
on the settled scene-M state (the last of a tick's ten launches).

    python3 profiles/snapshot.py --save 3000   (writes /tmp/lpe_snap.npz)
    LPE_LIB=profiles/_var/liblpe_ft.so python3 profiles/density_trace.py

The library must be built with -DLPE_FTRACE (profiles/trace_build.sh sph ft
-DLPE_FTRACE -DLPE_FTRACE_NOCPT).  Stamps (lpe_sph.hip DTR / DTRMAX): 0 start,
1 staged (barrier), 2 walk done (last wave), 3 tile filed (thread 0), 4 end
(last wave); 5 the tile's longest neighbour list, 6 its staged records."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe
SCENE = os.environ.get("SCENE")          # (C2 / C4: that config after its prep ticks instead of the M snapshot)
ctx = lpe.Context(0)
if SCENE:
    sys.path.insert(0, os.path.join(ROOT, "little-physics-engine_amd"))
    import scenes
    sc = scenes.scene(SCENE)
    b, v = scenes.to_bodies(sc["bodies"])
    fl = sc["fluid"]
    ctx.rigid_set_config(lpe.rigid_config(universe=sc["U"]))
    ctx.sph_set_config(lpe.default_fluid_config())
    ctx.rigid_upload(b, v)
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    ctx.world_set_coupling(None)
    ctx.world_tick(1 / 120, 30 if SCENE == "C2" else 90); ctx.sync()
    z = {"x": fl["x"]}
else:
    z = np.load("/tmp/lpe_snap.npz")
    ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
    ctx.sph_set_config(lpe.default_fluid_config())
    ctx.rigid_upload(z["bodies"], z["verts"])
    ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
    ctx.world_set_coupling(None)
    ctx.world_tick(1 / 120, 3); ctx.sync()
L = lpe.lib()
L.lpe_ftrace.argtypes = [C.c_int, C.c_void_p, C.c_int]
L.lpe_dtrace.argtypes = [C.c_void_p, C.c_int]
nb = (len(z["x"]) + 255) // 256
L.lpe_ftrace(1, None, 0)
ctx.world_tick(1 / 120, 1); ctx.sync()
buf = np.zeros(4096 * 8, np.uint64)
L.lpe_dtrace(buf.ctypes.data, buf.size)
L.lpe_ftrace(0, None, 0)
t = buf[: nb * 8].reshape(nb, 8).astype(np.int64)
ran = t[:, 0] > 0
t = t[ran]
t0 = t[:, 0].min()
us = lambda a, b: (t[:, b] - t[:, a]) / 100.0
start, end = (t[:, 0] - t0) / 100.0, (t[:, 4] - t0) / 100.0
rows = [("start", start), ("stage", us(0, 1)), ("walk", us(1, 2)), ("filing", us(2, 3)), ("write", us(3, 4)),
        ("end", end), ("longest list", t[:, 5].astype(float)), ("staged recs", t[:, 6].astype(float))]
print("tiles", int(ran.sum()), "of", nb, "kernel span us", end.max())
print("pctl          " + " ".join(f"{p:>8}" for p in ("0", "50", "90", "99", "100")))
for name, v in rows:
    print(f"{name:13s}", " ".join(f"{x:8.1f}" for x in np.percentile(v, [0, 50, 90, 99, 100])))
print("slowest tiles: tile start stage walk filing write end longest staged")
idx = np.flatnonzero(ran)
for k in np.argsort(-end)[:12]:
    print(idx[k], round(start[k], 1), round(us(0, 1)[k], 1), round(us(1, 2)[k], 1), round(us(2, 3)[k], 1),
          round(us(3, 4)[k], 1), round(end[k], 1), int(t[k, 5]), int(t[k, 6]))
ctx.close()
