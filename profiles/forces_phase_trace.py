"""Per-block phase times of k_forces_couple on the settled scene-M state.

    python3 profiles/snapshot.py --save 3000   (writes /tmp/lpe_snap.npz)
    LPE_LIB=profiles/_var/liblpe_ft.so python3 profiles/forces_phase_trace.py

The library must be built with -DLPE_FTRACE (profiles/trace_build.sh sph ft -DLPE_FTRACE)."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe
z = np.load("/tmp/lpe_snap.npz")
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_upload(z["bodies"], z["verts"])
ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
ctx.world_set_coupling(None)
ctx.world_tick(1 / 120, 3); ctx.sync()
L = lpe.lib()
L.lpe_ftrace.argtypes = [C.c_int, C.c_void_p, C.c_int]
buf = np.zeros(4096 * 8, np.uint64)
L.lpe_ftrace(1, None, 0)
ctx.world_tick(1 / 120, 1); ctx.sync()
L.lpe_ftrace(0, buf.ctypes.data, buf.size)
nb = (len(z["x"]) + 255) // 256
t = buf[: nb * 8].reshape(nb, 8).astype(np.int64)
t0 = t[:, 0].min()
st, a, b, e, pairs = (t[:, 0] - t0) / 100.0, (t[:, 1] - t[:, 0]) / 100.0, (t[:, 2] - t[:, 1]) / 100.0, (t[:, 3] - t[:, 2]) / 100.0, t[:, 4]
b = np.where(t[:, 2] > 0, b, 0); e = np.where(t[:, 2] > 0, e, (t[:, 3] - t[:, 1]) / 100.0)
end = (t[:, 3] - t0) / 100.0
print("kernel span us", end.max(), "blocks", nb)
for name, v in (("start", st), ("nbr+scan", a), ("pairs", b), ("fold+write", e), ("end", end), ("pairs/blk", pairs)):
    q = np.percentile(v, [0, 50, 90, 99, 100])
    print(f"{name:10s}", " ".join(f"{x:8.1f}" for x in q))
i = np.argsort(-end)[:8]
nl = (t[:, 5] - t[:, 0]) / 100.0
print("nbr-loop(max wave)", " ".join(f"{x:8.1f}" for x in np.percentile(nl, [0, 50, 90, 99, 100])))
print("max ncount/blk", " ".join(f"{x:8.1f}" for x in np.percentile(t[:, 6], [0, 50, 90, 99, 100])))
print("max cand/blk", " ".join(f"{x:8.1f}" for x in np.percentile(t[:, 7], [0, 50, 90, 99, 100])))
print("slowest blocks: start, nbrloop, nbr+count, pairs, fold, npairs, maxcnt, maxcand")
for k in i: print(k, round(st[k], 1), round(nl[k], 1), round(a[k], 1), round(b[k], 1), round(e[k], 1), pairs[k], t[k, 6], t[k, 7])
