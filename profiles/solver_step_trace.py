"""Per-colour-step times of k_pgs_colour / k_pos_colour on the rigid microbench fixture.

    LPE_LIB=profiles/_var/liblpe_pt.so python3 profiles/solver_step_trace.py

The library must be built with -DLPE_PTRACE (profiles/trace_build.sh rigid pt -DLPE_PTRACE)."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe
z = np.load(os.path.join(ROOT, "tests", "golden", "pile_M_t250.npz"))
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
ctx.rigid_upload(z["bodies"], z["verts"]); st = ctx.rigid_step()
ctx.rigid_upload(z["bodies"], z["verts"]); st = ctx.rigid_step()
L = lpe.lib(); L.lpe_ptrace.argtypes = [C.c_void_p]
buf = np.zeros(2 * 2048, np.uint64); L.lpe_ptrace(buf.ctypes.data)
ncol = st["pgsLevels"]
print("colours", ncol, "pairs", st["pairs"], "contacts", st["contacts"])
cb = buf[2048 + 1024: 2048 + 1024 + ncol + 1].astype(np.int64)
print("pairs per colour", np.diff(cb).tolist())
for w, name in ((0, "pgs"), (1, "pos")):
    t = buf[w * 2048:(w + 1) * 2048].astype(np.int64)
    n = 10 * ncol + 1
    d = np.diff(t[:n]) / 100.0
    print(name, "total us", round((t[n - 1] - t[0]) / 100.0, 1), "per-step mean", round(d.mean(), 2))
    print("  by colour (mean over iterations):", np.round(d.reshape(10, ncol).mean(0), 2).tolist())
