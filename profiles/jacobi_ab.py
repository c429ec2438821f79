"""Round 5: the contact solve alone on the metric pile fixture
(tests/golden/rigid_pileM_t1.npz: 10,156 pairs / 29,706 contacts), the
reference's Gauss-Seidel (striped, default) and the opt-in Jacobi solver, 30
steps each from the same upload -- run under rocprofv3 --kernel-trace --stats
for k_pgs_stripes vs k_pgs_jacobi."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe  # noqa: E402
z = dict(np.load(os.path.join(ROOT, "tests", "golden", "rigid_pileM_t1.npz")))
ctx = lpe.Context(0)
out = {}
ITERS = int(os.environ.get("ITERS", z["pgs_iterations"]))          # (an iteration-count sweep: ITERS=...)
MODES = [int(m) for m in os.environ.get("MODES", "0,1").split(",")]
for mode in MODES:
    ctx.rigid_set_config(lpe.rigid_config(universe=float(z["universe"]), pgs_iterations=ITERS, pgsMode=mode))
    ts = []
    for _ in range(30):
        ctx.rigid_upload(z["before_rigid"], z["verts"])
        ctx.sync()
        t0 = time.perf_counter()
        st = ctx.rigid_step(stats=True)
        ctx.sync()
        ts.append(time.perf_counter() - t0)
    out[["gauss_seidel", "jacobi"][mode]] = {"step_ms_median": round(1e3 * float(np.median(ts)), 3),
                                             "contacts": st["contacts"], "iters": ITERS}
ctx.close()
print(json.dumps(out), flush=True)
