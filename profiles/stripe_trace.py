"""Per-workgroup phase times of k_pgs_stripes / k_pos_stripes on the rigid
microbench fixture (tests/golden/pile_M_t250.npz).

    profiles/trace_build.sh rigid pt -DLPE_PTRACE
    LPE_LIB=profiles/_var/liblpe_pt.so python3 profiles/stripe_trace.py

Stamps (wall_clock64, 100 MHz) per workgroup: 0 kernel entry, 1 staged, then
per iteration: A start (after the wait + reload), A end, A published, B start,
B end, B published."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe
FIX = os.environ.get("FIXTURE")          # (a rigid_*.npz fixture instead of the metric pile, e.g. the C1 stack)
LIVE = os.environ.get("LIVE")            # (C1 / C3: the live scene after its settle, as small_probe.py runs it)
if LIVE:
    sys.path.insert(0, os.path.join(ROOT, "little-physics-engine_amd"))
    import scenes
    sc = scenes.rigid_scene(LIVE)
    b0, v0 = scenes.to_bodies(sc["bodies"])
    cfg = lpe.rigid_config(universe=sc["U"], pgs_iterations=sc["pgs_iterations"])
    c0 = lpe.Context(0)
    c0.rigid_set_config(cfg)
    c0.rigid_upload(b0, v0)
    c0.world_tick(1 / 120, 240 if LIVE == "C3" else 560)
    z = {"bodies": c0.rigid_download(), "verts": v0}
    c0.close()
elif FIX:
    z = dict(np.load(os.path.join(ROOT, "tests", "golden", FIX)))
    z["bodies"] = z["before_rigid"]
    cfg = lpe.rigid_config(universe=float(z["universe"]), pgs_iterations=int(z["pgs_iterations"]))
else:
    z = np.load(os.path.join(ROOT, "tests", "golden", "pile_M_t250.npz"))
    cfg = lpe.rigid_config(universe=32.0)
ctx = lpe.Context(0)
ctx.rigid_set_config(cfg)
for _ in range(3):
    ctx.rigid_upload(z["bodies"], z["verts"]); st = ctx.rigid_step()
print("pairs", st["pairs"], "contacts", st["contacts"], "colours", st["pgsLevels"])
L = lpe.lib(); L.lpe_strace.argtypes = [C.c_void_p]
buf = np.zeros(2 * 32 * 64, np.uint64); L.lpe_strace(buf.ctypes.data)
buf = buf.reshape(2, 32, 64).astype(np.int64)
it = cfg.pgsIterations
for w, name in ((0, "pgs"), (1, "pos")):
    t = buf[w]
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0
    print(f"{name}: entry spread {rel[:, 0].max():.2f} us, staged by {rel[:, 1].max():.2f} us, "
          f"end {rel[:, 7 + 6 * (it - 1)].max():.2f} us")
    ph = rel[:, 2:2 + 6 * it].reshape(32, it, 6)
    A = ph[:, :, 1] - ph[:, :, 0]; B = ph[:, :, 4] - ph[:, :, 3]
    pubA = ph[:, :, 2] - ph[:, :, 1]; waitB = ph[:, :, 3] - ph[:, :, 2]; pubB = ph[:, :, 5] - ph[:, :, 4]
    waitA = ph[:, 1:, 0] - ph[:, :-1, 5]
    for nm, a in (("A", A), ("B", B), ("pubA", pubA), ("waitB", waitB), ("pubB", pubB), ("waitA", waitA)):
        print(f"  {nm:6s} mean {a.mean():6.2f}  max {a.max():6.2f}  per-WG mean over it: "
              f"{np.round(a.mean(1)[:8], 2).tolist()}")
    print("  WG0 timeline it0-2:", np.round(ph[0, :3].ravel(), 2).tolist())
    print("  WG1 timeline it0-2:", np.round(ph[1, :3].ravel(), 2).tolist())
st = buf[0]
na, nbs, npr = st[:, 61], st[:, 62], st[:, 63]
used = npr > 0
print("pgs steps per WG: A", na[used].tolist(), "B", nbs[used].tolist(), "pairs", npr[used].tolist())
t = buf[0]; t0 = t[:, 0].min(); rel = (t - t0) / 100.0
ph = rel[:, 2:2 + 6 * it].reshape(32, it, 6)
A = (ph[:, :, 1] - ph[:, :, 0]).mean(1); B = (ph[:, :, 4] - ph[:, :, 3]).mean(1)
print("pgs us per step: A", np.round(A[used] / np.maximum(na[used], 1), 2).tolist())
print("pgs us per step: B", np.round(B[used] / np.maximum(nbs[used], 1), 2).tolist())

