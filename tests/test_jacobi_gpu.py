"""The opt-in Jacobi contact solver on the device (lpe_rigid_config.pgsMode =
LPE_PGS_JACOBI, lpe_rigid.hip k_pgs_jacobi) through the C ABI.

Not the reference's arithmetic (its solveLcpPgs, contact_solver.cpp:381-440,
is sequential Gauss-Seidel and stays the default), so the device is checked
(1) bit for bit against the numpy restatement of the same Jacobi iteration
(tests/jacobi_restated.py) on every rigid fixture, bench-scale piles
included, (2) for the LCP invariants (lamN >= 0, |lamF| <= mu lamN) and
(3) for reproducibility (integer impulse sums: the same bits every run).
The default mode's impulses (lpe_rigid_download_impulses) are checked for the
same invariants."""
import glob
import os

import numpy as np
import pytest

from conftest import ROOT, lpe, scenes
import jacobi_restated as jr

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(ROOT, "tests", "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "rigid_*.npz")))
VEL = ("vx", "vy", "omega")
DT = 1.0 / 120.0


def _step(ctx, z, mode, iters=None):
    cfg = lpe.rigid_config(universe=float(z["universe"]),
                           pgs_iterations=int(z["pgs_iterations"]) if iters is None else iters, pgsMode=mode)
    ctx.rigid_set_config(cfg)
    ctx.rigid_upload(z["before_rigid"], z["verts"])
    ctx.rigid_step()
    _, cs = ctx.rigid_contacts()
    ln, lf = ctx.rigid_impulses()
    return cfg, cs, ctx.rigid_download(), ln, lf


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_jacobi_matches_restatement(gpu_ctx, path):
    z = dict(np.load(path))
    cfg, cs, out, ln, lf = _step(gpu_ctx, z, lpe.PGS_JACOBI)
    assert len(cs) > 0
    ref, rln, rlf = jr.solve(z["before_rigid"], cs, cfg.frictionCoeff, cfg.pgsIterations)
    for k in VEL:
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(ln, rln)
    np.testing.assert_array_equal(lf, rlf)
    assert np.all(ln >= 0) and np.all(np.abs(lf) <= np.float32(cfg.frictionCoeff) * ln)
    print(f"{os.path.basename(path)}: {len(cs)} contacts, Jacobi = restatement")


def test_jacobi_reproducible_and_gauss_seidel_invariants(gpu_ctx):
    z = dict(np.load(os.path.join(GOLDEN, "rigid_pileM_t1.npz")))
    _, cs1, o1, l1, f1 = _step(gpu_ctx, z, lpe.PGS_JACOBI)
    _, cs2, o2, l2, f2 = _step(gpu_ctx, z, lpe.PGS_JACOBI)
    for k in VEL:
        np.testing.assert_array_equal(o1[k], o2[k])
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(f1, f2)
    cfg, cs, out, ln, lf = _step(gpu_ctx, z, lpe.PGS_GAUSS_SEIDEL)
    assert len(ln) == len(cs) > 20000
    assert np.all(ln >= 0) and np.all(np.abs(lf) <= np.float32(cfg.frictionCoeff) * ln)
    assert ln.max() > 0


def test_jacobi_converges(gpu_ctx):
    """More iterations, closer to resting: the worst approaching normal
    velocity shrinks with the iteration count (pile8 fixture)."""
    z = dict(np.load(os.path.join(GOLDEN, "rigid_pile8_t60.npz")))
    worst = []
    for iters in (10, 100, 1000):
        _, cs, out, _, _ = _step(gpu_ctx, z, lpe.PGS_JACOBI, iters)
        worst.append(float(jr.normal_velocity(z["before_rigid"], out, cs).min()))
    assert worst[0] < worst[1] < worst[2] and worst[2] > -0.05, worst


def test_world_tick_jacobi_mode():
    """Scene M (fluid + 4,096 pentagons) advanced 40 world ticks with the
    Jacobi solver: no solver fault, finite state, and its last tick's
    impulses inside the friction cone."""
    s = scenes.scene("M")
    b, v = scenes.to_bodies(s["bodies"])
    ctx = lpe.Context(0)
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"], pgsMode=lpe.PGS_JACOBI))
        ctx.rigid_upload(b, v)
        fl = s["fluid"]
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
        ctx.world_tick(DT, 40)
        ctx.sync()
        out = ctx.rigid_download()
        for k in ("x", "y", "vx", "vy", "omega"):
            assert np.all(np.isfinite(out[k])), k
        ln, lf = ctx.rigid_impulses()
        assert np.all(ln >= 0) and np.all(np.abs(lf) <= np.float32(0.5) * ln)
    finally:
        ctx.close()
