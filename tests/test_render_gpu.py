"""GPU parity of the screen-space fluid density field (lpe_render_density)
against the restatement (oracle/render_oracle.c).  The device sums each
cell's particles in bin order instead of particle order, so the density -
and through it the maximum and the normalised grid - agree to fp32
summation rounding: the bar is 1e-5 relative for the maximum and 1e-5
absolute for the normalised grid (values in [0, 1])."""
import numpy as np
import pytest

from conftest import lpe, scenes

pytestmark = pytest.mark.gpu
DT = 1.0 / 120.0


def _fluid_ctx(name):
    s = scenes.scene(name)
    fl = s["fluid"]
    ctx = lpe.Context(0)
    ctx.sph_set_config(lpe.default_fluid_config())
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    ctx.sph_upload_rigids(scenes.gather_rigids(s["bodies"]))
    return ctx, fl


def _check(ctx, x, y, oracle_mod, w, h, origin, cs=0.01, sr=10.0):
    got, mx = ctx.render_density(w, h, cs, origin, sr)
    ref = oracle_mod.render_density(x, y, w, h, cs, origin, sr)
    assert ref["max"] > 0
    assert abs(mx - ref["max"]) <= 1e-5 * ref["max"], (mx, ref["max"])
    np.testing.assert_allclose(got, ref["normalized"], rtol=0, atol=1e-5)
    return got


def test_render_density_lattice(oracle_mod):
    ctx, fl = _fluid_ctx("small64_0")
    try:
        _check(ctx, np.float32(fl["x"]), np.float32(fl["y"]), oracle_mod, 200, 200, (2.0, 4.0))
    finally:
        ctx.close()


def test_render_density_after_ticks_leaves_state_alone(oracle_mod):
    """Rendering between ticks sorts the current positions into the grid hash
    but does not change the simulation: two ticks with a render in between
    are bit-identical to two ticks without."""
    ctx, fl = _fluid_ctx("small64_8")
    ref_ctx, _ = _fluid_ctx("small64_8")
    try:
        ctx.sph_step(DT)
        ref_ctx.sph_step(DT)
        st = ctx.sph_download()
        _check(ctx, st["x"], st["y"], oracle_mod, 240, 220, (1.9, 3.9))
        ctx.sph_step(DT)
        ref_ctx.sph_step(DT)
        a, b = ctx.sph_download(), ref_ctx.sph_download()
        for k in ("x", "y", "vx", "vy", "density", "pressure"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    finally:
        ctx.close()
        ref_ctx.close()


def test_render_density_empty_and_args():
    ctx = lpe.Context(0)
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(*[np.zeros(0, np.float32)] * 5)
        g, mx = ctx.render_density(16, 8)
        assert mx == 0.0 and g.shape == (8, 16) and not g.any()
        with pytest.raises(lpe.LpeError):
            ctx.render_density(0, 8)
    finally:
        ctx.close()
