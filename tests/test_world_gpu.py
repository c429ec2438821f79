"""GPU parity of the resident full tick (lpe_world_tick: FluidSystem with
rigid coupling, Boundary, Gravity, RigidBodyCollision, Rotation, Movement,
Sleep) against the whole-tick oracle (oracle/rigid_oracle.cpp:lpeo_world_tick
over oracle/sph_oracle.c).

After one tick the fluid is bit-identical; the rigid velocities carry the
float-atomic accumulation order of the fluid->rigid forces (reference:
float atomics too, metal:892-898), so bodies are compared at 1e-5 relative,
and later ticks (which feed those bodies back into the fluid) by the
north_star bar of 1e-5 relative on fp32 positions."""
import numpy as np
import pytest

from conftest import lpe, scenes

pytestmark = pytest.mark.gpu
DT = 1.0 / 120.0


def setup(ctx, name):
    s = scenes.scene(name)
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    rcfg = lpe.rigid_config(universe=s["U"])
    fcfg = lpe.default_fluid_config()
    ctx.sph_set_config(fcfg)
    ctx.rigid_set_config(rcfg)
    ctx.rigid_upload(b, v)
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    couple = np.arange(len(b) - 1, -1, -1, dtype=np.int32)
    ctx.world_set_coupling(couple)
    return s, fl, b, v, rcfg, fcfg, couple


@pytest.mark.parametrize("name", ["small64_8", "small96_12"])
def test_world_one_tick(gpu_ctx, oracle_mod, name):
    s, fl, b, v, rcfg, fcfg, couple = setup(gpu_ctx, name)
    gpu_ctx.world_tick(DT, 1)
    out = gpu_ctx.sph_download()
    bodies = gpu_ctx.rigid_download()
    p, rb = oracle_mod.world_tick(fcfg, rcfg, scenes.particles_aos(fl), b, v, couple, DT, 1)
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], p[:, col], err_msg=k)
    for k in ("x", "y", "angle"):
        np.testing.assert_allclose(bodies[k], rb[k], rtol=1e-6, atol=1e-7, err_msg=k)
    for k in ("vx", "vy", "omega"):
        np.testing.assert_allclose(bodies[k], rb[k], rtol=1e-5, atol=1e-5, err_msg=k)


def test_world_multi_tick(gpu_ctx, oracle_mod):
    s, fl, b, v, rcfg, fcfg, couple = setup(gpu_ctx, "small64_8")
    gpu_ctx.world_tick(DT, 5)
    out = gpu_ctx.sph_download()
    bodies = gpu_ctx.rigid_download()
    p, rb = oracle_mod.world_tick(fcfg, rcfg, scenes.particles_aos(fl), b, v, couple, DT, 5)
    for k, col in (("x", 0), ("y", 1)):
        ok = np.isclose(out[k], p[:, col], rtol=1e-5, atol=1e-5)
        assert ok.mean() > 0.99, (k, ok.mean())
    for k in ("x", "y"):
        np.testing.assert_allclose(bodies[k], rb[k], rtol=1e-5, atol=1e-4, err_msg=k)
    assert np.isfinite(out["vx"]).all() and np.isfinite(bodies["vx"]).all()
