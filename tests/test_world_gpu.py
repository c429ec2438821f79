"""GPU parity of the resident full tick (lpe_world_tick: FluidSystem with
rigid coupling, Boundary, Gravity, RigidBodyCollision, Rotation, Movement,
Sleep) against the whole-tick oracle (oracle/rigid_oracle.cpp:lpeo_world_tick
over oracle/sph_oracle.c).

The fluid is bit-identical tick after tick (the fluid->rigid accumulators
are exact sums rounded once on both sides, so nothing on the path depends on
thread order).  So are the bodies: their fp64 geometry uses the sine and
cosine device and oracle share (csrc/lpe_trig.h; the platform libms differ
in the last bit), the rest is IEEE-exact arithmetic
(correctly rounded division and square root, no FMA contraction)."""
import numpy as np
import pytest

from conftest import lpe, scenes

pytestmark = pytest.mark.gpu
DT = 1.0 / 120.0
BODY_STATE = ("x", "y", "angle", "vx", "vy", "omega", "sleep_counter")


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
    for k in BODY_STATE:
        np.testing.assert_array_equal(bodies[k], rb[k], err_msg=k)


def test_world_multi_tick(gpu_ctx, oracle_mod):
    """Five full ticks (the next tick's first sub-step is prelaunched beside
    the rigid solvers): the fluid stays bit-identical to the oracle."""
    s, fl, b, v, rcfg, fcfg, couple = setup(gpu_ctx, "small64_8")
    gpu_ctx.world_tick(DT, 5)
    out = gpu_ctx.sph_download()
    bodies = gpu_ctx.rigid_download()
    p, rb = oracle_mod.world_tick(fcfg, rcfg, scenes.particles_aos(fl), b, v, couple, DT, 5)
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], p[:, col], err_msg=k)
    for k in BODY_STATE:
        np.testing.assert_array_equal(bodies[k], rb[k], err_msg=k)


def _world_run(name, nticks, serial, fluid=True):
    import os
    os.environ["LPE_SERIAL_TICK"] = "1" if serial else "0"
    try:
        ctx = lpe.Context(0)
        try:
            s = scenes.scene(name)
            fl = s["fluid"]
            b, v = scenes.to_bodies(s["bodies"])
            ctx.sph_set_config(lpe.default_fluid_config())
            ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            ctx.rigid_upload(b, v)
            if fluid:
                ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
            ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
            ctx.world_tick(DT, nticks)
            return (ctx.sph_download() if fluid else None), ctx.rigid_download()
        finally:
            ctx.close()
    finally:
        os.environ.pop("LPE_SERIAL_TICK", None)


@pytest.mark.parametrize("name", ["small64_0", "small96_12"])
def test_world_prelaunch_equals_serial(name):
    """The overlapped tick (detection on a side stream, the next tick's first
    sub-step prelaunched beside the solvers) equals the systems run in order
    on one stream (LPE_SERIAL_TICK=1), bit for bit, fluid and bodies, over
    5 ticks: pins every cross-stream dependency of the prelaunch."""
    fa, ba = _world_run(name, 5, serial=False)
    fb, bb = _world_run(name, 5, serial=True)
    for k in ("x", "y", "vx", "vy", "density", "pressure"):
        np.testing.assert_array_equal(fa[k], fb[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega", "flags", "sleep_counter"):
        np.testing.assert_array_equal(ba[k], bb[k], err_msg=k)


def _bounce_bodies(b):
    """Bodies of small64_8 moved past the boundary margin (0.15 m) towards
    the walls, so the boundary system clamps and reflects them in the tick."""
    b = b.copy()
    b["x"][4], b["vx"][4] = 0.08, -0.5          # left margin, against the left wall
    b["y"][5], b["vy"][5] = 5.95, 0.8           # top margin
    b["x"][6], b["vx"][6] = 5.9, 0.3            # right margin
    return b


def _rigid_only_run(b, v, rcfg, nticks, serial):
    import os
    os.environ["LPE_SERIAL_TICK"] = "1" if serial else "0"
    try:
        ctx = lpe.Context(0)
        try:
            ctx.rigid_set_config(rcfg)
            ctx.rigid_upload(b, v)
            ctx.world_tick(DT, nticks)
            return ctx.rigid_download()
        finally:
            ctx.close()
    finally:
        os.environ.pop("LPE_SERIAL_TICK", None)


def test_world_overlap_equals_serial_with_bounces():
    """The world tick runs collision detection and colouring on a side stream
    during the fluid step, with the boundary clamp moved to the start of the
    tick (k_boundary_pos / k_boundary_vel); a rigid-only run (deterministic)
    must equal the serial systems order bit for bit, bounces included."""
    s = scenes.scene("small64_8")
    b, v = scenes.to_bodies(s["bodies"])
    b = _bounce_bodies(b)
    rcfg = lpe.rigid_config(universe=s["U"])
    a = _rigid_only_run(b, v, rcfg, 30, serial=False)
    r = _rigid_only_run(b, v, rcfg, 30, serial=True)
    for k in ("x", "y", "angle", "vx", "vy", "omega", "flags"):
        np.testing.assert_array_equal(a[k], r[k], err_msg=k)
    assert a["x"][4] >= 0.15 - 1e-12 and a["y"][5] <= 6.0 - 0.15 + 1e-12


def test_world_one_tick_bounces(gpu_ctx, oracle_mod):
    """One full tick with fluid, coupling and bodies inside the boundary
    margin against the whole-tick oracle (tolerances of test_world_one_tick)."""
    s = scenes.scene("small64_8")
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    b = _bounce_bodies(b)
    rcfg = lpe.rigid_config(universe=s["U"])
    fcfg = lpe.default_fluid_config()
    gpu_ctx.sph_set_config(fcfg)
    gpu_ctx.rigid_set_config(rcfg)
    gpu_ctx.rigid_upload(b, v)
    gpu_ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    couple = np.arange(len(b) - 1, -1, -1, dtype=np.int32)
    gpu_ctx.world_set_coupling(couple)
    gpu_ctx.world_tick(DT, 1)
    out = gpu_ctx.sph_download()
    bodies = gpu_ctx.rigid_download()
    p, rb = oracle_mod.world_tick(fcfg, rcfg, scenes.particles_aos(fl), b, v, couple, DT, 1)
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3)):
        np.testing.assert_array_equal(out[k], p[:, col], err_msg=k)
    for k in BODY_STATE:
        np.testing.assert_array_equal(bodies[k], rb[k], err_msg=k)


def test_world_one_tick_calls_equal_multi_tick(oracle_mod):
    """The drop-in path calls lpe_world_tick once per ECSSimulator::tick; the
    next tick's first sub-step is prelaunched at the end of every call (it
    writes only scratch), so downloads, stats and a probe between the calls
    see the end-of-tick state, and 5 one-tick calls equal one 5-tick call
    bit for bit."""
    s = scenes.scene("small64_8")
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    runs = []
    for mode in ("loop", "one"):
        ctx = lpe.Context(0)
        try:
            ctx.sph_set_config(lpe.default_fluid_config())
            ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            ctx.rigid_upload(b, v)
            ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
            ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
            if mode == "loop":
                mids = []
                for t in range(5):
                    ctx.world_tick(DT, 1)
                    mids.append(ctx.sph_download())        # joins the pending prelaunch
                    ctx.sph_stats()
                # the state after tick 1 is the oracle's after one tick
                p1, _ = oracle_mod.world_tick(lpe.default_fluid_config(), lpe.rigid_config(universe=s["U"]),
                                              scenes.particles_aos(fl), b, v,
                                              np.arange(len(b) - 1, -1, -1, dtype=np.int32), DT, 1)
                np.testing.assert_array_equal(mids[0]["x"], p1[:, 0])
                np.testing.assert_array_equal(mids[0]["vy"], p1[:, 3])
            else:
                ctx.world_tick(DT, 5)
            runs.append((ctx.sph_download(), ctx.rigid_download()))
        finally:
            ctx.close()
    (fa, ba), (fb, bb) = runs
    for k in ("x", "y", "vx", "vy", "density", "pressure"):
        np.testing.assert_array_equal(fa[k], fb[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        np.testing.assert_array_equal(ba[k], bb[k], err_msg=k)


def test_prelaunch_voided_by_probe_and_upload(gpu_ctx):
    """A probe (its own hash) and a re-upload between world ticks discard the
    pending prelaunch; the following ticks equal a fresh run's."""
    s = scenes.scene("small64_0")
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])

    def fresh(nt):
        ctx = lpe.Context(0)
        try:
            ctx.sph_set_config(lpe.default_fluid_config())
            ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            ctx.rigid_upload(b, v)
            ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
            ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
            ctx.world_tick(DT, nt)
            return ctx.sph_download()
        finally:
            ctx.close()
    want = fresh(3)
    ctx = lpe.Context(0)
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        ctx.rigid_upload(b, v)
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
        ctx.world_tick(DT, 2)
        ctx.sph_probe_density()                  # voids the prelaunch
        ctx.world_tick(DT, 1)
        got = ctx.sph_download()
        # a re-upload of the start state voids it too: 3 ticks again
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.rigid_upload(b, v)
        ctx.world_tick(DT, 3)
        again = ctx.sph_download()
    finally:
        ctx.close()
    for k in ("x", "y", "vx", "vy", "density"):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
        np.testing.assert_array_equal(again[k], want[k], err_msg=k)


_SERIAL_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from conftest import lpe, scenes
s = scenes.scene("small96_12")
fl = s["fluid"]
b, v = scenes.to_bodies(s["bodies"])
ctx = lpe.Context(0)
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
ctx.rigid_upload(b, v)
ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
ctx.world_tick(1.0 / 120.0, 6)
f = ctx.sph_download()
r = ctx.rigid_download()          # (raises on a cross-stream wait's watchdog)
np.savez(sys.argv[2], **{"f_" + k: f[k] for k in ("x", "y", "vx", "vy")},
         **{"r_" + k: r[k] for k in ("x", "y", "angle", "vx", "vy", "omega")})
ctx.close()
"""


def test_world_tick_with_serialised_dispatches(tmp_path):
    """The world tick's cross-stream waits are device polls (k_wait_flag)
    when the context's streams run kernels together, which a probe checks
    once per context; with every dispatch serialised (AMD_SERIALIZE_KERNEL=3,
    as under rocprofv3 counter collection) a poller would hold its queue until
    its watchdog, so the tick must fall back to events: same bits as the
    overlapped tick in this process, and no watchdog fault."""
    import os
    import subprocess
    import sys
    out = tmp_path / "serial.npz"
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3")
    tests_dir = os.path.dirname(os.path.abspath(__file__))
    subprocess.run([sys.executable, "-c", _SERIAL_SCRIPT, tests_dir, str(out)], env=env, check=True, timeout=240)
    f, r = _world_run("small96_12", 6, serial=False)
    z = np.load(out)
    for k in ("x", "y", "vx", "vy"):
        np.testing.assert_array_equal(z["f_" + k], f[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        np.testing.assert_array_equal(z["r_" + k], r[k], err_msg=k)
