"""GPU parity of the device Barnes-Hut (lpe_bh_step, csrc/lpe_bh.hip) against
the restatement (oracle/bh_oracle.c, itself pinned to the reference's
barnes_hut.cpp by tests/test_oracle_bh.py) and against the reference
fixtures directly.  Bar: bit-exact fp64 velocities and identical tree
statistics (nodes, depth, inserted) - the device replays every node's
insertion sequence, so the centres of mass are the reference's bit for bit.

The larger scenes go past the reference's 1024-node pool, where the
reference itself is undefined (gen_bh_golden.py); there the restatement is
the bar."""
import glob
import os

import numpy as np
import pytest

from conftest import ROOT, lpe, scenes

pytestmark = pytest.mark.gpu
FIXTURES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "bh_*.npz")))


def device(ctx, cfg, x, y, vx, vy, m, dt, hv=None):
    ctx.bh_upload(x, y, vx, vy, m, hv)
    st = ctx.bh_step(cfg, dt)
    gx, gy = ctx.bh_download()
    return gx, gy, st


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_device_matches_reference_fixture(path, gpu_ctx):
    z = dict(np.load(path))
    o = z["order"]
    cfg = lpe.BhConfig(theta=float(z["theta"]), small_mass_threshold=float(z["small_mass_threshold"]),
                       universe_size=float(z["universe"]), softener=float(z["softener"]), G=float(z["G"]))
    gx, gy, _ = device(gpu_ctx, cfg, z["x"][o], z["y"][o], z["vx0"][o], z["vy0"][o], z["m"][o], float(z["dt"]),
                       z["has_vel"][o])
    ex, ey = np.empty_like(gx), np.empty_like(gy)
    ex[o], ey[o] = gx, gy
    np.testing.assert_array_equal(ex, z["vx"])
    np.testing.assert_array_equal(ey, z["vy"])


@pytest.mark.parametrize("kind,n", [("disk", 1000), ("disk", 20000), ("clustered", 4096), ("clustered", 65536)])
def test_device_matches_restatement(kind, n, gpu_ctx, oracle_mod):
    s = scenes.bh_disk(n) if kind == "disk" else scenes.bh_clustered(n)
    hv = np.ones(n, np.uint8)
    hv[::11] = 0
    cfg = lpe.bh_config(s["U"], softener=s["softener"])
    rx, ry, rst = oracle_mod.bh_step(cfg, s["x"], s["y"], s["vx"], s["vy"], s["m"], 0.75, has_vel=hv)
    gx, gy, gst = device(gpu_ctx, cfg, s["x"], s["y"], s["vx"], s["vy"], s["m"], 0.75, hv)
    assert gst == rst
    np.testing.assert_array_equal(gx, rx)
    np.testing.assert_array_equal(gy, ry)


def test_device_early_exit_and_no_threshold(gpu_ctx, oracle_mod):
    s = scenes.bh_clustered(3000, seed=8)
    m = np.full(3000, 10.0)
    cfg = lpe.bh_config(s["U"])
    gx, gy, st = device(gpu_ctx, cfg, s["x"], s["y"], s["vx"], s["vy"], m, 1.0)
    assert st["skipped"] == 1
    np.testing.assert_array_equal(gx, s["vx"])
    cfg0 = lpe.bh_config(s["U"], theta=0.3, small_mass_threshold=0.0)   # no skip at all
    rx, ry, rst = oracle_mod.bh_step(cfg0, s["x"], s["y"], s["vx"], s["vy"], m, 1.0)
    gx, gy, gst = device(gpu_ctx, cfg0, s["x"], s["y"], s["vx"], s["vy"], m, 1.0)
    assert gst == rst and gst["skipped"] == 0
    np.testing.assert_array_equal(gx, rx)
    np.testing.assert_array_equal(gy, ry)


def test_device_coincident_bodies(gpu_ctx, oracle_mod):
    # two bodies at one point: the boxes halve until bx + size no longer
    # contains them in fp64 (depth 55 here), where the reference's contains
    # test drops both (barnes_hut.hpp contains(), barnes_hut.cpp:139-141)
    x = np.array([10.0, 10.0, 30.0]); y = np.array([10.0, 10.0, 5.0]); m = np.array([1e6, 1e6, 1e6])
    v = np.zeros(3)
    cfg = lpe.bh_config(64.0)
    rx, ry, rst = oracle_mod.bh_step(cfg, x, y, v, v, m, 1.0)
    gx, gy, gst = device(gpu_ctx, cfg, x, y, v, v, m, 1.0)
    assert gst == rst and rst["depth"] == 55
    np.testing.assert_array_equal(gx, rx)
    np.testing.assert_array_equal(gy, ry)


def test_device_empty_and_single(gpu_ctx):
    gpu_ctx.bh_upload([], [], [], [], [])
    assert gpu_ctx.bh_step(lpe.bh_config(10.0), 1.0)["nodes"] == 0
    gx, gy, st = device(gpu_ctx, lpe.bh_config(10.0), [5.0], [5.0], [1.0], [2.0], [1e9], 1.0)
    assert st["nodes"] == 1 and gx[0] == 1.0 and gy[0] == 2.0


def _planet_world(n=48, seed=4, U=2000.0):
    """Massive circles far apart (no contacts): only Barnes-Hut couples them."""
    rng = np.random.default_rng(seed)
    b = scenes.Bodies()
    scenes.add_walls(b, U)
    g = int(np.ceil(np.sqrt(n)))
    for i in range(n):
        x = 200.0 + (i % g) * 150.0 + rng.uniform(-20, 20)
        y = 200.0 + (i // g) * 150.0 + rng.uniform(-20, 20)
        b.add(x=x, y=y, vx=rng.normal(0, 0.1), vy=rng.normal(0, 0.1), mass=10.0 ** rng.uniform(11, 14),
              circle=True, radius=1.0, shape_size=1.0, has_angvel=True, has_inertia=True, inertia=1.0)
    return scenes.to_bodies(b), U


def test_world_tick_runs_barnes_hut(gpu_ctx, oracle_mod):
    """lpe_world_tick's BarnesHutSystem (position 5 of sim.cpp:107-114) equals the
    systems run one by one: boundary + gravity, collision, Barnes-Hut on the
    bodies in EnTT view order (last body first, walls excluded) through the
    restatement, rotation + movement + sleep."""
    (bodies, verts), U = _planet_world()
    cfg = lpe.rigid_config(universe=U)
    dt = 1.0 / 120.0
    w = lpe.Context(0)
    try:
        w.rigid_set_config(cfg)
        w.rigid_upload(bodies, verts)
        w.world_tick(dt, 1)
        got = w.rigid_download()
    finally:
        w.close()
    m = lpe.Context(0)
    try:
        m.rigid_set_config(cfg)
        m.rigid_upload(bodies, verts)
        m.rigid_integrate(lpe.SYS_BOUNDARY | lpe.SYS_GRAVITY, dt)
        m.rigid_step(stats=False)
        mid = m.rigid_download()
        sel = [i for i in range(len(mid))[::-1]
               if (mid[i]["flags"] & lpe.BODY_HAS_MASS) and not (mid[i]["flags"] & lpe.BODY_BOUNDARY)]
        bc = lpe.bh_config(U)
        vx, vy, st = oracle_mod.bh_step(bc, mid["x"][sel], mid["y"][sel], mid["vx"][sel], mid["vy"][sel],
                                        mid["mass"][sel], dt)
        assert st["skipped"] == 0 and st["nodes"] > len(sel)
        mid["vx"][sel] = vx
        mid["vy"][sel] = vy
        m.rigid_upload(mid, verts)
        m.rigid_integrate(lpe.SYS_ROTATION | lpe.SYS_MOVEMENT | lpe.SYS_SLEEP, dt)
        ref = m.rigid_download()
    finally:
        m.close()
    assert np.any(ref["vx"] != bodies["vx"])
    for k in ("x", "y", "vx", "vy", "angle", "omega"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_world_tick_barnes_hut_off_and_fluid_guard(gpu_ctx):
    (bodies, verts), U = _planet_world(n=16)
    dt = 1.0 / 120.0
    a, b = lpe.Context(0), lpe.Context(0)
    try:
        for c in (a, b):
            c.rigid_set_config(lpe.rigid_config(universe=U))
            c.rigid_upload(bodies, verts)
        b.world_set_barnes_hut(False)
        a.world_tick(dt, 1)
        b.world_tick(dt, 1)
        assert np.any(a.rigid_download()["vx"] != b.rigid_download()["vx"])
    finally:
        a.close()
        b.close()
    # a heavy world with fluid particles: strict mode only (fails loudly)
    hb = scenes.Bodies()
    scenes.add_walls(hb, 20.0)
    for i in range(4):
        hb.add(x=4.0 + 4.0 * i, y=6.0, mass=1e12, circle=True, radius=0.5, shape_size=0.5, has_angvel=True,
               has_inertia=True)
    hbod, hverts = scenes.to_bodies(hb)
    fl = scenes.fluid_lattice(np.random.default_rng(1), 8, 8, 8.0, 14.0)
    c = lpe.Context(0)
    try:
        c.rigid_set_config(lpe.rigid_config(universe=20.0))
        c.rigid_upload(hbod, hverts)
        c.sph_set_config(lpe.default_fluid_config())
        c.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        with pytest.raises(lpe.LpeError, match="STATE|strict"):
            c.world_tick(dt, 1)
    finally:
        c.close()
