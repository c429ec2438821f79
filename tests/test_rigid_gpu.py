"""GPU parity of the rigid path (HIP, through the C ABI).

(1) Against the REFERENCE: golden fixtures recorded from the reference's own
    sources (tests/golden/rigid_*.npz); the device step replays the
    reference's pair order (quadtree) and PGS order (unordered_map) and must
    reproduce contacts, post-PGS velocities and post-position-solver poses.
(2) Against the restatement (oracle/rigid_oracle.cpp) in the canonical order
    the device runs by default, including the C3-scale pile.
Bar: bit-exact contact-pair lists (and contact topology a, b, pair); the
device uses the reference's operation order with no FMA contraction, but its
fp64 cos/sin (ROCm device libm) can differ from glibc's by an ulp, so contact
geometry is compared at 1e-12 relative / 1e-13 absolute (the bar of the CPU
restatement against the same fixtures, test_portable_trig_within_an_ulp_of_libm:
at the bench-scale piles a handful of near-zero penetrations and normal
components differ by 1-3e-14 m) and the solver outputs at 1e-7
(positions, fp64) / 1e-5 (velocities, fp32 rows) -- the north_star bar is
1e-5 relative.  Integrators use no transcendental and stay bit-exact.
"""
import glob
import os

import numpy as np
import pytest

from conftest import ROOT, lpe, scenes

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(ROOT, "tests", "golden")
FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "rigid_*.npz")))
DT = 1.0 / 120.0


def load(path):
    z = dict(np.load(path))
    cfg = lpe.rigid_config(universe=float(z["universe"]), pgs_iterations=int(z["pgs_iterations"]))
    return z, cfg


GEOM = ("nx", "ny", "pen", "px", "py")
POSE = ("x", "y", "angle")
VEL = ("vx", "vy", "omega")


def same(a, b, keys, rtol=0.0, atol=0.0):
    for k in keys:
        if rtol == 0.0:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        else:
            np.testing.assert_allclose(a[k], b[k], rtol=rtol, atol=atol, err_msg=k)


def close_state(out, ref):
    """Device vs the restatement in the canonical order: bit for bit (the
    trigonometry is the implementation both share, csrc/lpe_trig.h)."""
    same(out, ref, POSE)
    same(out, ref, VEL)


def ref_state(out, ref):
    """Device vs the reference's own fixture (its platform libm rounds sin/cos
    in the last bit differently): poses 1e-7, velocities 1e-5 relative."""
    same(out, ref, POSE, rtol=1e-7, atol=1e-9)
    same(out, ref, VEL, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_reference_orders_replay(gpu_ctx, path):
    z, cfg = load(path)
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(z["before_rigid"], z["verts"])
    st = gpu_ctx.rigid_step(pairs=z["pairs"], pgs_order=z["pgs_order"] if len(z["contacts"]) else None)
    pairs, cs = gpu_ctx.rigid_contacts()
    ref = z["contacts"]
    assert st["contacts"] == len(ref)
    same(cs, ref, ("a", "b"))
    same(cs, ref, GEOM, rtol=1e-12, atol=1e-13)
    out = gpu_ctx.rigid_download()
    if len(ref):
        ref_state(out, z["after_pos"])


def eid_pair_keys(bodies, pairs):
    e = bodies["eid"].astype(np.int64)
    a, b = e[pairs[:, 0]], e[pairs[:, 1]]
    return np.sort(np.minimum(a, b) * (1 << 32) + np.maximum(a, b))


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_device_own_detection_matches_reference(gpu_ctx, path):
    """The device's OWN canonical detection (no replayed order) against the
    reference's: the broadphase pair set equal to the reference quadtree's
    (broadphase.cpp:233-295) as a set of entity pairs, bit for bit, and every
    pair's narrowphase contacts (narrowphase.cpp:352-420) equal to the
    reference's for that pair, in order, geometry within 1e-12 rel / 1e-13 abs (the device's
    trigonometry vs glibc, test_portable_trig_within_an_ulp_of_libm).  The
    bench-scale fixtures (rigid_pileM_t1: 10,156 pairs / 29,706 contacts,
    rigid_C3_t240: 9,462 / 27,443) are one reference tick on the states the
    bench times."""
    z, cfg = load(path)
    pre = z["before_rigid"]
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(pre, z["verts"])
    st = gpu_ctx.rigid_step()
    pairs, cs = gpu_ctx.rigid_contacts()
    np.testing.assert_array_equal(eid_pair_keys(pre, pairs), eid_pair_keys(pre, z["pairs"]))
    ref = z["contacts"]
    assert st["contacts"] == len(ref) == len(cs)
    # group both contact lists by (a, b): narrowphase order within a pair is the
    # reference's clip order, the pairs' order differs (quadtree vs entity order)
    def grouped(c):
        key = c["a"].astype(np.int64) * len(pre) + c["b"]
        o = np.argsort(key, kind="stable")
        return key[o], c[o]
    kd, cd = grouped(cs)
    kr, cr = grouped(ref)
    np.testing.assert_array_equal(kd, kr)
    same(cd, cr, GEOM, rtol=1e-12, atol=1e-13)
    print(f"{os.path.basename(path)}: {len(pairs)} pairs, {len(cs)} contacts equal to the reference")


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_canonical_step_matches_restatement(gpu_ctx, oracle_mod, path):
    z, cfg = load(path)
    pre = z["before_rigid"]
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(pre, z["verts"])
    st = gpu_ctx.rigid_step()
    pairs, cs = gpu_ctx.rigid_contacts()
    ref_pairs = oracle_mod.broadphase(cfg, pre, z["verts"])
    np.testing.assert_array_equal(pairs, ref_pairs)          # bit-exact pair list, canonical order
    ref_cs = oracle_mod.narrowphase(pre, z["verts"], ref_pairs)
    same(cs, ref_cs, ("a", "b", "pair"))
    same(cs, ref_cs, GEOM)                                    # (shared trigonometry: exact)
    out = gpu_ctx.rigid_download()
    ref, rst = oracle_mod.rigid_update(cfg, pre, z["verts"])
    close_state(out, ref)
    assert st["pairs"] == rst.pairs and st["contacts"] == rst.contacts


@pytest.mark.parametrize("path", FIXTURES[:2], ids=[os.path.basename(p) for p in FIXTURES[:2]])
def test_integrators_match_reference(gpu_ctx, path):
    z, cfg = load(path)
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(z["tick_start"], z["verts"])
    gpu_ctx.rigid_integrate(lpe.SYS_BOUNDARY | lpe.SYS_GRAVITY, DT)
    same(gpu_ctx.rigid_download(), z["before_rigid"], ("x", "y", "angle", "vx", "vy", "omega"))
    gpu_ctx.rigid_upload(z["after_pos"], z["verts"])
    gpu_ctx.rigid_integrate(lpe.SYS_ROTATION | lpe.SYS_MOVEMENT | lpe.SYS_SLEEP, DT)
    same(gpu_ctx.rigid_download(), z["final"],
         ("x", "y", "angle", "vx", "vy", "omega", "sleep_counter", "flags"))


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_colour_order_matches_restatement(gpu_ctx, oracle_mod, path):
    """The canonical solver order (striped Gauss-Seidel, round 3): every
    pair's step on the device equals the restated one (integer work,
    bit-exact) and every step is proper: no movable body appears twice."""
    z, cfg = load(path)
    pre = z["before_rigid"]
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(pre, z["verts"])
    st = gpu_ctx.rigid_step()
    pairs, cs = gpu_ctx.rigid_contacts()
    col, ncol = gpu_ctx.rigid_colours()
    _, ref_col, ref_ncol, _ = oracle_mod.stripe_order(pre, cs, len(pairs))
    np.testing.assert_array_equal(col, ref_col)
    assert ncol == ref_ncol == st["pgsLevels"]
    inf = ((pre["flags"] & lpe.BODY_HAS_MASS) != 0) & (pre["mass"] > 1e29)
    rot = ((pre["flags"] & lpe.BODY_HAS_INERTIA) != 0) & (pre["inertia"] > 1e-12) & (pre["inertia"] < 1e29)
    movable = ~inf | rot
    for c in range(ncol):
        sel = pairs[col == c]
        ends = np.concatenate([sel[movable[sel[:, 0]], 0], sel[movable[sel[:, 1]], 1]])
        assert len(np.unique(ends)) == len(ends), f"colour {c} reuses a movable body"


def test_c3_pile_canonical(gpu_ctx, oracle_mod):
    """C3-scale pile (4096 polygons + 4 walls, 16 PGS iterations): warm the
    pile on the CPU restatement, then one RigidBodyCollisionSystem::update on
    the device against the restatement."""
    s = scenes.rigid_scene("C3")
    b, v = scenes.to_bodies(s["bodies"])
    cfg = lpe.rigid_config(universe=s["U"], pgs_iterations=16)
    for _ in range(40):
        b, _ = oracle_mod.rigid_tick(cfg, b, v, DT)
    b = oracle_mod.integrate(cfg, b, "boundary")
    b = oracle_mod.integrate(cfg, b, "gravity", DT)
    ref, rst = oracle_mod.rigid_update(cfg, b, v)
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(b, v)
    st = gpu_ctx.rigid_step()
    assert st["pairs"] == rst.pairs and st["contacts"] == rst.contacts and rst.contacts > 1000
    print(f"C3 pile: {st['pairs']} pairs, {st['contacts']} contacts, {st['pgsLevels']} colours")
    out = gpu_ctx.rigid_download()
    close_state(out, ref)


def test_metric_pile_canonical(gpu_ctx, oracle_mod):
    """The metric scene's own settled pile (scene M at tick 250, 4,096
    pentagons + walls, ~10k pairs / ~30k contacts: tests/golden/pile_M_t250.npz)
    through one RigidBodyCollisionSystem::update on the device against the
    restatement: the same broadphase pairs and contacts, the same canonical
    colouring, and the solved state within the rigid bars."""
    z = np.load(os.path.join(GOLDEN, "pile_M_t250.npz"))
    b, v = z["bodies"], z["verts"]
    cfg = lpe.rigid_config(universe=32.0)
    ref, rst = oracle_mod.rigid_update(cfg, b, v)
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(b, v)
    st = gpu_ctx.rigid_step()
    assert st["pairs"] == rst.pairs and st["contacts"] == rst.contacts and rst.contacts > 20000
    pairs, cs = gpu_ctx.rigid_contacts()
    col, ncol = gpu_ctx.rigid_colours()
    _, ref_col, ref_ncol, ns = oracle_mod.stripe_order(b, cs, len(pairs))
    np.testing.assert_array_equal(col, ref_col)
    assert ncol == ref_ncol and ns >= 16, (ncol, ns)
    close_state(gpu_ctx.rigid_download(), ref)


def test_multi_tick_device_matches_restatement(gpu_ctx, oracle_mod):
    """20 full rigid ticks resident on the device (Boundary, Gravity,
    collision, Rotation, Movement, Sleep) against the restatement."""
    s = scenes.rigid_scene("mix8")
    b, v = scenes.to_bodies(s["bodies"])
    cfg = lpe.rigid_config(universe=s["U"])
    gpu_ctx.rigid_set_config(cfg)
    gpu_ctx.rigid_upload(b, v)
    ref = b
    for _ in range(20):
        gpu_ctx.rigid_integrate(lpe.SYS_BOUNDARY | lpe.SYS_GRAVITY, DT)
        gpu_ctx.rigid_step(stats=False)
        gpu_ctx.rigid_integrate(lpe.SYS_ROTATION | lpe.SYS_MOVEMENT | lpe.SYS_SLEEP, DT)
        ref, _ = oracle_mod.rigid_tick(cfg, ref, v, DT)
    out = gpu_ctx.rigid_download()
    close_state(out, ref)
    same(out, ref, ("sleep_counter", "flags"))


def test_pair_buffer_grow_and_redo(oracle_mod):
    """Regression for the pair-buffer overflow fixed in round 1 (an
    out-of-bounds write on the first step of a larger pile): with the buffers
    deliberately sized for 16 pairs / 64 contacts, the step on the metric
    pile (~10k pairs) must grow them, redo its detection and still match the
    restatement exactly as test_metric_pile_canonical does."""
    z = np.load(os.path.join(GOLDEN, "pile_M_t250.npz"))
    b, v = z["bodies"], z["verts"]
    cfg = lpe.rigid_config(universe=32.0)
    ref, rst = oracle_mod.rigid_update(cfg, b, v)
    ctx = lpe.Context(0)
    try:
        ctx.rigid_set_config(cfg)
        ctx.rigid_upload(b, v)
        ctx.rigid_reserve(16, 64)
        assert ctx.rigid_buffer_info()["pairs"] == 16
        st = ctx.rigid_step()
        info = ctx.rigid_buffer_info()
        out = ctx.rigid_download()
    finally:
        ctx.close()
    assert info["regrows"] >= 2 and info["pairs"] >= rst.pairs and info["contacts"] >= rst.contacts, info
    assert st["pairs"] == rst.pairs and st["contacts"] == rst.contacts
    close_state(out, ref)


def test_pair_buffer_grow_in_world_tick():
    """The same overflow inside the world tick (detection on the side stream,
    rigid_tick_finish redoes it): bodies equal a run with roomy buffers."""
    z = np.load(os.path.join(GOLDEN, "pile_M_t250.npz"))
    b, v = z["bodies"], z["verts"]
    outs = []
    for tiny in (True, False):
        ctx = lpe.Context(0)
        try:
            ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
            ctx.rigid_upload(b, v)
            if tiny:
                ctx.rigid_reserve(8, 32)
            ctx.world_tick(DT, 3)
            outs.append((ctx.rigid_download(), ctx.rigid_buffer_info()))
        finally:
            ctx.close()
    assert outs[0][1]["regrows"] >= 1
    for k in ("x", "y", "angle", "vx", "vy", "omega", "flags"):
        np.testing.assert_array_equal(outs[0][0][k], outs[1][0][k], err_msg=k)


def test_lagged_overflow_reported_and_contained():
    """a pair/contact overflow in a tick whose counts are checked
    after the fact (lagged detection) must stay inside the buffers and fail
    loudly.  256 pentagons 0.3 m apart (no contact) in columns that close on
    each other at 14 m/s: the first, synchronous tick finds no pair and arms
    the lagged mode on buffers reserved for 64 pairs / 256 contacts; the next
    tick's detection finds ~4x more pairs than that.  The overflowing tick
    solves nothing (k_compact zeroes its counts), the check raises
    LPE_ERR_OVERFLOW, and the bodies stay finite."""
    U = 12.0
    b = scenes.Bodies()
    scenes.add_walls(b, U)
    for row in range(16):
        for col in range(16):
            verts = scenes.regular_polygon(5, 0.1)
            b.add(x=3.0 + col * 0.3, y=3.0 + row * 0.3, vx=(7.0 if col % 2 == 0 else -7.0), vy=0.0, mass=5.0,
                  verts=verts, shape_size=0.1, has_angvel=True, has_inertia=True,
                  inertia=scenes.polygon_inertia(verts, 5.0))
    bodies, verts = scenes.to_bodies(b)
    ctx = lpe.Context(0)
    try:
        ctx.rigid_set_config(lpe.rigid_config(universe=U))
        ctx.rigid_upload(bodies, verts)
        ctx.rigid_reserve(64, 256)
        with pytest.raises(lpe.LpeError, match="OVERFLOW"):
            ctx.world_tick(DT, 4)
            ctx.rigid_download()
        out = ctx.rigid_download()
    finally:
        ctx.close()
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        assert np.isfinite(out[k]).all(), k
    assert (out["x"][4:] > 0).all() and (out["x"][4:] < U).all()
