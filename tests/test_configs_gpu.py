"""Full-size parity at BASELINE.json's configs.

C2 (64k SPH dam break), C4 (256k SPH + 512 pentagons) and the metric scene M
(256k SPH + 4096 pentagons) are advanced on the device until they are in
motion (C2: the dam has broken; C4, M: the pentagons are in the fluid and M's
pile has settled), then ONE full world tick (lpe_world_tick: every system of
sim.cpp:107-114) from that exact state runs on the device and on the oracle
(OpenMP over particles; results are thread-count independent).  The fluid
and the bodies must be bit-identical (the rigid path's trigonometry is the
implementation device and oracle share, csrc/lpe_trig.h).  ("M", 3000) is
the state bench.py times: the metric scene after its 3,000 settle ticks;
("C4", 3000) likewise C4's timed state (round 5: C4 is timed settled, in the
reference's capped cells).

The reference cell-capacity mode (LPE_SPH_MODE_REF_CELL_CAP) is the
reference's own grid semantics; M's settled pool compresses cells past the
reference's 64 slots, so there the check covers the reference's dropped
inserts and cross-cell reads, and the default (unbounded) mode is checked
too.  C5 (2M particles, the 8-GPU config) is checked as 8 slab ranks through
the in-process transport against the single domain."""
import importlib.util
import os
import sys

import numpy as np
import pytest

from conftest import lpe, scenes

pytestmark = pytest.mark.gpu
DT = 1.0 / 120.0

_spec = importlib.util.spec_from_file_location(
    "slab", os.path.join(os.path.dirname(lpe.__file__), "slab.py"))
slab = importlib.util.module_from_spec(_spec)
sys.modules["slab"] = slab
_spec.loader.exec_module(slab)


def _world_ctx(U, fl, bodies, verts, mode=0):
    ctx = lpe.Context(0)
    ctx.sph_set_config(lpe.default_fluid_config())
    ctx.rigid_set_config(lpe.rigid_config(universe=U))
    ctx.rigid_upload(bodies, verts)
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    ctx.world_set_coupling(np.arange(len(bodies) - 1, -1, -1, dtype=np.int32))
    ctx.sph_set_mode(mode)
    return ctx


_STATE = {}


def _advanced(name, prep):
    """The scene after `prep` device ticks (cached per session)."""
    key = (name, prep)
    if key not in _STATE:
        s = scenes.scene(name)
        b, v = scenes.to_bodies(s["bodies"])
        ctx = _world_ctx(s["U"], s["fluid"], b, v)
        try:
            ctx.world_tick(DT, prep)
            out = ctx.sph_download()
            fl = dict(x=out["x"], y=out["y"], vx=out["vx"], vy=out["vy"], mass=s["fluid"]["mass"],
                      density=out["density"], pressure=out["pressure"])
            _STATE[key] = (s, fl, ctx.rigid_download(), v)
        finally:
            ctx.close()
    return _STATE[key]


@pytest.mark.parametrize("name,prep,mode", [
    ("C2", 30, lpe.SPH_MODE_REF_CELL_CAP),
    ("C4", 90, lpe.SPH_MODE_REF_CELL_CAP),
    ("C4", 3000, lpe.SPH_MODE_REF_CELL_CAP),
    ("C4", 3000, 0),
    ("M", 240, lpe.SPH_MODE_REF_CELL_CAP),
    ("M", 240, 0),
    ("M", 3000, lpe.SPH_MODE_REF_CELL_CAP),
    ("M", 3000, 0),
])
def test_config_world_tick_bit_exact(oracle_mod, name, prep, mode):
    s, fl, bodies, verts = _advanced(name, prep)
    ctx = _world_ctx(s["U"], fl, bodies, verts, mode)
    try:
        ctx.world_tick(DT, 1)
        out = ctx.sph_download()
        got_b = ctx.rigid_download()
        st = ctx.sph_stats()
    finally:
        ctx.close()
    oracle_mod.set_threads(0)
    oracle_mod.set_ref_cell_cap(bool(mode))
    try:
        couple = np.arange(len(bodies) - 1, -1, -1, dtype=np.int32)
        p, rb = oracle_mod.world_tick(lpe.default_fluid_config(), lpe.rigid_config(universe=s["U"]),
                                      scenes.particles_aos(fl), bodies, verts, couple, DT, 1)
        assert not oracle_mod.ref_undefined()
    finally:
        oracle_mod.set_ref_cell_cap(False)
    assert st["refUndefined"] == 0
    if name == "M" and prep == 240:  # the pool is still compressed past the reference's 64 slots
        assert st["overCapCells"] > 0 and st["maxCellOccupancy"] > 64
    if prep == 3000:  # the bench's timed states of M and C4 (a few cells may still exceed 64)
        print(f"{name}@3000 mode {mode}: overCapCells {st['overCapCells']}, max occupancy {st['maxCellOccupancy']}")
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], p[:, col], err_msg=(name, k, st))
    for k in ("x", "y", "angle", "vx", "vy", "omega", "sleep_counter"):
        np.testing.assert_array_equal(got_b[k], rb[k], err_msg=(name, k))


def test_mode_switch_voids_prelaunch_with_filed_tiles():
    """The bench's sequence: world ticks in one cell mode, then a switch to the
    reference's capped cells (which voids the pending prelaunched sub-step, its
    density pass having filed the heavy tiles), then world ticks.  The filing
    lists alternate by density pass and only a forces pass clears the other
    one's counts, so after a void the next pass files into a list whose counts
    no forces pass cleared: the forces pass's filed blocks must still run only
    the tiles this pass filed (the tile-flag check).  Equal, bit for bit, to
    the same ticks from the downloaded state in a fresh context (no pending
    prelaunch); the round-6 fault was a tile run twice, its particles counted
    twice into the next hash."""
    s, fl, bodies, verts = _advanced("M", 240)
    ctx = _world_ctx(s["U"], fl, bodies, verts, 0)
    try:
        ctx.world_tick(DT, 2)
        mid_f, mid_b = ctx.sph_download(), ctx.rigid_download()
        ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)       # voids the prelaunch
        ctx.world_tick(DT, 2)
        got_f, got_b = ctx.sph_download(), ctx.rigid_download()
        st = ctx.sph_stats()
    finally:
        ctx.close()
    fl2 = dict(x=mid_f["x"], y=mid_f["y"], vx=mid_f["vx"], vy=mid_f["vy"], mass=fl["mass"],
               density=mid_f["density"], pressure=mid_f["pressure"])
    ref = _world_ctx(s["U"], fl2, mid_b, verts, lpe.SPH_MODE_REF_CELL_CAP)
    try:
        ref.world_tick(DT, 2)
        want_f, want_b = ref.sph_download(), ref.rigid_download()
    finally:
        ref.close()
    assert st["refUndefined"] == 0
    for k in ("x", "y", "vx", "vy", "density", "pressure"):
        np.testing.assert_array_equal(got_f[k], want_f[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        np.testing.assert_array_equal(got_b[k], want_b[k], err_msg=k)


def _m_ticks(monkeypatch, q, h, ticks):
    """M from its 240-tick state advanced `ticks` world ticks, the tile
    scheduling's class thresholds set to (q, h) coupling pairs (None: default)."""
    for var, val in (("LPE_HEAVY_Q", q), ("LPE_HEAVY_H", h)):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, str(val))
    s, fl, bodies, verts = _advanced("M", 240)
    ctx = _world_ctx(s["U"], fl, bodies, verts)
    try:
        ctx.world_tick(DT, ticks)
        return ctx.sph_download(), ctx.rigid_download()
    finally:
        ctx.close()


@pytest.mark.parametrize("q,h", [(1, 1), (1 << 30, 1 << 30), (1, 1 << 30)],
                         ids=["all-quarters", "all-whole", "quarters-then-whole"])
def test_tile_scheduling_overflow_bit_exact(monkeypatch, q, h):
    """The forces pass's tile scheduling with its classes
    overfilled.  M couples ≈ 310 of its 1,024 tiles.  (1, 1) files every one
    of them as four part blocks: the 128 quarter slots fill, the next 160
    fall to halves, the rest to whole blocks.  (2^30, 2^30) files them all
    whole: 160 fit and ≈ 150 stay unfiled, run by their own tile blocks.
    (1, 2^30) fills the quarters and then the whole blocks, skipping halves,
    with some tiles left unfiled again.  Tiles with a single coupling pair
    split four ways leave empty part blocks.  Any partition of a tile's slots
    over blocks is the same arithmetic, so 3 world ticks must be bit-identical
    to the default thresholds (oracle-checked by
    test_config_world_tick_bit_exact)."""
    ref, rb_ref = _m_ticks(monkeypatch, None, None, 3)
    got, rb = _m_ticks(monkeypatch, q, h, 3)
    for k in ("x", "y", "vx", "vy", "density", "pressure"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        np.testing.assert_array_equal(rb[k], rb_ref[k], err_msg=k)


@pytest.mark.parametrize("cells", ["unbounded", "ref"])
def test_c5_eight_slab_ranks_bit_exact(cells):
    """C5 (2,097,152 particles): 8 x-slab ranks (in-process transport, one
    GPU) against the single domain, 2 full world ticks: every particle and
    wall bit for bit, in unbounded cells and in the reference's 64-particle
    cells (the ranks then file 3 ghost columns each side)."""
    s = scenes.scene("C5")
    fl = s["fluid"]
    n = len(fl["x"])
    b, v = scenes.to_bodies(s["bodies"])
    one = _world_ctx(s["U"], fl, b, v, mode=lpe.SPH_MODE_REF_CELL_CAP if cells == "ref" else 0)
    try:
        one.world_tick(DT, 2)
        ref = one.sph_download()
        rb_ref = one.rigid_download()
    finally:
        one.close()
    edges = slab.slab_edges(fl["x"], 8)
    ctxs = [lpe.Context(0) for _ in range(8)]
    try:
        for r, c in enumerate(ctxs):
            c.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            c.rigid_upload(b, v)
            slab.setup_rank(c, r, 8, fl, edges, lpe.default_fluid_config(), cells=cells)
            c.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
        lpe.mg_loopback_run(ctxs, 2, world=lpe.WorldConfig(DT, 1.0, 1.0, 1.0))
        parts = [c.sph_download_owned(cap=n) for c in ctxs]
        rbs = [c.rigid_download() for c in ctxs]
    finally:
        for c in ctxs:
            c.close()
    assert min(len(p["id"]) for p in parts) > 0
    got = slab.merge_owned(parts, n)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    for r in rbs:
        for k in ("x", "y", "vx", "vy"):
            np.testing.assert_array_equal(r[k], rb_ref[k], err_msg=k)


def test_short_division_equals_general():
    """The forces pass's pair term takes its quotients and square root by
    shortened sequences when the fluid config's thresholds keep the operands
    in range (SphStepParams.shortDiv).  A minimum density of
    1e-20 (no particle comes near it) turns them off: three world ticks of the
    metric scene in motion (M@240, the pile in the fluid) must give the same
    bits either way -- the shortened sequences equal the general ones."""
    s, fl, bodies, verts = _advanced("M", 240)

    def run(min_dens):
        ctx = lpe.Context(0)
        try:
            cfg = lpe.default_fluid_config()
            cfg.numericalConfig.minDensityThreshold = min_dens
            ctx.sph_set_config(cfg)
            ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            ctx.rigid_upload(bodies, verts)
            ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
            ctx.world_set_coupling(np.arange(len(bodies) - 1, -1, -1, dtype=np.int32))
            ctx.world_tick(DT, 3)
            return ctx.sph_download(), ctx.rigid_download()
        finally:
            ctx.close()

    short, rb_short = run(lpe.default_fluid_config().numericalConfig.minDensityThreshold)
    general, rb_general = run(1e-20)
    for k in ("x", "y", "vx", "vy", "density", "pressure"):
        np.testing.assert_array_equal(short[k], general[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        np.testing.assert_array_equal(rb_short[k], rb_general[k], err_msg=k)
