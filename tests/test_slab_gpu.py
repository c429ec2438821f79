"""GPU parity of the x-slab decomposition against the
single-domain HIP step, which tests/test_sph_gpu.py pins to the oracle.

Several ranks run on the one GPU of the box through the in-process loopback
transport (lpe_mg_loopback_run: one host thread per rank, every exchange and
reduction a kernel on the rank's stream ordered by events, reductions in
rank order); the RCCL transport differs only in how the same buffers move.
Ownership is decided per sub-step by cell column, ghosts carry global ids
and the reference grid comes from every rank's bbox record, so the merged
state is bit-identical to the single-domain run, tick after tick.  With
rigid coupling too: the rigid accumulators are exact fixed-point sums whose
limbs are all-reduced as int64, so the split over ranks cannot change a bit,
and full world ticks stay bit-identical to the single domain."""
import numpy as np
import pytest

from conftest import lpe, scenes
import importlib.util
import os
import sys

pytestmark = pytest.mark.gpu
DT = 1.0 / 120.0

_spec = importlib.util.spec_from_file_location(
    "slab", os.path.join(os.path.dirname(lpe.__file__), "slab.py"))
slab = importlib.util.module_from_spec(_spec)
sys.modules["slab"] = slab
_spec.loader.exec_module(slab)


def _single(fl, rig, nticks):
    ctx = lpe.Context(0)
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.sph_upload_rigids(rig)
        for _ in range(nticks):
            ctx.sph_step(DT)
        out = ctx.sph_download()
        r, acc = ctx.sph_download_rigids()
        return out, r, acc
    finally:
        ctx.close()


def _sharded(fl, rig, nticks, edges, wire_cap=None, rebalance=0):
    n = len(edges) - 1
    cfg = lpe.default_fluid_config()
    ctxs = [lpe.Context(0) for _ in range(n)]
    try:
        for r, c in enumerate(ctxs):
            slab.setup_rank(c, r, n, fl, edges, cfg, rig, wire_cap=wire_cap, rebalance=rebalance)
        counts0 = [c.n for c in ctxs]
        lpe.mg_loopback_run(ctxs, nticks, DT)
        parts = [c.sph_download_owned(cap=len(fl["x"])) for c in ctxs]
        rigs = [c.sph_download_rigids() for c in ctxs]
        return slab.merge_owned(parts, len(fl["x"])), rigs, counts0, [len(p["id"]) for p in parts]
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("nranks", [2, 3])
def test_slab_fluid_bit_exact(nranks):
    """Dam-break block (walls only, no particle touches them), 3 ticks."""
    s = scenes.scene("small96_0")
    fl = s["fluid"]
    rig = scenes.gather_rigids(s["bodies"])
    ref, _, _ = _single(fl, rig, 3)
    edges = slab.slab_edges(fl["x"], nranks)
    got, _, c0, c1 = _sharded(fl, rig, 3, edges)
    assert min(c0) > 0
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_slab_migration_and_empty_rank():
    """Edges through the moving fluid (particles cross slab edges and change
    owner inside a sub-step) and a rank that starts empty and receives
    particles."""
    s = scenes.scene("small64_0")
    fl = dict(s["fluid"])
    n = len(fl["x"])
    fl["vx"] = np.full(n, 4.0)      # the whole block drifts right 4 m/s (0.13 m in 4 ticks)
    rig = np.zeros(0, lpe.RIGID_DTYPE)
    ref, _, _ = _single(fl, rig, 4)
    cs = slab.cell_size()
    col = slab._columns(fl["x"])
    c_lo, c_hi = int(col.min()), int(col.max())
    edges = np.array([-np.inf, (c_hi - 8) * cs, (c_hi + 1) * cs, np.inf], np.float32)
    assert c_hi - 8 > c_lo
    got, _, c0, c1 = _sharded(fl, rig, 4, edges)
    assert c0[2] == 0 and c1[2] > 0, (c0, c1)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_slab_coupled_first_tick():
    """Pentagons sinking into the fluid across a slab edge: the fluid is
    bit-identical in tick 1, the summed accumulators and rigid velocities
    within float-atomic summation order."""
    s = scenes.scene("small96_12")
    fl = s["fluid"]
    rig = scenes.gather_rigids(s["bodies"])
    ref, rref, aref = _single(fl, rig, 1)
    edges = slab.slab_edges(fl["x"], 2)
    got, rigs, _, _ = _sharded(fl, rig, 1, edges)
    assert np.abs(aref).sum() > 0
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    for r_out, acc in rigs:                   # every rank holds the summed result
        np.testing.assert_array_equal(acc, aref)
        for k in ("vx", "vy", "omega"):
            np.testing.assert_array_equal(r_out[k], rref[k], err_msg=k)


def test_slab_spike_within_capacity():
    """Every exchange moves a fixed wire both ends know (no host round trip
    sizes it): a velocity jump after 2 ticks pushes many more particles over
    the edges within the capacity, and 3 more ticks stay bit-identical to the
    single domain; the reported wire is the capacity."""
    s = scenes.scene("small96_0")
    fl = dict(s["fluid"])
    fl["vx"] = np.full(len(fl["x"]), 0.8)
    rig = np.zeros(0, lpe.RIGID_DTYPE)
    ref2, _, _ = _single(fl, rig, 2)
    edges = slab.slab_edges(fl["x"], 3)
    cfg = lpe.default_fluid_config()
    cap = slab.wire_capacity(np.asarray(fl["x"], np.float32), edges, cfg)

    def loop(flin, nticks):
        ctxs = [lpe.Context(0) for _ in range(3)]
        try:
            for r, c in enumerate(ctxs):
                slab.setup_rank(c, r, 3, flin, edges, cfg, rig, wire_cap=cap)
            lpe.mg_loopback_run(ctxs, nticks, DT)
            wires = [c.sph_stats()["haloWire"] for c in ctxs]
            parts = [c.sph_download_owned(cap=len(flin["x"])) for c in ctxs]
        finally:
            for c in ctxs:
                c.close()
        return slab.merge_owned(parts, len(flin["x"])), wires

    got2, _ = loop(fl, 2)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got2[k], ref2[k], err_msg=k)

    def jumped(state):
        out = dict(x=state["x"], y=state["y"], vx=np.asarray(state["vx"], np.float32) + np.float32(3.0),
                   vy=state["vy"], mass=fl["mass"], density=state["density"], pressure=state["pressure"])
        return out

    ref5, _, _ = _single(jumped(ref2), rig, 3)
    got5, wires = loop(jumped(got2), 3)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got5[k], ref5[k], err_msg=k)
    assert wires[0][0] == 0 and wires[2][1] == 0            # no neighbour there
    for w in (wires[0][1], wires[1][0], wires[1][1], wires[2][0]):
        assert w == cap, (wires, cap)


def test_slab_halo_overflow_reported():
    """A wire too small for the edge band fails loudly."""
    s = scenes.scene("small64_0")
    fl = s["fluid"]
    edges = slab.slab_edges(fl["x"], 2)
    with pytest.raises(lpe.LpeError, match="OVERFLOW|overflow"):
        _sharded(fl, np.zeros(0, lpe.RIGID_DTYPE), 1, edges, wire_cap=8)


def _world_rank(ctx, r, n, s, edges):
    b, v = scenes.to_bodies(s["bodies"])
    ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
    ctx.rigid_upload(b, v)
    if edges is None:
        fl = s["fluid"]
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    else:
        slab.setup_rank(ctx, r, n, s["fluid"], edges, lpe.default_fluid_config())
    ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))


def test_slab_world_tick_replicated_rigids():
    """Full resident ticks (lpe_world_tick) with the fluid in 2 slabs and the
    rigid pass replicated: fluid and bodies bit-identical to the single domain
    after 1 and 5 ticks, the rigid replicas identical to each other."""
    s = scenes.scene("small96_12")
    n_glob = len(s["fluid"]["x"])
    for nt in (1, 5):
        one = lpe.Context(0)
        try:
            _world_rank(one, 0, 1, s, None)
            one.world_tick(DT, nt)
            ref = one.sph_download()
            rb_ref = one.rigid_download()
        finally:
            one.close()
        edges = slab.slab_edges(s["fluid"]["x"], 2)
        ctxs = [lpe.Context(0) for _ in range(2)]
        try:
            for r, c in enumerate(ctxs):
                _world_rank(c, r, 2, s, edges)
            lpe.mg_loopback_run(ctxs, nt, world=lpe.WorldConfig(DT, 1.0, 1.0, 1.0))
            got = slab.merge_owned([c.sph_download_owned(cap=n_glob) for c in ctxs], n_glob)
            rbs = [c.rigid_download() for c in ctxs]
        finally:
            for c in ctxs:
                c.close()
        for k in ("x", "y", "vx", "vy", "angle", "omega"):
            np.testing.assert_array_equal(rbs[0][k], rbs[1][k], err_msg=k)
        for k in slab.FIELDS:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=(nt, k))
        for k in ("x", "y", "angle", "vx", "vy", "omega"):
            np.testing.assert_array_equal(rbs[0][k], rb_ref[k], err_msg=(nt, k))


def test_rccl_transport_single_rank():
    """The RCCL transport initialises on the box (world size 1: a slab with no
    neighbours, so no traffic) and the step matches the single domain."""
    s = scenes.scene("small64_0")
    fl = s["fluid"]
    rig = scenes.gather_rigids(s["bodies"])
    ref, _, _ = _single(fl, rig, 2)
    ctx = lpe.Context(0)
    try:
        ctx.mg_init_rccl(1, 0, lpe.mg_unique_id())
        slab.setup_rank(ctx, 0, 1, fl, slab.slab_edges(fl["x"], 1), lpe.default_fluid_config(), rig)
        ctx.sph_step(DT)
        ctx.sph_step(DT)
        got = slab.merge_owned([ctx.sph_download_owned()], len(fl["x"]))
    finally:
        ctx.close()
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_slab_rebalance_bit_exact_and_model_edges():
    """Re-balancing every step on a left-heavy split: the edge moves a column
    per step towards equal counts -- exactly as slab.rebalance_edges
    restates it from the owned particles' columns -- while the merged state
    stays bit-identical to the single domain."""
    s = scenes.scene("small96_0")
    fl = s["fluid"]
    rig = np.zeros(0, lpe.RIGID_DTYPE)
    n = len(fl["x"])
    cfg = lpe.default_fluid_config()
    cs = slab.cell_size(cfg)
    col = slab._columns(fl["x"])
    edges = np.array([-np.inf, (int(col.min()) + 16) * cs, np.inf], np.float32)   # 16 of 24 columns left
    e_model = np.array([-(1 << 29), int(col.min()) + 16, 1 << 29])
    e0 = e_model.copy()
    ctxs = [lpe.Context(0) for _ in range(2)]
    try:
        for r, c in enumerate(ctxs):
            slab.setup_rank(c, r, 2, fl, edges, cfg, rig, rebalance=1)
        mv = ctxs[0].sph_slab_info()["mv"]
        col0 = int(e0[1]) - mv - 2
        ncols = int(e0[1]) + mv + 2 - col0 + 1
        for t in range(4):
            lpe.mg_loopback_run(ctxs, 1, DT)
            parts = [c.sph_download_owned(cap=n) for c in ctxs]
            allx = np.concatenate([p["x"] for p in parts])
            hist = np.bincount(np.clip(slab._columns(allx, cfg) - col0, 0, ncols - 1), minlength=ncols)
            e_model = slab.rebalance_edges(hist.astype(np.float32), col0, e_model, e0, 2, mv)
            for c in ctxs:
                got = c.sph_slab_info()["edges"]
                assert got[1] == e_model[1], (t, got, e_model)
        got = slab.merge_owned(parts, n)
    finally:
        for c in ctxs:
            c.close()
    assert e_model[1] < e0[1]
    ref, _, _ = _single(fl, rig, 4)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def test_slab_stats_and_prelaunch_one_tick_calls():
    """The slab path with the prelaunched sub-step 0 (world ticks one call at
    a time, as the drop-in does) equals multi-tick calls, and the stats
    report the owned counts and the ghosts received."""
    s = scenes.scene("small96_12")
    n_glob = len(s["fluid"]["x"])
    outs = []
    for per_call in (1, 3):
        edges = slab.slab_edges(s["fluid"]["x"], 3)
        ctxs = [lpe.Context(0) for _ in range(3)]
        try:
            for r, c in enumerate(ctxs):
                _world_rank(c, r, 3, s, edges)
            for _ in range(3 // per_call):
                lpe.mg_loopback_run(ctxs, per_call, world=lpe.WorldConfig(DT, 1.0, 1.0, 1.0))
            st = [c.sph_stats() for c in ctxs]
            outs.append(slab.merge_owned([c.sph_download_owned(cap=n_glob) for c in ctxs], n_glob))
        finally:
            for c in ctxs:
                c.close()
        assert sum(x["slabOwned"] for x in st) == n_glob
        assert st[0]["ghostsIn"][1] > 0 and st[1]["ghostsIn"][0] > 0 and st[1]["ghostsIn"][1] > 0
        assert all(x["slabSlots"] >= x["slabOwned"] for x in st)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def test_slab_drift_into_empty_rank_grows_grid_and_slots():
    """VERDICT r5 items 1-2 (profiles/r05/slab_capacity/repro.py, unpadded):
    C2's 65,536 particles drift right at 8 m/s into a rank that starts empty,
    with the domain at the pool's bbox + 1 m (slab.setup_rank's default) and a
    wire of 8,192 records, so 36,864 slots.  Round 5 faulted the GPU between
    ticks 20 and 30 (the fluid left the rank's device grid) and dropped ghosts
    once the slots were full.  Now the lagged checks (lpe_sph.hip
    sph_lag_service) grow the receiving rank's grid ahead of the fluid and its
    slots past half their use: after 100 ticks every particle is owned by a
    rank and the merged state equals the single domain's bit for bit."""
    s = scenes.scene("C2")
    fl = dict(s["fluid"])
    n = len(fl["x"])
    fl["vx"] = np.full(n, 8.0, np.float32)
    cfg = lpe.default_fluid_config()
    cs = slab.cell_size(cfg)
    c_hi = int(slab._columns(fl["x"], cfg).max())
    edges = np.array([-np.inf, (c_hi + 1) * cs, np.inf], np.float32)
    nt = 100
    ctxs = [lpe.Context(0) for _ in range(2)]
    try:
        for r, c in enumerate(ctxs):
            slab.setup_rank(c, r, 2, fl, edges, cfg, np.zeros(0, lpe.RIGID_DTYPE), wire_cap=8192)
        assert ctxs[1].n == 0
        lpe.mg_loopback_run(ctxs, nt, DT)
        st = [c.sph_stats() for c in ctxs]
        parts = [c.sph_download_owned(cap=n) for c in ctxs]
    finally:
        for c in ctxs:
            c.close()
    assert sum(x["slabOwned"] for x in st) == n
    assert st[1]["slabOwned"] > n // 2, st[1]
    assert st[1]["gridRegrows"] >= 1 and st[1]["slotRegrows"] >= 1, st[1]
    got = slab.merge_owned(parts, n)
    ref, _, _ = _single(fl, np.zeros(0, lpe.RIGID_DTYPE), nt)
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


def _m_state(prep):
    """Scene M after `prep` single-domain world ticks: (scene, fluid, bodies, verts)."""
    s = scenes.scene("M")
    b, v = scenes.to_bodies(s["bodies"])
    one = lpe.Context(0)
    try:
        _world_rank(one, 0, 1, s, None)
        one.world_tick(DT, prep)
        out = one.sph_download()
        bodies = one.rigid_download()
    finally:
        one.close()
    fl = dict(s["fluid"])
    fl.update({k: out[k] for k in ("x", "y", "vx", "vy", "density", "pressure")})
    return s, fl, bodies, v


@pytest.mark.parametrize("nranks", [2, 4])
def test_slab_capped_cells_bit_exact(nranks):
    """the reference's 64-particle cells on slab ranks.
    Scene M 240 ticks in (the pool compressed: cells of up to ~98), the edges
    put beside over-full cells (the over-full column the last owned column,
    the first ghost column, one further out), 3 world ticks in
    LPE_SPH_MODE_REF_CELL_CAP: the ranks (at least 3 ghost columns each side,
    one more per 65 particles the largest cell holds past 64 -- the capped
    cells keep compressing, 182, 259, 302 particles in a cell after 1, 2, 3
    ticks, profiles/r06/probe/capped_slab_diag.log; the literal loop's
    cross-cell reads on the global grid's flat order; values read as ids
    that are not on the rank skipped) equal the single domain in the same
    mode bit for bit, fluid and bodies."""
    s, fl, bodies, verts = _m_state(240)
    cfg = lpe.default_fluid_config()
    cs = slab.cell_size(cfg)
    eps = np.float32(cfg.gridConfig.gridEpsilon)
    col = np.floor((fl["x"] + eps) / np.float32(cs)).astype(np.int64)
    row = np.floor((fl["y"] + eps) / np.float32(cs)).astype(np.int64)
    cells, counts = np.unique(np.stack([col, row], 1), axis=0, return_counts=True)
    over = np.unique(cells[counts > 64][:, 0])
    assert len(over) >= nranks - 1, "no over-full cells at this state"
    pick = over[np.linspace(0, len(over) - 1, nranks + 1).astype(int)[1:-1]]
    cuts = sorted(set(int(c) + d for c, d in zip(pick, (1, 0, -1))))
    edges = np.array([-np.inf] + [c * cs for c in cuts] + [np.inf], np.float32)
    n = len(fl["x"])
    sf = dict(s)
    sf["fluid"] = fl
    one = lpe.Context(0)
    try:
        one.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        one.rigid_upload(bodies, verts)
        one.sph_set_config(cfg)
        one.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        one.world_set_coupling(np.arange(len(bodies) - 1, -1, -1, dtype=np.int32))
        one.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
        one.sph_diag(True)
        one.world_tick(DT, 3)
        ref = one.sph_download()
        rb_ref = one.rigid_download()
        st1 = one.sph_stats()
    finally:
        one.close()
    assert st1["overCapCellsTotal"] > 0, st1
    ctxs = [lpe.Context(0) for _ in range(len(edges) - 1)]
    try:
        for r, c in enumerate(ctxs):
            c.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            c.rigid_upload(bodies, verts)
            slab.setup_rank(c, r, len(ctxs), fl, edges, cfg, cells="ref",
                            wire_cap=slab.wire_capacity(fl["x"], edges, cfg, band=slab.BAND_MAX))
            c.world_set_coupling(np.arange(len(bodies) - 1, -1, -1, dtype=np.int32))
        lpe.mg_loopback_run(ctxs, 3, world=lpe.WorldConfig(DT, 1.0, 1.0, 1.0))
        got = slab.merge_owned([c.sph_download_owned(cap=n) for c in ctxs], n)
        rbs = [c.rigid_download() for c in ctxs]
    finally:
        for c in ctxs:
            c.close()
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    for r in rbs:
        for k in ("x", "y", "angle", "vx", "vy", "omega"):
            np.testing.assert_array_equal(r[k], rb_ref[k], err_msg=k)
