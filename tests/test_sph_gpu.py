"""GPU parity of the SPH path (HIP, through the C ABI) against the CPU oracle.

Bar (BASELINE.json north_star): bit-exact reference grid-cell indices; fp32
state within 1e-5 relative.  The HIP path is in fact held to bit-identity with
oracle/sph_oracle.c (same canonical orders, no FMA contraction, correctly
rounded div/sqrt, tanh/pow via fp64 rounded once), the rigid accumulators
included: both sides sum the fluid->rigid forces exactly and round once
(sph_coupling.h xacc_*; the reference's float atomics have no defined order).
"""
import numpy as np
import pytest

from conftest import lpe, scenes

pytestmark = pytest.mark.gpu
DT = 1.0 / 120.0


def _upload(ctx, fl, rigids=None, cfg=None):
    ctx.sph_set_config(cfg or lpe.default_fluid_config())
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    ctx.sph_upload_rigids(rigids if rigids is not None else np.zeros(0, lpe.RIGID_DTYPE))


def _close(a, b, rtol=1e-5, scale=None):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    sc = np.maximum(np.abs(b), scale if scale is not None else 0.0)
    return np.abs(a - b) <= rtol * sc + 1e-30


@pytest.mark.parametrize("name", ["small64_0", "small96_0"])
def test_cells_bit_exact(gpu_ctx, oracle_mod, name):
    s = scenes.scene(name)
    _upload(gpu_ctx, s["fluid"])
    cells, st = gpu_ctx.sph_probe_cells()
    ref, g = oracle_mod.cells(scenes.particles_aos(s["fluid"]))
    assert (st["gridMinX"], st["gridMinY"], st["gridDimX"], st["gridDimY"]) == \
        (g.gridMinX, g.gridMinY, g.gridDimX, g.gridDimY)
    np.testing.assert_array_equal(cells, ref)


def test_cells_not_inserted_edge(gpu_ctx, oracle_mod):
    """A particle within eps below a cell boundary at the global max is 'not
    inserted' (fluid.cpp:745-746 has no epsilon, metal:224-226 does)."""
    rng = np.random.default_rng(5)
    n = 2000
    x = rng.uniform(1.0, 2.0, n)
    y = rng.uniform(1.0, 2.0, n)
    x[0] = np.float32(2.3) - np.float32(5e-7)   # max x, just below the 2.3 boundary
    y[1] = np.float32(2.4) - np.float32(4e-7)
    fl = dict(x=x, y=y, vx=np.zeros(n), vy=np.zeros(n), mass=np.full(n, scenes.FLUID_MASS),
              density=np.zeros(n), pressure=np.zeros(n))
    _upload(gpu_ctx, fl)
    cells, st = gpu_ctx.sph_probe_cells()
    ref, g = oracle_mod.cells(scenes.particles_aos(fl))
    assert (ref < 0).sum() >= 1
    np.testing.assert_array_equal(cells, ref)
    assert st["notInserted"] == int((ref < 0).sum())


@pytest.mark.parametrize("name", ["small64_0", "small96_0"])
def test_density_bit_exact(gpu_ctx, oracle_mod, name):
    s = scenes.scene(name)
    _upload(gpu_ctx, s["fluid"])
    rho, p = gpu_ctx.sph_probe_density()
    rrho, rp, g, st = oracle_mod.density(scenes.particles_aos(s["fluid"]))
    np.testing.assert_array_equal(rho, rrho)
    np.testing.assert_array_equal(p, rp)


@pytest.mark.parametrize("kind,mode", [("C2", 0), ("jitter", 0), ("jitter_wide", 0), ("C2", 2), ("jitter", 2)])
def test_density_pair_kernel_staged_bit_exact(gpu_ctx, oracle_mod, kind, mode):
    """The two-particles-per-lane pure density pass (k_density_pair, 8-byte
    pair stores) on wide fluids, where its 512-slot tiles stage their
    neighbourhoods (no fallback): the C2 dam break, and a jittered lattice
    with uneven cells (pairs that straddle quadrants, cells and the tiles'
    two row runs).  mode 2 (LPE_SPH_MODE_PROBE_TICK_PASS): the same probe
    through the tick's k_density<true>, the microbench's second pass."""
    if kind == "C2":
        fl = scenes.scene("C2")["fluid"]
    else:
        rng = np.random.default_rng(12)
        # jitter_wide: ~1,560 tiles, several per block of the persistent pass
        fl = scenes.fluid_lattice(rng, *((1600, 500) if kind == "jitter_wide" else (700, 60)), 1.0, 1.0)
        fl["x"] = (fl["x"] + rng.uniform(-0.006, 0.006, len(fl["x"])))
        fl["y"] = (fl["y"] + rng.uniform(-0.006, 0.006, len(fl["y"])))
    _upload(gpu_ctx, fl)
    gpu_ctx.sph_set_mode(mode)
    gpu_ctx.sph_diag(True)
    rho, p = gpu_ctx.sph_probe_density()
    st = gpu_ctx.sph_stats()
    gpu_ctx.sph_set_mode(0)
    rrho, rp, g, _ = oracle_mod.density(scenes.particles_aos(fl))
    np.testing.assert_array_equal(rho, rrho)
    np.testing.assert_array_equal(p, rp)
    assert st["stageFallback"] == 0


def test_tick_walls_only_bit_exact(gpu_ctx, oracle_mod):
    """One full tick (10 sub-steps) with only the 4 walls (R > 0 dispatches the
    impulse kernel, but no particle touches a wall)."""
    s = scenes.scene("small64_0")
    rig = scenes.gather_rigids(s["bodies"])
    _upload(gpu_ctx, s["fluid"], rig)
    gpu_ctx.sph_step(DT)
    out = gpu_ctx.sph_download()
    ref, rref, acc, st = oracle_mod.fluid_tick(scenes.particles_aos(s["fluid"]), rig, DT)
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("vxHalf", 4), ("vyHalf", 5),
                   ("ax", 6), ("ay", 7), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], ref[:, col], err_msg=k)
    stats = gpu_ctx.sph_stats()
    assert stats["maxCellOccupancy"] == st.maxOcc
    assert stats["maxCellOccupancy"] <= lpe_max_per_cell()


def lpe_max_per_cell():
    return 64


@pytest.mark.parametrize("name", ["small64_8", "small96_12"])
def test_tick_coupled(gpu_ctx, oracle_mod, name):
    """One tick with pentagons sinking into the fluid: impulse + push-out.
    The fluid state, the rigid accumulators (exact sums rounded once) and the
    written-back rigid velocities are bit-identical to the oracle."""
    s = scenes.scene(name)
    rig = scenes.gather_rigids(s["bodies"])
    _upload(gpu_ctx, s["fluid"], rig)
    gpu_ctx.sph_step(DT)
    out = gpu_ctx.sph_download()
    r_out, acc = gpu_ctx.sph_download_rigids()
    ref, rref, racc, st = oracle_mod.fluid_tick(scenes.particles_aos(s["fluid"]), rig, DT)
    assert np.abs(racc).sum() > 0, "scene must exercise the coupling"
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("vxHalf", 4), ("vyHalf", 5),
                   ("ax", 6), ("ay", 7), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], ref[:, col], err_msg=k)
    np.testing.assert_array_equal(acc, racc)
    for k in ("vx", "vy", "omega"):
        np.testing.assert_array_equal(r_out[k], rref[k], err_msg=k)


def test_tick_coupled_deterministic(oracle_mod):
    """Two runs of several coupled ticks give the same bits (no float atomics
    left on the path: the accumulators are exact sums)."""
    s = scenes.scene("small96_12")
    rig = scenes.gather_rigids(s["bodies"])
    outs = []
    for _ in range(2):
        ctx = lpe.Context(0)
        try:
            _upload(ctx, s["fluid"], rig)
            for _ in range(4):
                ctx.sph_step(DT)
            out = ctx.sph_download()
            r_out, acc = ctx.sph_download_rigids()
            outs.append((out, r_out, acc))
        finally:
            ctx.close()
    (a, ra, aa), (b, rb, ab) = outs
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    np.testing.assert_array_equal(aa, ab)
    np.testing.assert_array_equal(ra.view(np.uint8), rb.view(np.uint8))


def test_multi_tick_invariants(gpu_ctx):
    """Several resident ticks: finite state, occupancy within the reference cap."""
    s = scenes.scene("small96_12")
    rig = scenes.gather_rigids(s["bodies"])
    _upload(gpu_ctx, s["fluid"], rig)
    for _ in range(5):
        gpu_ctx.sph_step(DT)
    out = gpu_ctx.sph_download()
    for k in ("x", "y", "vx", "vy", "density"):
        assert np.isfinite(out[k]).all(), k
    st = gpu_ctx.sph_stats()
    assert st["capacityOverflow"] == 0
    assert 0 < st["maxCellOccupancy"] <= 64


# ---- reference cell-capacity mode (LPE_SPH_MODE_REF_CELL_CAP) ----------------
from test_oracle_sph import compressed_scene  # noqa: E402


def _crowd_rigids():
    """Walls of a 3 m universe and two pentagons over the crowded region."""
    b = scenes.Bodies()
    scenes.add_walls(b, 3.0)
    for (x, y, r) in ((1.12, 1.1, 0.08), (1.3, 1.33, 0.1)):
        v = scenes.regular_polygon(5, r)
        b.add(x=x, y=y, vx=0.1, vy=0.3, mass=5.0, verts=v, has_angvel=True, has_inertia=True,
              inertia=scenes.polygon_inertia(v, 5.0), omega=0.5)
    return scenes.gather_rigids(b)


def test_ref_cell_cap_density_bit_exact(gpu_ctx, oracle_mod):
    """An over-full cell (> 64): the device's literal reference walk equals
    the oracle's 65-int grid buffer read, bit for bit."""
    fl = compressed_scene()
    _upload(gpu_ctx, fl)
    gpu_ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
    try:
        rho, p = gpu_ctx.sph_probe_density()
        st = gpu_ctx.sph_stats()
    finally:
        gpu_ctx.sph_set_mode(0)
    oracle_mod.set_ref_cell_cap(True)
    try:
        rrho, rp, g, ost = oracle_mod.density(scenes.particles_aos(fl))
    finally:
        oracle_mod.set_ref_cell_cap(False)
    assert st["overCapCells"] == ost.overCap == 1 and st["refUndefined"] == 0
    np.testing.assert_array_equal(rho, rrho)
    np.testing.assert_array_equal(p, rp)
    rho0, _ = gpu_ctx.sph_probe_density()             # default mode: unbounded lists
    assert (rho0 != rho).sum() > 0


@pytest.mark.parametrize("extra", [90, 300])
def test_ref_cell_cap_tick_bit_exact(gpu_ctx, oracle_mod, extra):
    """One coupled tick (10 sub-steps) in the capacity mode with an over-full
    cell (300 extra: the unclamped read runs several cells ahead)."""
    fl = compressed_scene(extra=extra)
    rig = _crowd_rigids()
    _upload(gpu_ctx, fl, rig)
    gpu_ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
    try:
        gpu_ctx.sph_step(DT)
        out = gpu_ctx.sph_download()
        r_out, acc = gpu_ctx.sph_download_rigids()
        st = gpu_ctx.sph_stats()
    finally:
        gpu_ctx.sph_set_mode(0)
    oracle_mod.set_ref_cell_cap(True)
    try:
        ref, rref, racc, ost = oracle_mod.fluid_tick(scenes.particles_aos(fl), rig, DT)
        assert not oracle_mod.ref_undefined()
    finally:
        oracle_mod.set_ref_cell_cap(False)
    assert st["overCapCells"] == ost.overCap > 0
    assert np.abs(racc).sum() > 0
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("vxHalf", 4), ("vyHalf", 5),
                   ("ax", 6), ("ay", 7), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], ref[:, col], err_msg=k)
    np.testing.assert_array_equal(acc, racc)


@pytest.mark.parametrize("extra", [90, 300])
def test_tick_over_full_bins_bit_exact(gpu_ctx, oracle_mod, extra):
    """Default mode, one coupled tick with 90 / 300 extra particles in one
    cell: the grid hash files at most 32 ids per (cell, quadrant) bin and the
    rest in its overflow list (k_bucket_permute); the in-bin order, and so
    every sum, stays the oracle's (ascending id)."""
    fl = compressed_scene(extra=extra)
    rig = _crowd_rigids()
    _upload(gpu_ctx, fl, rig)
    gpu_ctx.sph_step(DT)
    out = gpu_ctx.sph_download()
    r_out, acc = gpu_ctx.sph_download_rigids()
    st = gpu_ctx.sph_stats()
    ref, rref, racc, ost = oracle_mod.fluid_tick(scenes.particles_aos(fl), rig, DT)
    assert st["maxCellOccupancy"] == ost.maxOcc > 64     # (its quadrants hold 34 / 82 particles)
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("vxHalf", 4), ("vyHalf", 5),
                   ("ax", 6), ("ay", 7), ("density", 11), ("pressure", 12)):
        np.testing.assert_array_equal(out[k], ref[:, col], err_msg=k)
    np.testing.assert_array_equal(acc, racc)


def test_ref_cell_cap_equals_default_below_64(gpu_ctx, oracle_mod):
    s = scenes.scene("small64_8")
    rig = scenes.gather_rigids(s["bodies"])
    _upload(gpu_ctx, s["fluid"], rig)
    gpu_ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
    try:
        gpu_ctx.sph_step(DT)
        out = gpu_ctx.sph_download()
        assert gpu_ctx.sph_stats()["overCapCells"] == 0
    finally:
        gpu_ctx.sph_set_mode(0)
    ref, _, _, _ = oracle_mod.fluid_tick(scenes.particles_aos(s["fluid"]), rig, DT)
    for k, col in (("x", 0), ("y", 1), ("vx", 2), ("vy", 3), ("density", 11)):
        np.testing.assert_array_equal(out[k], ref[:, col], err_msg=k)


def test_drift_grows_device_grid_bit_exact():
    """the device grid follows the fluid, as the
    reference's grid follows its bbox every sub-step (fluid.cpp:740-755).  C2
    drifting at 8 m/s for 200 lpe_sph_step calls (13 m, past the upload's
    margin of 64 cells) regrows the grid at call boundaries (lpe_sph.hip
    sph_lag_service) and equals, bit for bit, the same run on a grid that
    covered the whole path from the start (lpe_sph_set_domain)."""
    s = scenes.scene("C2")
    fl = dict(s["fluid"])
    fl["vx"] = np.full(len(fl["x"]), 8.0, np.float32)
    nt = 200
    outs, stats = [], []
    for cover in (False, True):
        ctx = lpe.Context(0)
        try:
            ctx.sph_set_config(lpe.default_fluid_config())
            ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
            if cover:
                ctx.sph_set_domain(float(fl["x"].min()) - 2.0, float(fl["y"].min()) - 2.0,
                                   float(fl["x"].max()) + 8.0 * nt * DT + 4.0, float(fl["y"].max()) + 2.0)
            for _ in range(nt):
                ctx.sph_step(DT)
            outs.append(ctx.sph_download())
            stats.append(ctx.sph_stats())
        finally:
            ctx.close()
    assert stats[0]["gridRegrows"] >= 1 and stats[1]["gridRegrows"] == 0, stats
    assert stats[0]["capacityOverflow"] == 0
    for k in ("x", "y", "vx", "vy", "density", "pressure"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def test_fluid_leaving_the_grid_fails_with_capacity_error():
    """VERDICT r5 item 1 / ADVICE r5: a fluid that leaves the device grid
    within one call (C2 at 2,000 m/s: 17 m a tick against a 6.4 m margin)
    ends in LPE_ERR_CAPACITY, not in a GPU fault: bin_key clamps the bins,
    the density plans take their cells from the bins and the reference grid
    is clipped to the device grid, so no walk leaves the grid's buffers.  The
    error is sticky until the next upload; the context then steps normally
    (bit-exact against a fresh context)."""
    s = scenes.scene("C2")
    fl = dict(s["fluid"])
    fast = dict(fl)
    fast["vx"] = np.full(len(fl["x"]), 2000.0, np.float32)
    ctx = lpe.Context(0)
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fast["x"], fast["y"], fast["vx"], fast["vy"], fast["mass"], fast["density"], fast["pressure"])
        with pytest.raises(lpe.LpeError, match="left the device grid"):
            for _ in range(3):              # (reported by the lagged check or by the download)
                ctx.sph_step(DT)
            ctx.sph_download()
        assert ctx.sph_stats()["capacityOverflow"] != 0
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        for _ in range(2):
            ctx.sph_step(DT)
        got = ctx.sph_download()
    finally:
        ctx.close()
    ctx = lpe.Context(0)
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        for _ in range(2):
            ctx.sph_step(DT)
        ref = ctx.sph_download()
    finally:
        ctx.close()
    for k in ("x", "y", "vx", "vy", "density"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
