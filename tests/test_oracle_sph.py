"""CPU tests of the SPH oracle (oracle/sph_oracle.c).

The reference SPH path is Metal-only with no fixtures: the
oracle is pinned by (1) known-answer cases recomputed here independently in
numpy fp32 from fluid_kernels.metal's formulas, (2) the reference's grid
rules (fluid.cpp:717-752, metal:224-236) including the "not inserted" edge,
and (3) regression vectors in tests/golden/ (made by the oracle itself).
"""
import os

import numpy as np
import pytest

from conftest import ROOT, lpe, scenes

f32 = np.float32
PI_F = f32(np.pi)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def aos(x, y, m=scenes.FLUID_MASS, vx=None, vy=None):
    n = len(x)
    p = np.zeros((n, 13), np.float32)
    p[:, 0] = x
    p[:, 1] = y
    if vx is not None:
        p[:, 2] = vx
        p[:, 4] = vx
    if vy is not None:
        p[:, 3] = vy
        p[:, 5] = vy
    p[:, 8] = m
    p[:, 9] = 0.05
    return p


def ref_cells_numpy(p, eps=f32(1e-6)):
    """fluid.cpp:717-752 + metal:224-236 in numpy fp32."""
    x = p[:, 0].astype(f32)
    y = p[:, 1].astype(f32)
    cs = f32(2.0) * f32(0.05)
    minX = f32(x.min()) - f32(1e-6)
    minY = f32(y.min()) - f32(1e-6)
    gmx = int(np.floor(f32(minX / cs)))
    gmy = int(np.floor(f32(minY / cs)))
    dx = int(np.floor(f32(x.max() / cs))) - gmx + 1
    dy = int(np.floor(f32(y.max() / cs))) - gmy + 1
    gx = np.floor((x + eps) / cs).astype(np.int64) - gmx
    gy = np.floor((y + eps) / cs).astype(np.int64) - gmy
    ok = (gx >= 0) & (gx < dx) & (gy >= 0) & (gy < dy)
    return np.where(ok, gy * dx + gx, -1).astype(np.int32), (gmx, gmy, dx, dy)


def test_cells_match_numpy_restatement(oracle_mod):
    s = scenes.scene("small48_0")
    p = scenes.particles_aos(s["fluid"])
    cells, g = oracle_mod.cells(p)
    ref, grid = ref_cells_numpy(p)
    assert (g.gridMinX, g.gridMinY, g.gridDimX, g.gridDimY) == grid
    np.testing.assert_array_equal(cells, ref)


def test_not_inserted_edge(oracle_mod):
    """fluid.cpp:745-746 floors max/cs without epsilon, metal:224-226 adds it:
    the particle just below a cell boundary at the maximum is not inserted."""
    x = np.array([1.0, 1.5, f32(2.3) - f32(5e-7)], np.float32)
    y = np.array([1.0, 1.2, 1.1], np.float32)
    p = aos(x, y)
    cells, g = oracle_mod.cells(p)
    ref, _ = ref_cells_numpy(p)
    np.testing.assert_array_equal(cells, ref)
    assert cells[2] == -1 and cells[0] >= 0
    # and it misses its own density term: density is exactly zero
    rho, pr, g2, st = oracle_mod.density(p)
    assert rho[2] == 0.0 and st.notInserted == 1


def test_density_known_answer(oracle_mod):
    """Two particles at distance d < h (metal:246-307): rho_i = m * poly6 *
    ((h^2)^3 + (h^2 - d^2)^3) accumulated in stencil order in fp32."""
    d = f32(0.03)
    p = aos(np.array([1.0, 1.0 + d], np.float32), np.array([1.0, 1.0], np.float32))
    rho, pr, g, st = oracle_mod.density(p)
    h = f32(0.05)
    h2 = h * h
    h4 = h2 * h2
    poly6 = f32(4.0) / (PI_F * (h4 * h4))
    m = f32(scenes.FLUID_MASS)
    dx = f32(p[0, 0]) - f32(p[1, 0])
    r2 = dx * dx
    w_self = poly6 * h2 * h2 * h2
    w_pair = poly6 * (h2 - r2) * (h2 - r2) * (h2 - r2)
    # both particles share a cell; within it the order is (quadrant, index)
    q = [int(np.floor(f32(2) * ((p[i, 0] + f32(1e-6)) / f32(0.1)))) % 2 for i in range(2)]
    order0 = [0, 1] if q[0] <= q[1] else [1, 0]
    terms = {0: m * w_self, 1: m * w_pair}
    acc = f32(0)
    for j in order0:
        acc = f32(acc + terms[j])
    assert rho[0] == acc
    assert pr[0] == max(f32(0), f32(200.0) * (acc - f32(0.5)))


def test_lattice_rest_density(oracle_mod):
    """m = rho0 s^2 on an s = h/2 lattice gives rho ~ rho0 in the bulk."""
    s = scenes.scene("small48_0")
    p = scenes.particles_aos(s["fluid"])
    rho, pr, g, st = oracle_mod.density(p)
    x, y = p[:, 0], p[:, 1]
    bulk = (x > x.min() + 0.15) & (x < x.max() - 0.15) & (y > y.min() + 0.15) & (y < y.max() - 0.15)
    assert 0.45 < np.median(rho[bulk]) < 0.56
    assert st.maxOcc <= 64


@pytest.mark.parametrize("name", ["small64_8", "small48_0"])
def test_golden_regression(oracle_mod, name):
    z = np.load(os.path.join(GOLDEN, f"sph_{name}.npz"))
    out, rout, acc, st = oracle_mod.fluid_tick(z["particles_in"], z["rigids_in"], 1.0 / 120.0)
    np.testing.assert_array_equal(out, z["particles_out"])
    np.testing.assert_array_equal(acc, z["accum"])
    np.testing.assert_array_equal(rout.view(np.uint8), z["rigids_out"].view(np.uint8))
    cells, g = oracle_mod.cells(z["particles_in"])
    np.testing.assert_array_equal(cells, z["cells_in"])


def test_tick_invariants(oracle_mod):
    s = scenes.scene("small64_8")
    p = scenes.particles_aos(s["fluid"])
    rig = scenes.gather_rigids(s["bodies"])
    out, rout, acc, st = oracle_mod.fluid_tick(p, rig, 1.0 / 120.0)
    assert np.isfinite(out).all()
    # gather semantics: a tick starts from a = 0, and a is an acceleration
    assert np.abs(acc).sum() > 0            # the pentagons touch the fluid
    assert (out[:, 0] >= 0).all() and (out[:, 1] >= 0).all()   # push-out clamp
    # walls have mass 1e30 -> write-back v += F * 1e-30 keeps them ~at rest
    assert np.abs(rout["vx"][:4]).max() < 1e-20


def _round_f32_exact(fr):
    """Nearest float32 to the rational fr, ties to even (independent of the
    oracle: candidates around float64(fr), compared exactly)."""
    from fractions import Fraction
    c = np.float32(float(fr))
    best = None
    for cand in (np.nextafter(c, f32(-np.inf)), c, np.nextafter(c, f32(np.inf))):
        err = abs(Fraction(float(cand)) - fr)
        key = (err, int(np.frombuffer(np.float32(cand).tobytes(), np.uint32)[0]) & 1)
        if best is None or key < best[0]:
            best = (key, cand)
    return f32(best[1])


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_xacc_sum_is_correctly_rounded(oracle_mod, seed):
    """The rigid accumulators' exact sum (sph_oracle.c xacc_*): equal to the
    correctly rounded rational sum, for mixed signs, magnitudes from
    denormals to 1e6, and massive cancellation; order does not matter."""
    from fractions import Fraction
    rng = np.random.default_rng(seed)
    n = 2000
    mag = 10.0 ** rng.uniform(-44, 6, n)
    v = (rng.choice([-1.0, 1.0], n) * mag).astype(np.float32)
    v[:10] = np.array([1e-45, -1e-45, 3e-39, 0.15, -0.15, 0.1, 1e6, -1e6, 0.0, -0.0], np.float32)
    exact = sum((Fraction(float(x)) for x in v), Fraction(0))
    want = _round_f32_exact(exact)
    got = oracle_mod.xacc_sum(v)
    assert got == want, (got, want)
    assert oracle_mod.xacc_sum(v[::-1]) == got
    assert oracle_mod.xacc_sum(rng.permutation(v)) == got


def test_xacc_sum_cancellation_and_ties(oracle_mod):
    one = f32(1.0)
    eps = np.float32(2.0 ** -24)
    # 1 + 2^-24 is a tie between 1 and 1 + 2^-23: rounds to even (1.0)
    assert oracle_mod.xacc_sum(np.array([one, eps], np.float32)) == one
    # 1 + 2^-24 + 2^-40 is above the tie: rounds up
    assert oracle_mod.xacc_sum(np.array([one, eps, 2.0 ** -40], np.float32)) == np.nextafter(one, f32(2))
    # huge cancellation leaves the tiny term exactly
    v = np.array([1e6, 3e-30, -1e6], np.float32)
    assert oracle_mod.xacc_sum(v) == f32(3e-30)
    assert oracle_mod.xacc_sum(np.array([-0.5, -0.25], np.float32)) == f32(-0.75)
    assert oracle_mod.xacc_sum(np.zeros(0, np.float32)) == f32(0)
    assert oracle_mod.xacc_sum(np.array([2.0 ** 64], np.float32)) == f32(-1e30)   # range error


def compressed_scene(extra=90, seed=3):
    """A 16 x 16 lattice (16 particles per 2h cell) plus `extra` particles
    squeezed into one cell: that cell exceeds GPU_MAX_PER_CELL = 64."""
    rng = np.random.default_rng(seed)
    s = scenes.LATTICE_S
    gx, gy = np.meshgrid(np.arange(16), np.arange(16))
    x = 1.0 + (gx.ravel() + 0.5) * s + rng.uniform(-0.1, 0.1, 256) * s
    y = 1.0 + (gy.ravel() + 0.5) * s + rng.uniform(-0.1, 0.1, 256) * s
    cx, cy = 1.2 + 0.05, 1.2 + 0.05                       # inside cell (12, 12) of the 0.1 m grid
    x = np.concatenate([x, cx + rng.uniform(-0.045, 0.045, extra)])
    y = np.concatenate([y, cy + rng.uniform(-0.045, 0.045, extra)])
    n = len(x)
    return dict(x=x, y=y, vx=rng.uniform(-0.1, 0.1, n), vy=rng.uniform(-0.1, 0.1, n),
                mass=np.full(n, scenes.FLUID_MASS), density=np.zeros(n), pressure=np.zeros(n))


def ref_cap_density_numpy(p):
    """computeDensity (metal:246-307) over the reference's GPUGridCell buffer
    (count + 64 indices per cell, memset each sub-step, fluid.hpp:56-61,
    fluid.cpp:821-824; inserts past 64 dropped, metal:237-240), read with the
    unclamped loop (metal:281-283), insertion order = cell quadrant then
    index.  Plain numpy fp32, independent of the oracle."""
    cells, (gmx, gmy, dx, dy) = ref_cells_numpy(p)
    n = len(p)
    cs = f32(0.1)
    eps = f32(1e-6)
    C = dx * dy
    buf = np.zeros(65 * C, np.int64)
    quad = []
    for i in range(n):
        tx = (p[i, 0] + eps) / cs
        ty = (p[i, 1] + eps) / cs
        qx = int(np.floor(f32(2) * tx)) - 2 * int(np.floor(tx))
        qy = int(np.floor(f32(2) * ty)) - 2 * int(np.floor(ty))
        quad.append(qy * 2 + qx)
    for c in range(C):
        mem = sorted((quad[i], i) for i in np.nonzero(cells == c)[0])
        buf[65 * c] = len(mem)
        for k, (_, i) in enumerate(mem[:64]):
            buf[65 * c + 1 + k] = i
    h = f32(0.05)
    h2 = h * h
    h4 = h2 * h2
    poly6 = f32(4.0) / (PI_F * (h4 * h4))
    rho = np.zeros(n, np.float32)
    for i in range(n):
        xi, yi = p[i, 0], p[i, 1]
        cX = int(np.floor((xi + eps) / cs)) - gmx
        cY = int(np.floor((yi + eps) / cs)) - gmy
        acc = f32(0)
        for ny in (-1, 0, 1):
            for nx in (-1, 0, 1):
                cx, cy = cX + nx, cY + ny
                if cx < 0 or cx >= dx or cy < 0 or cy >= dy:
                    continue
                c = cy * dx + cx
                for k in range(int(buf[65 * c])):
                    pos = 65 * c + 1 + k
                    assert pos < 65 * C
                    j = int(buf[pos])
                    if j >= n:
                        continue
                    ddx = xi - p[j, 0]
                    ddy = yi - p[j, 1]
                    r2 = ddx * ddx + ddy * ddy
                    if r2 < h2:
                        diff = h2 - r2
                        acc = f32(acc + p[j, 8] * (poly6 * diff * diff * diff))
        rho[i] = acc
    return rho


def test_ref_cell_cap_density_known_answer(oracle_mod):
    """The oracle's reference cell-capacity mode equals the literal numpy
    restatement bit for bit on a scene with an over-full cell, and differs
    from the unbounded default there (the reference drops and mis-reads)."""
    fl = compressed_scene()
    p = scenes.particles_aos(fl)
    want = ref_cap_density_numpy(p)
    oracle_mod.set_ref_cell_cap(True)
    try:
        rho, pr, g, st = oracle_mod.density(p)
    finally:
        oracle_mod.set_ref_cell_cap(False)
    assert st.overCap == 1 and st.maxOcc > 64
    np.testing.assert_array_equal(rho, want)
    rho0, _, _, _ = oracle_mod.density(p)
    assert (rho0 != rho).sum() > 0


def test_ref_cell_cap_is_default_below_64(oracle_mod):
    """Without an over-full cell the capacity mode is the default, bit for bit."""
    s = scenes.scene("small64_8")
    p = scenes.particles_aos(s["fluid"])
    rig = scenes.gather_rigids(s["bodies"])
    a = oracle_mod.fluid_tick(p, rig, 1.0 / 120.0)
    oracle_mod.set_ref_cell_cap(True)
    try:
        b = oracle_mod.fluid_tick(p, rig, 1.0 / 120.0)
    finally:
        oracle_mod.set_ref_cell_cap(False)
    assert b[3].overCap == 0
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[2], b[2])
