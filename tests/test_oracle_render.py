"""CPU known-answer tests of the density-field restatement
(oracle/render_oracle.c: fluid_renderer_kernels.metal:20-124 and
fluid_renderer.cpp:407-447).  Parity unpinned by execution: the reference
renderer is Metal-only and has no fixtures, so the restatement is pinned by
these hand-computed cases."""
import numpy as np

from conftest import ROOT  # noqa: F401  (puts oracle/ on sys.path)
import oracle


def test_single_particle_density_and_symmetry():
    c = 20                      # particle at the centre of cell (20, 20) of a 41 x 41 grid
    cs = np.float32(0.01)
    x = np.float32((c + 0.5) * cs)
    r = oracle.render_density([x], [x], 41, 41, float(cs), (0.0, 0.0), 10.0)
    h = np.float32(10.0) * cs
    hsq = h * h
    d = r["density"]
    assert d[c, c] == hsq * hsq * hsq               # distance 0: (h^2)^3
    assert d[0, 0] == 0.0 and d[c, c + 10] == 0.0   # outside h (|r| >= h)
    assert d[c, c + 9] > 0.0
    np.testing.assert_allclose(d, d[:, ::-1], rtol=1e-4, atol=1e-4 * d.max())  # mirror (cell centres round)
    np.testing.assert_array_equal(d, d.T)           # x and y take the same arithmetic
    assert r["max"] == r["blurred"].max() > 0
    assert r["normalized"][c, c] == 1.0 and r["normalized"].min() >= 0.0


def test_blur_of_a_delta():
    """Two 5x5 mean blurs of one non-zero cell: the interior weights are the
    5x5 mean of the 5x5 mean (1/25 each pass), edges divide by the in-bounds
    count (metal:84-97)."""
    cs = 0.01
    r = oracle.render_density([np.float32(0.105)], [np.float32(0.105)], 21, 21, cs, (0.0, 0.0), 0.5)
    d = r["density"]
    assert np.count_nonzero(d) == 1 and d[10, 10] > 0
    b = r["blurred"]
    v = d[10, 10]
    assert np.isclose(b[10, 10], v * 25 / 625, rtol=1e-6)
    assert b[10, 15] == 0.0 and b[10, 14] > 0.0      # support 9 x 9 after two passes


def test_no_particles():
    r = oracle.render_density(np.zeros(0, np.float32), np.zeros(0, np.float32), 8, 8)
    assert r["max"] == 0.0 and not r["normalized"].any()
