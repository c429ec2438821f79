"""Restatement of the opt-in Jacobi contact solver (lpe_rigid.hip
k_pgs_jacobi, lpe_rigid_config.pgsMode = LPE_PGS_JACOBI) in numpy, for the
tests: the device must reproduce it bit for bit.

Test infrastructure, not the product: the Jacobi mode is not the reference's
arithmetic (the reference runs sequential Gauss-Seidel, solveLcpPgs,
contact_solver.cpp:381-440), so there is no reference output to pin it to.
It is pinned here by restatement and, in the tests, by the LCP invariants
(lamN >= 0, |lamF| <= mu lamN, separating or resting normal velocities once
converged).

Per iteration every contact pair reads the previous iteration's body
velocities, runs its contacts' normal and friction rows in order
(contact_solver.cpp:399-437) on a copy of its two bodies whose inverse mass /
inertia are scaled by the body's pair count (mass splitting), and contributes
its impulses (applyImpulse, :315-356, unscaled masses) to the bodies in
2^-40 fixed point; the sums are exact integers, so their order does not
matter.  The rows are
buildConstraintRows / computeEffectiveMass's (contact_solver.cpp:133-253):
direction = normalised contact normal, lever arms from the pre-solve poses,
fp32.  Everything is float32 arithmetic with no fused operations, as the
device is built (-ffp-contract=off)."""
import numpy as np

from conftest import lpe

F = np.float32
SCALE, INV = 2.0 ** 40, 2.0 ** -40


def _can_rotate(b):
    f = b["flags"]
    return (((f & lpe.BODY_HAS_ANGVEL) != 0) & ((f & lpe.BODY_HAS_INERTIA) != 0)
            & (b["inertia"] > 1e-12) & (b["inertia"] < 1e29))


def _infinite(b):
    return ((b["flags"] & lpe.BODY_HAS_MASS) != 0) & (b["mass"] > 1e29)


def rows(bodies, contacts):
    """Per contact (contact order): body indices a, b (-1: infinite mass),
    dir (x, y), lever arms, inverse masses / inertias -- k_prep_items."""
    b = bodies
    cr = _can_rotate(b)
    with np.errstate(divide="ignore"):
        im = np.where(b["mass"] > 1e29, F(0), (1.0 / b["mass"]).astype(F)).astype(F)
        ii = np.where(cr & (b["inertia"] > 1e-12) & (b["inertia"] < 1e29),
                      (1.0 / b["inertia"]).astype(F), F(0)).astype(F)
    inf = _infinite(b)
    ca, cb = contacts["a"].astype(np.int64), contacts["b"].astype(np.int64)
    a = np.where(inf[ca], -1, ca)
    bb = np.where(inf[cb], -1, cb)
    nx, ny = contacts["nx"], contacts["ny"]
    ln = np.sqrt(nx * nx + ny * ny)
    ok = ln > 1e-9
    with np.errstate(invalid="ignore", divide="ignore"):
        ux = np.where(ok, nx / ln, 1.0)
        uy = np.where(ok, ny / ln, 0.0)
    r = {"a": a, "b": bb, "dx": ux.astype(F), "dy": uy.astype(F),
         "rxA": (contacts["px"] - b["x"][ca]).astype(F), "ryA": (contacts["py"] - b["y"][ca]).astype(F),
         "rxB": (contacts["px"] - b["x"][cb]).astype(F), "ryB": (contacts["py"] - b["y"][cb]).astype(F)}
    r["imA"] = np.where(a >= 0, im[np.maximum(a, 0)], F(0)).astype(F)
    r["iiA"] = np.where(a >= 0, ii[np.maximum(a, 0)], F(0)).astype(F)
    r["imB"] = np.where(bb >= 0, im[np.maximum(bb, 0)], F(0)).astype(F)
    r["iiB"] = np.where(bb >= 0, ii[np.maximum(bb, 0)], F(0)).astype(F)
    return r


def _eff(r, dx, dy, mA, iA, mB, iB):
    rAxn = r["rxA"] * dy - r["ryA"] * dx
    rBxn = r["rxB"] * dy - r["ryB"] * dx
    s = mA + mB + (rAxn * rAxn) * iA + (rBxn * rBxn) * iB
    with np.errstate(divide="ignore"):
        return np.where(s < F(1e-12), F(0), F(1) / s).astype(F)


def solve(bodies, contacts, mu, iters):
    """Returns (bodies after the solve, lamN, lamF) -- the velocity fields of
    the bodies in contact (k_pgs_writeback's set), the impulses per contact.
    `contacts` in narrowphase order (each pair's contacts contiguous, in its
    clip order: lpe_rigid_download_contacts)."""
    b = bodies
    nb, nc = len(b), len(contacts)
    r = rows(b, contacts)
    # pairs: runs of equal contacts["pair"]
    first = np.flatnonzero(np.r_[True, contacts["pair"][1:] != contacts["pair"][:-1]]) if nc else np.zeros(0, int)
    cnt_p = np.diff(np.r_[first, nc])
    npairs = len(first)
    a, bb = r["a"][first], r["b"][first]
    hasA, hasB = a >= 0, bb >= 0
    ia, ib = np.maximum(a, 0), np.maximum(bb, 0)
    cr = _can_rotate(b)
    v0 = np.stack([b["vx"].astype(F), b["vy"].astype(F), np.where(cr, b["omega"].astype(F), F(0))], 1)
    cnt = np.bincount(a[hasA], minlength=nb) + np.bincount(bb[hasB], minlength=nb)
    fA = np.where(hasA, cnt[ia].astype(F), F(1)).astype(F)
    fB = np.where(hasB, cnt[ib].astype(F), F(1)).astype(F)
    imA, iiA, imB, iiB = r["imA"][first], r["iiA"][first], r["imB"][first], r["iiB"][first]
    smA, siA, smB, siB = fA * imA, fA * iiA, fB * imB, fB * iiB
    # the rows' effective masses on the scaled copies (per contact, its pair's copies)
    pid = np.repeat(np.arange(npairs), cnt_p)
    effN = _eff(r, r["dx"], r["dy"], smA[pid], siA[pid], smB[pid], siB[pid])
    effF = _eff(r, -r["dy"], r["dx"], smA[pid], siA[pid], smB[pid], siB[pid])
    mu = F(mu)
    S = np.zeros((nb, 3), np.int64)
    lamN = np.zeros(nc, F)
    lamF = np.zeros(nc, F)
    zero = np.zeros(npairs, F)
    for _ in range(iters):
        V = v0 + (S.astype(np.float64) * INV).astype(F)
        vxA = np.where(hasA, V[ia, 0], zero); vyA = np.where(hasA, V[ia, 1], zero); wA = np.where(hasA, V[ia, 2], zero)
        vxB = np.where(hasB, V[ib, 0], zero); vyB = np.where(hasB, V[ib, 1], zero); wB = np.where(hasB, V[ib, 2], zero)
        D = [zero.copy() for _ in range(6)]
        for j in range(int(cnt_p.max()) if npairs else 0):       # the pairs' j-th contacts, in order
            on = cnt_p > j
            k = first[on] + j
            sel = lambda x: x[on]
            for row in range(2):
                dx = r["dx"][k] if row == 0 else -r["dy"][k]
                dy = r["dy"][k] if row == 0 else r["dx"][k]
                eff = effN[k] if row == 0 else effF[k]
                rxA, ryA, rxB, ryB = r["rxA"][k], r["ryA"][k], r["rxB"][k], r["ryB"][k]
                ax = sel(vxA) + (-ryA) * sel(wA)
                ay = sel(vyA) + rxA * sel(wA)
                bx = sel(vxB) + (-ryB) * sel(wB)
                by = sel(vyB) + rxB * sel(wB)
                vrel = (bx - ax) * dx + (by - ay) * dy
                if row == 0:
                    old = lamN[k]
                    lo, hi = np.full(len(k), F(0)), np.full(len(k), F(1e20))
                else:
                    old = lamF[k]
                    limit = mu * lamN[k]
                    lo, hi = -limit, limit
                dl = (-eff) * (vrel + F(0))
                nl = old + dl
                nl = np.where(nl < lo, lo, nl)
                nl = np.where(nl > hi, hi, nl)
                dl = nl - old
                if row == 0:
                    lamN[k] = nl
                else:
                    lamF[k] = nl
                app = ~(np.abs(dl) < F(1e-15))
                cA = rxA * dy - ryA * dx
                cB = rxB * dy - ryB * dx
                uA, uB = app & sel(hasA), app & sel(hasB)
                vxA[on] = np.where(uA, sel(vxA) - dx * (dl * sel(smA)), sel(vxA))
                vyA[on] = np.where(uA, sel(vyA) - dy * (dl * sel(smA)), sel(vyA))
                wA[on] = np.where(uA, sel(wA) - cA * dl * sel(siA), sel(wA))
                D[0][on] = np.where(uA, D[0][on] - dx * (dl * sel(imA)), D[0][on])
                D[1][on] = np.where(uA, D[1][on] - dy * (dl * sel(imA)), D[1][on])
                D[2][on] = np.where(uA, D[2][on] - cA * dl * sel(iiA), D[2][on])
                vxB[on] = np.where(uB, sel(vxB) + dx * (dl * sel(smB)), sel(vxB))
                vyB[on] = np.where(uB, sel(vyB) + dy * (dl * sel(smB)), sel(vyB))
                wB[on] = np.where(uB, sel(wB) + cB * dl * sel(siB), sel(wB))
                D[3][on] = np.where(uB, D[3][on] + dx * (dl * sel(imB)), D[3][on])
                D[4][on] = np.where(uB, D[4][on] + dy * (dl * sel(imB)), D[4][on])
                D[5][on] = np.where(uB, D[5][on] + cB * dl * sel(iiB), D[5][on])
        q = [np.rint(d.astype(np.float64) * SCALE).astype(np.int64) for d in D]
        for u in range(3):
            np.add.at(S[:, u], a[hasA], q[u][hasA])
            np.add.at(S[:, u], bb[hasB], q[3 + u][hasB])
    V = v0 + (S.astype(np.float64) * INV).astype(F)
    out = b.copy()
    inC = np.zeros(nb, bool)
    inC[contacts["a"]] = True
    inC[contacts["b"]] = True
    w = inC & ~_infinite(b)
    out["vx"] = np.where(w, V[:, 0].astype(np.float64), b["vx"])
    out["vy"] = np.where(w, V[:, 1].astype(np.float64), b["vy"])
    out["omega"] = np.where(w & cr, V[:, 2].astype(np.float64), b["omega"])
    return out, lamN, lamF


def normal_velocity(bodies_pre, bodies_post, contacts):
    """Relative normal velocity at each contact (getRelativeVelocity,
    contact_solver.cpp:285-313) from the post-solve velocities and the
    pre-solve lever arms, in float64 (an invariant check, not a restatement)."""
    b, o = bodies_pre, bodies_post
    ca, cb = contacts["a"], contacts["b"]
    n = np.stack([contacts["nx"], contacts["ny"]], 1)
    n = n / np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-300)
    rA = np.stack([contacts["px"] - b["x"][ca], contacts["py"] - b["y"][ca]], 1)
    rB = np.stack([contacts["px"] - b["x"][cb], contacts["py"] - b["y"][cb]], 1)
    cr = _can_rotate(b)
    wA = np.where(cr[ca], o["omega"][ca], 0.0)
    wB = np.where(cr[cb], o["omega"][cb], 0.0)
    vA = np.stack([o["vx"][ca] - wA * rA[:, 1], o["vy"][ca] + wA * rA[:, 0]], 1)
    vB = np.stack([o["vx"][cb] - wB * rB[:, 1], o["vy"][cb] + wB * rB[:, 0]], 1)
    return ((vB - vA) * n).sum(1)
