// sph_coupling.h — per-particle rigid–fluid coupling (device functions).
//
// Restates rigidFluidImpulseSolver (fluid_kernels.metal:679-924) and
// rigidFluidPositionSolver (fluid_kernels.metal:533-668) for ONE particle,
// over a candidate list of rigids in ascending rigid index (the reference
// loops over all R rigids in ascending order; non-candidates fail its AABB
// test, so the candidate walk is equivalent).
#pragma once
#include "lpe_internal.h"

namespace lpe {

__device__ __forceinline__ bool pointInPolygon(float px, float py, const lpe_gpu_rigid &b) {
    int vCount = b.vertCount;
    if (vCount < 3) return false;
    bool inside = false;
    for (int i = 0, j = vCount - 1; i < vCount; j = i++) {
        float xi = b.vertsX[i], yi = b.vertsY[i];
        float xj = b.vertsX[j], yj = b.vertsY[j];
        bool intersect = ((yi > py) != (yj > py)) &&
                         (px < (xj - xi) * (py - yi) / (yj - yi) + xi);
        if (intersect) inside = !inside;
    }
    return inside;
}

__device__ __forceinline__ void closestPointOnPolygon(float px, float py, const lpe_gpu_rigid &b,
                                                      float &ox, float &oy) {
    int vCount = b.vertCount;
    ox = px; oy = py;
    if (vCount < 2) return;
    float minDistSq = 1e12f;
    for (int i = 0; i < vCount; i++) {
        int j = (i + 1) % vCount;
        float x1 = b.vertsX[i], y1 = b.vertsY[i];
        float x2 = b.vertsX[j], y2 = b.vertsY[j];
        float ex = x2 - x1, ey = y2 - y1;
        float eLenSq = ex * ex + ey * ey;
        if (eLenSq < 1e-16f) continue;
        float dx = px - x1, dy = py - y1;
        float t = (dx * ex + dy * ey) / eLenSq;
        if (t < 0.f) t = 0.f;
        if (t > 1.f) t = 1.f;
        float cx = x1 + t * ex, cy = y1 + t * ey;
        float cdx = px - cx, cdy = py - cy;
        float distSq = cdx * cdx + cdy * cdy;
        if (distSq < minDistSq) { minDistSq = distSq; ox = cx; oy = cy; }
    }
}

__device__ __forceinline__ float f2len(float x, float y) { return sqrtf(x * x + y * y); }

// The coupling's view of a rigid, rebuilt once per tick (k_rig_couple):
// 16-B aligned, so a (particle, rigid) pair loads everything it may need in
// one round of wide loads instead of a chain of scalar field loads.
//   h = (posX, posY, radius, flags: shapeType | vertCount << 8 | fast << 16)
//   v = (vx, vy, omega, mass), w = (inertia, -, -, -)
//   vt[k] = (x_2k, y_2k, x_2k+1, y_2k+1): the polygon, interleaved
// fast = the impulse solver's velocity test (metal:705-709), same arithmetic.
static constexpr int RIGC_F4 = 3 + LPE_MAX_POLY_VERTS / 2;   // float4s per record
struct RigC {
    float px, py, radius;
    int shape, nv;
    bool fast;
    float vx, vy, omega, mass, inertia;
};

// the compact record of rigid r (k_rig_couple); the polygon stays in the
// record (vert(i) reads it, L1-resident)
__device__ __forceinline__ const float4 *rigc_load(const float4 *__restrict__ rc, int r, RigC &b) {
    const float4 *q = rc + (size_t)r * RIGC_F4;
    const float4 h = q[0], v = q[1], w = q[2];
    const int fl = __float_as_int(h.w);
    b.px = h.x; b.py = h.y; b.radius = h.z;
    b.shape = fl & 0xff; b.nv = (fl >> 8) & 0xff; b.fast = (fl >> 16) & 1;
    b.vx = v.x; b.vy = v.y; b.omega = v.z; b.mass = v.w; b.inertia = w.x;
    return q + 3;
}
__device__ __forceinline__ float2 rigc_vert(const float4 *__restrict__ vt, int i) {
    const float4 p = vt[i >> 1];
    return (i & 1) ? make_float2(p.z, p.w) : make_float2(p.x, p.y);
}

// the compact AABB (minX, maxX, minY, maxY) of coupling rigid r and its
// compact coupling record (sph_coupling.h RigC), nr AABBs first
__device__ __forceinline__ void rig_couple_one(const lpe_gpu_rigid &b, int r, int nr, float maxSafeVelocitySq,
                                               float4 *__restrict__ aabb) {
    aabb[r] = make_float4(b.minX, b.maxX, b.minY, b.maxY);
    float4 *q = aabb + nr + (size_t)r * RIGC_F4;
    const bool fast = (b.vx * b.vx + b.vy * b.vy + b.omega * b.omega) > maxSafeVelocitySq;
    const int nv = min(max(b.vertCount, 0), LPE_MAX_POLY_VERTS);
    const int fl = (b.shapeType & 0xff) | ((b.shapeType == 1 ? nv : 0) << 8) | ((fast ? 1 : 0) << 16);
    q[0] = make_float4(b.posX, b.posY, b.radius, __int_as_float(b.shapeType == 0 || b.shapeType == 1 ? fl : 0xff));
    q[1] = make_float4(b.vx, b.vy, b.omega, b.mass);
    q[2] = make_float4(b.inertia, 0.f, 0.f, 0.f);
    for (int k = 0; k < LPE_MAX_POLY_VERTS / 2; k++)
        q[3 + k] = make_float4(b.vertsX[2 * k], b.vertsY[2 * k], b.vertsX[2 * k + 1], b.vertsY[2 * k + 1]);
}

// pointInPolygon / closestPointOnPolygon (above) on the compact record's
// vertices (n <= LPE_MAX_POLY_VERTS), each edge's vertices loaded once.  The
// parity test's toggles commute; the closest-point scan keeps the original
// edge order (first minimum wins).
__device__ __forceinline__ bool pip_rec(float px, float py, int n, const float4 *__restrict__ vt) {
    if (n < 3) return false;
    bool inside = false;
    float2 pj = rigc_vert(vt, n - 1);
    for (int i = 0; i < n; i++) {
        const float2 pi = rigc_vert(vt, i);
        const float xi = pi.x, yi = pi.y, xj = pj.x, yj = pj.y;
        const bool intersect = ((yi > py) != (yj > py)) && (px < (xj - xi) * (py - yi) / (yj - yi) + xi);
        if (intersect) inside = !inside;
        pj = pi;
    }
    return inside;
}
__device__ __forceinline__ void closest_rec(float px, float py, int n, const float4 *__restrict__ vt,
                                            float &ox, float &oy) {
    ox = px; oy = py;
    if (n < 2) return;
    float minDistSq = 1e12f;
    const float2 p0 = rigc_vert(vt, 0);
    float2 p1 = p0;
    for (int i = 0; i < n; i++) {
        const float2 p2 = i + 1 < n ? rigc_vert(vt, i + 1) : p0;
        float x1 = p1.x, y1 = p1.y, x2 = p2.x, y2 = p2.y;
        p1 = p2;
        float ex = x2 - x1, ey = y2 - y1;
        float eLenSq = ex * ex + ey * ey;
        if (eLenSq < 1e-16f) continue;
        float dx = px - x1, dy = py - y1;
        float t = (dx * ex + dy * ey) / eLenSq;
        if (t < 0.f) t = 0.f;
        if (t > 1.f) t = 1.f;
        float cx = x1 + t * ex, cy = y1 + t * ey;
        float cdx = px - cx, cdy = py - cy;
        float distSq = cdx * cdx + cdy * cdy;
        if (distSq < minDistSq) { minDistSq = distSq; ox = cx; oy = cy; }
    }
}

// tanh / pow of the impulse solver (metal:810, :822): fp64 rounded once to
// fp32, the same definition as oracle/sph_oracle.c.
__device__ __forceinline__ float lpe_tanhf(float x) { return (float)tanh((double)x); }
__device__ __forceinline__ float lpe_powf(float x, float e) { return (float)pow((double)x, (double)e); }

struct CoupleParams {
    float gravity, restDensity, viscosity;
    float maxForce, maxTorque, viscosityScale, depthScale, depthTransitionRate;
    float pressureForceRatio, viscousForceRatio, angDampThr, angDampFactor;
    float depthEstimateScale, maxSafeVelocitySq, minPenetration, minRelVelocity;
    float fluidForceScale, fluidForceMax, buoyancyStrength;
    float safetyMargin, relaxFactor, minSafeDistance, minPositionChange, maxCorrection;
    float boundaryOffset;
    int bx0, by0, bW, bH;
    float bcs;
    int nr;
};

// Particle state entering the coupling (after velocityVerletFinish).
struct CoupleState {
    float x, y, vx, vy, vhx, vhy, ax, ay, mass, rho, p;
};

// ---------------------------------------------------------------------------
// Rigid accumulators (accumFx, accumFy, accumTorque).  The reference adds the
// per-particle forces with float atomics (metal:892-898), in no defined
// order.  Here every accumulator is an EXACT fixed-point sum: 8 limbs of 32
// bits (held in 64-bit words, so carries can wait) covering 2^-160 .. 2^96,
// i.e. every fp32 value below 2^64 (denormals included) lands exactly; after
// the sub-steps the sum is rounded once, to nearest even, to fp32.  The
// result is the correctly rounded sum, which every order of float additions
// approximates: independent of thread scheduling, of the sort order, and of
// how the particles are split over slab ranks (the limbs all-reduce exactly
// as int64).  oracle/sph_oracle.c restates the same arithmetic.
static constexpr int XACC_LIMBS = 8;      // limb k holds bits [32k, 32k + 32) of the value * 2^160
static constexpr int XACC_BIAS = 160;

__device__ __forceinline__ void xacc_add(unsigned long long *__restrict__ acc, float f,
                                         int32_t *__restrict__ status, int range_slot) {
    const uint32_t u = __float_as_uint(f);
    const uint32_t e = (u >> 23) & 0xffu, m = u & 0x7fffffu;
    if (e == 0u && m == 0u) return;                              // +-0
    if (e >= 127u + 64u) { atomicOr(&status[range_slot], 1); return; }   // |f| >= 2^64, inf, nan
    const uint32_t M = e ? (m | 0x800000u) : m;
    const int pos = (e ? (int)e - 150 : -149) + XACC_BIAS;     // bit index of M's lsb, >= 11
    const unsigned long long v = (unsigned long long)M << (pos & 31);
    unsigned long long lo = v & 0xffffffffull, hi = v >> 32;
    if (u >> 31) { lo = 0ull - lo; hi = 0ull - hi; }             // two's complement limbs
    if (lo) atomicAdd(&acc[pos >> 5], lo);
    if (hi) atomicAdd(&acc[(pos >> 5) + 1], hi);
}

// The exact sum rounded to nearest even.
__host__ __device__ __forceinline__ float xacc_round(const unsigned long long *acc) {
    uint32_t d[XACC_LIMBS];
    long long carry = 0;
    for (int i = 0; i < XACC_LIMBS; i++) {
        const long long t = (long long)acc[i] + carry;
        d[i] = (uint32_t)((unsigned long long)t & 0xffffffffull);
        carry = t >> 32;                                         // floor division
    }
    const bool neg = carry < 0;
    if (neg) {                                                   // magnitude of the 256-bit value
        unsigned long long c = 1;
        for (int i = 0; i < XACC_LIMBS; i++) {
            const unsigned long long t = (unsigned long long)(uint32_t)~d[i] + c;
            d[i] = (uint32_t)t;
            c = t >> 32;
        }
    }
    int b = -1;
#pragma unroll
    for (int i = XACC_LIMBS - 1; i >= 0; i--)
        if (b < 0 && d[i]) b = i * 32 + 31 - __builtin_clz(d[i]);
    if (b < 0) return 0.0f;
    const int p = b - 23 > 11 ? b - 23 : 11;                      // lsb kept; bit 11 is 2^-149
    // kept = bits [p, b] (<= 24 bits, inside the 64-bit window of limbs
    // p/32 and p/32 + 1); guard = bit p - 1; sticky = any bit below it.
    // The limbs are picked by unrolled compares (no dynamic register index).
    const int li = p >> 5;
    const int gb = p - 1, gl = gb >> 5;
    uint32_t wlo = 0u, whi = 0u, gw = 0u;
    bool sticky = false;
#pragma unroll
    for (int i = 0; i < XACC_LIMBS; i++) {
        if (i == li) wlo = d[i];
        if (i == li + 1) whi = d[i];
        if (i == gl) gw = d[i];
        if (i < gl) sticky |= d[i] != 0u;
    }
    const unsigned long long win = (unsigned long long)wlo | ((unsigned long long)whi << 32);
    uint32_t kept = (uint32_t)((win >> (p & 31)) & ((1ull << (b - p + 1)) - 1ull));
    const uint32_t guard = (gw >> (gb & 31)) & 1u;
    sticky |= (gw & ((1u << (gb & 31)) - 1u)) != 0u;
    if (guard && (sticky || (kept & 1u))) kept++;
    const float r = ldexpf((float)kept, p - XACC_BIAS);          // exact
    return neg ? -r : r;
}

// One rigid's contribution to the impulse solver (metal:792-900), given the
// penetration, lever arm and normal of the particle inside it;
// effectiveArea = pow(m / densityF, 2/3), a per-particle value (couple_in).
__device__ __forceinline__ void impulse_term(const CoupleState &st, const CoupleParams &cp, float dt,
                                             const RigC &rb, float effectiveArea, int r, float pen, float relx,
                                             float rely, float nx, float ny, float densityF,
                                             float pressureF, unsigned long long *__restrict__ acq,
                                             int32_t *__restrict__ status, float &tfx_out,
                                             float &tfy_out) {
    const float py = st.y;
    float rotx = -rb.omega * rely, roty = rb.omega * relx;
    float rvx = rb.vx + rotx, rvy = rb.vy + roty;
    float relVx = st.vx - rvx, relVy = st.vy - rvy;
    float depthFactor = lpe_tanhf(cp.depthTransitionRate * pen / cp.depthScale);
    float normalVel = relVx * nx + relVy * ny;
    float nvx = nx * normalVel, nvy = ny * normalVel;
    float tvx = relVx - nvx, tvy = relVy - nvy;
    float depth = fminf(py / cp.depthEstimateScale, 1.0f);
    float hydro = densityF * cp.gravity * depth;
    float totalPressure = pressureF + hydro;
    float pressureForce = totalPressure * effectiveArea * depthFactor;
    float pfm = fminf(pressureForce, cp.maxForce * cp.pressureForceRatio);
    float pfx = nx * pfm, pfy = ny * pfm;
    float tangentVelMag = f2len(tvx, tvy);
    if (tangentVelMag > cp.minRelVelocity) {
        float tdx = tvx / tangentVelMag, tdy = tvy / tangentVelMag;
        float viscosityCoef = cp.viscosity * cp.viscosityScale;
        float viscousForce = viscosityCoef * tangentVelMag * densityF * depthFactor * dt;
        float vfm = fminf(viscousForce, cp.maxForce * cp.viscousForceRatio);
        pfx += -tdx * vfm;
        pfy += -tdy * vfm;
    }
    if (rb.mass > 0.1f) {
        float bxf = 0.0f * cp.buoyancyStrength * pen * effectiveArea * cp.gravity * densityF;
        float byf = -1.0f * cp.buoyancyStrength * pen * effectiveArea * cp.gravity * densityF;
        float cbx = pfx + bxf, cby = pfy + byf;
        if (f2len(cbx, cby) <= cp.maxForce) { pfx = cbx; pfy = cby; }
    }
    float tfx = pfx, tfy = pfy;
    float forceMag = f2len(tfx, tfy);
    if (forceMag > cp.maxForce) {
        float sc = cp.maxForce / forceMag;
        tfx = tfx * sc; tfy = tfy * sc;
    }
    float torque = relx * tfy - rely * tfx;
    torque = fminf(fmaxf(torque, -cp.maxTorque), cp.maxTorque);
    if (fabsf(rb.omega) > cp.angDampThr) {
        float sgn = (rb.omega > 0.f) ? 1.f : ((rb.omega < 0.f) ? -1.f : 0.f);
        torque -= cp.angDampFactor * sgn * fabsf(rb.omega) * rb.inertia;
    }
    unsigned long long *a = acq + (size_t)r * (3 * XACC_LIMBS);
    xacc_add(a, tfx, status, ST_XACC_RANGE);
    xacc_add(a + XACC_LIMBS, tfy, status, ST_XACC_RANGE);
    xacc_add(a + 2 * XACC_LIMBS, torque, status, ST_XACC_RANGE);
    tfx_out = tfx;
    tfy_out = tfy;
}

// The position solver's clamp, move, boundary offset and velocity projection
// (metal:640-668).
__device__ __forceinline__ void position_tail(CoupleState &st, const CoupleParams &cp, float oldx, float oldy,
                                              float acx, float acy, bool hadCollision) {
    float cm = f2len(acx, acy);
    if (cm > cp.maxCorrection) {
        acx = (acx / cm) * cp.maxCorrection;
        acy = (acy / cm) * cp.maxCorrection;
    }
    st.x -= acx;
    st.y -= acy;
    if (st.x < 0.f) st.x = cp.boundaryOffset;
    if (st.y < 0.f) st.y = cp.boundaryOffset;
    if (hadCollision) {
        float pdx = st.x - oldx, pdy = st.y - oldy;
        float pdm = f2len(pdx, pdy);
        if (pdm > cp.minPositionChange) {
            float cdx = pdx / pdm, cdy = pdy / pdm;
            float cvx = st.vx, cvy = st.vy;
            float va = cvx * cdx + cvy * cdy;
            if (va < 0.0f) {
                float restitution = 0.0f;
                cvx -= (1.0f + restitution) * va * cdx;
                cvy -= (1.0f + restitution) * va * cdy;
                st.vx = cvx; st.vy = cvy;
                st.vhx = st.vx; st.vhy = st.vy;
            }
        }
    }
}

// One (particle, rigid) pair of the two coupling solvers, for a rigid whose
// AABB holds the particle: the terms the particle's accumulators take from
// it.  Both solvers accumulate in ascending rigid order; a term is stored
// with its sign so that the fold is an addition (x - y is x + (-y) in IEEE
// arithmetic, so folding the signed terms is bit-identical to the
// reference's -= / +=).  flags: PT_COLL the particle is inside (position
// solver term in ax, ay), PT_IMP the impulse solver ran (fluid force term in
// fx, fy; rigid accumulators already added).
struct PairTerm { float ax, ay, fx, fy; };
static constexpr int PT_COLL = 1, PT_IMP = 2;

// the particle's inputs of the pair computation
struct CoupleIn {
    float x, y, vx, vy, mass, densityF, pressureF, effArea;
};

// (trace builds, -DLPE_FTRACE: the stages of one pair, each after a wait for
// its memory operations, as the maximum over lanes of the time since the
// pair's start -- profiles/forces_trace.py; the shipped build has no stamps)
#if defined(LPE_FTRACE) && !defined(LPE_FTRACE_NOCPT)
#define CPT0() const unsigned long long cpt0_ = wall_clock64()
#define CPT(k) do { if (cp_tr) { __builtin_amdgcn_s_waitcnt(0); atomicMax(cp_tr + (k), wall_clock64() - cpt0_); } } while (0)
#else
#define CPT0() do {} while (0)
#define CPT(k) do {} while (0)
#endif
__device__ __forceinline__ int couple_pair(const CoupleIn &in, const CoupleParams &cp, float dt, bool impulse,
                                           const float4 *__restrict__ rc, int r,
                                           unsigned long long *__restrict__ acq, int32_t *__restrict__ status,
                                           PairTerm &t, unsigned long long *cp_tr = nullptr) {
    (void)cp_tr;
    CPT0();
    RigC rb;
    const float4 *vt = rigc_load(rc, r, rb);
#if defined(LPE_FTRACE) && !defined(LPE_FTRACE_NOCPT)
    if (rb.nv == 255) t.ax = rb.px;        // (consumes the record before the first stamp)
#endif
    CPT(0);
    const float px = in.x, py = in.y;
    CoupleState st;                    // the fields impulse_term reads
    st.x = px; st.y = py; st.vx = in.vx; st.vy = in.vy; st.mass = in.mass;
    st.vhx = st.vhy = st.ax = st.ay = st.rho = st.p = 0.f;
    const bool doImp = impulse && !rb.fast;
    int flags = 0;
    float tfx = 0.f, tfy = 0.f;
    if (rb.shape == 0) {
        const float rx = px - rb.px, ry = py - rb.py;
        const float dist2 = rx * rx + ry * ry;
        const float radius = rb.radius;
        if (!(dist2 < radius * radius)) return 0;
        const float dist0 = sqrtf(dist2);
        if (doImp) {
            float dist = dist0;
            if (dist < cp.minPenetration) dist = cp.minPenetration;
            float pen = radius - dist;
            if (pen < 0.0f) pen = 0.0f;
            if (!(pen < cp.minPenetration)) {
                impulse_term(st, cp, dt, rb, in.effArea, r, pen, rx, ry, rx / dist, ry / dist, in.densityF,
                             in.pressureF, acq, status, tfx, tfy);
                flags |= PT_IMP;
            }
        }
        float dist = dist0, dx = rx, dy = ry;
        if (dist < cp.minSafeDistance) { dist = cp.minSafeDistance; dx = 1.0f; dy = 0.0f; }
        const float pen = (radius - dist) + cp.safetyMargin;
        const float dirx = dx / dist, diry = dy / dist;
        t.ax = -(dirx * pen * cp.relaxFactor);                 // acx -= ...
        t.ay = -(diry * pen * cp.relaxFactor);
    } else if (rb.shape == 1) {
        if (rb.nv < 3 || !pip_rec(px, py, rb.nv, vt)) { CPT(1); return 0; }
        CPT(1);
        float cx, cy;
        closest_rec(px, py, rb.nv, vt, cx, cy);
        const float dx = px - cx, dy = py - cy;
        const float d0 = sqrtf(dx * dx + dy * dy);
        CPT(2);
        if (doImp) {
            float d = d0;
            if (d < cp.minPenetration) d = cp.minPenetration;
            float pen = d;
            if (pen < 0.0f) pen = 0.0f;
            if (!(pen < cp.minPenetration)) {
                impulse_term(st, cp, dt, rb, in.effArea, r, pen, px - rb.px, py - rb.py, dx / d, dy / d,
                             in.densityF, in.pressureF, acq, status, tfx, tfy);
                flags |= PT_IMP;
            }
        }
        CPT(3);
        float d = d0, cdx = dx, cdy = dy;
        if (d < cp.minSafeDistance) { d = cp.minSafeDistance; cdx = 1.0f; cdy = 0.0f; }
        const float pen = d + cp.safetyMargin;
        const float dirx = cdx / d, diry = cdy / d;
        t.ax = dirx * pen * cp.relaxFactor;                    // acx += ...
        t.ay = diry * pen * cp.relaxFactor;
    } else {
        return 0;
    }
    t.fx = -(tfx * cp.fluidForceScale);                        // tffx -= tfx * fluidForceScale
    t.fy = -(tfy * cp.fluidForceScale);
    return flags | PT_COLL;
}

// couple_pair in two halves, so the forces pass can compute the geometry
// (containment, closest point, penetration, normal, the position solver's
// term) while the particle's fluid forces are still being summed, and the
// impulse solver's term (which needs the finished velocity) afterwards.  The
// same operations in the same order as couple_pair: bit-identical terms.
// PT_WANT: the impulse solver runs for the pair (pen, nx, ny hold its input).
static constexpr int PT_WANT = 4;
struct PairGeo { float ax, ay, pen, nx, ny; };

__device__ __forceinline__ int couple_geom(float px, float py, const CoupleParams &cp, bool impulse,
                                           const float4 *__restrict__ rc, int r, PairGeo &g) {
    RigC rb;
    const float4 *vt = rigc_load(rc, r, rb);
    const bool doImp = impulse && !rb.fast;
    int flags = 0;
    g.pen = g.nx = g.ny = 0.f;
    if (rb.shape == 0) {
        const float rx = px - rb.px, ry = py - rb.py;
        const float dist2 = rx * rx + ry * ry;
        const float radius = rb.radius;
        if (!(dist2 < radius * radius)) return 0;
        const float dist0 = sqrtf(dist2);
        if (doImp) {
            float dist = dist0;
            if (dist < cp.minPenetration) dist = cp.minPenetration;
            float pen = radius - dist;
            if (pen < 0.0f) pen = 0.0f;
            if (!(pen < cp.minPenetration)) {
                g.pen = pen; g.nx = rx / dist; g.ny = ry / dist;
                flags |= PT_WANT;
            }
        }
        float dist = dist0, dx = rx, dy = ry;
        if (dist < cp.minSafeDistance) { dist = cp.minSafeDistance; dx = 1.0f; dy = 0.0f; }
        const float pen = (radius - dist) + cp.safetyMargin;
        const float dirx = dx / dist, diry = dy / dist;
        g.ax = -(dirx * pen * cp.relaxFactor);                 // acx -= ...
        g.ay = -(diry * pen * cp.relaxFactor);
    } else if (rb.shape == 1) {
        if (rb.nv < 3 || !pip_rec(px, py, rb.nv, vt)) return 0;
        float cx, cy;
        closest_rec(px, py, rb.nv, vt, cx, cy);
        const float dx = px - cx, dy = py - cy;
        const float d0 = sqrtf(dx * dx + dy * dy);
        if (doImp) {
            float d = d0;
            if (d < cp.minPenetration) d = cp.minPenetration;
            float pen = d;
            if (pen < 0.0f) pen = 0.0f;
            if (!(pen < cp.minPenetration)) {
                g.pen = pen; g.nx = dx / d; g.ny = dy / d;
                flags |= PT_WANT;
            }
        }
        float d = d0, cdx = dx, cdy = dy;
        if (d < cp.minSafeDistance) { d = cp.minSafeDistance; cdx = 1.0f; cdy = 0.0f; }
        const float pen = d + cp.safetyMargin;
        const float dirx = cdx / d, diry = cdy / d;
        g.ax = dirx * pen * cp.relaxFactor;                    // acx += ...
        g.ay = diry * pen * cp.relaxFactor;
    } else {
        return 0;
    }
    return flags | PT_COLL;
}

// the impulse solver's half of a pair whose geometry asked for it (PT_WANT):
// the rigid accumulators take the force, the particle the returned term
__device__ __forceinline__ void couple_imp(const CoupleIn &in, const CoupleParams &cp, float dt,
                                           const float4 *__restrict__ rc, int r, float pen, float nx, float ny,
                                           unsigned long long *__restrict__ acq, int32_t *__restrict__ status,
                                           float &fx, float &fy) {
    RigC rb;
    (void)rigc_load(rc, r, rb);
    CoupleState st;                    // the fields impulse_term reads
    st.x = in.x; st.y = in.y; st.vx = in.vx; st.vy = in.vy; st.mass = in.mass;
    st.vhx = st.vhy = st.ax = st.ay = st.rho = st.p = 0.f;
    float tfx, tfy;
    // lever arm: px - rb.px (circle: rx; polygon: px - rb.px, metal:856-857)
    impulse_term(st, cp, dt, rb, in.effArea, r, pen, in.x - rb.px, in.y - rb.py, nx, ny, in.densityF,
                 in.pressureF, acq, status, tfx, tfy);
    fx = -(tfx * cp.fluidForceScale);                          // tffx -= tfx * fluidForceScale
    fy = -(tfy * cp.fluidForceScale);
}

// the per-particle accumulators of the two solvers
struct CoupleAcc {
    float tffx = 0.f, tffy = 0.f, acx = 0.f, acy = 0.f;
    bool had = false, hadCollision = false;
    __device__ __forceinline__ void fold(const PairTerm &t, int flags) {
        if (!(flags & PT_COLL)) return;
        if (flags & PT_IMP) { tffx = tffx + t.fx; tffy = tffy + t.fy; had = true; }
        hadCollision = true;
        acx = acx + t.ax;
        acy = acy + t.ay;
    }
};

// area: the particle has impulse-solver candidates (pow only then)
__device__ __forceinline__ CoupleIn couple_in(const CoupleState &st, const CoupleParams &cp, bool area) {
    CoupleIn in;
    in.x = st.x; in.y = st.y; in.vx = st.vx; in.vy = st.vy; in.mass = st.mass;
    in.densityF = st.rho > 0.0f ? st.rho : cp.restDensity;
    in.pressureF = st.p;
    in.effArea = area ? lpe_powf(st.mass / in.densityF, 2.0f / 3.0f) : 0.f;   // metal:818-822
    return in;
}

// the impulse solver's fluid force on the particle and the position solver's
// move (metal:900-924, :640-668), after every pair was folded
__device__ __forceinline__ void couple_finish(CoupleState &st, const CoupleParams &cp, const CoupleAcc &a) {
    const float oldx = st.x, oldy = st.y;
    if (a.had) {
        float tffx = a.tffx, tffy = a.tffy;
        float fm = f2len(tffx, tffy);
        if (fm > cp.fluidForceMax) {
            float sc = cp.fluidForceMax / fm;
            tffx = tffx * sc; tffy = tffy * sc;
        }
        float invMass = (st.mass > 0.0001f) ? 1.0f / st.mass : 1.0f;
        st.ax += tffx * invMass;
        st.ay += tffy * invMass;
    }
    position_tail(st, cp, oldx, oldy, a.acx, a.acy, a.hadCollision);
}

// rigidFluidImpulseSolver (metal:679-924) followed by rigidFluidPositionSolver
// (metal:533-668; always dispatched, fluid.cpp:929-942) for one particle, in
// one pass over its candidate rigids.  The position solver tests exactly the
// rigids whose AABB holds the particle (the impulse solver additionally skips
// fast rigids), at the same position (the impulse solver only changes the
// acceleration), so the containment and closest-point geometry is computed
// once per (particle, rigid) and each solver accumulates in candidate order
// exactly as the two separate loops.  aabb[k] = (minX, maxX, minY, maxY) of
// candidate list[k] (bin order): one 16-B load per candidate, the compact
// record only for AABB hits.
__device__ __forceinline__ bool aabb_holds(const float4 &bb, float px, float py) {
    return !(px < bb.x || px > bb.y || py < bb.z || py > bb.w);
}
__device__ __forceinline__ void couple_both(CoupleState &st, const CoupleParams &cp, float dt, bool impulse,
                                           const float4 *__restrict__ rc, const float4 *__restrict__ aabb,
                                           const int32_t *__restrict__ list, int k0, int k1,
                                           unsigned long long *__restrict__ acq,
                                           int32_t *__restrict__ status) {
    const CoupleIn in = couple_in(st, cp, impulse && k1 > k0);
    CoupleAcc a;
    constexpr int U = 4;
    for (int k = k0; k < k1; k += U) {
        int rr[U];
        float4 bb[U];
#pragma unroll
        for (int u = 0; u < U; u++) rr[u] = list[min(k + u, k1 - 1)];
#pragma unroll
        for (int u = 0; u < U; u++) bb[u] = aabb[min(k + u, k1 - 1)];   // bin-ordered AABBs
#pragma unroll
        for (int u = 0; u < U; u++)
            if (k + u < k1 && aabb_holds(bb[u], in.x, in.y)) {
                PairTerm t;
                const int f = couple_pair(in, cp, dt, impulse, rc, rr[u], acq, status, t);
                a.fold(t, f);
            }
    }
    couple_finish(st, cp, a);
}

}  // namespace lpe
