// lpe_rigid.hip — rigid-body path of the MI355X backend
// (Systems::RigidBodyCollisionSystem, src/systems/rigid/*.cpp, and the
// integrator systems src/systems/{boundary,gravity,rotation,movement,sleep}.cpp).
//
// Device pipeline of one RigidBodyCollisionSystem::update
// (rigid_body_collision.cpp:24-50):
//   k_rb_prep       per-body AABB (computeAABB, broadphase.cpp:158-191) and
//                   the candidate test (Solid + Mass + Phase, inside the
//                   quadtree root, broadphase.cpp:200-223)
//   k_bg_*          uniform-grid broadphase in entity-id order: the pair SET
//                   of detectCollisions (broadphase.cpp:233-295), which equals
//                   brute force over the inserted boxes; emitted in canonical
//                   (eid_a, eid_b) order by count -> scan -> fill -> segment sort
//   k_narrow        one thread per pair, fp64: GJK (gjk.cpp:73-123), EPA
//                   (epa.cpp:32-97), single contacts or reference-face
//                   clipping (narrowphase.cpp:126-350); contacts compacted in
//                   pair order
//   PGS             rows in fp32 (contact_solver.cpp:133-253); the sequential
//                   Gauss-Seidel sweep (solveLcpPgs, :381-440) is executed
//                   level by level: an item's level is one more than the level
//                   of the previous item (in sweep order) sharing a dynamic
//                   body, so every level is a set of independent rows and the
//                   result is bit-identical to the sequential sweep in the same
//                   order.  One 1024-thread workgroup, body velocities in LDS.
//   position solver the same schedule over contacts in narrowphase order,
//                   fp64 (position_solver.cpp:215-290), body poses in LDS.
// Orders: canonical (pairs by entity id; manifolds = pairs) by default, or
// caller-supplied (lpe_rigid_step_ordered) to replay the reference's quadtree
// and std::unordered_map orders bit for bit.
#include <atomic>
#include "lpe_internal.h"
#include "rigid_dev.h"
#include "lpe_trig.h"
#include "lpe_trace.h"
#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

namespace lpe {

RigidDev *rigid_dev(lpe_ctx *ctx) {
    if (!ctx->rigid) ctx->rigid = new RigidDev();
    return (RigidDev *)ctx->rigid;
}
static RigidDev *rdev(lpe_ctx *ctx) { return rigid_dev(ctx); }

// ---------------------------------------------------------------------------
// generic exclusive scan of n ints (3 launches); start has n+1 entries
__device__ __forceinline__ int r_wave_incl(int v) {
    int lane = threadIdx.x & 63;
    for (int off = 1; off < 64; off <<= 1) {
        int t = __shfl_up(v, off);
        if (lane >= off) v += t;
    }
    return v;
}
__device__ __forceinline__ int r_block_excl(int v, int *total) {
    __shared__ int wsum[RTPB / 64];
    int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = r_wave_incl(v);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int off = 0, tot = 0;
    for (int k = 0; k < RTPB / 64; k++) { if (k < w) off += wsum[k]; tot += wsum[k]; }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}
__global__ void __launch_bounds__(RTPB) k_rscan_reduce(const int32_t *nptr, int ncap,
                                                       const int32_t *__restrict__ cnt,
                                                       int32_t *__restrict__ bsum) {
    int n = nptr ? min(*nptr, ncap) : ncap;   // a count past the capacity (overflow, redone) is clipped
    int base = blockIdx.x * 1024;
    int s = 0;
    for (int k = 0; k < 4; k++) {
        int c = base + k * RTPB + threadIdx.x;
        if (c < n) s += cnt[c];
    }
    int tot;
    (void)r_block_excl(s, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(RTPB) k_rscan_blocks(const int32_t *nptr, int ncap,
                                                       int32_t *__restrict__ bsum,
                                                       int32_t *__restrict__ start) {
    int n = nptr ? min(*nptr, ncap) : ncap;   // a count past the capacity (overflow, redone) is clipped
    int nb = (n + 1023) / 1024;
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += RTPB) {
        int b = b0 + threadIdx.x;
        int v = (b < nb) ? bsum[b] : 0;
        int tot;
        int ex = r_block_excl(v, &tot);
        if (b < nb) bsum[b] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) start[n] = carry;
}
// fused (<= 1,024 tiles): bsum holds the raw tile totals and each block sums
// the ones before it (k_rscan_blocks' work, one launch fewer); block 0 stores
// the total at start[n]
__global__ void __launch_bounds__(RTPB) k_rscan_final(const int32_t *nptr, int ncap,
                                                      const int32_t *__restrict__ cnt,
                                                      const int32_t *__restrict__ bsum,
                                                      int32_t *__restrict__ start,
                                                      int32_t *__restrict__ cursor, int fused) {
    int n = nptr ? min(*nptr, ncap) : ncap;   // a count past the capacity (overflow, redone) is clipped
    int base = blockIdx.x * 1024 + threadIdx.x * 4;
    int pfx = 0;
    if (fused) {
        const int nt = (n + 1023) / 1024;
        int pre = 0, all = 0;
        for (int t = threadIdx.x; t < nt; t += RTPB) {
            const int v = bsum[t];
            pre += t < (int)blockIdx.x ? v : 0;
            all += v;
        }
        int tp, ta;
        (void)r_block_excl(pre, &tp);
        (void)r_block_excl(all, &ta);
        pfx = tp;
        if (blockIdx.x == 0 && threadIdx.x == 0) start[n] = ta;
    } else if (base < n || threadIdx.x == 0) {
        pfx = bsum[blockIdx.x];
    }
    int v[4], s = 0;
    for (int k = 0; k < 4; k++) { int c = base + k; v[k] = (c < n) ? cnt[c] : 0; s += v[k]; }
    int tot;
    int ex = r_block_excl(s, &tot) + pfx;
    for (int k = 0; k < 4; k++) {
        int c = base + k;
        if (c < n) { start[c] = ex; if (cursor) cursor[c] = ex; }
        ex += v[k];
    }
}

// the whole scan in one block (capacities of a few tiles: one launch instead
// of two), tile by tile with a running carry; also copies the total to
// *total_out when given (the pair count the narrowphase reads)
__global__ void __launch_bounds__(RTPB) k_rscan_single(const int32_t *nptr, int ncap,
                                                       const int32_t *__restrict__ cnt,
                                                       int32_t *__restrict__ start,
                                                       int32_t *__restrict__ cursor,
                                                       int32_t *__restrict__ total_out) {
    const int n = nptr ? min(*nptr, ncap) : ncap;   // a count past the capacity (overflow, redone) is clipped
    int carry = 0;
    for (int t0 = 0; t0 < n; t0 += 1024) {
        const int base = t0 + threadIdx.x * 4;
        int v[4], s = 0;
        for (int k = 0; k < 4; k++) { const int c = base + k; v[k] = (c < n) ? cnt[c] : 0; s += v[k]; }
        int tot;
        int ex = r_block_excl(s, &tot) + carry;
        for (int k = 0; k < 4; k++) {
            const int c = base + k;
            if (c < n) { start[c] = ex; if (cursor) cursor[c] = ex; }
            ex += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        start[n] = carry;
        if (total_out) *total_out = carry;
    }
}
static constexpr int RSCAN_SINGLE_MAX = 4096;   // capacities scanned by k_rscan_single

// ---------------------------------------------------------------------------
// geometry (fp64), restating vector_math.cpp / polygon.hpp
struct D2 { double x, y; };
__device__ __forceinline__ D2 d2(double x, double y) { D2 r; r.x = x; r.y = y; return r; }
__device__ __forceinline__ D2 sub(D2 a, D2 b) { return d2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ D2 add(D2 a, D2 b) { return d2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ D2 neg(D2 a) { return d2(-a.x, -a.y); }
__device__ __forceinline__ D2 mul(D2 a, double s) { return d2(a.x * s, a.y * s); }
__device__ __forceinline__ double dot(D2 a, D2 b) { return a.x * b.x + a.y * b.y; }
__device__ __forceinline__ double crs(D2 a, D2 b) { return a.x * b.y - a.y * b.x; }
__device__ __forceinline__ D2 nrm(D2 a) {                       // vector_math.cpp:130-137
    double len = sqrt(a.x * a.x + a.y * a.y);
    if (len > 1e-9) return d2(a.x / len, a.y / len);
    return d2(1.0, 0.0);
}

struct DShape {
    bool circle;
    double radius;
    D2 pos;
    double angle;
    const double *lv;
    int nv;
};
__device__ __forceinline__ DShape dshape(const lpe_body &b, const double *verts) {
    DShape s;
    s.circle = (b.flags & LPE_BODY_CIRCLE) != 0;
    s.radius = s.circle ? b.radius : 0.0;
    s.pos = d2(b.x, b.y);
    s.angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
    s.lv = verts + 2 * (size_t)b.vert_off;
    s.nv = s.circle ? 0 : b.vert_cnt;
    return s;
}
__device__ D2 support1(const DShape &s, D2 d) {
    if (s.circle) {                                               // polygon.hpp:90-101
        double len = sqrt(d.x * d.x + d.y * d.y);
        D2 dn = d;
        if (len > 1e-9) { dn.x /= len; dn.y /= len; }
        return d2(s.pos.x + dn.x * s.radius, s.pos.y + dn.y * s.radius);
    }
    double c = lpe_cos(s.angle), sn = lpe_sin(s.angle);                 // polygon.hpp:55-76
    double best = -1e9;
    D2 bp = d2(0.0, 0.0);
    for (int i = 0; i < s.nv; i++) {
        double lx = s.lv[2 * i], ly = s.lv[2 * i + 1];
        double wx = s.pos.x + (lx * c - ly * sn);
        double wy = s.pos.y + (lx * sn + ly * c);
        double proj = wx * d.x + wy * d.y;
        if (proj > best) { best = proj; bp = d2(wx, wy); }
    }
    return bp;
}
__device__ __forceinline__ D2 support(const DShape &A, const DShape &B, D2 d) {
    D2 pA = support1(A, d);
    D2 pB = support1(B, d2(-d.x, -d.y));
    return d2(pA.x - pB.x, pA.y - pB.y);
}

// GJKIntersect (gjk.cpp:73-123) with handleSimplex (:9-71); pts[0] oldest
__device__ bool gjk(const DShape &A, const DShape &B, D2 *pts, int &np) {
    D2 dir = d2(1, 0);
    np = 0;
    pts[np++] = support(A, B, dir);
    if (dot(pts[0], dir) < 0) return false;
    dir = neg(pts[0]);
    int it = 0;
    while (true) {
        it++;
        if (it > 100) return false;
        D2 p = support(A, B, dir);
        double proj = dot(p, dir);
        if (proj < 0) return false;
        pts[np++] = p;
        if (np == 2) {
            D2 a = pts[1], b = pts[0];
            D2 ab = sub(b, a), ao = neg(a);
            if (dot(ab, ao) > 0) {
                D2 perp = d2(-ab.y, ab.x);
                if (dot(perp, ao) < 0) perp = d2(ab.y, -ab.x);
                dir = perp;
            } else {
                pts[0] = a; np = 1;
                dir = ao;
            }
        } else {
            D2 a = pts[2], b = pts[1], c = pts[0];
            D2 ab = sub(b, a), ac = sub(c, a), ao = neg(a);
            D2 abPerp = d2(ab.y, -ab.x);
            if (dot(abPerp, ac) > 0) abPerp = d2(-ab.y, ab.x);
            D2 acPerp = d2(ac.y, -ac.x);
            if (dot(acPerp, ab) > 0) acPerp = d2(-ac.y, ac.x);
            if (dot(ab, ao) > 0 && dot(abPerp, ao) > 0) {
                pts[0] = pts[1]; pts[1] = pts[2]; np = 2;       // erase(begin)
                dir = abPerp;
            } else if (dot(ac, ao) > 0 && dot(acPerp, ao) > 0) {
                pts[1] = pts[2]; np = 2;                         // erase(begin + 1)
                dir = acPerp;
            } else {
                return true;
            }
        }
    }
}

// EPA (epa.cpp:32-97)
__device__ bool epa(const DShape &A, const DShape &B, const D2 *simplex, D2 &n, double &pen) {
    D2 poly[EPA_MAX];
    int np = 3;
    poly[0] = simplex[0]; poly[1] = simplex[1]; poly[2] = simplex[2];
    {
        D2 ab = sub(poly[1], poly[0]), ac = sub(poly[2], poly[0]);
        if (fabs(crs(ab, ac)) < 1e-14) return false;
    }
    {
        double cv = (poly[1].x - poly[0].x) * (poly[2].y - poly[0].y) -
                    (poly[1].y - poly[0].y) * (poly[2].x - poly[0].x);
        if (cv < 0) { D2 t = poly[0]; poly[0] = poly[2]; poly[2] = t; }
    }
    for (int iter = 0; iter < 100; iter++) {
        double closest = 1.7976931348623157e308;
        int ce = -1;
        D2 en = d2(0, 0);
        for (int i = 0; i < np; i++) {
            int j = (i + 1) % np;
            D2 e = sub(poly[j], poly[i]);
            D2 nn = nrm(d2(e.y, -e.x));
            double dist = dot(nn, poly[i]);
            if (dist < 0) { nn.x = -nn.x; nn.y = -nn.y; dist = -dist; }
            if (dist < closest) { closest = dist; ce = i; en = nn; }
        }
        if (ce < 0) return false;
        D2 p = support(A, B, en);
        double d = dot(p, en);
        if (d - closest < 1e-9) { n = en; pen = d; return true; }
        int at = (ce + 1) % np;
        for (int k = np; k > at; k--) poly[k] = poly[k - 1];
        poly[at] = p;
        np++;
    }
    return false;
}

__device__ __forceinline__ void world_verts(const DShape &s, D2 *v) {  // narrowphase.cpp:56-81
    for (int i = 0; i < s.nv; i++) {
        double lx = s.lv[2 * i], ly = s.lv[2 * i + 1];
        double rx = lx * lpe_cos(s.angle) - ly * lpe_sin(s.angle);
        double ry = lx * lpe_sin(s.angle) + ly * lpe_cos(s.angle);
        v[i] = d2(s.pos.x + rx, s.pos.y + ry);
    }
}
__device__ int clip_face(const D2 *in, int n, D2 pn, double off, D2 *out) {  // :203-234
    int m = 0;
    for (int i = 0; i < n; i++) {
        int j = (i + 1) % n;
        D2 p1 = in[i], p2 = in[j];
        double dd1 = dot(pn, p1) - off, dd2 = dot(pn, p2) - off;
        bool in1 = dd1 <= 0.0, in2 = dd2 <= 0.0;
        if (in1 && m < CLIP_MAX) out[m++] = p1;
        if (in1 != in2 && m < CLIP_MAX) {
            double t = dd1 / (dd1 - dd2);
            out[m++] = add(p1, mul(sub(p2, p1), t));
        }
    }
    return m;
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ bool body_candidate(const lpe_body &b) {
    return (b.flags & LPE_BODY_HAS_MASS) && (b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_SOLID);
}

// (also zeroes what the detection after it counts into: counts [0..3], [6],
// [10], [11], the per-body pair counts and the broadphase cell counts -- six
// memset launches fewer at the head of the detection)
__global__ void k_rb_prep(int nb, const lpe_body *__restrict__ bodies, const double *__restrict__ verts,
                          double lo, double hi, double4 *__restrict__ aabb, int32_t *__restrict__ cand,
                          int32_t *__restrict__ counts, int32_t *__restrict__ pcount, int32_t *__restrict__ bgCount,
                          int cells, int32_t *__restrict__ inContact) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i == 0) {
        counts[0] = counts[1] = counts[2] = counts[3] = 0;
        counts[6] = counts[10] = counts[11] = 0;
    }
    for (int c = i; c < cells; c += (int)gridDim.x * RTPB) bgCount[c] = 0;
    if (i < nb) {
        pcount[i] = 0;
        inContact[i] = 0;                // (and the solvers' contact marks, for colour_prep)
        inContact[nb + i] = 0;
    }
    if (i >= nb) return;
    const lpe_body b = bodies[i];
    double mnx, mny, mxx, mxy;
    double angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
    if (b.flags & LPE_BODY_CIRCLE) {
        double r = b.radius;
        mnx = b.x - r; mxx = b.x + r; mny = b.y - r; mxy = b.y + r;
    } else {
        mnx = b.x; mxx = b.x; mny = b.y; mxy = b.y;
        const double *lv = verts + 2 * (size_t)b.vert_off;
        for (int k = 0; k < b.vert_cnt; k++) {
            double vx = lv[2 * k], vy = lv[2 * k + 1];
            double rx = vx * lpe_cos(angle) - vy * lpe_sin(angle);
            double ry = vx * lpe_sin(angle) + vy * lpe_cos(angle);
            double wx = b.x + rx, wy = b.y + ry;
            if (wx < mnx) mnx = wx;
            if (wx > mxx) mxx = wx;
            if (wy < mny) mny = wy;
            if (wy > mxy) mxy = wy;
        }
    }
    aabb[i] = make_double4(mnx, mny, mxx, mxy);
    bool ok = body_candidate(b) && !(mxx < lo || mnx > hi || mxy < lo || mny > hi);
    cand[i] = ok ? 1 : 0;
}

// each body's pair list sorted by partner rank (the ranks in a list are
// distinct), four bodies per block: a list of up to BP_SHORT entries by its
// wave, in registers (an entry's place is the number of smaller keys); a
// longer one (the walls' lists, filled by many threads in arrival order) by
// the whole block afterwards, bitonic-sorted in LDS
static constexpr int BP_SHORT = 64;
static constexpr int BP_LONG = 4096;       // longest list sorted in LDS (longer: one thread)
__global__ void __launch_bounds__(RTPB)
k_bp_sort(int nb, const int32_t *__restrict__ pstart, int2 *__restrict__ pairs,
          int32_t *__restrict__ rk, int cap_pairs) {
    const int r0 = blockIdx.x * (RTPB / 64);
    const int r = r0 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r < nb) {
        const int s = pstart[r], e = min(pstart[r + 1], cap_pairs), n = e - s;
        if (n > BP_LONG) {                                   // (never expected) one lane, in place
            if (lane == 0)
                for (int k = s + 1; k < e; k++) {
                    int v = rk[k];
                    int2 p = pairs[k];
                    int j = k - 1;
                    while (j >= s && rk[j] > v) { rk[j + 1] = rk[j]; pairs[j + 1] = pairs[j]; j--; }
                    rk[j + 1] = v; pairs[j + 1] = p;
                }
        } else if (n > 1 && n <= BP_SHORT) {
            const int key = lane < n ? rk[s + lane] : 0x7fffffff;
            const int2 val = lane < n ? pairs[s + lane] : make_int2(0, 0);
            int rank = 0;
            for (int j = 0; j < n; j++) rank += __shfl(key, j) < key ? 1 : 0;
            if (lane < n) { rk[s + rank] = key; pairs[s + rank] = val; }
        }
    }
    __shared__ int key[BP_LONG];
    __shared__ int2 val[BP_LONG];
    for (int w = 0; w < RTPB / 64; w++) {                    // (block-uniform)
        const int rb = r0 + w;
        if (rb >= nb) break;
        const int s = pstart[rb], e = min(pstart[rb + 1], cap_pairs), n = e - s;
        if (n <= BP_SHORT || n > BP_LONG) continue;
        int m = 1;
        while (m < n) m <<= 1;
        for (int i = threadIdx.x; i < m; i += RTPB) {
            key[i] = i < n ? rk[s + i] : 0x7fffffff;
            val[i] = i < n ? pairs[s + i] : make_int2(0, 0);
        }
        __syncthreads();
        for (int size = 2; size <= m; size <<= 1)
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int i = threadIdx.x; i < m; i += RTPB) {
                    const int j = i ^ stride;
                    if (j > i) {
                        const bool up = (i & size) == 0;
                        if ((key[i] > key[j]) == up) {
                            const int tk = key[i]; key[i] = key[j]; key[j] = tk;
                            const int2 tv = val[i]; val[i] = val[j]; val[j] = tv;
                        }
                    }
                }
                __syncthreads();
            }
        for (int i = threadIdx.x; i < n; i += RTPB) { rk[s + i] = key[i]; pairs[s + i] = val[i]; }
        __syncthreads();                                     // (LDS reused by the next long list)
    }
}

// ---- uniform-grid broadphase --------------------------------------------
// The reference's pair set (broadphase.cpp:35-295: AABB overlap, not two
// boundary bodies, not two small particles) in entity-id order (pairs of the
// lower-ranked body, partners sorted by rank by k_bp_sort), from a uniform
// grid: a body whose AABB extent is at most the cell size g and whose AABB
// min corner lies on the grid is keyed by that corner's cell; two such bodies
// can only overlap if their keys are at most one cell apart.  The others
// ("special": walls, bodies off the grid) are tested against every candidate.
__device__ __forceinline__ bool bp_pair_ok(const double4 &A, const double4 &B, bool aB, bool bB, double sa,
                                           double sb, double small) {
    if (A.z < B.x || A.x > B.z) return false;               // boxesOverlap (broadphase.cpp:35-39)
    if (A.w < B.y || A.y > B.w) return false;
    if (aB && bB) return false;
    if (sa < small && sb < small) return false;
    return true;
}

__global__ void k_bg_key(int nb, const int32_t *__restrict__ byRank, const double4 *__restrict__ aabb,
                         const int32_t *__restrict__ cand, double org, double g, int G,
                         int32_t *__restrict__ key, int32_t *__restrict__ cellCount,
                         int32_t *__restrict__ special, int32_t *__restrict__ nspecial) {
    int r = blockIdx.x * RTPB + threadIdx.x;
    if (r >= nb) return;
    const int ia = byRank[r];
    int k = -1;                                              // not a candidate
    if (cand[ia]) {
        const double4 A = aabb[ia];
        const double ext = fmax(A.z - A.x, A.w - A.y);
        const double fx = floor((A.x - org) / g), fy = floor((A.y - org) / g);
        if (ext <= g && fx >= 0.0 && fy >= 0.0 && fx < (double)G && fy < (double)G) {
            k = (int)fy * G + (int)fx;
            atomicAdd(&cellCount[k], 1);
        } else {
            k = -2;
            special[atomicAdd(nspecial, 1)] = r;
        }
    }
    key[r] = k;
}

__global__ void k_bg_fill(int nb, const int32_t *__restrict__ key, int32_t *__restrict__ cursor,
                          int32_t *__restrict__ list) {
    int r = blockIdx.x * RTPB + threadIdx.x;
    if (r >= nb) return;
    const int k = key[r];
    if (k >= 0) list[atomicAdd(&cursor[k], 1)] = r;
}

// mode 0 counts (pcount of the lower rank), 1 fills (cursor from pstart).
// One wave per body rank: the lanes take the candidates of its (up to 3x3)
// cells as one flat index space, then the special bodies, so a body's tests
// run in parallel instead of as a chain of dependent loads.  The emission
// order is free (each body's list is sorted by partner rank afterwards).
static constexpr int BG_WAVES = RTPB / 64;                 // bodies per block
__global__ void __launch_bounds__(RTPB)
k_bg_pairs(int nb, int mode, const int32_t *__restrict__ byRank,
           const lpe_body *__restrict__ bodies, const double4 *__restrict__ aabb,
           double small, int G, const int32_t *__restrict__ key,
           const int32_t *__restrict__ cellStart, const int32_t *__restrict__ list,
           const int32_t *__restrict__ special, const int32_t *__restrict__ nspecial,
           int32_t *__restrict__ pcount, int32_t *__restrict__ pcursor,
           int2 *__restrict__ pairs, int32_t *__restrict__ pairRankB, int cap_pairs,
           int32_t *__restrict__ status) {
    const int r = blockIdx.x * BG_WAVES + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nb) return;                                     // (whole wave)
    const int k = key[r];
    if (k == -1) return;
    const int ia = byRank[r];
    const double4 A = aabb[ia];
    const bool aB = (bodies[ia].flags & LPE_BODY_BOUNDARY) != 0;
    const double sa = fmax(A.z - A.x, A.w - A.y);
    auto emit = [&](int lo, int hi) {                        // ranks: the pair belongs to lo
        if (mode == 0) {
            atomicAdd(&pcount[lo], 1);
        } else {
            const int slot = atomicAdd(&pcursor[lo], 1);
            if (slot < cap_pairs) { pairs[slot] = make_int2(byRank[lo], byRank[hi]); pairRankB[slot] = hi; }
            else atomicOr(&status[0], 1);
        }
    };
    auto test = [&](int rb) {
        const int ib = byRank[rb];
        const double4 B = aabb[ib];
        const bool bB = (bodies[ib].flags & LPE_BODY_BOUNDARY) != 0;
        return bp_pair_ok(A, B, aB, bB, sa, fmax(B.z - B.x, B.w - B.y), small);
    };
    const int ns = *nspecial;
    if (k >= 0) {
        const int cx = k % G, cy = k / G;
        int cs[9], pre[10];                                  // cell starts, flat prefix
        pre[0] = 0;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const int x = cx - 1 + i % 3, y = cy - 1 + i / 3;
            int b0 = 0, n = 0;
            if (x >= 0 && x < G && y >= 0 && y < G) {
                const int c = y * G + x;
                b0 = cellStart[c];
                n = cellStart[c + 1] - b0;
            }
            cs[i] = b0;
            pre[i + 1] = pre[i] + n;
        }
        for (int t = lane; t < pre[9]; t += 64) {
            int j = 0;
#pragma unroll
            for (int i = 0; i < 9; i++)
                if (t >= pre[i] && t < pre[i + 1]) j = cs[i] + (t - pre[i]);
            const int rb = list[j];
            if (rb > r && test(rb)) emit(r, rb);
        }
        for (int j = lane; j < ns; j += 64) {                // regular - special pairs
            const int rb = special[j];
            if (test(rb)) emit(min(r, rb), max(r, rb));
        }
    } else {
        for (int j = lane; j < ns; j += 64) {                // special - special pairs
            const int rb = special[j];
            if (rb > r && test(rb)) emit(r, rb);
        }
    }
}

// narrowPhase (narrowphase.cpp:352-420): one thread per pair
__global__ void __launch_bounds__(128)
k_narrow(const int32_t *__restrict__ npptr, int cap, const int2 *__restrict__ pairs,
         const lpe_body *__restrict__ bodies, const double *__restrict__ verts,
         lpe_contact *__restrict__ slots, int32_t *__restrict__ ccount, int32_t *__restrict__ counts) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    // the pair count can exceed the buffers when they overflowed (the step
    // then grows them and redoes the broadphase): never past the capacity
    if (k >= min(*npptr, cap)) return;
    int2 pr = pairs[k];
    const lpe_body ba = bodies[pr.x], bb = bodies[pr.y];
    DShape A = dshape(ba, verts), B = dshape(bb, verts);
    int cnt = 0;
    D2 simplex[4];
    int ns;
    lpe_contact *out = slots + (size_t)k * MAXC;
    if (gjk(A, B, simplex, ns)) {
        D2 n;
        double pen;
        if (epa(A, B, simplex, n, pen)) {
            lpe_contact c;
            c.a = pr.x; c.b = pr.y; c.pair = k; c.pad = 0;
            c.nx = n.x; c.ny = n.y; c.pen = pen;
            if (A.circle || B.circle) {
                D2 cp;
                if (A.circle && B.circle) cp = sub(B.pos, mul(n, B.radius));
                else if (A.circle) cp = add(A.pos, mul(n, A.radius));
                else cp = sub(B.pos, mul(n, B.radius));
                c.px = cp.x; c.py = cp.y;
                out[cnt++] = c;
            } else {
                // buildPolygonPolygonContacts (narrowphase.cpp:304-350), reference face on A
                D2 av[MAXV], bv[CLIP_MAX], t1[CLIP_MAX], t2[CLIP_MAX];
                int na = min(A.nv, MAXV), nbv = min(B.nv, MAXV);
                world_verts(A, av);
                DShape Bc = B; Bc.nv = nbv;
                world_verts(Bc, bv);
                int fa = 0;
                double bestDot = -1e30;
                for (int i = 0; i < na; i++) {                   // findBestFace (:126-145)
                    int j = (i + 1) % na;
                    D2 e = sub(av[j], av[i]);
                    D2 fn = nrm(d2(-e.y, e.x));
                    double d = dot(fn, n);
                    if (d > bestDot) { bestDot = d; fa = i; }
                }
                D2 v1 = av[fa], v2 = av[(fa + 1) % na];
                D2 ea = sub(v2, v1);
                D2 refN = nrm(d2(-ea.y, ea.x));
                double faceOff = dot(refN, v1);
                D2 edge = nrm(sub(v2, v1));
                D2 botN = neg(edge);
                int m1 = clip_face(bv, nbv, refN, faceOff, t1);
                int m2 = clip_face(t1, m1, edge, dot(edge, v2), t2);
                int m3 = clip_face(t2, m2, botN, dot(botN, v1), t1);
                double planeOff = dot(refN, v1);
                // at most nbv + 3 <= 35 < MAXC clipped points (MAXV = 32):
                // never truncated, but a truncation would be reported
                if (m3 > MAXC) atomicOr(&counts[11], 1);
                for (int q = 0; q < m3 && cnt < MAXC; q++) {
                    c.pen = -(dot(refN, t1[q]) - planeOff);
                    c.px = t1[q].x; c.py = t1[q].y;
                    out[cnt++] = c;
                }
            }
        }
    }
    ccount[k] = cnt;
}

// (also the contact count: counts[1] = the contacts kept, at most cap;
// counts[14] = the contacts found -- more than cap is an overflow;
// counts[15] = the pairs found.)  An overflowing detection (pairs past
// cap_pairs or the pair-overflow flag, contacts past cap) zeroes the pair and
// contact counts, so every kernel after it -- the striped order, the rows,
// the solvers -- sees an empty tick and stays inside its buffers; only a
// lagged detection gets here with an overflow (the synchronous one grows and
// redoes first), and its check reports it from counts[15] / [14] / [6].
// host (lagged detection): thread 0 also stores the 16 counts straight into
// the pinned host slot the lagged check reads (no copy launch after it);
// every other count is final by then (earlier kernels in stream order)
__global__ void k_compact(int32_t *__restrict__ npptr, int cap_pairs, const lpe_contact *__restrict__ slots,
                          const int32_t *__restrict__ ccount, const int32_t *__restrict__ cstart,
                          lpe_contact *__restrict__ out, int cap, int32_t *__restrict__ counts,
                          int32_t *__restrict__ host) {
    int k = blockIdx.x * RTPB + threadIdx.x;
    const int raw = *npptr;
    const int np = min(raw, cap_pairs);
    if (k == 0) {
        const int tot = cstart[np];
        const bool over = counts[6] != 0 || raw > cap_pairs || tot > cap;
        counts[1] = over ? 0 : tot;
        counts[14] = tot;
        counts[15] = raw;
        if (over) *npptr = 0;          // (blocks that read it first compact within the capacities)
        if (host) {
            // (npptr is counts + 0: its value as just left)
            for (int i = 0; i < 16; i++) host[i] = i == 0 ? (over ? 0 : raw) : counts[i];
            __threadfence_system();
        }
    }
    if (k >= np) return;
    int s = cstart[k];
    for (int j = 0; j < ccount[k]; j++)
        if (s + j < cap) out[s + j] = slots[(size_t)k * MAXC + j];
}

// ---------------------------------------------------------------------------
// PGS preparation (contact_solver.cpp:42-253)
__device__ __forceinline__ bool infinite_mass(const lpe_body &b) {
    return (b.flags & LPE_BODY_HAS_MASS) && b.mass > 1e29;
}
__device__ __forceinline__ bool can_rotate(const lpe_body &b) {
    if (!(b.flags & LPE_BODY_HAS_ANGVEL) || !(b.flags & LPE_BODY_HAS_INERTIA)) return false;
    return b.inertia > 1e-12 && b.inertia < 1e29;
}

__global__ void k_mark_contacts(const int32_t *__restrict__ ncptr, const lpe_contact *__restrict__ cs,
                                int32_t *__restrict__ inContact) {
    int k = blockIdx.x * RTPB + threadIdx.x;
    if (k >= *ncptr) return;
    inContact[cs[k].a] = 1;
    inContact[cs[k].b] = 1;
}

// loading the solver's bodies (contact_solver.cpp:480-507): what & 1 the
// inverse masses (constant during the tick), what & 2 the velocities
__global__ void k_pgs_bodies(int nb, const lpe_body *__restrict__ bodies, float *__restrict__ vel0,
                             float *__restrict__ imii, int what) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    const lpe_body b = bodies[i];
    bool cr = can_rotate(b);
    if (what & 1) {
        double m = b.mass;
        float im = (m > 1e29) ? 0.f : (float)(1.0 / m);
        float iv = 0.f;
        if (cr) {
            double I = b.inertia;
            if (I > 1e-12 && I < 1e29) iv = (float)(1.0 / I);
        }
        imii[2 * i] = im; imii[2 * i + 1] = iv;
    }
    if (what & 2) {
        vel0[3 * i] = (float)b.vx;
        vel0[3 * i + 1] = (float)b.vy;
        vel0[3 * i + 2] = cr ? (float)b.omega : 0.f;
    }
}

__device__ __forceinline__ float cross2f(float ax, float ay, float bx, float by) {
    float l0 = ax * by, l1 = ay * bx;                      // cross2fNeon (:207-214)
    return l0 - l1;
}

// buildConstraintRows (:133-197) + computeEffectiveMass (:216-253), item t
__global__ void k_pgs_rows(const int32_t *__restrict__ ncptr, const int32_t *__restrict__ order,
                           const lpe_contact *__restrict__ cs, const lpe_body *__restrict__ bodies,
                           const float *__restrict__ imii, float4 *__restrict__ rowN,
                           float4 *__restrict__ rowR, int2 *__restrict__ rowAB,
                           float4 *__restrict__ rowM, int32_t *__restrict__ sItemA,
                           int32_t *__restrict__ sItemB) {
    int t = blockIdx.x * RTPB + threadIdx.x;
    if (t >= *ncptr) return;
    const lpe_contact c = cs[order ? order[t] : t];
    const lpe_body A = bodies[c.a], B = bodies[c.b];
    int a = infinite_mass(A) ? -1 : c.a;
    int b = infinite_mass(B) ? -1 : c.b;
    D2 u = nrm(d2(c.nx, c.ny));
    float dirX = (float)u.x, dirY = (float)u.y;
    float rxA = (float)(c.px - A.x), ryA = (float)(c.py - A.y);
    float rxB = (float)(c.px - B.x), ryB = (float)(c.py - B.y);
    float imA = 0.f, imB = 0.f, iiA = 0.f, iiB = 0.f;
    if (a >= 0) { imA = imii[2 * a]; iiA = imii[2 * a + 1]; }
    if (b >= 0) { imB = imii[2 * b]; iiB = imii[2 * b + 1]; }
    float effN, effF;
    {
        float rAxn = cross2f(rxA, ryA, dirX, dirY), rBxn = cross2f(rxB, ryB, dirX, dirY);
        float sum = imA + imB + (rAxn * rAxn) * iiA + (rBxn * rBxn) * iiB;
        effN = (sum < 1e-12F) ? 0.F : 1.F / sum;
    }
    {
        float fx = -dirY, fy = dirX;
        float rAxn = cross2f(rxA, ryA, fx, fy), rBxn = cross2f(rxB, ryB, fx, fy);
        float sum = imA + imB + (rAxn * rAxn) * iiA + (rBxn * rBxn) * iiB;
        effF = (sum < 1e-12F) ? 0.F : 1.F / sum;
    }
    rowN[t] = make_float4(dirX, dirY, effN, effF);
    rowR[t] = make_float4(rxA, ryA, rxB, ryB);
    rowAB[t] = make_int2(a, b);
    rowM[t] = make_float4(imA, iiA, imB, iiB);
    sItemA[t] = a;
    sItemB[t] = b;
}

// ---------------------------------------------------------------------------
// Exact sequential Gauss-Seidel on the device, by dataflow.
//
// A sweep visits items (PGS contacts / position-solver contacts) in a fixed
// order; an item reads and writes the state of at most two movable bodies.
// The sequential result is reproduced exactly when every body sees its items
// in sweep order, sweep after sweep.  Each body carries a version counter (in
// LDS) = the number of its items already applied; item t of sweep `it` may
// run once its bodies' counters reach it * cnt + rank (cnt = items of the
// body, rank = items of the body before t).  No level schedule, no barrier:
// items run as soon as their inputs are final, and sweeps overlap.
//
// Work split: thread j owns items j, j + 1024, ... of every sweep and runs
// them in (sweep, item) order.  Every thread's queue is a subsequence of the
// global sequential order, so the earliest unfinished item is always at the
// head of its queue with its inputs final: progress is guaranteed.
__global__ void k_sched_count(const int32_t *__restrict__ kptr, const int32_t *__restrict__ ia,
                              const int32_t *__restrict__ ib, int32_t *__restrict__ bcount) {
    int t = blockIdx.x * RTPB + threadIdx.x;
    if (t >= *kptr) return;
    if (ia[t] >= 0) atomicAdd(&bcount[ia[t]], 1);
    if (ib[t] >= 0) atomicAdd(&bcount[ib[t]], 1);
}
__global__ void k_sched_fill(const int32_t *__restrict__ kptr, const int32_t *__restrict__ ia,
                             const int32_t *__restrict__ ib, int32_t *__restrict__ cursor,
                             int32_t *__restrict__ ent) {
    int t = blockIdx.x * RTPB + threadIdx.x;
    if (t >= *kptr) return;
    if (ia[t] >= 0) ent[atomicAdd(&cursor[ia[t]], 1)] = t;
    if (ib[t] >= 0) ent[atomicAdd(&cursor[ib[t]], 1)] = t;
}
// per item: (rank, cnt) on each of its bodies
__global__ void k_sched_rank(const int32_t *__restrict__ kptr, const int32_t *__restrict__ ia,
                             const int32_t *__restrict__ ib, const int32_t *__restrict__ bstart,
                             const int32_t *__restrict__ ent, int4 *__restrict__ ver) {
    int t = blockIdx.x * RTPB + threadIdx.x;
    if (t >= *kptr) return;
    int4 v = make_int4(0, 0, 0, 0);
    int a = ia[t], b = ib[t];
    if (a >= 0) {
        int s0 = bstart[a], e0 = bstart[a + 1], r = 0;
        for (int k = s0; k < e0; k++) r += ent[k] < t ? 1 : 0;
        v.x = r; v.y = e0 - s0;
    }
    if (b >= 0) {
        int s0 = bstart[b], e0 = bstart[b + 1], r = 0;
        for (int k = s0; k < e0; k++) r += ent[k] < t ? 1 : 0;
        v.z = r; v.w = e0 - s0;
    }
    ver[t] = v;
}

// Canonical solver order (lpe_rigid_step): graph-coloured Gauss-Seidel
// (SURVEY.md §7.1 step 7).  The contact pairs are edge-coloured so that no
// two pairs of one colour share a movable body; the solvers then visit the
// pairs colour by colour, each pair's contacts in narrowphase order.  The
// reference's PGS order is an unordered_map's (contact_manager.cpp:169-245)
// and its position-solver order the quadtree's pair order, so any such order
// is a valid restatement; this one keeps the dependency depth of a sweep at
// about (colours x contacts per pair) instead of the length of the longest
// chain of contacts in entity-id order.  Pairs of one colour touch disjoint
// movable bodies, so the order inside a colour does not change a single bit.
//
// Colouring (deterministic, restated by oracle/rigid_oracle.cpp
// lpeo_colour_order): rounds; every uncoloured pair claims its movable
// bodies with the priority (hash(p), p) -- the lowest wins a body; a pair that
// wins all of them takes a colour free on both and marks it used: with more
// pairs than one solver slot (SOLVE_TPB), the first free colour of the first
// K = ceil(pairs / 960) in a rotation hashed from the pair (r = hash(p ^
// 0x9e3779b9) * K >> 32: colours r .. K - 1, then 0 .. r - 1), else the lowest
// free colour.  A colour step costs a pair chain's latency per slot, so
// balanced colours of at most one slot each (10 steps per sweep on the
// metric pile's fixture instead of 14 slots in 9 lowest-first colours of up
// to 1,785 pairs) shorten both solvers.
// Hashed priorities keep the chains of "waits for a lower pair" short (pair
// indices follow entity ids, i.e. space, so plain index priorities chain
// across the pile).  One 1024-thread workgroup, per-body state in LDS.
// Outputs: order (contact per row, colour-major, each pair's rows
// contiguous), seg (row start, count) per coloured pair in colour-major pair
// order, cbase (first seg of each colour; cbase[ncol] = coloured pairs).
static constexpr int MAX_COLOURS = 64;
__host__ __device__ __forceinline__ uint32_t colour_hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ bool colour_dep(const lpe_body &b) {
    // a body the PGS writes (finite mass, contact_solver.cpp:70-98) or the
    // position solver moves (invM != 0 or rotatable, position_solver.cpp:125-168)
    bool inf = (b.flags & LPE_BODY_HAS_MASS) && b.mass > 1e29;
    bool rot = (b.flags & LPE_BODY_HAS_INERTIA) && b.inertia > 1e-12 && b.inertia < 1e29;
    return !inf || rot;
}
__global__ void __launch_bounds__(SOLVE_TPB)
k_pair_colour(int nb, const int32_t *__restrict__ npptr, const int2 *__restrict__ pairs,
              const int32_t *__restrict__ ccount, const int32_t *__restrict__ cstart,
              const lpe_body *__restrict__ bodies, int32_t *__restrict__ pcol,
              int32_t *__restrict__ order, int2 *__restrict__ seg, int32_t *__restrict__ cbase,
              int32_t *__restrict__ counts) {
    extern __shared__ unsigned long long su[];              // colours used, per body
    unsigned long long *claim = su + nb;                     // best claiming priority, per body
    unsigned char *dep = (unsigned char *)(claim + nb);      // movable body
    // pairs of a colour are placed by row count, largest first, so the waves
    // of a colour step run pairs of equal length (a wave executes as many
    // rows as its longest pair); the order inside a colour has no effect on
    // the result (its pairs share no movable body)
    constexpr int NCLS = 6;                                  // row-count classes: >= 6, 5, 4, 3, 2, 1
    __shared__ int colCnt[MAX_COLOURS * NCLS], colCur[MAX_COLOURS * NCLS];
    __shared__ int colPairs[MAX_COLOURS * NCLS], colPCur[MAX_COLOURS * NCLS];
    __shared__ int grpQ0[MAX_COLOURS * NCLS], grpRow0[MAX_COLOURS * NCLS];
    __shared__ int s_left, s_fault, s_ncol, s_m;
    const unsigned long long NONE = ~0ull;
    const int np = *npptr;
    for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
        su[i] = 0ull;
        claim[i] = NONE;
        dep[i] = colour_dep(bodies[i]) ? 1 : 0;
    }
    if (threadIdx.x == 0) { s_fault = 0; s_ncol = 0; s_m = 0; }
    __syncthreads();
    // Pairs p = tid + k*TPB (k < PK) live in registers for all rounds (a
    // round is then LDS work only); pairs beyond PK*TPB use global memory.
    // Colour state: -1 pair without contacts (no item), -2 uncoloured,
    // <= -3 coloured this round (-3 - colour), >= 0 colour.
    constexpr int PK = 12;
    int rab[PK], rc[PK];            // movable bodies packed as two int16 (-1: none)
#pragma unroll
    for (int k = 0; k < PK; k++) {
        const int p = threadIdx.x + k * SOLVE_TPB;
        rab[k] = -1; rc[k] = -1;
        if (p < np) {
            int2 pr = pairs[p];
            int a = dep[pr.x] ? pr.x : -1, b = dep[pr.y] ? pr.y : -1;
            rab[k] = (a & 0xffff) | (b << 16);
            rc[k] = ccount[p] > 0 ? -2 : -1;
            if (rc[k] == -2) atomicAdd(&s_m, 1);
        }
    }
    auto A = [](int ab) { return (int)(short)(ab & 0xffff); };
    auto B = [](int ab) { return ab >> 16; };
    for (int p = threadIdx.x + PK * SOLVE_TPB; p < np; p += SOLVE_TPB) {
        pcol[p] = ccount[p] > 0 ? -2 : -1;
        if (ccount[p] > 0) atomicAdd(&s_m, 1);
    }
    __syncthreads();
    constexpr int FILL = SOLVE_TPB - SOLVE_TPB / 16;           // target pairs per balanced colour
    const int K = s_m > SOLVE_TPB ? min((s_m + FILL - 1) / FILL, MAX_COLOURS) : 0;
    auto prio = [](int p) {
        return ((unsigned long long)colour_hash((uint32_t)p) << 32) | (uint32_t)p;
    };
    auto claimOf = [&](int p, int a, int b, int col) {
        if (col != -2) return;
        if (a >= 0) atomicMin(&claim[a], prio(p));
        if (b >= 0) atomicMin(&claim[b], prio(p));
    };
    auto pick = [&](int p, int a, int b, int &col) {
        if (col != -2) return;
        const unsigned long long pri = prio(p);
        if ((a < 0 || claim[a] == pri) && (b < 0 || claim[b] == pri)) {
            unsigned long long forb = (a >= 0 ? su[a] : 0ull) | (b >= 0 ? su[b] : 0ull);
            int c = -1;
            if (K > 0) {
                // the first free colour of the first K in the rotation r
                const uint32_t r = (uint32_t)(((unsigned long long)colour_hash((uint32_t)p ^ 0x9e3779b9u) *
                                               (unsigned)K) >> 32);
                const unsigned long long av = ~forb & (K == 64 ? ~0ull : (1ull << K) - 1);
                const unsigned long long hi = av & (~0ull << r);      // colours r .. K - 1 first
                if (av) c = __ffsll((long long)(hi ? hi : av)) - 1;
            }
            if (c < 0) c = __ffsll((long long)~forb) - 1;
            if (c < 0 || c >= MAX_COLOURS) { s_fault = 1; c = 0; }
            col = -3 - c;                                          // coloured this round
        } else {
            s_left = 1;
        }
    };
    auto commit = [&](int a, int b, int &col) {
        if (col == -1 || col >= 0) return;
        if (col <= -3) {
            const int c = -3 - col;
            col = c;
            if (a >= 0) su[a] |= 1ull << c;                        // one winner per body
            if (b >= 0) su[b] |= 1ull << c;
        }
        if (a >= 0) claim[a] = NONE;
        if (b >= 0) claim[b] = NONE;
    };
    auto gpair = [&](int p, int &a, int &b) {
        int2 pr = pairs[p];
        a = dep[pr.x] ? pr.x : -1;
        b = dep[pr.y] ? pr.y : -1;
    };
    for (int round = 0;; round++) {
        if (threadIdx.x == 0) s_left = 0;
#pragma unroll
        for (int k = 0; k < PK; k++) claimOf(threadIdx.x + k * SOLVE_TPB, A(rab[k]), B(rab[k]), rc[k]);
        for (int p = threadIdx.x + PK * SOLVE_TPB; p < np; p += SOLVE_TPB) {
            int a, b; gpair(p, a, b); claimOf(p, a, b, pcol[p]);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PK; k++) pick(threadIdx.x + k * SOLVE_TPB, A(rab[k]), B(rab[k]), rc[k]);
        for (int p = threadIdx.x + PK * SOLVE_TPB; p < np; p += SOLVE_TPB) {
            int a, b, col = pcol[p]; gpair(p, a, b); pick(p, a, b, col); pcol[p] = col;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PK; k++) commit(A(rab[k]), B(rab[k]), rc[k]);
        for (int p = threadIdx.x + PK * SOLVE_TPB; p < np; p += SOLVE_TPB) {
            int a, b, col = pcol[p]; gpair(p, a, b); commit(a, b, col); pcol[p] = col;
        }
        __syncthreads();
        const bool more = s_left && !s_fault && round < (1 << 20);
        __syncthreads();              // every thread has read s_left before it is reset
        if (!more) {
            if (threadIdx.x == 0) counts[9] = round + 1;
            break;
        }
    }
#pragma unroll
    for (int k = 0; k < PK; k++) {
        const int p = threadIdx.x + k * SOLVE_TPB;
        if (p < np) pcol[p] = rc[k];
    }
    __syncthreads();
    // colour-major order, and inside a colour groups of pairs with the same
    // row count (longest first).  A group of g pairs with n rows stores its
    // rows transposed, row j of its i-th pair at base + j * g + i, so the
    // lanes of a wave (consecutive pairs of one group) load row j of their
    // pairs from consecutive slots; pairs with >= NCLS rows keep theirs
    // contiguous.  seg[q] = (slot of row 0, n | stride << 8).
    auto cls = [](int n) { return NCLS - min(n, NCLS); };
    for (int i = threadIdx.x; i < MAX_COLOURS * NCLS; i += SOLVE_TPB) {
        colPairs[i] = 0; colPCur[i] = 0; colCnt[i] = 0; colCur[i] = 0;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < np; p += SOLVE_TPB) {
        int c = pcol[p];
        if (c >= 0) {
            const int gi = c * NCLS + cls(ccount[p]);
            atomicAdd(&colCnt[gi], ccount[p]);
            atomicAdd(&colPairs[gi], 1);
            atomicMax(&s_ncol, c + 1);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0, pacc = 0;
        for (int c = 0; c < MAX_COLOURS; c++) {
            if (c <= s_ncol) cbase[c] = pacc;
            for (int k = 0; k < NCLS; k++) {
                const int gi = c * NCLS + k;
                grpQ0[gi] = pacc; colPCur[gi] = pacc; pacc += colPairs[gi];
                grpRow0[gi] = acc; colCur[gi] = acc; acc += colCnt[gi];
            }
        }
        cbase[s_ncol] = pacc;
        counts[8] = s_ncol;
        if (s_fault) counts[7] = 1;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < np; p += SOLVE_TPB) {
        int c = pcol[p];
        if (c < 0) continue;
        const int n = ccount[p], s0 = cstart[p], k = cls(n), gi = c * NCLS + k;
        const int q = atomicAdd(&colPCur[gi], 1);
        int pos, stride;
        if (k == 0) {                                   // >= NCLS rows: contiguous
            pos = atomicAdd(&colCur[gi], n);
            stride = 1;
        } else {
            pos = grpRow0[gi] + (q - grpQ0[gi]);
            stride = colPairs[gi];
        }
        seg[q] = make_int2(pos, n | (stride << 8));
        for (int j = 0; j < n; j++) order[pos + j * stride] = s0 + j;
    }
}

// Colour-synchronous Gauss-Seidel sweeps (canonical order): for each colour,
// every thread runs whole pairs of that colour (their rows in order), then a
// barrier.  Equal bit for bit to the sequential sweep in colour-major order.
// solveLcpPgs (contact_solver.cpp:381-440), rows of buildConstraintRows
// (:133-197) in fp32, body velocities in LDS.
// one contact row (normal, then friction) on the pair's velocities in registers
#ifndef PGS_BRANCHLESS
#define PGS_BRANCHLESS 0
#endif
typedef float pk2 __attribute__((ext_vector_type(2)));
// The x/y halves of the row are computed as packed fp32 pairs (v_pk_mul_f32 /
// v_pk_add_f32: each lane of a packed op is the IEEE scalar op, unfused), so
// the results are the scalar code's bit for bit with fewer VALU issues.
template <bool BL>
__device__ __forceinline__ void pgs_row_t(float4 rn, float4 rr, float imA, float iiA, float imB, float iiB,
                                          bool hasA, bool hasB, float mu, float &ln, float &lf, float &vxA,
                                          float &vyA, float &wA, float &vxB, float &vyB, float &wB) {
    pk2 vA = {vxA, vyA}, vB = {vxB, vyB};
    const pk2 lA = {-rr.y, rr.x}, lB = {-rr.w, rr.z};
#pragma unroll
    for (int row = 0; row < 2; row++) {
        const pk2 d = row == 0 ? pk2{rn.x, rn.y} : pk2{-rn.y, rn.x};
        float eff = row == 0 ? rn.z : rn.w;
        // a = vA + wA * (-rA.y, rA.x): x - w*ry == x + w*(-ry) exactly
        const pk2 a = vA + lA * wA, b = vB + lB * wB;
        const pk2 rel = b - a;
        const pk2 pr = rel * d;
        float vrel = pr.x + pr.y;
        float old, lo, hi;
        if (row == 0) { old = ln; lo = 0.0f; hi = 1e20f; }
        else {
            old = lf;
            float limit = mu * ln;
            lo = -limit; hi = limit;
        }
        float dl = -eff * (vrel + 0.0f);
        float nl = old + dl;
        if (nl < lo) nl = lo;
        if (nl > hi) nl = hi;
        dl = nl - old;
        if (row == 0) ln = nl; else lf = nl;
        if constexpr (BL) {
        // the skipped / absent-body cases as selects of the unchanged values
        // (bit-identical to the branches; keeps exec-mask updates and their
        // VALU -> SALU hazards out of the row chain)
        const bool apply = !(fabsf(dl) < 1e-15F);
        const float crossA = rr.x * d.y - rr.y * d.x, crossB = rr.z * d.y - rr.w * d.x;
        const pk2 nvA = vA - d * (dl * imA), nvB = vB + d * (dl * imB);
        const float nwA = wA - crossA * dl * iiA, nwB = wB + crossB * dl * iiB;
        const bool uA = apply && hasA, uB = apply && hasB;
        vA.x = uA ? nvA.x : vA.x; vA.y = uA ? nvA.y : vA.y; wA = uA ? nwA : wA;
        vB.x = uB ? nvB.x : vB.x; vB.y = uB ? nvB.y : vB.y; wB = uB ? nwB : wB;
        } else {
        if (fabsf(dl) < 1e-15F) continue;
        if (hasA) {
            vA -= d * (dl * imA);
            float crossA = rr.x * d.y - rr.y * d.x;
            wA -= crossA * dl * iiA;
        }
        if (hasB) {
            vB += d * (dl * imB);
            float crossB = rr.z * d.y - rr.w * d.x;
            wB += crossB * dl * iiB;
        }
        }
    }
    vxA = vA.x; vyA = vA.y; vxB = vB.x; vyB = vB.y;
}
// The striped solver's row (k_pgs_stripes): pgs_row_t's arithmetic with the
// crosses precomputed (rowC, the same expressions) and the skipped update as
// a zero increment instead of selects -- a body whose impulse is skipped, or
// absent (zero inverse mass and inertia), gets v - d (0 m) = v: the same
// value (a zero velocity may change the sign of its zero, which no later
// operation of the tick turns into a different non-zero value); for the same
// reason vn + rhs (rhs = 0, :404) is vn
// (lv: the lever arms' perpendiculars (-r_A.y, r_A.x, -r_B.y, r_B.x), as the
// stripe workgroups stage them once per solve -- exact sign flips -- so the
// row does not rebuild them with a negate and a move per contact)
__device__ __forceinline__ void pgs_row_l(float4 rn, float4 lv, float4 rc, float imA, float iiA, float imB,
                                          float iiB, float mu, float &ln, float &lf, float &vxA, float &vyA,
                                          float &wA, float &vxB, float &vyB, float &wB) {
    pk2 vA = {vxA, vyA}, vB = {vxB, vyB};
    const pk2 lA = {lv.x, lv.y}, lB = {lv.z, lv.w};
#pragma unroll
    for (int row = 0; row < 2; row++) {
        const pk2 d = row == 0 ? pk2{rn.x, rn.y} : pk2{-rn.y, rn.x};
        const float eff = row == 0 ? rn.z : rn.w;
        const pk2 a = vA + lA * wA, b = vB + lB * wB;
        const pk2 rel = b - a;
        const pk2 pr = rel * d;
        float vrel = pr.x + pr.y;
        float old, lo, hi;
        if (row == 0) { old = ln; lo = 0.0f; hi = 1e20f; }
        else {
            old = lf;
            float limit = mu * ln;
            lo = -limit; hi = limit;
        }
        float dl = -eff * vrel;          // (the reference's + rhs, rhs = 0, changes only a zero's sign)
        // the clamp (lo <= hi) as one v_med3_f32: the compare / select pairs
        // cost two SGPR-mask hazard waits each on one wave; for a non-zero
        // value the same result, a zero only possibly of the other sign,
        // which dl = nl - old and the skip test below make +0 either way
        const float nl = __builtin_amdgcn_fmed3f(old + dl, lo, hi);
        dl = nl - old;
        if (row == 0) ln = nl; else lf = nl;
        const float da = fabsf(dl) < 1e-15F ? 0.0f : dl;
        const float crossA = row == 0 ? rc.x : rc.z, crossB = row == 0 ? rc.y : rc.w;
        vA = vA - d * (da * imA);
        vB = vB + d * (da * imB);
        wA = wA - crossA * da * iiA;
        wB = wB + crossB * da * iiB;
    }
    vxA = vA.x; vyA = vA.y; vxB = vB.x; vyB = vB.y;
}
__device__ __forceinline__ float4 lever_perp(float4 rr) { return make_float4(-rr.y, rr.x, -rr.w, rr.z); }
__device__ __forceinline__ void pgs_row_c(float4 rn, float4 rr, float4 rc, float imA, float iiA, float imB,
                                          float iiB, float mu, float &ln, float &lf, float &vxA, float &vyA,
                                          float &wA, float &vxB, float &vyB, float &wB) {
    pgs_row_l(rn, lever_perp(rr), rc, imA, iiA, imB, iiB, mu, ln, lf, vxA, vyA, wA, vxB, vyB, wB);
}
__device__ __forceinline__ void pgs_row_regs(float4 rn, float4 rr, float imA, float iiA, float imB,
                                             float iiB, bool hasA, bool hasB, float mu, float &ln,
                                             float &lf, float &vxA, float &vyA, float &wA, float &vxB,
                                             float &vyB, float &wB) {
    pgs_row_t<PGS_BRANCHLESS != 0>(rn, rr, imA, iiA, imB, iiB, hasA, hasB, mu, ln, lf, vxA, vyA, wA, vxB, vyB, wB);
}

// A colour step is latency-bound (one workgroup; a pair's rows are a chain),
// so the global round trips per step are kept to one: colour bases and the
// coloured pairs' row segments are cached in LDS (when they fit: segLds), and
// all rows of a pair (up to RB) are loaded before its sequential updates.
// The rows of a pair share its two bodies (and their masses): the bodies'
// state is read from LDS once per pair and kept in registers across its rows.

// A colour step's barrier: the step's LDS writes (velocities / poses) are
// visible to every wave after it; outstanding global loads (the next step's
// prefetch) stay in flight across it (__syncthreads() would drain them).
// Global data written inside the sweeps (the PGS multipliers) is re-read only
// by the thread that wrote it (static pair -> thread map).
// Buffer loads / stores with a 32-bit byte offset (one address VGPR per
// operation instead of two); descriptors built from kernel arguments only,
// so they stay in SGPRs.  No range limit beyond the 32-bit offset.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, 0x7fffffff, 0x00020000);
}
// A lane without work passes ok = false: its offset is out of range, so the
// load returns zeros without touching memory while the wave keeps a fixed
// count of memory operations (what lets the compiler's waits stay partial).
static constexpr uint32_t BOOB = 0x80000000u;
__device__ __forceinline__ float4 bld_f4(__amdgpu_buffer_rsrc_t r, uint32_t i, bool ok = true) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(ok ? i * 16u : BOOB), 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ int2 bld_i2(__amdgpu_buffer_rsrc_t r, uint32_t i, bool ok = true) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(ok ? i * 8u : BOOB), 0, 0);
    return make_int2((int)v.x, (int)v.y);
}
__device__ __forceinline__ float bld_f(__amdgpu_buffer_rsrc_t r, uint32_t i, bool ok = true) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(ok ? i * 4u : BOOB), 0, 0));
}
__device__ __forceinline__ void bst_f(__amdgpu_buffer_rsrc_t r, uint32_t i, float v, bool ok = true) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)(ok ? i * 4u : BOOB), 0, 0);
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

#ifndef PGS_PF
#define PGS_PF 2    // rows of a pair prefetched with it
#endif
#ifndef PGS_TL
#define PGS_TL 1    // further rows loaded at the start of its slot (waves with longer pairs)
#endif
#ifndef PGS_ILV
#define PGS_ILV 1   // the next slot's rows loaded between the current pair's rows
#endif
__global__ void __launch_bounds__(SOLVE_TPB)
k_pgs_colour(int nb, const int32_t *__restrict__ counts, const int32_t *__restrict__ cbase,
             const int2 *__restrict__ seg, int segLds, const float4 *__restrict__ rowN,
             const float4 *__restrict__ rowR, const int2 *__restrict__ rowAB,
             const float4 *__restrict__ rowM, float *__restrict__ vel, int iters, float mu,
             float *__restrict__ lamN, float *__restrict__ lamF, lpe_body *__restrict__ bodies,
             const int32_t *__restrict__ inContact) {
    extern __shared__ float sv[];   // 3 floats per body
    __shared__ int scb[MAX_COLOURS + 1];
    const int ncol = counts[8];
    if (bodies) {   // k_pgs_bodies (velocities) in the prologue
        for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
            const lpe_body &b = bodies[i];
            const bool cr = can_rotate(b);
            sv[3 * i] = (float)b.vx;
            sv[3 * i + 1] = (float)b.vy;
            sv[3 * i + 2] = cr ? (float)b.omega : 0.f;
        }
    } else {
        for (int i = threadIdx.x; i < 3 * nb; i += SOLVE_TPB) sv[i] = vel[i];
    }
    for (int c = threadIdx.x; c <= ncol; c += SOLVE_TPB) scb[c] = cbase[c];
    __syncthreads();
    (void)segLds;
    // Slots: a colour's pairs are split into ceil(n / SOLVE_TPB) slots of at
    // most one pair per thread (pairs of one colour share no movable body,
    // so any split is the same sweep); the barrier follows a colour's last
    // slot.  Slots are software-pipelined: the global loads of the thread's
    // pair of the NEXT slot (bodies, masses, its first PF rows and their
    // multipliers) are issued before the current pair is solved, and the
    // segment of the slot after that one slot earlier still, so they arrive
    // during the solve and the barrier.  The two slot buffers alternate (no
    // register copy, which would wait for the loads), and every prefetch and
    // every store of the first PF rows is issued unconditionally (a thread
    // without a next pair, or a pair with fewer rows, reads out of range:
    // zeros, no memory traffic; a pair with fewer rows re-stores its last
    // row), so the counts of memory operations in flight are static and each
    // wait covers only the buffer it needs.  Row data are constant
    // during the solve; a pair's multipliers are written only by the thread
    // that owns it (static q -> thread map), and the next slot's pair
    // differs from the current one (an iteration has at least two slots).
    // Rows in canonical order, arithmetic unchanged: bit-identical to the
    // unpipelined sweep.
    constexpr int PF = PGS_PF, TL = PGS_TL;
    constexpr bool ILV = PGS_ILV;
    struct Row { float4 n, r; float ln, lf; };
    struct Pf {
        int2 sg, ab;
        float4 m;
        Row r[PF];
    };
    const auto rN = brsrc(rowN), rR = brsrc(rowR), rAB = brsrc(rowAB), rM = brsrc(rowM);
    const auto rLN = brsrc(lamN), rLF = brsrc(lamF), rSeg = brsrc(seg);
    auto ldrow = [&](int t, bool ok, Row &w) {
        w.n = bld_f4(rN, t, ok); w.r = bld_f4(rR, t, ok);
        w.ln = bld_f(rLN, t, ok); w.lf = bld_f(rLF, t, ok);
    };
    // row j of the pair with segment sg (rows past its last: clamped to it,
    // not loaded; no pair: an out-of-range segment, nrow 0)
    auto ldrow_j = [&](int2 sg, int j, Row &w) {
        const int nrow = sg.y & 0xff, stride = sg.y >> 8;
        ldrow(sg.x + min(j, max(nrow - 1, 0)) * stride, j < nrow, w);
    };
    auto ldpair = [&](int2 sg, Pf &f) {
        f.sg = sg;
        const bool ok = (sg.y & 0xff) > 0;
        f.ab = bld_i2(rAB, sg.x, ok);
        f.m = bld_f4(rM, sg.x, ok);
    };
    auto ucb = [&](int c) { return __builtin_amdgcn_readfirstlane(scb[c]); };
    auto nslot0 = [&](int c) { return (ucb(c + 1) - ucb(c) + SOLVE_TPB - 1) / SOLVE_TPB; };
    int S = 0;
    for (int c = 0; c < ncol; c++) S += nslot0(c);
    // an iteration of one slot gets an empty second slot: the multipliers
    // prefetched for the next iteration are then loaded after this one's
    // stores (the prefetch is always valid)
    const int pad = S == 1 ? 1 : 0;
    auto nslot = [&](int c) { return nslot0(c) + pad; };
    const int total = iters * (S + pad);
    PTR(0, 0);
    if (threadIdx.x <= ncol) PTR_SET(1, 1024 + threadIdx.x, scb[threadIdx.x]);
    // slot positions (colour, slot of the colour, iteration) of slots s, s+1, s+2
    struct SP { int c, k, it; };
    auto adv = [&](SP p) {
        if (++p.k == nslot(p.c)) { p.k = 0; if (++p.c == ncol) { p.c = 0; p.it++; } }
        return p;
    };
    auto seg_of = [&](SP p) {
        const int q = ucb(p.c) + threadIdx.x + p.k * SOLVE_TPB;
        return bld_i2(rSeg, q, q < ucb(p.c + 1) && p.it < iters);
    };
    SP p0{0, 0, 0}, p1 = adv(p0), p2 = adv(p1);
    // one slot: [the current pairs' rows PF.. PF+TL-1 when the wave has
    // longer pairs] [segment of slot s+2 into sgZ] [bodies, masses of slot
    // s+1 into Y], then the current pair X row by row, each row followed by
    // the load of Y's row of that index (the next slot's data streams in
    // during the solve instead of stalling the wave's issue at its start),
    // barrier after the colour's last slot.  The multipliers are stored for
    // every row slot, out of range where there is none.
    auto slot = [&](auto tail, Pf &X, Pf &Y, int2 sgY, int2 &sgZ) {
        constexpr bool TAIL = decltype(tail)::value;
        const int it = p0.it;
        const int nrow = X.sg.y & 0xff, stride = X.sg.y >> 8;
        const bool hx = nrow > 0;
        Row T[TL > 0 ? TL : 1];
        if constexpr (TAIL) {
#pragma unroll
            for (int j = 0; j < TL; j++) ldrow_j(X.sg, PF + j, T[j]);
        }
        sgZ = seg_of(p2);
        ldpair(sgY, Y);
        if constexpr (!ILV) {
#pragma unroll
            for (int j = 0; j < PF; j++) ldrow_j(sgY, j, Y.r[j]);
        }
        const int2 ab = X.ab;
        const float4 m = X.m;
        const bool hasA = hx && ab.x >= 0, hasB = hx && ab.y >= 0;
        float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
        if (hasA) { vxA = sv[3 * ab.x]; vyA = sv[3 * ab.x + 1]; wA = sv[3 * ab.x + 2]; }
        if (hasB) { vxB = sv[3 * ab.y]; vyB = sv[3 * ab.y + 1]; wB = sv[3 * ab.y + 2]; }
        auto row = [&](int j, Row &w) {
            float ln = it ? w.ln : 0.f, lf = it ? w.lf : 0.f;
            if (j < nrow)
                pgs_row_regs(w.n, w.r, m.x, m.y, m.z, m.w, hasA, hasB, mu, ln, lf, vxA, vyA, wA, vxB, vyB, wB);
            const int t = X.sg.x + min(j, max(nrow - 1, 0)) * stride;
            bst_f(rLN, t, ln, j < nrow); bst_f(rLF, t, lf, j < nrow);
        };
#pragma unroll
        for (int j = 0; j < PF; j++) {
            row(j, X.r[j]);
            if constexpr (ILV) {
                __builtin_amdgcn_sched_barrier(0);
                ldrow_j(sgY, j, Y.r[j]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (TAIL) {
#pragma unroll
            for (int j = 0; j < TL; j++) row(PF + j, T[j]);
        }
        for (int j = TAIL ? PF + TL : PF; j < nrow; j++) {   // longer pairs: on demand
            Row w;
            ldrow(X.sg.x + j * stride, true, w);
            row(j, w);
        }
        if (hasA) { sv[3 * ab.x] = vxA; sv[3 * ab.x + 1] = vyA; sv[3 * ab.x + 2] = wA; }
        if (hasB) { sv[3 * ab.y] = vxB; sv[3 * ab.y + 1] = vyB; sv[3 * ab.y + 2] = wB; }
        if (p1.k == 0) {
            lds_barrier();
            PTR(0, p0.it * ncol + p0.c + 1);
        }
        p0 = p1; p1 = p2; p2 = adv(p2);
    };
    auto step = [&](Pf &X, Pf &Y, int2 sgY, int2 &sgZ) {
        if (TL > 0 && __builtin_amdgcn_ballot_w64((X.sg.y & 0xff) > PF) != 0)
            slot(std::true_type{}, X, Y, sgY, sgZ);
        else
            slot(std::false_type{}, X, Y, sgY, sgZ);
    };
    Pf bufA{}, bufB{};
    int2 sgA = make_int2(0, 0), sgB = make_int2(0, 0);
    if (total > 0) {
        const int2 sg0 = seg_of(p0);
        ldpair(sg0, bufA);
#pragma unroll
        for (int j = 0; j < PF; j++) ldrow_j(sg0, j, bufA.r[j]);
        sgB = seg_of(p1);
    }
    // slot s solves the buffer of s's parity and fills the other; the
    // segment registers hold slot s+1's (parity of s+1) and s+2's
    for (int s = 0; s < total; s += 2) {
        step(bufA, bufB, sgB, sgA);
        if (s + 1 < total) step(bufB, bufA, sgA, sgB);
    }
    if (total == 0) __syncthreads();   // (no sweep: the prologue's LDS writes)
    if (bodies) {   // k_pgs_writeback in the epilogue (only the velocity fields: the
                    // position solver writes the poses of the same bodies concurrently)
        for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
            if (!inContact[i]) continue;
            lpe_body &b = bodies[i];
            if (infinite_mass(b)) continue;
            b.vx = sv[3 * i];
            b.vy = sv[3 * i + 1];
            if (can_rotate(b)) b.omega = sv[3 * i + 2];
        }
    } else {
        for (int i = threadIdx.x; i < 3 * nb; i += SOLVE_TPB) vel[i] = sv[i];
    }
}

// a wave that sees no progress for this many passes gives up and raises
// counts[7] (never expected: the schedule is deadlock free by construction)
static constexpr unsigned FLOW_WATCHDOG = 1u << 24;

__device__ __forceinline__ int ver_acquire(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void ver_release(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// solveLcpPgs (contact_solver.cpp:381-440): per contact the normal row then
// the friction row (:449-543), applyImpulse (:315-356); body velocities in LDS.
// A lane holds its current item and the next one of its queue in registers
// (loaded one item ahead), so a pass never waits on a global load.
struct PgsItem {
    float4 rn, rr, rm;   // dir + eff, lever arms, inverse masses / inertias
    int2 ab;             // bodies (-1 = static)
    int4 rv;             // rank/cnt on A, rank/cnt on B
};
__global__ void __launch_bounds__(SOLVE_TPB)
k_pgs_flow(int nb, const int32_t *__restrict__ ncptr, const float4 *__restrict__ rowN,
           const float4 *__restrict__ rowR, const int2 *__restrict__ rowAB,
           const float4 *__restrict__ rowM, const int4 *__restrict__ rowV,
           float *__restrict__ vel, int iters, float mu, float *__restrict__ lamN,
           float *__restrict__ lamF, int32_t *__restrict__ fault) {
    extern __shared__ float sv[];   // 3 floats per body, then one version counter per body
    int *ver = (int *)(sv + 3 * nb);
    for (int i = threadIdx.x; i < 3 * nb; i += SOLVE_TPB) sv[i] = vel[i];
    for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) ver[i] = 0;
    __syncthreads();
    const int K = *ncptr;
    const int j = threadIdx.x;
    const int R = (K > j) ? (K - j + SOLVE_TPB - 1) / SOLVE_TPB : 0;
    const int total = iters * R;
    auto load = [&](int tt) {
        PgsItem q;
        q.rn = rowN[tt]; q.rr = rowR[tt]; q.rm = rowM[tt]; q.ab = rowAB[tt]; q.rv = rowV[tt];
        return q;
    };
    int done = 0, it = 0, r = 0, t = j;
    PgsItem cur{}, nxt{};
    cur.ab = make_int2(-1, -1);
    float ln = 0.f, lf = 0.f, nln = 0.f, nlf = 0.f;
    int nit = 0, nr = 0, nt = j;            // queue position of nxt (R > 1)
    if (total > 0) cur = load(t);
    if (R > 1) { nr = 1; nt = j + SOLVE_TPB; nxt = load(nt); }
    // drain the preheader loads here: otherwise the wait for them lands at
    // the loop top, where it would also wait out every later prefetch
    __builtin_amdgcn_s_waitcnt(0);
    unsigned idle = 0;   // watchdog: passes of this wave without progress
    bool prog = false;
    while (__any(done < total)) {
        idle = __any(prog) ? 0u : idle + 1u;
        prog = false;
        if (idle > FLOW_WATCHDOG) {
            if (threadIdx.x % 64 == 0) atomicOr(fault, 1);
            break;
        }
        if (done < total) {
            const int2 ab = cur.ab;
            const int4 rv = cur.rv;
            const int needA = it * rv.y + rv.x, needB = it * rv.w + rv.z;
            bool ready = true;
            if (ab.x >= 0) ready = ver_acquire(&ver[ab.x]) == needA;
            if (ready && ab.y >= 0) ready = ver_acquire(&ver[ab.y]) == needB;
            if (ready) {
                const float4 rn = cur.rn, rr = cur.rr;
                const float imA = cur.rm.x, iiA = cur.rm.y, imB = cur.rm.z, iiB = cur.rm.w;
                float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
                if (ab.x >= 0) { vxA = sv[3 * ab.x]; vyA = sv[3 * ab.x + 1]; wA = sv[3 * ab.x + 2]; }
                if (ab.y >= 0) { vxB = sv[3 * ab.y]; vyB = sv[3 * ab.y + 1]; wB = sv[3 * ab.y + 2]; }
#pragma unroll
                for (int row = 0; row < 2; row++) {
                    float dX = row == 0 ? rn.x : -rn.y;
                    float dY = row == 0 ? rn.y : rn.x;
                    float eff = row == 0 ? rn.z : rn.w;
                    float ax = vxA - wA * rr.y, ay = vyA + wA * rr.x;
                    float bx = vxB - wB * rr.w, by = vyB + wB * rr.z;
                    float relX = bx - ax, relY = by - ay;
                    float vrel = relX * dX + relY * dY;
                    float old, lo, hi;
                    if (row == 0) { old = ln; lo = 0.0f; hi = 1e20f; }
                    else {
                        old = lf;
                        float limit = mu * ln;
                        lo = -limit; hi = limit;
                    }
                    float dl = -eff * (vrel + 0.0f);
                    float nl = old + dl;
                    if (nl < lo) nl = lo;
                    if (nl > hi) nl = hi;
                    dl = nl - old;
                    if (row == 0) ln = nl; else lf = nl;
                    if (fabsf(dl) < 1e-15F) continue;
                    if (ab.x >= 0) {
                        vxA -= dX * (dl * imA);
                        vyA -= dY * (dl * imA);
                        float crossA = rr.x * dY - rr.y * dX;
                        wA -= crossA * dl * iiA;
                    }
                    if (ab.y >= 0) {
                        vxB += dX * (dl * imB);
                        vyB += dY * (dl * imB);
                        float crossB = rr.z * dY - rr.w * dX;
                        wB += crossB * dl * iiB;
                    }
                }
                if (ab.x >= 0) {
                    sv[3 * ab.x] = vxA; sv[3 * ab.x + 1] = vyA; sv[3 * ab.x + 2] = wA;
                    ver_release(&ver[ab.x], needA + 1);
                }
                if (ab.y >= 0) {
                    sv[3 * ab.y] = vxB; sv[3 * ab.y + 1] = vyB; sv[3 * ab.y + 2] = wB;
                    ver_release(&ver[ab.y], needB + 1);
                }
                done++;
                prog = true;
                if (R == 1) {
                    it++;                       // same row next sweep: lambdas stay in registers
                } else {
                    // lane-private lambdas: park this row's; the next item's were
                    // fetched one item ahead (stored >= 1 item before that fetch)
                    lamN[t] = ln; lamF[t] = lf;
                    cur = nxt; ln = nln; lf = nlf;
                    it = nit; r = nr; t = nt;
                    nr = r + 1; nit = it;
                    if (nr == R) { nr = 0; nit++; }
                    nt = j + nr * SOLVE_TPB;
                    if (done + 1 < total) {
                        nxt = load(nt);
                        nln = nit > 0 ? lamN[nt] : 0.f;
                        nlf = nit > 0 ? lamF[nt] : 0.f;
                    }
                }
            }
        }
        // every lane rejoins here each pass: keeps the compiler from turning
        // the not-ready path into an inner loop that lanes which progressed
        // would have to wait out (a SIMT deadlock)
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * nb; i += SOLVE_TPB) vel[i] = sv[i];
}

// write velocities of dynamic bodies in the DOF table (:516-529)
__global__ void k_pgs_writeback(int nb, lpe_body *__restrict__ bodies, const float *__restrict__ vel,
                                const int32_t *__restrict__ inContact) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb || !inContact[i]) return;
    lpe_body &b = bodies[i];
    if (infinite_mass(b)) return;
    b.vx = vel[3 * i];
    b.vy = vel[3 * i + 1];
    if (can_rotate(b)) b.omega = vel[3 * i + 2];
}

// ---------------------------------------------------------------------------
// position solver (position_solver.cpp)
__device__ __forceinline__ bool solid_body(const lpe_body &b) {
    return (b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_SOLID);
}
// loadBodyData (:125-168): invM, invI, canRotate(bit0), valid(bit1), solid(bit2)
__global__ void k_pos_bodies(int nb, const lpe_body *__restrict__ bodies, double *__restrict__ st) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    const lpe_body b = bodies[i];
    double invM = (b.mass > 1e29) ? 0.0 : (1.0 / b.mass);
    double invI = 0.0;
    int fl = 0;
    if (b.flags & LPE_BODY_HAS_INERTIA) {
        double I = b.inertia;
        if (I < 1e29 && I > 1e-12) { fl |= 1; invI = 1.0 / I; }
    }
    if (b.flags & LPE_BODY_HAS_MASS) fl |= 2;
    if (solid_body(b)) fl |= 4;
    st[3 * i] = invM;
    st[3 * i + 1] = invI;
    st[3 * i + 2] = (double)fl;
}
// gatherPositionData (:67-120): keep contacts with at least one Solid body;
// a body is a dependency only if it can move (invM != 0 or canRotate)
// u = position in the solver order (order[u] = contact; NULL: narrowphase order)
__global__ void k_pos_items(const int32_t *__restrict__ ncptr, const int32_t *__restrict__ order,
                            const lpe_contact *__restrict__ cs, const lpe_body *__restrict__ bodies,
                            const double *__restrict__ st, int32_t *__restrict__ keep) {
    int u = blockIdx.x * RTPB + threadIdx.x;
    if (u >= *ncptr) return;
    const lpe_contact c = cs[order ? order[u] : u];
    keep[u] = (solid_body(bodies[c.a]) || solid_body(bodies[c.b])) ? 1 : 0;
}
// gatherPositionData (:67-120) for the kept contact at order position u ->
// item t, packed with everything of the item that does not change during
// the solve (normal, correction, inverse masses, static skips)
__global__ void k_pos_fill(const int32_t *__restrict__ ncptr, const int32_t *__restrict__ order,
                           const int32_t *__restrict__ keep,
                           const int32_t *__restrict__ kstart, const lpe_contact *__restrict__ cs,
                           const double *__restrict__ st, PosRec *__restrict__ rec,
                           int32_t *__restrict__ ia, int32_t *__restrict__ ib,
                           int32_t *__restrict__ inPos, double baumgarte, double slop) {
    int u = blockIdx.x * RTPB + threadIdx.x;
    if (u >= *ncptr || !keep[u]) return;
    int t = kstart[u];
    const lpe_contact c = cs[order ? order[u] : u];
    auto movable = [&](int b) {
        return st[3 * b] != 0.0 || ((int)st[3 * b + 2] & 1);
    };
    ia[t] = movable(c.a) ? c.a : -1;
    ib[t] = movable(c.b) ? c.b : -1;
    inPos[c.a] = 1;
    inPos[c.b] = 1;
    int fa = (int)st[3 * c.a + 2], fb = (int)st[3 * c.b + 2];
    PosRec q;
    q.a = c.a; q.b = c.b;
    int fl = 0;
    if (!(fa & 2) || !(fb & 2)) fl |= 1;                       // solvePositionConstraint (:201-297)
    if (!(fa & 4) && !(fb & 4)) fl |= 1;
    double pen = c.pen - slop;
    if (pen <= 0.0) fl |= 1;
    if (fa & 1) fl |= 2;
    if (fb & 1) fl |= 4;
    D2 n = nrm(d2(c.nx, c.ny));
    q.nx = n.x; q.ny = n.y;
    q.corr = baumgarte * pen;
    q.px = c.px; q.py = c.py;
    q.invMA = st[3 * c.a]; q.invMB = st[3 * c.b];
    q.invIA = st[3 * c.a + 1]; q.invIB = st[3 * c.b + 1];
    q.flags = fl;
    q.pad = 0;
    rec[t] = q;
}
// Position solver, canonical order: every contact keeps its row position u
// (non-kept contacts become skipped items), so the colour segments of the PGS
// apply unchanged; colour-synchronous sweeps (see k_pgs_colour), body poses
// in LDS (fp64).  solvePositionContactsOnce (position_solver.cpp:215-290).
// The rows are stored as arrays (44 bytes a row, the pair's bodies and
// masses with each row and read from its first), carved from posRec's
// allocation: lanes of a wave read consecutive 16-byte pieces.
struct PosRows {
    double2 *n, *c, *m, *i;    // (nx, ny), (corr, px), (invMA, invMB), (invIA, invIB)
    double *py;
    int2 *ab;                  // bodies
    int32_t *fl;               // 1 skipped, 2 A rotates, 4 B rotates
};
__global__ void k_pos_fill_rows(const int32_t *__restrict__ ncptr, const int32_t *__restrict__ order,
                                const lpe_contact *__restrict__ cs, const lpe_body *__restrict__ bodies,
                                const double *__restrict__ st, PosRows out,
                                int32_t *__restrict__ inPos, double baumgarte, double slop) {
    int u = blockIdx.x * RTPB + threadIdx.x;
    if (u >= *ncptr) return;
    const lpe_contact c = cs[order[u]];
    const bool kept = solid_body(bodies[c.a]) || solid_body(bodies[c.b]);   // gatherPositionData (:67-120)
    int fa = (int)st[3 * c.a + 2], fb = (int)st[3 * c.b + 2];
    int fl = kept ? 0 : 1;
    if (kept) { inPos[c.a] = 1; inPos[c.b] = 1; }
    if (!(fa & 2) || !(fb & 2)) fl |= 1;
    if (!(fa & 4) && !(fb & 4)) fl |= 1;
    double pen = c.pen - slop;
    if (pen <= 0.0) fl |= 1;
    if (fa & 1) fl |= 2;
    if (fb & 1) fl |= 4;
    D2 n = nrm(d2(c.nx, c.ny));
    out.n[u] = make_double2(n.x, n.y);
    out.c[u] = make_double2(baumgarte * pen, c.px);
    out.py[u] = c.py;
    out.fl[u] = fl;
    out.m[u] = make_double2(st[3 * c.a], st[3 * c.b]);
    out.i[u] = make_double2(st[3 * c.a + 1], st[3 * c.b + 1]);
    out.ab[u] = make_int2(c.a, c.b);
}

// The solver preparation in two launches (colour_prep; the same arithmetic as
// the five kernels above, which the replay path keeps): per body the PGS's
// inverse masses (k_pgs_bodies, what = 1), the position solver's body data
// (k_pos_bodies) and the contact marks cleared; then per solver-order item
// the body marks (k_mark_contacts: the same set of bodies, marked from the
// same contacts), the PGS row (k_pgs_rows) and the position row
// (k_pos_fill_rows).
__global__ void k_prep_bodies(int nb, const lpe_body *__restrict__ bodies, float *__restrict__ imii,
                              double *__restrict__ st, int32_t *__restrict__ inContact) {
    const int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    const lpe_body b = bodies[i];
    {
        const bool cr = can_rotate(b);
        const double m = b.mass;
        const float im = (m > 1e29) ? 0.f : (float)(1.0 / m);
        float iv = 0.f;
        if (cr) {
            const double I = b.inertia;
            if (I > 1e-12 && I < 1e29) iv = (float)(1.0 / I);
        }
        imii[2 * i] = im; imii[2 * i + 1] = iv;
    }
    {
        const double invM = (b.mass > 1e29) ? 0.0 : (1.0 / b.mass);
        double invI = 0.0;
        int fl = 0;
        if (b.flags & LPE_BODY_HAS_INERTIA) {
            const double I = b.inertia;
            if (I < 1e29 && I > 1e-12) { fl |= 1; invI = 1.0 / I; }
        }
        if (b.flags & LPE_BODY_HAS_MASS) fl |= 2;
        if (solid_body(b)) fl |= 4;
        st[3 * i] = invM;
        st[3 * i + 1] = invI;
        st[3 * i + 2] = (double)fl;
    }
    inContact[i] = 0;
    inContact[nb + i] = 0;
}
__global__ void k_prep_items(const int32_t *__restrict__ ncptr, const int32_t *__restrict__ order,
                             const lpe_contact *__restrict__ cs, const lpe_body *__restrict__ bodies,
                             const float *__restrict__ imii, const double *__restrict__ st, float4 *__restrict__ rowN,
                             float4 *__restrict__ rowR, int2 *__restrict__ rowAB, float4 *__restrict__ rowM,
                             int32_t *__restrict__ sItemA, int32_t *__restrict__ sItemB, PosRows out,
                             int32_t *__restrict__ inContact, int32_t *__restrict__ inPos, double baumgarte,
                             double slop, int32_t *__restrict__ rowOf, float4 *__restrict__ rowC) {
    const int t = blockIdx.x * RTPB + threadIdx.x;
    if (t >= *ncptr) return;
    const lpe_contact c = cs[order[t]];
    rowOf[order[t]] = t;                          // (the Jacobi solver reads the rows by contact)
    const lpe_body A = bodies[c.a], B = bodies[c.b];
    inContact[c.a] = 1;
    inContact[c.b] = 1;
    {   // k_pgs_rows
        const int a = infinite_mass(A) ? -1 : c.a;
        const int b = infinite_mass(B) ? -1 : c.b;
        const D2 u = nrm(d2(c.nx, c.ny));
        const float dirX = (float)u.x, dirY = (float)u.y;
        const float rxA = (float)(c.px - A.x), ryA = (float)(c.py - A.y);
        const float rxB = (float)(c.px - B.x), ryB = (float)(c.py - B.y);
        float imA = 0.f, imB = 0.f, iiA = 0.f, iiB = 0.f;
        if (a >= 0) { imA = imii[2 * a]; iiA = imii[2 * a + 1]; }
        if (b >= 0) { imB = imii[2 * b]; iiB = imii[2 * b + 1]; }
        float effN, effF;
        {
            const float rAxn = cross2f(rxA, ryA, dirX, dirY), rBxn = cross2f(rxB, ryB, dirX, dirY);
            const float sum = imA + imB + (rAxn * rAxn) * iiA + (rBxn * rBxn) * iiB;
            effN = (sum < 1e-12F) ? 0.F : 1.F / sum;
        }
        {
            const float fx = -dirY, fy = dirX;
            const float rAxn = cross2f(rxA, ryA, fx, fy), rBxn = cross2f(rxB, ryB, fx, fy);
            const float sum = imA + imB + (rAxn * rAxn) * iiA + (rBxn * rBxn) * iiB;
            effF = (sum < 1e-12F) ? 0.F : 1.F / sum;
        }
        rowN[t] = make_float4(dirX, dirY, effN, effF);
        rowR[t] = make_float4(rxA, ryA, rxB, ryB);
        rowAB[t] = make_int2(a, b);
        rowM[t] = make_float4(imA, iiA, imB, iiB);
        // applyImpulse's crosses (:338-355) per direction, as pgs_row_t forms
        // them: r x d with d = (dirX, dirY), then d = (-dirY, dirX)
        rowC[t] = make_float4(rxA * dirY - ryA * dirX, rxB * dirY - ryB * dirX,
                              rxA * dirX - ryA * (-dirY), rxB * dirX - ryB * (-dirY));
        sItemA[t] = a;
        sItemB[t] = b;
    }
    {   // k_pos_fill_rows
        const bool kept = solid_body(A) || solid_body(B);
        const int fa = (int)st[3 * c.a + 2], fb = (int)st[3 * c.b + 2];
        int fl = kept ? 0 : 1;
        if (kept) { inPos[c.a] = 1; inPos[c.b] = 1; }
        if (!(fa & 2) || !(fb & 2)) fl |= 1;
        if (!(fa & 4) && !(fb & 4)) fl |= 1;
        const double pen = c.pen - slop;
        if (pen <= 0.0) fl |= 1;
        if (fa & 1) fl |= 2;
        if (fb & 1) fl |= 4;
        const D2 n = nrm(d2(c.nx, c.ny));
        out.n[t] = make_double2(n.x, n.y);
        out.c[t] = make_double2(baumgarte * pen, c.px);
        out.py[t] = c.py;
        out.fl[t] = fl;
        out.m[t] = make_double2(st[3 * c.a], st[3 * c.b]);
        out.i[t] = make_double2(st[3 * c.a + 1], st[3 * c.b + 1]);
        out.ab[t] = make_int2(c.a, c.b);
    }
}

// one item on the pair's poses in registers (the colour solver): the items of
// a pair share its bodies, their inverse masses and rotation flags
__device__ __forceinline__ void pos_item_regs(double nx, double ny, double corr, double px, double py,
                                              int flags, double invMA, double invMB, double invIA,
                                              double invIB, double &xA, double &yA, double &tA,
                                              double &xB, double &yB, double &tB) {
    if (flags & 1) return;
    D2 rA = d2(px - xA, py - yA);
    D2 rB = d2(px - xB, py - yB);
    D2 n = d2(nx, ny);
    double rAn = crs(rA, n), rBn = crs(rB, n);
    double denom = invMA + invMB + (rAn * rAn) * invIA + (rBn * rBn) * invIB;
    if (denom < 1e-12) return;
    double sc = corr / denom;
    double dx = n.x * sc, dy = n.y * sc;
    if (invMA != 0.0 || (flags & 2)) {
        xA -= dx * invMA;
        yA -= dy * invMA;
        if (flags & 2) tA -= rAn * sc * invIA;
    }
    if (invMB != 0.0 || (flags & 4)) {
        xB += dx * invMB;
        yB += dy * invMB;
        if (flags & 4) tB += rBn * sc * invIB;
    }
}

// the same, the skip and the static-body cases as selects of the unchanged
// values (bit-identical: every value that is kept is computed by the same
// operations; a skipped item's arithmetic is discarded)
// The striped position solver's item (pos_item's arithmetic in registers),
// the skipped item as a zero correction instead of selects: a skipped item (flags & 1, or denom < 1e-12) gets sc = 0, and a
// body that does not move (invM = 0) or turn (invI = 0 exactly when its
// rotation flag is clear, k_prep_bodies) gets x - n sc 0 = x -- the same
// value (a pose of exactly zero may change the sign of its zero, which no
// later operation of the tick turns into a different non-zero value)
__device__ __forceinline__ void pos_item_z(double nx, double ny, double corr, double px, double py,
                                           int flags, double invMA, double invMB, double invIA,
                                           double invIB, double &xA, double &yA, double &tA,
                                           double &xB, double &yB, double &tB) {
    D2 rA = d2(px - xA, py - yA);
    D2 rB = d2(px - xB, py - yB);
    D2 n = d2(nx, ny);
    double rAn = crs(rA, n), rBn = crs(rB, n);
    double denom = invMA + invMB + (rAn * rAn) * invIA + (rBn * rBn) * invIB;
    const bool apply = !(flags & 1) && !(denom < 1e-12);
    const double sc = apply ? corr / denom : 0.0;
    double dx = n.x * sc, dy = n.y * sc;
    xA = xA - dx * invMA; yA = yA - dy * invMA; tA = tA - rAn * sc * invIA;
    xB = xB + dx * invMB; yB = yB + dy * invMB; tB = tB + rBn * sc * invIB;
}
__device__ __forceinline__ void pos_item(const PosRec &q, double *sp) {
    if (q.flags & 1) return;
    const int a = q.a, b = q.b;
    D2 rA = d2(q.px - sp[3 * a], q.py - sp[3 * a + 1]);
    D2 rB = d2(q.px - sp[3 * b], q.py - sp[3 * b + 1]);
    D2 n = d2(q.nx, q.ny);
    double rAn = crs(rA, n), rBn = crs(rB, n);
    double denom = q.invMA + q.invMB + (rAn * rAn) * q.invIA + (rBn * rBn) * q.invIB;
    if (denom < 1e-12) return;
    double sc = q.corr / denom;
    double dx = n.x * sc, dy = n.y * sc;
    // an immovable body (invM = 0, no rotation) would get x - 0: skipped, so
    // pairs of one colour never write a shared static body
    if (q.invMA != 0.0 || (q.flags & 2)) {
        sp[3 * a] -= dx * q.invMA;
        sp[3 * a + 1] -= dy * q.invMA;
        if (q.flags & 2) sp[3 * a + 2] -= rAn * sc * q.invIA;
    }
    if (q.invMB != 0.0 || (q.flags & 4)) {
        sp[3 * b] += dx * q.invMB;
        sp[3 * b + 1] += dy * q.invMB;
        if (q.flags & 4) sp[3 * b + 2] += rBn * sc * q.invIB;
    }
}

#ifndef POS_PF
#define POS_PF 1    // rows of a pair prefetched with it
#endif
#ifndef POS_TL
#define POS_TL 2    // further rows loaded at the start of its slot (waves with longer pairs)
#endif
#ifndef POS_ILV
#define POS_ILV 0   // the next slot's rows loaded between the current pair's rows
#endif
__device__ __forceinline__ double2 bld_d2(__amdgpu_buffer_rsrc_t r, uint32_t i, bool ok = true) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(ok ? i * 16u : BOOB), 0, 0);
    return make_double2(__hiloint2double((int)v.y, (int)v.x), __hiloint2double((int)v.w, (int)v.z));
}
__device__ __forceinline__ double bld_d(__amdgpu_buffer_rsrc_t r, uint32_t i, bool ok = true) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(ok ? i * 8u : BOOB), 0, 0);
    return __hiloint2double((int)v.y, (int)v.x);
}
__device__ __forceinline__ int bld_i(__amdgpu_buffer_rsrc_t r, uint32_t i, bool ok = true) {
    return (int)__builtin_amdgcn_raw_buffer_load_b32(r, (int)(ok ? i * 4u : BOOB), 0, 0);
}
// Slot-pipelined like k_pgs_colour (see there): a colour's pairs in slots of
// at most one pair per thread, the next slot's pair (bodies, masses, first
// POS_PF rows) prefetched into the other buffer, the segment of the slot
// after it one slot earlier, idle lanes reading out of range.  A wave whose
// current pairs have more rows loads rows POS_PF.. POS_PF+POS_TL-1 at the
// start of the slot (before the prefetch, so each wait stays exact); rows
// beyond those are read on demand.  Rows in canonical order, arithmetic
// unchanged: bit-identical to the sequential sweep in colour-major order.
__global__ void __launch_bounds__(SOLVE_TPB)
k_pos_colour(int nb, const int32_t *__restrict__ counts, const int32_t *__restrict__ cbase,
             const int2 *__restrict__ seg, PosRows rows,
             lpe_body *__restrict__ bodies, const double *__restrict__ st,
             const int32_t *__restrict__ inPos, int iters) {
    extern __shared__ double sp[];   // x, y, angle per body
    __shared__ int scb[MAX_COLOURS + 1];
    const int ncol = counts[8];
    for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
        const lpe_body &b = bodies[i];
        sp[3 * i] = b.x; sp[3 * i + 1] = b.y;
        sp[3 * i + 2] = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
    }
    for (int c = threadIdx.x; c <= ncol; c += SOLVE_TPB) scb[c] = cbase[c];
    __syncthreads();
    const auto rN = brsrc(rows.n), rC = brsrc(rows.c), rMm = brsrc(rows.m), rI = brsrc(rows.i);
    const auto rPy = brsrc(rows.py), rAB = brsrc(rows.ab), rF = brsrc(rows.fl), rSeg = brsrc(seg);
    constexpr int PF = POS_PF, TL = POS_TL;
    constexpr bool ILV = POS_ILV;
    struct Row { double nx, ny, cr, px, py; int fl; };
    struct Pf {
        int2 sg;
        int a, b;
        double iMA, iMB, iIA, iIB;
        Row r[PF];
    };
    auto ldrow = [&](int t, bool ok, Row &w) {
        const double2 n = bld_d2(rN, t, ok), c = bld_d2(rC, t, ok);
        w.nx = n.x; w.ny = n.y; w.cr = c.x; w.px = c.y;
        w.py = bld_d(rPy, t, ok);
        w.fl = bld_i(rF, t, ok);
    };
    // row j of the pair with segment sg (rows past its last: clamped to it,
    // not loaded; no pair: an out-of-range segment, nrow 0)
    auto ldrow_j = [&](int2 sg, int j, Row &w) {
        const int nrow = sg.y & 0xff, stride = sg.y >> 8;
        ldrow(sg.x + min(j, max(nrow - 1, 0)) * stride, j < nrow, w);
    };
    auto ldpair = [&](int2 sg, Pf &f) {
        f.sg = sg;
        const bool ok = (sg.y & 0xff) > 0;
        const int2 ab = bld_i2(rAB, sg.x, ok);
        f.a = ab.x; f.b = ab.y;
        const double2 m = bld_d2(rMm, sg.x, ok), ii = bld_d2(rI, sg.x, ok);
        f.iMA = m.x; f.iMB = m.y; f.iIA = ii.x; f.iIB = ii.y;
    };
    auto ucb = [&](int c) { return __builtin_amdgcn_readfirstlane(scb[c]); };
    auto nslot0 = [&](int c) { return (ucb(c + 1) - ucb(c) + SOLVE_TPB - 1) / SOLVE_TPB; };
    int S = 0;
    for (int c = 0; c < ncol; c++) S += nslot0(c);
    const int total = iters * S;
    struct SP { int c, k, it; };
    auto adv = [&](SP p) {
        if (++p.k == nslot0(p.c)) { p.k = 0; if (++p.c == ncol) { p.c = 0; p.it++; } }
        return p;
    };
    auto seg_of = [&](SP p) {
        const int q = ucb(p.c) + threadIdx.x + p.k * SOLVE_TPB;
        return bld_i2(rSeg, q, q < ucb(p.c + 1) && p.it < iters);
    };
    SP p0{0, 0, 0}, p1 = adv(p0), p2 = adv(p1);
    PTR(1, 0);
    // one slot, laid out as k_pgs_colour's
    auto slot = [&](auto tail, Pf &X, Pf &Y, int2 sgY, int2 &sgZ) {
        constexpr bool TAIL = decltype(tail)::value;
        const int nrow = X.sg.y & 0xff, stride = X.sg.y >> 8;
        const bool hx = nrow > 0;
        Row T[TL > 0 ? TL : 1];
        if constexpr (TAIL) {
#pragma unroll
            for (int j = 0; j < TL; j++) ldrow_j(X.sg, PF + j, T[j]);
        }
        sgZ = seg_of(p2);
        ldpair(sgY, Y);
        if constexpr (!ILV) {
#pragma unroll
            for (int j = 0; j < PF; j++) ldrow_j(sgY, j, Y.r[j]);
        }
        const int a = X.a, b = X.b;
        double xA = 0.0, yA = 0.0, tA = 0.0, xB = 0.0, yB = 0.0, tB = 0.0;
        if (hx) {
            xA = sp[3 * a]; yA = sp[3 * a + 1]; tA = sp[3 * a + 2];
            xB = sp[3 * b]; yB = sp[3 * b + 1]; tB = sp[3 * b + 2];
        }
        auto row = [&](int j, const Row &w) {
            if (j < nrow)
                pos_item_regs(w.nx, w.ny, w.cr, w.px, w.py, w.fl, X.iMA, X.iMB, X.iIA, X.iIB, xA, yA, tA, xB,
                              yB, tB);
        };
#pragma unroll
        for (int j = 0; j < PF; j++) {
            row(j, X.r[j]);
            if constexpr (ILV) {
                __builtin_amdgcn_sched_barrier(0);
                ldrow_j(sgY, j, Y.r[j]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (TAIL) {
#pragma unroll
            for (int j = 0; j < TL; j++) row(PF + j, T[j]);
        }
        for (int j = TAIL ? PF + TL : PF; j < nrow; j++) {   // longer pairs: on demand
            Row w;
            ldrow(X.sg.x + j * stride, true, w);
            row(j, w);
        }
        // a static body (invM = 0, no rotation) is never written: pairs of
        // one colour may share it
        const int fl0 = X.r[0].fl;
        if (hx && (X.iMA != 0.0 || (fl0 & 2))) { sp[3 * a] = xA; sp[3 * a + 1] = yA; sp[3 * a + 2] = tA; }
        if (hx && (X.iMB != 0.0 || (fl0 & 4))) { sp[3 * b] = xB; sp[3 * b + 1] = yB; sp[3 * b + 2] = tB; }
        if (p1.k == 0) {
            lds_barrier();
            PTR(1, p0.it * ncol + p0.c + 1);
        }
        p0 = p1; p1 = p2; p2 = adv(p2);
    };
    auto step = [&](Pf &X, Pf &Y, int2 sgY, int2 &sgZ) {
        if (TL > 0 && __builtin_amdgcn_ballot_w64((X.sg.y & 0xff) > PF) != 0)
            slot(std::true_type{}, X, Y, sgY, sgZ);
        else
            slot(std::false_type{}, X, Y, sgY, sgZ);
    };
    Pf bufA{}, bufB{};
    int2 sgA = make_int2(0, 0), sgB = make_int2(0, 0);
    if (total > 0) {
        const int2 sg0 = seg_of(p0);
        ldpair(sg0, bufA);
#pragma unroll
        for (int j = 0; j < PF; j++) ldrow_j(sg0, j, bufA.r[j]);
        sgB = seg_of(p1);
    }
    for (int s = 0; s < total; s += 2) {
        step(bufA, bufB, sgB, sgA);
        if (s + 1 < total) step(bufB, bufA, sgA, sgB);
    }
    __syncthreads();
    // storeBodyData (:176-197)
    for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
        if (!inPos[i]) continue;
        int f = (int)st[3 * i + 2];
        if (!(f & 2)) continue;
        lpe_body &b = bodies[i];
        b.x = sp[3 * i]; b.y = sp[3 * i + 1];
        if ((f & 1) && (b.flags & LPE_BODY_HAS_ANGPOS)) b.angle = sp[3 * i + 2];
    }
}

// PositionSolver::positionalSolver (:299-325) by dataflow; x, y, angle of
// every body in LDS (fp64); item data double-buffered as in k_pgs_flow
struct PosItem {
    PosRec q;
    int4 rv;
    int da, db;          // movable dependency bodies (-1 none)
};
__global__ void __launch_bounds__(SOLVE_TPB)
k_pos_flow(int nb, const int32_t *__restrict__ kptr, const PosRec *__restrict__ rec,
           const int4 *__restrict__ rowV, const int32_t *__restrict__ ia,
           const int32_t *__restrict__ ib, lpe_body *__restrict__ bodies,
           const double *__restrict__ st, const int32_t *__restrict__ inPos, int iters,
           int32_t *__restrict__ fault) {
    extern __shared__ double sp[];   // x, y, angle per body, then one version counter per body
    int *ver = (int *)(sp + 3 * nb);
    for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
        const lpe_body &b = bodies[i];
        sp[3 * i] = b.x; sp[3 * i + 1] = b.y;
        sp[3 * i + 2] = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
        ver[i] = 0;
    }
    __syncthreads();
    const int K = *kptr;
    const int j = threadIdx.x;
    const int R = (K > j) ? (K - j + SOLVE_TPB - 1) / SOLVE_TPB : 0;
    const int total = iters * R;
    auto load = [&](int tt) {
        PosItem p;
        p.q = rec[tt]; p.rv = rowV[tt]; p.da = ia[tt]; p.db = ib[tt];
        return p;
    };
    int done = 0, it = 0, r = 0;
    PosItem cur{}, nxt{};
    cur.da = cur.db = -1;
    int nit = 0, nr = 0;
    if (total > 0) cur = load(j);
    if (R > 1) { nr = 1; nxt = load(j + SOLVE_TPB); }
    __builtin_amdgcn_s_waitcnt(0);     // see k_pgs_flow
    unsigned idle = 0;
    bool prog = false;
    while (__any(done < total)) {
        idle = __any(prog) ? 0u : idle + 1u;
        prog = false;
        if (idle > FLOW_WATCHDOG) {
            if (threadIdx.x % 64 == 0) atomicOr(fault, 1);
            break;
        }
        if (done < total) {
            const int da = cur.da, db = cur.db;
            const int needA = it * cur.rv.y + cur.rv.x, needB = it * cur.rv.w + cur.rv.z;
            bool ready = true;
            if (da >= 0) ready = ver_acquire(&ver[da]) == needA;
            if (ready && db >= 0) ready = ver_acquire(&ver[db]) == needB;
            if (ready) {
                const PosRec &q = cur.q;
                if (!(q.flags & 1)) {
                    const int a = q.a, b = q.b;
                    D2 rA = d2(q.px - sp[3 * a], q.py - sp[3 * a + 1]);
                    D2 rB = d2(q.px - sp[3 * b], q.py - sp[3 * b + 1]);
                    D2 n = d2(q.nx, q.ny);
                    double rAn = crs(rA, n), rBn = crs(rB, n);
                    double denom = q.invMA + q.invMB + (rAn * rAn) * q.invIA + (rBn * rBn) * q.invIB;
                    if (!(denom < 1e-12)) {
                        double sc = q.corr / denom;
                        double dx = n.x * sc, dy = n.y * sc;
                        // a body that cannot move (invM = 0, no rotation) is left
                        // untouched: its update is x - 0
                        if (da >= 0) {
                            sp[3 * a] -= dx * q.invMA;
                            sp[3 * a + 1] -= dy * q.invMA;
                            if (q.flags & 2) sp[3 * a + 2] -= rAn * sc * q.invIA;
                        }
                        if (db >= 0) {
                            sp[3 * b] += dx * q.invMB;
                            sp[3 * b + 1] += dy * q.invMB;
                            if (q.flags & 4) sp[3 * b + 2] += rBn * sc * q.invIB;
                        }
                    }
                }
                if (da >= 0) ver_release(&ver[da], needA + 1);
                if (db >= 0) ver_release(&ver[db], needB + 1);
                done++;
                prog = true;
                if (R == 1) {
                    it++;
                } else {
                    cur = nxt; it = nit; r = nr;
                    nr = r + 1; nit = it;
                    if (nr == R) { nr = 0; nit++; }
                    if (done + 1 < total) nxt = load(j + nr * SOLVE_TPB);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();   // reconvergence point (see k_pgs_flow)
    }
    __syncthreads();
    // storeBodyData (:176-197)
    for (int i = threadIdx.x; i < nb; i += SOLVE_TPB) {
        if (!inPos[i]) continue;
        int f = (int)st[3 * i + 2];
        if (!(f & 2)) continue;
        lpe_body &b = bodies[i];
        b.x = sp[3 * i]; b.y = sp[3 * i + 1];
        if ((f & 1) && (b.flags & LPE_BODY_HAS_ANGPOS)) b.angle = sp[3 * i + 2];
    }
}

// ---------------------------------------------------------------------------
// integrator systems (per body, fp64)
// ===========================================================================
// Striped Gauss-Seidel: the canonical solver order since round 3 (restated by
// oracle/rigid_oracle.cpp lpeo_stripe_order; see there for the definition).
// The movable bodies of the contact pairs are cut into S x-stripes no
// narrower than the longest pair; band j = stripes 2j and 2j+1, seam j =
// the stripe pair 2j+1 | 2j+2.  A pair lies inside one band or across one
// seam; each band's and each seam's pairs are coloured greedily.  A sweep is
// phase A (every band) then phase B (every seam); the bands touch disjoint
// bodies and so do the seams, so workgroup j runs band j, then seam j,
// concurrently with the others: only stripes 2j and 2j+2 are shared with a
// neighbour, handed over through global memory with one flag per phase
// (write-through stores and loads, MI355X_MICROARCH.md hand-off table, first
// row).  W = S/2 workgroups (one per CU) instead of one: a sweep's critical
// path is one band's colours plus one seam's (about 10 steps at scene M)
// instead of every colour of the scene, each step 1/W of the pairs.
static constexpr int STRIPES_MAX = 64;
static constexpr int SGROUPS = 2 * STRIPES_MAX;          // (S groups are used: S/2 bands, S/2 - 1 seams)
static constexpr int SCOLS = 64;                 // colours per group (a greedy colouring needs degree + 1)
static constexpr int STEPS_MAX = SGROUPS * SCOLS;
#ifndef LPE_STPB
#define LPE_STPB 256
#endif
static constexpr int STPB = LPE_STPB;             // threads of a stripe workgroup
// At most this many pairs with contacts: one stripe (one workgroup, no
// hand-overs).  A small scene's colours are few (a box stack's are two), so
// its sweeps are a handful of steps, while the stripes' per-phase hand-overs
// (~1-3 us each) were most of its solve (C1: 153 us with 40 stripes).
static constexpr int STRIPE_MIN_PAIRS = 1024;

struct StripeBufs {
    int32_t *bstripe;      // [nb] stripe of a movable body in a contact pair, else -1
    int32_t *bpos;         // [nb] slot of a contact-pair body in sbList, else -1
    double *bred;          // [4 per block of k_stripe_pairs] x min, x max, longest pair, pairs with contacts
    int32_t *pflag;        // [cap_pairs] 1 has contacts, 2 A movable, 4 B movable
    double2 *px;           // [cap_pairs] x of A and B
    int32_t *pgroup;       // [cap_pairs] group of a pair with contacts, else -1
    int32_t *pcolg;        // [cap_pairs] colour inside its group
    int32_t *prank;        // [cap_pairs] rank inside (group, colour)
    int32_t *prowoff;      // [cap_pairs] first row inside (group, colour)
    int32_t *glist;        // [cap_pairs] pairs by group, ascending inside a group
    int32_t *gla, *glb, *gln;  // [cap_pairs] by glist position: the pair's two movable bodies' slots in its
                               // group's stripes (-1: static) and its contact count (k_group_colour)
    int32_t *gstart;       // [SGROUPS + 1]
    int32_t *gcnt;         // [SGROUPS][SCOLS][2] pairs, rows per (group, colour); [SGROUPS*SCOLS*2 + g]: colours of g
    int32_t *stepIdx;      // [SGROUPS * SCOLS] canonical step of (group, colour)
    int32_t *stepPair;     // [STEPS_MAX + 1] first coloured-pair slot of a step
    int32_t *stepRow;      // [STEPS_MAX + 1] first row of a step
    int32_t *wgStep;       // [STRIPES_MAX / 2][4] phase A [first, end), phase B [first, end)
    int32_t *sbStart;      // [STRIPES_MAX + 2] bodies of each stripe; [STRIPES_MAX + 1]: end of the static ones
    int32_t *sbList;       // [nb] movable contact-pair bodies by stripe, then the static ones
    uint32_t *sflag;       // [2][STRIPES_MAX / 2] hand-over flags (phase A, phase B) per solver
    unsigned long long *gvt;   // [3 nb] velocities handed over (PGS) with their epochs, by sbList slot
    double *gpos;          // [3 nb] poses handed over (position solver), by sbList slot
};

__device__ __forceinline__ int stripe_of(double x, double x0, double w, int S) {
    if (S == 1) return 0;
    const double f = floor((x - x0) / w);
    return (int)fmin((double)(S - 1), fmax(0.0, f));
}

// per pair with contacts: which bodies move and their x; per block the range
// of the movable bodies' x, the longest pair and the pairs with contacts
// (sb.bred, 4 doubles a block)
__global__ void __launch_bounds__(RTPB)
k_stripe_pairs(const int32_t *__restrict__ npptr, const int2 *__restrict__ pairs,
               const int32_t *__restrict__ ccount, const lpe_body *__restrict__ bodies, StripeBufs sb) {
    __shared__ double wr[3][RTPB / 64];
    __shared__ int wc[RTPB / 64];
    const int p = blockIdx.x * RTPB + threadIdx.x;
    const int np = *npptr;
    if ((int)(blockIdx.x * RTPB) >= np) return;
    double mn = 1.7976931348623157e308, mx = -1.7976931348623157e308, sp = 0.0;
    bool has = false;
    if (p < np) {
        int f = 0;
        double2 x = make_double2(0.0, 0.0);
        if (ccount[p] > 0) {
            const int2 pr = pairs[p];
            const lpe_body &A = bodies[pr.x], &B = bodies[pr.y];
            const bool da = colour_dep(A), db = colour_dep(B);
            x = make_double2(A.x, B.x);
            f = 1 | (da ? 2 : 0) | (db ? 4 : 0);
            has = true;
            if (da) { mn = fmin(mn, x.x); mx = fmax(mx, x.x); }
            if (db) { mn = fmin(mn, x.y); mx = fmax(mx, x.y); }
            if (da && db) sp = fabs(x.x - x.y);
        }
        sb.pflag[p] = f;
        sb.px[p] = x;
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, off));
        mx = fmax(mx, __shfl_xor(mx, off));
        sp = fmax(sp, __shfl_xor(sp, off));
    }
    const int w = threadIdx.x >> 6;
    const int c = __popcll(__ballot(has));
    if ((threadIdx.x & 63) == 0) { wr[0][w] = mn; wr[1][w] = mx; wr[2][w] = sp; wc[w] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int n = wc[0];
        for (int k = 1; k < RTPB / 64; k++) {
            mn = fmin(mn, wr[0][k]); mx = fmax(mx, wr[1][k]); sp = fmax(sp, wr[2][k]); n += wc[k];
        }
        sb.bred[4 * blockIdx.x] = mn;
        sb.bred[4 * blockIdx.x + 1] = mx;
        sb.bred[4 * blockIdx.x + 2] = sp;
        sb.bred[4 * blockIdx.x + 3] = (double)n;
    }
}

// One workgroup: the stripe count and width, the stripes' body lists (then
// the static bodies of contact pairs), the pairs' groups and the groups'
// sizes (counts[12] = S, counts[13] = workgroups).  The stripe count comes
// first, from k_stripe_pairs' partials alone, so one pass over the pairs
// marks their bodies, checks the one-stripe rule and files them in groups
// (round 4: the pair loops batched, SETUP_U pairs a thread in flight; three
// passes of dependent loads were ~50 us at scene M).
static constexpr int SETUP_U = 4;

__global__ void __launch_bounds__(SOLVE_TPB)
k_stripe_setup(int nb, const int32_t *__restrict__ npptr, const int2 *__restrict__ pairs,
               const lpe_body *__restrict__ bodies, StripeBufs sb, int32_t *__restrict__ counts, int smax) {
    extern __shared__ unsigned int bmark[];                 // [2][words]: movable / static contact-pair bodies
    __shared__ double wr[3][SOLVE_TPB / 64];
    __shared__ int wn[SOLVE_TPB / 64];
    __shared__ double sx0, sw;
    __shared__ int sS, sViol, nstat, statcur;
    __shared__ int scnt[STRIPES_MAX], scur[STRIPES_MAX], gcount[SGROUPS];
    STP(0);
    const int np = *npptr;
    const int words = (nb + 31) >> 5;
    for (int i = threadIdx.x; i < 2 * words; i += SOLVE_TPB) bmark[i] = 0u;
    for (int i = threadIdx.x; i < STRIPES_MAX; i += SOLVE_TPB) scnt[i] = 0;
    for (int i = threadIdx.x; i < SGROUPS; i += SOLVE_TPB) gcount[i] = 0;
    if (threadIdx.x == 0) { sViol = 0; nstat = 0; }
    double mn = 1.7976931348623157e308, mx = -1.7976931348623157e308, sp = 0.0;
    int npairs = 0;                                        // pairs with contacts
    const int nblk = (np + RTPB - 1) / RTPB;
    for (int k = threadIdx.x; k < nblk; k += SOLVE_TPB) {
        mn = fmin(mn, sb.bred[4 * k]); mx = fmax(mx, sb.bred[4 * k + 1]); sp = fmax(sp, sb.bred[4 * k + 2]);
        npairs += (int)sb.bred[4 * k + 3];
    }
    for (int off = 32; off > 0; off >>= 1) {
        mn = fmin(mn, __shfl_xor(mn, off));
        mx = fmax(mx, __shfl_xor(mx, off));
        sp = fmax(sp, __shfl_xor(sp, off));
        npairs += __shfl_xor(npairs, off);
    }
    if ((threadIdx.x & 63) == 0) {
        wr[0][threadIdx.x >> 6] = mn; wr[1][threadIdx.x >> 6] = mx; wr[2][threadIdx.x >> 6] = sp;
        wn[threadIdx.x >> 6] = npairs;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < SOLVE_TPB / 64; k++) {
            mn = fmin(mn, wr[0][k]); mx = fmax(mx, wr[1][k]); sp = fmax(sp, wr[2][k]); npairs += wn[k];
        }
        int S = 1;
        if (mx > mn && npairs > STRIPE_MIN_PAIRS) {
            const double q = (mx - mn) / sp;          // (span 0: +inf)
            // (smax: the two solvers' S / 2 workgroups each must be co-resident,
            // one per CU -- stripe_cap)
            if (q >= 2.0 && smax >= 2) S = min(smax, (int)floor(fmin(q, 1e9))) & ~1;
        }
        sS = S;
        sx0 = mn;
        sw = (mx - mn) / S;
    }
    __syncthreads();
    STP(1);
    int S = sS;
    const double x0 = sx0, w = sw;
    // one pass over the pairs: the bodies' marks, the one-stripe rule (a pair
    // more than one stripe apart, a rounding edge), the groups for S
    for (int p0 = 0; p0 < np; p0 += SETUP_U * SOLVE_TPB) {
        int f[SETUP_U];
        int2 pr[SETUP_U];
        double2 x[SETUP_U];
#pragma unroll
        for (int u = 0; u < SETUP_U; u++) {
            const int p = p0 + u * SOLVE_TPB + (int)threadIdx.x;
            f[u] = 0;
            if (p < np) { f[u] = sb.pflag[p]; pr[u] = pairs[p]; x[u] = sb.px[p]; }
        }
#pragma unroll
        for (int u = 0; u < SETUP_U; u++) {
            const int p = p0 + u * SOLVE_TPB + (int)threadIdx.x;
            if (p >= np) continue;
            int g = -1;
            if (f[u] & 1) {
                atomicOr(&bmark[((f[u] & 2) ? 0 : words) + (pr[u].x >> 5)], 1u << (pr[u].x & 31));
                atomicOr(&bmark[((f[u] & 4) ? 0 : words) + (pr[u].y >> 5)], 1u << (pr[u].y & 31));
                int sa = (f[u] & 2) ? stripe_of(x[u].x, x0, w, S) : -1;
                int sb2 = (f[u] & 4) ? stripe_of(x[u].y, x0, w, S) : -1;
                if (sa >= 0 && sb2 >= 0 && abs(sa - sb2) > 1) sViol = 1;
                if (sa < 0) sa = sb2;
                if (sb2 < 0) sb2 = sa;
                if (sa < 0) sa = sb2 = 0;
                g = (sa >> 1) == (sb2 >> 1) ? 2 * (sa >> 1) : 2 * (min(sa, sb2) >> 1) + 1;
                atomicAdd(&gcount[g], 1);
            }
            sb.pgroup[p] = g;
        }
    }
    __syncthreads();
    STP(2);
    if (sViol) {                                       // (block-uniform) one stripe after all
        S = 1;
        for (int p = threadIdx.x; p < np; p += SOLVE_TPB) sb.pgroup[p] = (sb.pflag[p] & 1) ? 0 : -1;
        for (int i = threadIdx.x; i < SGROUPS; i += SOLVE_TPB) gcount[i] = i == 0 ? npairs : 0;
        __syncthreads();
    }
    for (int b = threadIdx.x; b < nb; b += SOLVE_TPB) {
        int s = -1;
        if ((bmark[b >> 5] >> (b & 31)) & 1u) {
            s = stripe_of(bodies[b].x, x0, w, S);
            atomicAdd(&scnt[s], 1);
        } else if ((bmark[words + (b >> 5)] >> (b & 31)) & 1u) {
            atomicAdd(&nstat, 1);
        }
        sb.bstripe[b] = s;
    }
    __syncthreads();
    STP(3);
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int s = 0; s < STRIPES_MAX; s++) { sb.sbStart[s] = acc; scur[s] = acc; acc += scnt[s]; }
        sb.sbStart[STRIPES_MAX] = acc;
        statcur = acc;
        sb.sbStart[STRIPES_MAX + 1] = acc + nstat;
        acc = 0;
        for (int g = 0; g < SGROUPS; g++) { sb.gstart[g] = acc; acc += gcount[g]; }
        sb.gstart[SGROUPS] = acc;
        counts[12] = S;
        counts[13] = (S + 1) / 2;
    }
    __syncthreads();
    STP(4);
    for (int b = threadIdx.x; b < nb; b += SOLVE_TPB) {
        const int s = sb.bstripe[b];
        int i = -1;
        if (s >= 0) i = atomicAdd(&scur[s], 1);
        else if ((bmark[words + (b >> 5)] >> (b & 31)) & 1u) i = atomicAdd(&statcur, 1);
        if (i >= 0) sb.sbList[i] = b;
        sb.bpos[b] = i;
    }
    STP(5);
}

// one wave per group: greedy colouring of its pairs in ascending order (the
// lowest colour free on the pair's movable bodies), the pair's rank and row
// offset inside its (group, colour), the group's colour sizes.  The bodies'
// colour masks live in LDS by stripe-list slot (the group's bodies lie in
// its one or two stripes) between chunks of 32 pairs; inside a chunk they
// live in the lanes of the pairs that last changed them.  The colouring is
// one sequential chain, run by the whole wave on wave-uniform values: each
// body's source lane is found before the chain from the chunk's body lists
// alone, colour c's pair / row counters live in lane c, so a pair costs four
// lane reads, the first free colour and a lane write (round 4: ~30
// instructions a pair, from ~115 with the masks indexed by slot).
// The block first lists its group's pairs in ascending order (a stable
// compaction by all RTPB threads), then wave 0 colours them.  (Round 4
// measured a block-wide Jones-Plassmann colouring with ascending-order
// priority -- the same colours as the sequential pass -- and dropped it: in
// entity order a pair's lower neighbours form chains as long as the scene,
// so the rounds were 2-3x slower than the chain.)

__global__ void __launch_bounds__(RTPB)
k_group_colour(const int32_t *__restrict__ npptr, const int32_t *__restrict__ counts, const int2 *__restrict__ pairs,
               const int32_t *__restrict__ ccount, StripeBufs sb) {
    extern __shared__ unsigned long long used[];             // per stripe-list slot of the group's stripes
    const int g = (int)blockIdx.x;
    const int S = counts[12];
    if (g >= S) return;                                // groups: bands 0, 2, .. and seams 1, 3, .. < S
    CTR(0, wall_clock64());
    const int s = (g >> 1) * 2 + (g & 1);               // band j: stripes 2j, 2j+1; seam j: 2j+1, 2j+2
    const int u0 = sb.sbStart[s], u1 = sb.sbStart[min(s + 2, S)];
    const int g0 = sb.gstart[g], g1 = sb.gstart[g + 1];
    {
        // the list: wave w files the group's pairs of its quarter of the
        // pairs in ascending order (ballots; the group tests batched LIST_U
        // loads deep, counted in a first pass, filed in a second), then each
        // listed pair's body slots and contact count, one pair a thread (the
        // colouring chain below reads three plain arrays)
        constexpr int LIST_U = 8;
        __shared__ int wcount[RTPB / 64];
        const int np = *npptr;
        const int wv = (int)threadIdx.x >> 6, ln = (int)threadIdx.x & 63;
        const int seg = ((np + RTPB - 1) / RTPB) * 64;    // (a multiple of 64 a wave)
        const int s0 = min(np, wv * seg), s1 = min(np, s0 + seg);
        auto pass = [&](bool file, int off) {
            int cnt = 0;
            for (int b0 = s0; b0 < s1; b0 += 64 * LIST_U) {
                int gv[LIST_U];
#pragma unroll
                for (int u = 0; u < LIST_U; u++) {
                    const int p = b0 + 64 * u + ln;
                    gv[u] = p < s1 ? sb.pgroup[p] : -1;
                }
#pragma unroll
                for (int u = 0; u < LIST_U; u++) {
                    const bool hit = gv[u] == g;
                    const unsigned long long m = __ballot(hit);
                    if (file && hit) sb.glist[off + cnt + __popcll(m & ((1ull << ln) - 1ull))] = b0 + 64 * u + ln;
                    cnt += __popcll(m);
                }
            }
            return cnt;
        };
        const int mine = pass(false, 0);
        if (ln == 0) wcount[wv] = mine;
        __syncthreads();
        int off = g0;
        for (int k = 0; k < wv; k++) off += wcount[k];
        pass(true, off);
        __syncthreads();                               // (the list, in global memory)
        for (int t = g0 + (int)threadIdx.x; t < g1; t += RTPB) {
            const int p = sb.glist[t];
            const int2 pr = pairs[p];
            const int fl = sb.pflag[p];
            const int n = ccount[p];
            const int ba = sb.bpos[pr.x], bb = sb.bpos[pr.y];
            sb.gla[t] = (fl & 2) ? ba - u0 : -1;
            sb.glb[t] = (fl & 4) ? bb - u0 : -1;
            sb.gln[t] = n;
        }
    }
    CTR(1, wall_clock64());
    for (int i = (int)threadIdx.x; i < u1 - u0; i += RTPB) used[i] = 0ull;
    __syncthreads();                                   // (the list's slots and counts, and the masks)
    CTR(2, wall_clock64());
    if (threadIdx.x >= 64) return;
    const int lane = (int)threadIdx.x;
    int ncol = 0, fault = 0;
    int cp = 0, cr = 0;                                   // lane c: colour c's pairs and rows so far
    // Chunks of 32 pairs; lane l is the pair (l & 31)'s body on side l >> 5
    // (A, B).  Its register R holds that body's colour mask: on entry the
    // mask after the earlier chunks (from LDS), after the pair its mask with
    // the pair's colour added.  A pair reads each body's mask from the lane of
    // the chunk's last earlier pair on that body (src: found before the
    // chain, from the body lists alone), or from its own lane, so the chain is
    // two 64-bit reads, the first free colour and two lane writes per pair.
    const int side = lane >> 5, k = lane & 31;
    auto fetch = [&](int c0, int &p, int &body, int &n) {
        const int t = c0 + k;
        p = -1; body = -1; n = 0;
        if (t < g1) {
            body = side ? sb.glb[t] : sb.gla[t];
            if (!side) { p = sb.glist[t]; n = sb.gln[t]; }
        }
    };
    int np_, nbody, nn;
    fetch(g0, np_, nbody, nn);                            // (one chunk ahead: off the chain)
    for (int c0 = g0; c0 < g1; c0 += 32) {
        const int p = np_, body = nbody, n = nn;
        fetch(c0 + 32, np_, nbody, nn);
        const int m = min(32, g1 - c0);
        const unsigned long long R0 = body >= 0 ? used[body] : 0ull;
        uint32_t Rlo = (uint32_t)R0, Rhi = (uint32_t)(R0 >> 32);
        // (a static body's key is unique to its lane: it matches no other)
        const int key = body >= 0 ? body : -2 - lane;
        int src = lane;                                   // the lane holding the body's mask before the pair
        int later = 0;                                    // a later pair of the chunk has the body
        for (int j = 0; j < m; j++) {
            const int s0 = __builtin_amdgcn_readlane(key, j), s1 = __builtin_amdgcn_readlane(key, j + 32);
            const bool before = j < k;
            src = (before && s0 == key) ? j : src;
            src = (before && s1 == key) ? j + 32 : src;
            later |= (j > k) & ((s0 == key) | (s1 == key));
        }
        int myc = 0, myrank = 0, myrow = 0;
        for (int i = 0; i < m; i++) {
            const int sa = __builtin_amdgcn_readlane(src, i), sb_ = __builtin_amdgcn_readlane(src, i + 32);
            const int ni = __builtin_amdgcn_readlane(n, i);
            const unsigned long long ua =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)Rhi, sa) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)Rlo, sa);
            const unsigned long long ub =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)Rhi, sb_) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)Rlo, sb_);
            const unsigned long long forb = ua | ub;      // (a static body's lane holds 0)
            const int c = forb == ~0ull ? 0 : __ffsll((long long)~forb) - 1;
            fault |= forb == ~0ull;
            const unsigned long long bit = 1ull << c;
            const unsigned long long na = ua | bit, nb = ub | bit;
            const bool ia = lane == i, ib = lane == i + 32;
            Rlo = ia ? (uint32_t)na : (ib ? (uint32_t)nb : Rlo);
            Rhi = ia ? (uint32_t)(na >> 32) : (ib ? (uint32_t)(nb >> 32) : Rhi);
            ncol = max(ncol, c + 1);
            // rank and row offset in ascending order
            const int rank = __builtin_amdgcn_readlane(cp, c), row = __builtin_amdgcn_readlane(cr, c);
            const bool ic = lane == c;
            cp += ic ? 1 : 0;
            cr += ic ? ni : 0;
            myc = ia ? c : myc;
            myrank = ia ? rank : myrank;
            myrow = ia ? row : myrow;
        }
        // (one writer per body; read by the next chunk)
        if (body >= 0 && !later) used[body] = ((unsigned long long)Rhi << 32) | Rlo;
        if (!side && p >= 0) {
            sb.pcolg[p] = myc;
            sb.prank[p] = myrank;
            sb.prowoff[p] = myrow;
        }
    }
    CTR(3, wall_clock64());
    CTR(4, (unsigned long long)*npptr);
    CTR(5, (unsigned long long)(g1 - g0));
    CTR(6, (unsigned long long)(u1 - u0));
    CTR(7, (unsigned long long)ncol);
    int32_t *gc = sb.gcnt + (size_t)g * SCOLS * 2;
    gc[2 * lane] = cp;
    gc[2 * lane + 1] = cr;
    if (lane == 0) {
        sb.gcnt[SGROUPS * SCOLS * 2 + g] = ncol;
        if (fault) atomicOr((int *)&counts[7], 1);
    }
}

// the canonical step sequence: phase A (the bands, groups 0, 2, 4, ..), then
// phase B (the seams, groups 1, 3, ..), colours ascending.  Thread t is the
// t-th group of that sequence (phase t >> 6, band / seam j = t & 63); one
// block scan gives every group's first step, pair slot and row.
__global__ void __launch_bounds__(RTPB)
k_stripe_layout(StripeBufs sb, int32_t *__restrict__ counts) {
    const int S = counts[12];
    const int t = (int)threadIdx.x;
    const int ph = t >> 6, j = t & 63, g = 2 * j + ph;
    const bool valid = t < SGROUPS && 2 * j + ph < S;
    const int nc = valid ? sb.gcnt[SGROUPS * SCOLS * 2 + g] : 0;
    int gp = 0, gr = 0;
    const int32_t *gc = sb.gcnt + (size_t)(valid ? g : 0) * SCOLS * 2;
    for (int c = 0; c < nc; c++) { gp += gc[2 * c]; gr += gc[2 * c + 1]; }
    int ts, tp, trw;
    const int s0 = r_block_excl(nc, &ts), p0 = r_block_excl(gp, &tp), q0 = r_block_excl(gr, &trw);
    int pa = p0, ra = q0;
    for (int c = 0; c < nc; c++) {
        sb.stepIdx[g * SCOLS + c] = s0 + c;
        sb.stepPair[s0 + c] = pa;
        sb.stepRow[s0 + c] = ra;
        pa += gc[2 * c];
        ra += gc[2 * c + 1];
    }
    if (t < SGROUPS && j < STRIPES_MAX / 2) {       // workgroup j runs band j and seam j
        sb.wgStep[4 * j + 2 * ph] = s0;
        sb.wgStep[4 * j + 2 * ph + 1] = s0 + nc;
    }
    if (t == 0) {
        sb.stepPair[ts] = tp;
        sb.stepRow[ts] = trw;
        counts[8] = ts;
    }
}

// each pair's slot in the step sequence (seg: its rows, contiguous) and its
// rows' contact indices (order); pcol = the pair's step (-1: no contact)
__global__ void k_stripe_fill(const int32_t *__restrict__ npptr, const int32_t *__restrict__ ccount,
                              const int32_t *__restrict__ cstart, StripeBufs sb, int32_t *__restrict__ pcol,
                              int2 *__restrict__ seg, int32_t *__restrict__ order) {
    const int p = blockIdx.x * RTPB + threadIdx.x;
    if (p >= *npptr) return;
    const int g = sb.pgroup[p];
    if (g < 0) { pcol[p] = -1; return; }
    const int st = sb.stepIdx[g * SCOLS + sb.pcolg[p]];
    const int q = sb.stepPair[st] + sb.prank[p];
    const int rs = sb.stepRow[st] + sb.prowoff[p];
    const int n = ccount[p], c0 = cstart[p];
    seg[q] = make_int2(rs, n | (1 << 8));
    for (int j = 0; j < n; j++) order[rs + j] = c0 + j;
    pcol[p] = st;
}

// ---- hand-over of a stripe's bodies between neighbouring workgroups --------
// (MI355X_MICROARCH.md, inter-workgroup hand-off table, first row: every
// store and load of the handed-over values write-through / L1-bypassing
// (relaxed agent-scope atomics: global_store / global_load ... sc1), each
// storing wave drained before the workgroup barrier, one lane's sc1 flag
// store; the consumer's lane 0 polls the flag with sc1 loads, the others load
// after the barrier it joins.  One workgroup per CU, hipMalloc memory.)
// Values travel by stripe-list slot; lv holds them by slot - s0.
template <typename T>
__device__ __forceinline__ void stripe_publish(const StripeBufs &sb, int s, int s0, const T *lv, T *g) {
    const int b0 = 3 * sb.sbStart[s], b1 = 3 * sb.sbStart[s + 1];
    for (int i = b0 + (int)threadIdx.x; i < b1; i += STPB)
        __hip_atomic_store(&g[i], lv[i - 3 * s0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void stripe_reload(const StripeBufs &sb, int s, int s0, T *lv, const T *g) {
    const int b0 = 3 * sb.sbStart[s], b1 = 3 * sb.sbStart[s + 1];
    for (int i = b0 + (int)threadIdx.x; i < b1; i += STPB)
        lv[i - 3 * s0] = __hip_atomic_load(&g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stripe_signal(uint32_t *flag, uint32_t v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // this wave's hand-over stores are done
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a wait that sees no progress for ~0.2 s gives up and raises counts[7] bit 2
// (never expected: the schedule is deadlock free and every workgroup is
// resident); the solve's result is then wrong and the next detection fails
__device__ __forceinline__ void stripe_wait(const uint32_t *flag, uint32_t v, int32_t *fault) {
    if (threadIdx.x == 0) {
        unsigned spins = 0;
        while ((int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - v) < 0) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 22)) { atomicOr(fault, 2); break; }
        }
    }
    __syncthreads();
}

// What workgroup j works on: bodies of stripes 2j .. 2j+2 (sbList slots
// [s0, s1)), phase A steps [a0, a1) (stripe 2j's two groups) and phase B
// steps [b0, b1) (stripe 2j+1's), and their pairs and rows, each a contiguous
// range of the step sequence with A before B.  The LDS copies number pairs
// and rows A first, then B (lpair / lrow); local step k = lstep(st).
struct StripeView {
    int S, j, s0, s1, nDyn, nAll;
    int a0, a1, b0, b1;
    int pA0, nA, pB0, nB;
    int rA0, nRA, rB0, nRB;
    __device__ int lpair(int q) const { return q < pA0 + nA ? q - pA0 : nA + q - pB0; }
    __device__ int lrow(int r) const { return r < rA0 + nRA ? r - rA0 : nRA + r - rB0; }
    __device__ int lstep(int st) const { return st < a1 ? st - a0 : (a1 - a0) + st - b0; }
    __device__ int nsteps() const { return (a1 - a0) + (b1 - b0); }
    __device__ int npairs() const { return nA + nB; }
    __device__ int nrows() const { return nRA + nRB; }
    __device__ int nloc() const { return s1 - s0; }
};
__device__ __forceinline__ StripeView stripe_view(const StripeBufs &sb, const int32_t *counts, int j) {
    StripeView v;
    v.S = counts[12]; v.j = j;
    v.s0 = sb.sbStart[2 * j];
    v.s1 = sb.sbStart[min(2 * j + 3, v.S)];
    v.nDyn = sb.sbStart[STRIPES_MAX];
    v.nAll = sb.sbStart[STRIPES_MAX + 1];
    v.a0 = sb.wgStep[4 * j]; v.a1 = sb.wgStep[4 * j + 1];
    v.b0 = sb.wgStep[4 * j + 2]; v.b1 = sb.wgStep[4 * j + 3];
    v.pA0 = sb.stepPair[v.a0]; v.nA = sb.stepPair[v.a1] - v.pA0;
    v.pB0 = sb.stepPair[v.b0]; v.nB = sb.stepPair[v.b1] - v.pB0;
    v.rA0 = sb.stepRow[v.a0]; v.nRA = sb.stepRow[v.a1] - v.rA0;
    v.rB0 = sb.stepRow[v.b0]; v.nRB = sb.stepRow[v.b1] - v.rB0;
    return v;
}
// the local steps' first local pairs (and the end), into LDS
__device__ __forceinline__ void stripe_steps_lds(const StripeBufs &sb, const StripeView &v, int *stepL) {
    const int ns = v.nsteps();
    for (int k = threadIdx.x; k <= ns; k += STPB) {
        const int st = k < v.a1 - v.a0 ? v.a0 + k : v.b0 + (k - (v.a1 - v.a0));
        stepL[k] = k == ns ? v.npairs() : v.lpair(sb.stepPair[st]);
    }
}

// Does every colour step of this workgroup hold at most one wave of pairs?
// Then wave 0 runs the steps alone (stripe_sweeps, `single`): a step's
// pairs touch disjoint bodies, and one wave's LDS stores are visible to its
// own later loads once they have completed (s_waitcnt), so consecutive steps
// need no workgroup barrier -- the barrier, and the three idle waves'
// re-issue, were a third of a step's latency (profiles/r03/pgs_step_cost.txt).
// stepL: the LDS step table (or null: the global one).  Every thread calls it.
__device__ __forceinline__ bool stripe_single_wave(const StripeBufs &sb, const StripeView &v, const int *stepL) {
    __shared__ int s_big;
    if (threadIdx.x == 0) s_big = 0;
    __syncthreads();
    const int ns = v.nsteps();
    for (int k = threadIdx.x; k < ns; k += STPB) {
        int len;
        if (stepL) {
            len = stepL[k + 1] - stepL[k];
        } else {
            const int st = k < v.a1 - v.a0 ? v.a0 + k : v.b0 + (k - (v.a1 - v.a0));
            len = sb.stepPair[st + 1] - sb.stepPair[st];
        }
        if (len > 64) s_big = 1;
    }
    __syncthreads();
    return s_big == 0;
}

// The sweeps of one stripe pair per workgroup (the loop shared by both
// solvers): phase A = stripe 2j's steps, phase B = stripe 2j+1's; before a
// phase the shared stripe a neighbour changed last is reloaded, after it the
// one the neighbour needs next is published.  solve(st, it) runs one step.
// single: wave 0 runs the steps without workgroup barriers between them
// (stripe_single_wave); the workgroup joins at the phase's end.
// wave 0's steps [s0, s1) one after the other (the `single` schedule)
template <typename Solve>
__device__ __forceinline__ void wave_steps(int s0, int s1, int it, Solve &solve) {
    if (threadIdx.x < 64) {
        for (int st = s0; st < s1; st++) {
            solve(st, it);
            // this wave's LDS stores complete before its next step's loads
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_s_waitcnt(0xc07f);        // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
        }
    }
}
// Tagged hand-over (the PGS's fp32 velocities): each value travels with the
// epoch of the phase that wrote it in one 64-bit word (value bits | epoch <<
// 32, relaxed agent-scope atomic stores and loads), and a consumer polls the
// values themselves until every one carries the epoch it waits for -- one
// memory round trip instead of a flag poll followed by a reload.  A stripe's
// words are rewritten only after their consumer has read them (the phases'
// dependency chain), so a consumer never sees a later epoch than the one it
// waits for.
__device__ __forceinline__ void stripe_publish_tag(const StripeBufs &sb, int s, int s0, const float *lv,
                                                   unsigned long long *g, uint32_t tag) {
    const int b0 = 3 * sb.sbStart[s], b1 = 3 * sb.sbStart[s + 1];
    for (int i = b0 + (int)threadIdx.x; i < b1; i += STPB)
        __hip_atomic_store(&g[i], ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(lv[i - 3 * s0]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stripe_reload_tag(const StripeBufs &sb, int s, int s0, float *lv,
                                                  const unsigned long long *g, uint32_t tag, int32_t *fault) {
    const int b0 = 3 * sb.sbStart[s], b1 = 3 * sb.sbStart[s + 1];
    // (once a wait has timed out -- this thread's, or any, seen in
    // the fault word -- the remaining words are not waited for: one timeout
    // period per stuck solve, not one per word)
    bool gave_up = (__hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2) != 0;
    for (int i = b0 + (int)threadIdx.x; i < b1; i += STPB) {
        unsigned long long w = __hip_atomic_load(&g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (!gave_up && (uint32_t)(w >> 32) != tag) {
            __builtin_amdgcn_s_sleep(1);
            ++spins;
            if (spins > (1u << 22)) { atomicOr(fault, 2); gave_up = true; break; }      // (as stripe_wait)
            if (!(spins & 1023u) && (__hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2)) {
                gave_up = true;
                break;
            }
            w = __hip_atomic_load(&g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        lv[i - 3 * s0] = __uint_as_float((uint32_t)w);
    }
}

// single: `phase(s0, s1, it)` runs wave 0's steps (wave_steps, or a solver's
// own pipelined loop); the workgroup joins at the phase's end.  G = unsigned
// long long: the tagged hand-over (T = float; the flags are not used, the
// epochs are base + 2 it + 1 after phase A, + 2 after phase B).
template <typename T, typename G, typename Solve, typename Phase>
__device__ __forceinline__ void stripe_sweeps(const StripeBufs &sb, const StripeView &v, int iters, uint32_t base,
                                              uint32_t *flagA, uint32_t *flagB, T *lv, G *g, int32_t *fault,
                                              Solve solve, int tw, bool single, Phase phase) {
    constexpr bool tagged = std::is_same<G, unsigned long long>::value;
    const int j = v.j;
    const bool right = 2 * j + 2 < v.S;             // seam j (phase B) exists
    (void)tw;
    auto steps = [&](int s0, int s1, int it) {
        if (single) {
            phase(s0, s1, it);
            __syncthreads();
        } else {
            for (int st = s0; st < s1; st++) { solve(st, it); __syncthreads(); }
        }
    };
    STR(tw, j, 1);
    for (int it = 0; it < iters; it++) {
        if (it > 0 && j > 0) {                    // stripe 2j, after the left neighbour's phase B of it - 1
            if constexpr (tagged) {
                stripe_reload_tag(sb, 2 * j, v.s0, lv, g, base + 2 * it, fault);
            } else {
                stripe_wait(&flagB[j - 1], base + it, fault);
                stripe_reload(sb, 2 * j, v.s0, lv, g);
            }
            __syncthreads();
        }
        STR(tw, j, 2 + 6 * it);
        steps(v.a0, v.a1, it);
        STR(tw, j, 3 + 6 * it);
        if (j > 0) {
            if constexpr (tagged) {
                stripe_publish_tag(sb, 2 * j, v.s0, lv, g, base + 2 * it + 1);
            } else {
                stripe_publish(sb, 2 * j, v.s0, lv, g);
                stripe_signal(&flagA[j], base + it + 1);
            }
        }
        STR(tw, j, 4 + 6 * it);
        if (!right) continue;
        {                                         // stripe 2j+2, after the right neighbour's phase A of it
            if constexpr (tagged) {
                stripe_reload_tag(sb, 2 * j + 2, v.s0, lv, g, base + 2 * it + 1, fault);
            } else {
                stripe_wait(&flagA[j + 1], base + it + 1, fault);
                stripe_reload(sb, 2 * j + 2, v.s0, lv, g);
            }
            __syncthreads();
        }
        STR(tw, j, 5 + 6 * it);
        steps(v.b0, v.b1, it);
        STR(tw, j, 6 + 6 * it);
        if constexpr (tagged) {
            stripe_publish_tag(sb, 2 * j + 2, v.s0, lv, g, base + 2 * it + 2);
        } else {
            stripe_publish(sb, 2 * j + 2, v.s0, lv, g);
            stripe_signal(&flagB[j], base + it + 1);
        }
        STR(tw, j, 7 + 6 * it);
    }
}
// the stripes whose final values this workgroup holds: 2j+1, 2j+2, and 0
__device__ __forceinline__ bool stripe_owned(int s, int j, int S) {
    return s >= 0 && s < S && (s == 2 * j + 1 || s == 2 * j + 2 || (j == 0 && s == 0));
}

// bytes of LDS a stripe workgroup may use (one workgroup per CU)
static constexpr int STRIPE_LDS = 150 * 1024;
__host__ __device__ constexpr int lds_align(int b) { return (b + 15) & ~15; }

// PGS (solveLcpPgs, contact_solver.cpp:381-440) over the striped order.  The
// workgroup's rows, pairs, multipliers and its bodies' velocities live in LDS
// for the whole solve (staged once: rows are 40 bytes, pairs 32); a
// workgroup whose rows do not fit reads them from global memory instead.
__global__ void __launch_bounds__(STPB)
k_pgs_stripes(const int32_t *__restrict__ counts, StripeBufs sb, const int2 *__restrict__ seg,
              const float4 *__restrict__ rowN, const float4 *__restrict__ rowR, const float4 *__restrict__ rowC,
              const int2 *__restrict__ rowAB,
              const float4 *__restrict__ rowM, int iters, float mu, float *__restrict__ lamN,
              float *__restrict__ lamF, lpe_body *__restrict__ bodies, const int32_t *__restrict__ inContact,
              uint32_t base, int32_t *__restrict__ fault) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int j = (int)blockIdx.x;
    if (j >= counts[13]) return;
    __builtin_amdgcn_s_setprio(3);   // (the tick's critical path: issue ahead of co-resident fluid waves)
    STR(0, j, 0);
    const StripeView v = stripe_view(sb, counts, j);
    const int NR = v.nrows(), NP = v.npairs(), NL = v.nloc(), NS = v.nsteps();
    if (threadIdx.x == 0) {   // (trace slots 61-63: phase A / B steps, pairs)
        STR_SET(0, j, 61, v.a1 - v.a0); STR_SET(0, j, 62, v.b1 - v.b0); STR_SET(0, j, 63, NP);
    }
    // layout: rn, rr, rc [NR] float4 | pr [NP] int4 | pm [NP] float4 | ln, lf [NR] | lv [3 NL] | stepL [NS + 1]
    const int oRR = 16 * NR, oRC = oRR + 16 * NR, oPR = oRC + 16 * NR, oPM = oPR + 16 * NP, oLN = oPM + 16 * NP,
              oLF = oLN + 4 * NR,
              oLV = oLF + 4 * NR, oST = oLV + 12 * NL, total = oST + 4 * (NS + 1);
    const bool inL = total <= STRIPE_LDS;
    float *lv = inL ? (float *)(smem + oLV) : (float *)smem;
    for (int i = v.s0 + (int)threadIdx.x; i < v.s1; i += STPB) {
        const lpe_body &b = bodies[sb.sbList[i]];
        float *o = lv + 3 * (i - v.s0);
        o[0] = (float)b.vx; o[1] = (float)b.vy; o[2] = can_rotate(b) ? (float)b.omega : 0.f;
    }
    const int *bpos = sb.bpos;
    auto lbody = [&](int b) { return b >= 0 ? bpos[b] - v.s0 : -1; };
    if (inL) {
        float4 *rn = (float4 *)smem, *rr = (float4 *)(smem + oRR), *rc = (float4 *)(smem + oRC),
               *pm = (float4 *)(smem + oPM);
        int4 *pr = (int4 *)(smem + oPR);
        float *ln = (float *)(smem + oLN), *lf = (float *)(smem + oLF);
        int *stepL = (int *)(smem + oST);
        for (int r = threadIdx.x; r < NR; r += STPB) {
            const int g = r < v.nRA ? v.rA0 + r : v.rB0 + (r - v.nRA);
            rn[r] = rowN[g]; rr[r] = lever_perp(rowR[g]); rc[r] = rowC[g];   // (rr: staged as lever_perp)
            ln[r] = 0.f; lf[r] = 0.f;
        }
        for (int q = threadIdx.x; q < NP; q += STPB) {
            const int gq = q < v.nA ? v.pA0 + q : v.pB0 + (q - v.nA);
            const int2 sg = seg[gq];
            const int2 ab = rowAB[sg.x];
            pr[q] = make_int4(v.lrow(sg.x), sg.y & 0xff, lbody(ab.x), lbody(ab.y));
            pm[q] = rowM[sg.x];
        }
        stripe_steps_lds(sb, v, stepL);
        __syncthreads();
        const bool single = stripe_single_wave(sb, v, stepL);
        auto solve = [&](int st, int) {
            const int k = v.lstep(st);
            const int q1 = stepL[k + 1];
            for (int q = stepL[k] + (int)threadIdx.x; q < q1; q += STPB) {
                const int4 p = pr[q];
                const float4 m = pm[q];
                const bool hasA = p.z >= 0, hasB = p.w >= 0;
                float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
                if (hasA) { vxA = lv[3 * p.z]; vyA = lv[3 * p.z + 1]; wA = lv[3 * p.z + 2]; }
                if (hasB) { vxB = lv[3 * p.w]; vyB = lv[3 * p.w + 1]; wB = lv[3 * p.w + 2]; }
                constexpr int U = 4;                    // rows loaded together
                for (int j0 = 0; j0 < p.y; j0 += U) {
                    float4 a[U], c[U], x[U];
                    float n[U], f[U];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        const int t = p.x + min(j0 + u, p.y - 1);
                        a[u] = rn[t]; c[u] = rr[t]; x[u] = rc[t]; n[u] = ln[t]; f[u] = lf[t];
                    }
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        if (j0 + u >= p.y) break;
                        pgs_row_l(a[u], c[u], x[u], m.x, m.y, m.z, m.w, mu, n[u], f[u], vxA, vyA, wA, vxB, vyB, wB);
                        ln[p.x + j0 + u] = n[u];
                        lf[p.x + j0 + u] = f[u];
                    }
                }
                if (hasA) { lv[3 * p.z] = vxA; lv[3 * p.z + 1] = vyA; lv[3 * p.z + 2] = wA; }
                if (hasB) { lv[3 * p.w] = vxB; lv[3 * p.w + 1] = vyB; lv[3 * p.w + 2] = wB; }
            }
        };
        // the single-wave schedule, software-pipelined: a step's pair record,
        // masses and first U rows (with their multipliers) do not depend on
        // the velocities, so the next step's are loaded before this step's
        // row math; only the bodies' velocities are read after the previous
        // step's stores (one wave: its LDS operations complete in order).
        // Same rows, same order, same arithmetic as `solve`.
        auto phase = [&](int s0, int s1, int) {
            if (threadIdx.x >= 64 || s0 >= s1) return;
            constexpr int U = 4;
            struct Nx { int4 p; float4 m; float4 a[U], c[U], x[U]; float n[U], f[U]; };
            auto fetch = [&](int st, Nx &x) {
                const int k = v.lstep(st);
                const int q = stepL[k] + (int)threadIdx.x;
                const bool ok = q < stepL[k + 1];
                x.p = ok ? pr[q] : make_int4(0, 0, -1, -1);
                x.m = pm[ok ? q : 0];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int t = x.p.x + max(min(u, x.p.y - 1), 0);
                    x.a[u] = rn[t]; x.c[u] = rr[t]; x.x[u] = rc[t]; x.n[u] = ln[t]; x.f[u] = lf[t];
                }
            };
            Nx cur, nxt;
            fetch(s0, cur);
            for (int st = s0; st < s1; st++) {
                if (st + 1 < s1) fetch(st + 1, nxt);
                const int4 p = cur.p;
                const float4 m = cur.m;
                const bool hasA = p.z >= 0, hasB = p.w >= 0;
                float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
                if (hasA) { vxA = lv[3 * p.z]; vyA = lv[3 * p.z + 1]; wA = lv[3 * p.z + 2]; }
                if (hasB) { vxB = lv[3 * p.w]; vyB = lv[3 * p.w + 1]; wB = lv[3 * p.w + 2]; }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    if (u >= p.y) break;
                    float n = cur.n[u], f = cur.f[u];
                    pgs_row_l(cur.a[u], cur.c[u], cur.x[u], m.x, m.y, m.z, m.w, mu, n, f, vxA, vyA, wA, vxB, vyB,
                              wB);
                    ln[p.x + u] = n;
                    lf[p.x + u] = f;
                }
                for (int jr = U; jr < p.y; jr++) {       // (pairs of more than U rows: the rest on demand)
                    const int t = p.x + jr;
                    float n = ln[t], f = lf[t];
                    pgs_row_l(rn[t], rr[t], rc[t], m.x, m.y, m.z, m.w, mu, n, f, vxA, vyA, wA, vxB, vyB, wB);
                    ln[t] = n;
                    lf[t] = f;
                }
                if (hasA) { lv[3 * p.z] = vxA; lv[3 * p.z + 1] = vyA; lv[3 * p.z + 2] = wA; }
                if (hasB) { lv[3 * p.w] = vxB; lv[3 * p.w + 1] = vyB; lv[3 * p.w + 2] = wB; }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // (program order of the LDS accesses)
                cur = nxt;
            }
        };
        stripe_sweeps(sb, v, iters, base, sb.sflag, sb.sflag + STRIPES_MAX / 2, lv, sb.gvt, fault, solve, 0,
                      single, phase);
        __syncthreads();
        for (int r = threadIdx.x; r < NR; r += STPB) {    // (the impulses, lpe_rigid_download_impulses)
            const int g = r < v.nRA ? v.rA0 + r : v.rB0 + (r - v.nRA);
            lamN[g] = ln[r]; lamF[g] = lf[r];
        }
    } else {
        __syncthreads();
        const bool single = stripe_single_wave(sb, v, nullptr);
        auto solve = [&](int st, int it) {
            const int q1 = sb.stepPair[st + 1];
            for (int q = sb.stepPair[st] + (int)threadIdx.x; q < q1; q += STPB) {
                const int2 sg = seg[q];
                const int rs = sg.x, nrow = sg.y & 0xff;
                const int2 ab = rowAB[rs];
                const float4 m = rowM[rs];
                const int la = lbody(ab.x), lb = lbody(ab.y);
                const bool hasA = la >= 0, hasB = lb >= 0;
                float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
                if (hasA) { vxA = lv[3 * la]; vyA = lv[3 * la + 1]; wA = lv[3 * la + 2]; }
                if (hasB) { vxB = lv[3 * lb]; vyB = lv[3 * lb + 1]; wB = lv[3 * lb + 2]; }
                for (int t = rs; t < rs + nrow; t++) {
                    float n = it ? lamN[t] : 0.f, f = it ? lamF[t] : 0.f;
                    pgs_row_c(rowN[t], rowR[t], rowC[t], m.x, m.y, m.z, m.w, mu, n, f, vxA, vyA, wA, vxB, vyB, wB);
                    lamN[t] = n;
                    lamF[t] = f;
                }
                if (hasA) { lv[3 * la] = vxA; lv[3 * la + 1] = vyA; lv[3 * la + 2] = wA; }
                if (hasB) { lv[3 * lb] = vxB; lv[3 * lb + 1] = vyB; lv[3 * lb + 2] = wB; }
            }
        };
        stripe_sweeps(sb, v, iters, base, sb.sflag, sb.sflag + STRIPES_MAX / 2, lv, sb.gvt, fault, solve, 0,
                      single,
                      [&](int a0, int a1, int itv) { wave_steps(a0, a1, itv, solve); });
    }
    __syncthreads();
    // k_pgs_writeback for the stripes this workgroup finished last (only the
    // velocity fields: the position solver writes the poses concurrently)
    for (int s = 2 * j; s <= 2 * j + 2; s++) {
        if (!stripe_owned(s, j, v.S)) continue;
        for (int i = sb.sbStart[s] + (int)threadIdx.x; i < sb.sbStart[s + 1]; i += STPB) {
            const int b = sb.sbList[i];
            if (!inContact[b]) continue;
            lpe_body &bd = bodies[b];
            if (infinite_mass(bd)) continue;
            const float *o = lv + 3 * (i - v.s0);
            bd.vx = o[0];
            bd.vy = o[1];
            if (can_rotate(bd)) bd.omega = o[2];
        }
    }
}

// ---- opt-in Jacobi contact solver (lpe_rigid_config.pgsMode = LPE_PGS_JACOBI)
// north_star's "Jacobi-style" parallel solve, beside the reference's
// Gauss-Seidel (solveLcpPgs, contact_solver.cpp:381-440), which stays the
// default.  The unit is a contact pair (narrowphase pair, its contacts in
// narrowphase order): every pair of an iteration reads the bodies'
// velocities of the previous iteration and runs its contacts' normal and
// friction rows in order (the reference's sequence, :399-437) on its own copy
// of its two bodies, whose inverse mass and inertia are scaled by the body's
// pair count n (mass splitting: the copies' average is the body's new
// velocity, which makes the iteration a relaxed block Jacobi that converges
// for any contact graph).  The pair's impulses, applied with the unscaled
// masses (applyImpulse, :315-356), are summed per body in 2^-40 fixed point
// (int64 atomics: integer sums commute, so the result does not depend on the
// order of the pairs or the schedule, and is bit-reproducible); the
// iteration after reads v0 + sum.  Restated for the tests in
// tests/jacobi_restated.py.
//
// One launch, a persistent grid (every block resident) with one grid barrier
// an iteration.  Block j owns the pairs whose first contact lies in its
// contact range (contacts of a pair are contiguous, cstart) and keeps their
// rows -- built once, as k_prep_items builds them, with the effective masses
// of the scaled copies -- and impulses in LDS for the whole solve; each
// iteration touches global memory only for the body sums (two loads and one
// atomic per body and velocity component).  The sums ping-pong between two
// buffers, the one written by iteration k also taking the pair's iteration
// k - 1 share, so no buffer is cleared inside the launch.
static constexpr double JAC_SCALE = 0x1p40, JAC_INV = 0x1p-40;
static constexpr int JAC_TPB = 256, JAC_BLOCKS_MAX = 256;
static constexpr int JAC_CPB = 384;                  // contacts a block owns (at most, + one pair's)
static constexpr int JAC_LDS_ROWS = JAC_CPB + MAXC;
struct JacBufs {              // carved from one allocation (jac_bufs)
    uint32_t *bar;            // grid barrier arrivals (zeroed per launch)
    int32_t *cnt;             // [nb] pairs per body (zeroed per launch)
    long long *S0, *S1;       // [3 nb] the velocity sums, ping-pong (zeroed per launch)
    float *v0;                // [3 nb] the velocities the solve starts from
};
__device__ __forceinline__ void jac_grid_barrier(uint32_t *bar, uint32_t target, int32_t *fault) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");           // this wave's atomics are performed
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while ((int)(__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 22)) { atomicOr(fault, 4); break; }     // (never expected: every block is resident)
        }
    }
    __syncthreads();
}
__device__ __forceinline__ float jac_vel(const float *v0, const long long *S, int k) {
    const long long q = __hip_atomic_load(&S[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v0[k] + (float)((double)q * JAC_INV);
}
__device__ __forceinline__ long long jac_fix(float x) { return __double2ll_rn((double)x * JAC_SCALE); }
// the effective mass of a row on the scaled copies (computeEffectiveMass, :216-253)
__device__ __forceinline__ float jac_eff(float rxA, float ryA, float rxB, float ryB, float dx, float dy, float mA,
                                         float iA, float mB, float iB) {
    const float rAxn = cross2f(rxA, ryA, dx, dy), rBxn = cross2f(rxB, ryB, dx, dy);
    const float sum = mA + mB + (rAxn * rAxn) * iA + (rBxn * rBxn) * iB;
    return (sum < 1e-12F) ? 0.F : 1.F / sum;
}
__device__ __forceinline__ int jac_lower_bound(const int32_t *a, int n, int v) {   // first i with a[i] >= v
    int lo = 0, hi = n;
    while (lo < hi) { const int m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}
__global__ void __launch_bounds__(JAC_TPB)
k_pgs_jacobi(int nb, const int32_t *__restrict__ npptr, const int32_t *__restrict__ ncptr,
             const int32_t *__restrict__ ccount, const int32_t *__restrict__ cstart,
             const int32_t *__restrict__ rowOf, const float4 *__restrict__ rowN, const float4 *__restrict__ rowR,
             const int2 *__restrict__ rowAB, const float4 *__restrict__ rowM, int iters, float mu,
             float *__restrict__ lamN, float *__restrict__ lamF, lpe_body *__restrict__ bodies,
             const int32_t *__restrict__ inContact, JacBufs jb, int32_t *__restrict__ fault) {
    // the block's rows and pairs, resident in LDS for the whole solve.  The
    // rows are k_prep_items's (rowOf: contact -> row), built before the
    // position solver (running beside this kernel) moves the poses.
    __shared__ float4 lrn[JAC_LDS_ROWS];        // dir, effN, effF (scaled copies)
    __shared__ float4 lrr[JAC_LDS_ROWS];        // lever arms
    __shared__ float2 llam[JAC_LDS_ROWS];       // lamN, lamF
    __shared__ int4 lpr[JAC_LDS_ROWS];          // per pair: first row (block-local), rows, body a, body b (-1: static)
    __shared__ float4 lps[JAC_LDS_ROWS];        // per pair: scaled inverse masses / inertias smA, siA, smB, siB
    __shared__ float4 lpm[JAC_LDS_ROWS];        // per pair: imA, iiA, imB, iiB
    __shared__ long long ldp[6 * JAC_LDS_ROWS]; // per pair: its share of the previous iteration
    __shared__ int lrange[4], lnp;
    const int np = *npptr, nc = *ncptr;
    // the blocks in use: JAC_CPB contacts each (the grid is sized by the
    // capacity when the count is on the device only; the others leave at
    // once and take no part in the barriers, so they hold no CU)
    const int G = max(1, min((int)gridDim.x, (nc + JAC_CPB - 1) / JAC_CPB));
    if ((int)blockIdx.x >= G) return;
    const int stride = G * JAC_TPB, t0 = (int)(blockIdx.x * JAC_TPB + threadIdx.x);
    const int tid = (int)threadIdx.x;
    uint32_t arrivals = 0;
    for (int i = t0; i < nb; i += stride) {       // (k_pgs_bodies, what = 2: velocities, never moved by the position solver)
        const lpe_body &b = bodies[i];
        jb.v0[3 * i] = (float)b.vx; jb.v0[3 * i + 1] = (float)b.vy;
        jb.v0[3 * i + 2] = can_rotate(b) ? (float)b.omega : 0.f;
    }
    // the block's pairs: first contact in [j C, (j + 1) C)
    if (tid == 0) {
        const int C = (nc + G - 1) / G;
        const int p0 = jac_lower_bound(cstart, np, min(nc, (int)blockIdx.x * C));
        const int p1 = jac_lower_bound(cstart, np, min(nc, ((int)blockIdx.x + 1) * C));
        lrange[0] = p0; lrange[1] = p1;
        lrange[2] = cstart[p0]; lrange[3] = cstart[p1];
        lnp = 0;
        if (cstart[p1] - cstart[p0] > JAC_LDS_ROWS) atomicOr(fault, 8);   // (never: C <= JAC_CPB by the grid)
    }
    __syncthreads();
    const int p0 = lrange[0], p1 = lrange[1], k0 = lrange[2], k1 = min(lrange[3], k0 + JAC_LDS_ROWS);
    // the block's pairs with contacts (any order: the result does not depend on
    // it) and their movable bodies' pair counts
    for (int p = p0 + tid; p < p1; p += JAC_TPB) {
        const int n = ccount[p], c0 = cstart[p];
        if (n == 0 || c0 + n > k1) continue;
        const int2 ab = rowAB[rowOf[c0]];
        if (ab.x >= 0) atomicAdd(&jb.cnt[ab.x], 1);
        if (ab.y >= 0) atomicAdd(&jb.cnt[ab.y], 1);
        lpr[atomicAdd(&lnp, 1)] = make_int4(c0 - k0, n, ab.x, ab.y);
    }
    arrivals += G;
    jac_grid_barrier(jb.bar, arrivals, fault);
    const int npl = lnp;
    // the pairs' scaled copies, and the rows with their effective masses
    for (int m = tid; m < npl; m += JAC_TPB) {
        const int4 pr = lpr[m];
        const float4 im = rowM[rowOf[k0 + pr.x]];
        float fA = 1.f, fB = 1.f;
        if (pr.z >= 0) fA = (float)__hip_atomic_load(&jb.cnt[pr.z], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pr.w >= 0) fB = (float)__hip_atomic_load(&jb.cnt[pr.w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const float4 sc = make_float4(fA * im.x, fA * im.y, fB * im.z, fB * im.w);
        lpm[m] = im; lps[m] = sc;
        for (int j = 0; j < pr.y; j++) {
            const int l = pr.x + j, t = rowOf[k0 + l];
            const float4 rn = rowN[t], rr = rowR[t];
            lrn[l] = make_float4(rn.x, rn.y, jac_eff(rr.x, rr.y, rr.z, rr.w, rn.x, rn.y, sc.x, sc.y, sc.z, sc.w),
                                 jac_eff(rr.x, rr.y, rr.z, rr.w, -rn.y, rn.x, sc.x, sc.y, sc.z, sc.w));
            lrr[l] = rr;
            llam[l] = make_float2(0.f, 0.f);
        }
    }
    __syncthreads();
    for (int it = 0; it < iters; it++) {
        const long long *Sc = (it & 1) ? jb.S1 : jb.S0;
        long long *Sn = (it & 1) ? jb.S0 : jb.S1;
        for (int m = tid; m < npl; m += JAC_TPB) {
            const int4 pr = lpr[m];
            const int a = pr.z, b = pr.w;
            const bool hasA = a >= 0, hasB = b >= 0;
            float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
            if (hasA) { vxA = jac_vel(jb.v0, Sc, 3 * a); vyA = jac_vel(jb.v0, Sc, 3 * a + 1); wA = jac_vel(jb.v0, Sc, 3 * a + 2); }
            if (hasB) { vxB = jac_vel(jb.v0, Sc, 3 * b); vyB = jac_vel(jb.v0, Sc, 3 * b + 1); wB = jac_vel(jb.v0, Sc, 3 * b + 2); }
            const float4 im = lpm[m], sc = lps[m];
            float DxA = 0.f, DyA = 0.f, DwA = 0.f, DxB = 0.f, DyB = 0.f, DwB = 0.f;
            for (int j = 0; j < pr.y; j++) {
                const int l = pr.x + j;
                const float4 rn = lrn[l], rr = lrr[l];
                float2 lam = llam[l];
#pragma unroll
                for (int row = 0; row < 2; row++) {
                    const float dx = row == 0 ? rn.x : -rn.y, dy = row == 0 ? rn.y : rn.x;
                    const float eff = row == 0 ? rn.z : rn.w;
                    // getRelativeVelocity (:285-313) on the copies
                    const float ax = vxA + (-rr.y) * wA, ay = vyA + rr.x * wA;
                    const float bx = vxB + (-rr.w) * wB, by = vyB + rr.z * wB;
                    const float vrel = (bx - ax) * dx + (by - ay) * dy;
                    float old, lo, hi;
                    if (row == 0) { old = lam.x; lo = 0.0f; hi = 1e20f; }
                    else { old = lam.y; const float limit = mu * lam.x; lo = -limit; hi = limit; }
                    float dl = -eff * (vrel + 0.0f);
                    float nl = old + dl;
                    if (nl < lo) nl = lo;
                    if (nl > hi) nl = hi;
                    dl = nl - old;
                    if (row == 0) lam.x = nl; else lam.y = nl;
                    if (fabsf(dl) < 1e-15F) continue;
                    const float crossA = rr.x * dy - rr.y * dx, crossB = rr.z * dy - rr.w * dx;
                    if (hasA) {
                        vxA -= dx * (dl * sc.x); vyA -= dy * (dl * sc.x); wA -= crossA * dl * sc.y;
                        DxA -= dx * (dl * im.x); DyA -= dy * (dl * im.x); DwA -= crossA * dl * im.y;
                    }
                    if (hasB) {
                        vxB += dx * (dl * sc.z); vyB += dy * (dl * sc.z); wB += crossB * dl * sc.w;
                        DxB += dx * (dl * im.z); DyB += dy * (dl * im.z); DwB += crossB * dl * im.w;
                    }
                }
                llam[l] = lam;
            }
            const long long q[6] = {jac_fix(DxA), jac_fix(DyA), jac_fix(DwA), jac_fix(DxB), jac_fix(DyB), jac_fix(DwB)};
#pragma unroll
            for (int u = 0; u < 6; u++) {
                const long long prev = it ? ldp[6 * m + u] : 0ll;
                const int body = u < 3 ? a : b;
                if (body >= 0) atomicAdd((unsigned long long *)&Sn[3 * body + (u % 3)],
                                         (unsigned long long)(q[u] + prev));
                ldp[6 * m + u] = q[u];
            }
        }
        arrivals += G;
        jac_grid_barrier(jb.bar, arrivals, fault);
    }
    // the impulses by contact index (lpe_rigid_download_impulses)
    for (int k = k0 + tid; k < k1; k += JAC_TPB) { lamN[k] = llam[k - k0].x; lamF[k] = llam[k - k0].y; }
    // k_pgs_writeback (velocity fields only: the position solver writes the poses concurrently)
    const long long *Sf = (iters & 1) ? jb.S1 : jb.S0;
    for (int i = t0; i < nb; i += stride) {
        if (!inContact[i]) continue;
        lpe_body &bd = bodies[i];
        if (infinite_mass(bd)) continue;
        bd.vx = jac_vel(jb.v0, Sf, 3 * i);
        bd.vy = jac_vel(jb.v0, Sf, 3 * i + 1);
        if (can_rotate(bd)) bd.omega = jac_vel(jb.v0, Sf, 3 * i + 2);
    }
}

// Position solver (solvePositionContactsOnce, position_solver.cpp:215-290)
// over the striped order.  The poses (fp64) of the workgroup's stripes and of
// the static bodies its pairs touch, its rows (44 bytes) and pairs (48) live
// in LDS; a workgroup whose rows do not fit reads them from global memory.
__global__ void __launch_bounds__(STPB)
k_pos_stripes(const int32_t *__restrict__ counts, StripeBufs sb, const int2 *__restrict__ seg, PosRows rows,
              lpe_body *__restrict__ bodies, const double *__restrict__ st, const int32_t *__restrict__ inPos,
              int iters, uint32_t base, int32_t *__restrict__ fault) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int j = (int)blockIdx.x;
    if (j >= counts[13]) return;
    __builtin_amdgcn_s_setprio(3);
    STR(1, j, 0);
    const StripeView v = stripe_view(sb, counts, j);
    const int NR = v.nrows(), NP = v.npairs(), NS = v.nsteps();
    const int NL = v.nloc() + (v.nAll - v.nDyn);      // the stripes' bodies, then the static ones
    // layout: n, c [NR] double2 | pm, pi [NP] double2 | pr [NP] int4 | py [NR] | lp [3 NL] | fl [NR] | stepL
    const int oC = 16 * NR, oPM = oC + 16 * NR, oPI = oPM + 16 * NP, oPR = oPI + 16 * NP, oPY = oPR + 16 * NP,
              oLP = oPY + 8 * NR, oFL = oLP + 24 * NL, oST = oFL + 4 * NR, total = oST + 4 * (NS + 1);
    const bool inL = total <= STRIPE_LDS;
    double *lp = inL ? (double *)(smem + oLP) : (double *)smem;
    for (int i = threadIdx.x; i < NL; i += STPB) {
        const int slot = i < v.nloc() ? v.s0 + i : v.nDyn + (i - v.nloc());
        const lpe_body &b = bodies[sb.sbList[slot]];
        lp[3 * i] = b.x; lp[3 * i + 1] = b.y;
        lp[3 * i + 2] = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
    }
    const int *bpos = sb.bpos;
    auto lbody = [&](int b) {
        const int p = bpos[b];
        return p >= v.nDyn ? v.nloc() + (p - v.nDyn) : p - v.s0;
    };
    // one pair's rows against the poses in lp (a static body, invM = 0 and no
    // rotation, is never written: pairs of one step may share it)
    auto pair_rows = [&](int a, int b, double2 mm, double2 ii, int nrow, auto row) {
        double xA = lp[3 * a], yA = lp[3 * a + 1], tA = lp[3 * a + 2];
        double xB = lp[3 * b], yB = lp[3 * b + 1], tB = lp[3 * b + 2];
        const int fl0 = row(0, mm, ii, xA, yA, tA, xB, yB, tB);
        for (int k = 1; k < nrow; k++) row(k, mm, ii, xA, yA, tA, xB, yB, tB);
        if (mm.x != 0.0 || (fl0 & 2)) { lp[3 * a] = xA; lp[3 * a + 1] = yA; lp[3 * a + 2] = tA; }
        if (mm.y != 0.0 || (fl0 & 4)) { lp[3 * b] = xB; lp[3 * b + 1] = yB; lp[3 * b + 2] = tB; }
    };
    if (inL) {
        double2 *ln = (double2 *)smem, *lc = (double2 *)(smem + oC), *pm = (double2 *)(smem + oPM),
                *pi = (double2 *)(smem + oPI);
        int4 *pr = (int4 *)(smem + oPR);
        double *py = (double *)(smem + oPY);
        int *fl = (int *)(smem + oFL), *stepL = (int *)(smem + oST);
        for (int r = threadIdx.x; r < NR; r += STPB) {
            const int g = r < v.nRA ? v.rA0 + r : v.rB0 + (r - v.nRA);
            ln[r] = rows.n[g]; lc[r] = rows.c[g]; py[r] = rows.py[g]; fl[r] = rows.fl[g];
        }
        for (int q = threadIdx.x; q < NP; q += STPB) {
            const int gq = q < v.nA ? v.pA0 + q : v.pB0 + (q - v.nA);
            const int2 sg = seg[gq];
            const int2 ab = rows.ab[sg.x];
            pr[q] = make_int4(v.lrow(sg.x), sg.y & 0xff, lbody(ab.x), lbody(ab.y));
            pm[q] = rows.m[sg.x];
            pi[q] = rows.i[sg.x];
        }
        stripe_steps_lds(sb, v, stepL);
        __syncthreads();
        const bool single = stripe_single_wave(sb, v, stepL);
        auto solve = [&](int stp, int) {
            const int k = v.lstep(stp);
            const int q1 = stepL[k + 1];
            for (int q = stepL[k] + (int)threadIdx.x; q < q1; q += STPB) {
                const int4 p = pr[q];
                const int r0 = p.x;
                pair_rows(p.z, p.w, pm[q], pi[q], p.y,
                          [&](int k2, double2 mm, double2 ii, double &xA, double &yA, double &tA, double &xB,
                              double &yB, double &tB) {
                              const int t = r0 + k2;
                              const double2 n = ln[t], c = lc[t];
                              const int f = fl[t];
                              pos_item_z(n.x, n.y, c.x, c.y, py[t], f, mm.x, mm.y, ii.x, ii.y, xA, yA, tA, xB,
                                            yB, tB);
                              return f;
                          });
            }
        };
        // the single-wave schedule, software-pipelined as the PGS's: the next
        // step's pair record and first U rows are loaded before this step's
        // rows run; only the poses are read after the previous step's stores
        auto phase = [&](int s0, int s1, int) {
            if (threadIdx.x >= 64 || s0 >= s1) return;
            constexpr int U = 4;
            struct Nx { int4 p; double2 mm, ii; double2 n[U], c[U]; double y[U]; int f[U]; };
            auto fetch = [&](int stp, Nx &x) {
                const int k = v.lstep(stp);
                const int q = stepL[k] + (int)threadIdx.x;
                const bool ok = q < stepL[k + 1];
                x.p = ok ? pr[q] : make_int4(0, 0, 0, 0);
                x.mm = pm[ok ? q : 0];
                x.ii = pi[ok ? q : 0];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int t = x.p.x + max(min(u, x.p.y - 1), 0);
                    x.n[u] = ln[t]; x.c[u] = lc[t]; x.y[u] = py[t]; x.f[u] = fl[t];
                }
            };
            Nx cur, nxt;
            fetch(s0, cur);
            for (int stp = s0; stp < s1; stp++) {
                if (stp + 1 < s1) fetch(stp + 1, nxt);
                const int4 p = cur.p;
                if (p.y > 0) {
                    const int a = p.z, b = p.w;
                    const double2 mm = cur.mm, ii = cur.ii;
                    double xA = lp[3 * a], yA = lp[3 * a + 1], tA = lp[3 * a + 2];
                    double xB = lp[3 * b], yB = lp[3 * b + 1], tB = lp[3 * b + 2];
#pragma unroll
                    for (int u = 0; u < U; u++) {
                        if (u >= p.y) break;
                        pos_item_z(cur.n[u].x, cur.n[u].y, cur.c[u].x, cur.c[u].y, cur.y[u], cur.f[u], mm.x, mm.y,
                                     ii.x, ii.y, xA, yA, tA, xB, yB, tB);
                    }
                    for (int k2 = U; k2 < p.y; k2++) {       // (pairs of more than U rows: the rest on demand)
                        const int t = p.x + k2;
                        const double2 n = ln[t], c = lc[t];
                        pos_item_z(n.x, n.y, c.x, c.y, py[t], fl[t], mm.x, mm.y, ii.x, ii.y, xA, yA, tA, xB, yB, tB);
                    }
                    const int fl0 = cur.f[0];
                    if (mm.x != 0.0 || (fl0 & 2)) { lp[3 * a] = xA; lp[3 * a + 1] = yA; lp[3 * a + 2] = tA; }
                    if (mm.y != 0.0 || (fl0 & 4)) { lp[3 * b] = xB; lp[3 * b + 1] = yB; lp[3 * b + 2] = tB; }
                }
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // (program order of the LDS accesses)
                cur = nxt;
            }
        };
        stripe_sweeps(sb, v, iters, base, sb.sflag + STRIPES_MAX, sb.sflag + STRIPES_MAX + STRIPES_MAX / 2, lp,
                      sb.gpos, fault, solve, 1, single, phase);
    } else {
        __syncthreads();
        const bool single = stripe_single_wave(sb, v, nullptr);
        auto solve = [&](int stp, int) {
            const int q1 = sb.stepPair[stp + 1];
            for (int q = sb.stepPair[stp] + (int)threadIdx.x; q < q1; q += STPB) {
                const int2 sg = seg[q];
                const int rs = sg.x;
                const int2 ab = rows.ab[rs];
                pair_rows(lbody(ab.x), lbody(ab.y), rows.m[rs], rows.i[rs], sg.y & 0xff,
                          [&](int k2, double2 mm, double2 ii, double &xA, double &yA, double &tA, double &xB,
                              double &yB, double &tB) {
                              const int t = rs + k2;
                              const double2 n = rows.n[t], c = rows.c[t];
                              const int f = rows.fl[t];
                              pos_item_z(n.x, n.y, c.x, c.y, rows.py[t], f, mm.x, mm.y, ii.x, ii.y, xA, yA, tA,
                                            xB, yB, tB);
                              return f;
                          });
            }
        };
        stripe_sweeps(sb, v, iters, base, sb.sflag + STRIPES_MAX, sb.sflag + STRIPES_MAX + STRIPES_MAX / 2, lp,
                      sb.gpos, fault, solve, 1, single,
                      [&](int a0, int a1, int itv) { wave_steps(a0, a1, itv, solve); });
    }
    __syncthreads();
    // storeBodyData (:176-197) for the stripes this workgroup finished last
    for (int s = 2 * j; s <= 2 * j + 2; s++) {
        if (!stripe_owned(s, j, v.S)) continue;
        for (int i = sb.sbStart[s] + (int)threadIdx.x; i < sb.sbStart[s + 1]; i += STPB) {
            const int b = sb.sbList[i];
            if (!inPos[b]) continue;
            const int f = (int)st[3 * b + 2];
            if (!(f & 2)) continue;
            lpe_body &bd = bodies[b];
            const double *o = lp + 3 * (i - v.s0);
            bd.x = o[0]; bd.y = o[1];
            if ((f & 1) && (bd.flags & LPE_BODY_HAS_ANGPOS)) bd.angle = o[2];
        }
    }
}

__global__ void k_boundary(int nb, lpe_body *__restrict__ bodies, double m, double U, double damp,
                           double maxSpeed) {   // boundary.cpp:13-70
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    lpe_body b = bodies[i];
    if (!(b.flags & LPE_BODY_HAS_VEL)) return;
    if ((b.flags & LPE_BODY_HAS_SLEEP) && (b.flags & LPE_BODY_ASLEEP)) return;
    bool bounced = false;
    if (b.x < m) { b.x = m; b.vx = fabs(b.vx) * damp; bounced = true; }
    else if (b.x > U - m) { b.x = U - m; b.vx = -fabs(b.vx) * damp; bounced = true; }
    if (b.y < m) { b.y = m; b.vy = fabs(b.vy) * damp; bounced = true; }
    else if (b.y > U - m) { b.y = U - m; b.vy = -fabs(b.vy) * damp; bounced = true; }
    if (bounced) {
        double sp = sqrt(b.vx * b.vx + b.vy * b.vy);
        if (sp > maxSpeed) { b.vx = (b.vx / sp) * maxSpeed; b.vy = (b.vy / sp) * maxSpeed; }
    }
    bodies[i] = b;
}
// The world tick splits the boundary system in two so that collision
// detection can start at the beginning of the tick: the position clamp
// depends on positions only, which nothing before the boundary system changes
// (the fluid step and gravity only write velocities; the fluid reads its own
// gathered copy of the bodies, taken before the clamp), and the velocity part
// is applied at the boundary system's place in the tick from the recorded
// bounce bits.  Together they equal k_boundary.
// A cross-stream signal without a marker packet: the launch's last
// workgroup (arrival count) releases its writes and every earlier launch's
// (stream order) and stores `value` into *flag; k_wait_flag polls it.
__device__ __forceinline__ void grid_done_signal(uint32_t *ctr, uint32_t *flag, uint32_t value) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(ctr, 1u) == gridDim.x - 1) {
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence();
            __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// One wave on the waiting stream: returns once *flag has reached `want`
// (wrapping compare); a watchdog (limit polls: ~3 s in the tick) raises
// `bit` in *fault and returns, so the stream never hangs on a signal that was
// not launched.
__global__ void k_wait_flag(const uint32_t *__restrict__ flag, uint32_t want, int32_t *__restrict__ fault,
                            uint32_t limit, int32_t bit) {
    if (threadIdx.x != 0) return;
    for (uint32_t n = 0;; n++) {
        const uint32_t v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if ((int32_t)(v - want) >= 0) return;
        if (n == limit) {
            atomicOr(fault, bit);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}
__global__ void k_set_flag(uint32_t *__restrict__ flag, uint32_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_boundary_pos(int nb, lpe_body *__restrict__ bodies, double m, double U,
                               int32_t *__restrict__ bits, uint32_t *__restrict__ sig, uint32_t value) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i < nb) {
        lpe_body &b = bodies[i];
        int f = 0;
        const int flags = b.flags;
        if ((flags & LPE_BODY_HAS_VEL) && !((flags & LPE_BODY_HAS_SLEEP) && (flags & LPE_BODY_ASLEEP))) {
            const double x = b.x, y = b.y;
            if (x < m) { b.x = m; f |= 1; }
            else if (x > U - m) { b.x = U - m; f |= 2; }
            if (y < m) { b.y = m; f |= 4; }
            else if (y > U - m) { b.y = U - m; f |= 8; }
        }
        bits[i] = f;
    }
    if (sig) grid_done_signal(sig + 3, sig + 2, value);
}
__device__ __forceinline__ void boundary_vel_one(lpe_body &b, int f, double damp, double maxSpeed) {
    double vx = b.vx, vy = b.vy;
    if (f & 1) vx = fabs(vx) * damp;
    else if (f & 2) vx = -fabs(vx) * damp;
    if (f & 4) vy = fabs(vy) * damp;
    else if (f & 8) vy = -fabs(vy) * damp;
    double sp = sqrt(vx * vx + vy * vy);
    if (sp > maxSpeed) { vx = (vx / sp) * maxSpeed; vy = (vy / sp) * maxSpeed; }
    b.vx = vx; b.vy = vy;
}
__global__ void k_boundary_vel(int nb, lpe_body *__restrict__ bodies, const int32_t *__restrict__ bits,
                               double damp, double maxSpeed) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    const int f = bits[i];
    if (!f) return;
    boundary_vel_one(bodies[i], f, damp, maxSpeed);
}
__device__ __forceinline__ bool gravity_view(const lpe_body &b) {
    return (b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_HAS_VEL) &&
           (b.flags & LPE_BODY_HAS_MASS) && !(b.flags & LPE_BODY_BOUNDARY);
}
__global__ void k_gravity_check(int nb, const lpe_body *__restrict__ bodies, double thr,
                                int32_t *__restrict__ heavy) {   // gravity.cpp:43-51
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    if (thr > 0.0 && gravity_view(bodies[i]) && bodies[i].mass >= thr) atomicOr(heavy, 1);
}
__global__ void k_gravity(int nb, lpe_body *__restrict__ bodies, double g, double dt,
                          const int32_t *__restrict__ heavy) {   // gravity.cpp:53-57
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb || *heavy) return;
    if (gravity_view(bodies[i])) bodies[i].vy += g * dt;
}
// BoundarySystem's velocity half then BasicGravitySystem, per body (the world
// tick: nothing between them touches the bodies)
__global__ void k_boundary_vel_gravity(int nb, lpe_body *__restrict__ bodies, const int32_t *__restrict__ bits,
                                       double damp, double maxSpeed, double g, double dt,
                                       const int32_t *__restrict__ heavy, uint32_t *__restrict__ sig,
                                       uint32_t value) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i < nb) {
        const int f = bits[i];
        lpe_body &b = bodies[i];
        if (f) boundary_vel_one(b, f, damp, maxSpeed);
        if (!*heavy && gravity_view(b)) b.vy += g * dt;
    }
    if (sig) grid_done_signal(sig + 1, sig, value);
}
// RotationSystem, MovementSystem, SleepSystem on one body (each returns
// whether it wrote the body; the kernels below store it back only then)
__device__ __forceinline__ bool rotation_one(lpe_body &b, double dt, double damping, double maxw) {   // rotation.cpp:18-60
    if (!(b.flags & LPE_BODY_HAS_ANGPOS) || !(b.flags & LPE_BODY_HAS_ANGVEL)) return false;
    if (b.flags & LPE_BODY_BOUNDARY) return false;
    const double Pi = 3.141592654;
    b.angle += b.omega * dt;
    if (damping < 1.0) b.omega *= damping;
    if (maxw > 0) {
        if (b.omega > maxw) b.omega = maxw;
        if (b.omega < -maxw) b.omega = -maxw;
    }
    if (b.angle > 2.0 * Pi) b.angle -= 2.0 * Pi;
    else if (b.angle < 0) b.angle += 2.0 * Pi;
    return true;
}
__device__ __forceinline__ bool movement_one(lpe_body &b, double dt) {   // movement.cpp:13-39
    if (!(b.flags & LPE_BODY_HAS_VEL) || (b.flags & LPE_BODY_BOUNDARY)) return false;
    if ((b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_LIQUID)) return false;
    b.x += b.vx * dt;
    b.y += b.vy * dt;
    return true;
}
__device__ __forceinline__ bool sleep_one(lpe_body &b, double lin, double ang, int frames) {   // sleep.cpp:19-67
    const uint32_t need = LPE_BODY_HAS_VEL | LPE_BODY_HAS_PHASE | LPE_BODY_HAS_MASS | LPE_BODY_HAS_SLEEP;
    if ((b.flags & need) != need || (b.flags & LPE_BODY_BOUNDARY)) return false;
    double speed = sqrt(b.vx * b.vx + b.vy * b.vy);
    double as = (b.flags & LPE_BODY_HAS_ANGVEL) ? fabs(b.omega) : 0.0;
    bool asleep = (b.flags & LPE_BODY_ASLEEP) != 0;
    if (speed < lin && as < ang) {
        if (!asleep) {
            b.sleep_counter++;
            if (b.sleep_counter > frames) asleep = true;
        }
    } else {
        b.sleep_counter = 0;
        asleep = false;
    }
    if (asleep) {
        b.flags |= LPE_BODY_ASLEEP;
        b.vx = 0; b.vy = 0;
        if (b.flags & LPE_BODY_HAS_ANGVEL) b.omega = 0;
    } else {
        b.flags &= ~LPE_BODY_ASLEEP;
    }
    return true;
}
__global__ void k_rotation(int nb, lpe_body *__restrict__ bodies, double dt, double damping, double maxw) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    lpe_body b = bodies[i];
    if (rotation_one(b, dt, damping, maxw)) bodies[i] = b;
}
__global__ void k_movement(int nb, lpe_body *__restrict__ bodies, double dt) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    lpe_body b = bodies[i];
    if (movement_one(b, dt)) bodies[i] = b;
}
__global__ void k_sleep(int nb, lpe_body *__restrict__ bodies, double lin, double ang, int frames) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    lpe_body b = bodies[i];
    if (sleep_one(b, lin, ang, frames)) bodies[i] = b;
}
// the three in one launch (sim.cpp:112-114 order, per body)
__global__ void k_rotation_movement_sleep(int nb, lpe_body *__restrict__ bodies, double dt_state, double damping,
                                          double maxw, double dt_move, double lin, double ang, int frames) {
    int i = blockIdx.x * RTPB + threadIdx.x;
    if (i >= nb) return;
    lpe_body b = bodies[i];
    bool w = rotation_one(b, dt_state, damping, maxw);
    w |= movement_one(b, dt_move);
    w |= sleep_one(b, lin, ang, frames);
    if (w) bodies[i] = b;
}

}  // namespace lpe

using namespace lpe;

// ===========================================================================
// host side
static inline int rblk(long n, int t = RTPB) { return (int)((n + t - 1) / t); }

template <typename T>
static int rgrow(lpe_ctx *ctx, T **p, size_t n) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    hipError_t e = hipMalloc((void **)p, sizeof(T) * std::max<size_t>(n, 1));
    if (e != hipSuccess) { ctx->err = std::string("hipMalloc: ") + hipGetErrorString(e); return LPE_ERR_HIP; }
    return LPE_OK;
}

static int rigid_lag_drain(lpe_ctx *ctx, RigidDev *d);
static void rigid_lag_off(lpe_ctx *ctx, RigidDev *d);

int lpe_rigid_destroy_internal(lpe_ctx *ctx) {
    RigidDev *d = (RigidDev *)ctx->rigid;
    if (!d) return LPE_OK;
    rigid_lag_off(ctx, d);
    if (d->side) (void)hipStreamSynchronize(d->side);      // nothing may still use the buffers
    if (d->psolve) (void)hipStreamSynchronize(d->psolve);
    void *ptrs[] = {d->bodies, d->verts, d->rank, d->byRank, d->aabb, d->cand, d->pcount, d->pstart,
                    d->pcursor, d->pairs, d->pairRankB, d->cslots, d->ccount, d->cstart, d->contacts,
                    d->bsum, d->order, d->rowN, d->rowR, d->rowAB, d->vel0, d->imii, d->inContact,
                    d->posState, d->posRec, d->posKeep, d->posStart, d->rowM, d->sItemA, d->sItemB,
                    d->sVer, d->lamN, d->lamF, d->rowOf, d->rowC, d->sBCount, d->sBStart, d->sBCursor, d->sEnt,
                    d->counts, d->pcol, d->cseg, d->cbase, d->bgCount, d->bgStart, d->bgCursor,
                    d->bgList, d->bgKey, d->bgSpecial, d->bbits, d->jac};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    if (StripeBufs *sb = (StripeBufs *)d->stripes) {
        void *sp[] = {sb->bstripe, sb->pgroup, sb->pcolg, sb->prank, sb->prowoff, sb->glist, sb->gstart, sb->gcnt,
                      sb->stepIdx, sb->stepPair, sb->stepRow, sb->wgStep, sb->sbStart, sb->sbList, sb->sflag,
                      sb->gvt, sb->gpos, sb->bpos, sb->pflag, sb->px, sb->bred};
        for (void *p : sp) if (p) (void)hipFree(p);
        delete sb;
    }
    if (d->hc) (void)hipHostFree(d->hc);
    if (d->hcr) (void)hipHostFree(d->hcr);
    if (d->tsync) (void)hipFree(d->tsync);
    hipEvent_t evs[] = {d->evStart, d->evDetect, d->evColour, d->evFork, d->evJoin, d->evHc[0], d->evHc[1], d->evBvg};
    for (hipEvent_t e : evs) if (e) (void)hipEventDestroy(e);
    if (d->side) (void)hipStreamDestroy(d->side);
    if (d->psolve) (void)hipStreamDestroy(d->psolve);
    delete d;
    ctx->rigid = nullptr;
    return LPE_OK;
}

extern "C" int lpe_rigid_config_default(lpe_rigid_config *c) {
    if (!c) return LPE_ERR_ARG;
    std::memset(c, 0, sizeof(*c));
    c->universeSize = 6.0; c->metersPerPixel = 0.01; c->quadtreeCapacity = 8;
    c->boundaryBuffer = 500.0; c->smallParticleThreshold = 0.01; c->pgsIterations = 10;
    c->frictionCoeff = 0.5f; c->posIterations = 10; c->baumgarte = 0.02; c->slop = 0.001;
    c->gravity = 9.8; c->planetaryMassThreshold = 1e10; c->angularDamping = 0.98;
    c->maxAngularSpeed = 20.0; c->marginPixels = 15.0; c->bounceDamping = 0.7; c->maxSpeed = 1.0;
    c->linearSleepThreshold = 0.5; c->angularSleepThreshold = 0.5; c->sleepFramesThreshold = 60;
    return LPE_OK;
}

extern "C" int lpe_rigid_set_config(lpe_ctx *ctx, const lpe_rigid_config *cfg) {
    if (!ctx || !cfg) return LPE_ERR_ARG;
    if (cfg->pgsMode != LPE_PGS_GAUSS_SEIDEL && cfg->pgsMode != LPE_PGS_JACOBI) {
        ctx->err = "rigid config: pgsMode must be LPE_PGS_GAUSS_SEIDEL or LPE_PGS_JACOBI";
        return LPE_ERR_ARG;
    }
    RigidDev *d = rdev(ctx);
    // the cached mass checks stay valid across an unchanged config (the
    // resident host path re-sets it every tick)
    if (!d->cfg_set || std::memcmp(&d->cfg, cfg, sizeof(*cfg)) != 0) {
        d->heavy_valid = false;
        d->gen++;
        rigid_lag_off(ctx, d);
    }
    d->cfg = *cfg;
    d->cfg_set = true;
    return LPE_OK;
}

static int rigid_alloc_bodies(lpe_ctx *ctx, RigidDev *d, int nb) {
    if (nb <= d->cap_nb && d->bodies) return LPE_OK;
    int st = 0;
    size_t N = (size_t)nb;
    if ((st = rgrow(ctx, &d->bodies, N))) return st;
    if ((st = rgrow(ctx, &d->rank, N))) return st;
    if ((st = rgrow(ctx, &d->byRank, N))) return st;
    if ((st = rgrow(ctx, &d->aabb, N))) return st;
    if ((st = rgrow(ctx, &d->cand, N))) return st;
    if ((st = rgrow(ctx, &d->pcount, N))) return st;
    if ((st = rgrow(ctx, &d->pstart, N + 1))) return st;
    if ((st = rgrow(ctx, &d->pcursor, N))) return st;
    if ((st = rgrow(ctx, &d->vel0, 3 * N))) return st;
    if ((st = rgrow(ctx, &d->imii, 2 * N))) return st;
    if ((st = rgrow(ctx, &d->inContact, 2 * N))) return st;
    if ((st = rgrow(ctx, &d->posState, 3 * N))) return st;
    if ((st = rgrow(ctx, &d->sBCount, N))) return st;
    if ((st = rgrow(ctx, &d->sBStart, N + 1))) return st;
    if ((st = rgrow(ctx, &d->sBCursor, N))) return st;
    if ((st = rgrow(ctx, &d->bbits, N))) return st;
    if (!d->counts) {
        if ((st = rgrow(ctx, &d->counts, 16))) return st;
        LPE_HIP(ctx, hipMemsetAsync(d->counts, 0, sizeof(int32_t) * 16, ctx->stream));
    }
    d->cap_nb = nb;
    return LPE_OK;
}

static int rigid_alloc_pairs(lpe_ctx *ctx, RigidDev *d, int cap_pairs) {
    if (cap_pairs <= d->cap_pairs && d->pairs) return LPE_OK;
    int st = 0;
    size_t P = (size_t)cap_pairs;
    if ((st = rgrow(ctx, &d->pairs, P))) return st;
    if ((st = rgrow(ctx, &d->pairRankB, P))) return st;
    if ((st = rgrow(ctx, &d->cslots, P * MAXC))) return st;
    if ((st = rgrow(ctx, &d->ccount, P))) return st;
    if ((st = rgrow(ctx, &d->cstart, P + 1))) return st;
    d->cap_pairs = cap_pairs;
    return LPE_OK;
}

static int rigid_alloc_contacts(lpe_ctx *ctx, RigidDev *d, int cap) {
    if (cap <= d->cap_contacts && d->contacts) return LPE_OK;
    int st = 0;
    size_t K = (size_t)cap;
    if ((st = rgrow(ctx, &d->contacts, K))) return st;
    if ((st = rgrow(ctx, &d->order, K))) return st;
    if ((st = rgrow(ctx, &d->rowN, K))) return st;
    if ((st = rgrow(ctx, &d->rowR, K))) return st;
    if ((st = rgrow(ctx, &d->rowAB, K))) return st;
    if ((st = rgrow(ctx, &d->rowM, K))) return st;
    if ((st = rgrow(ctx, &d->rowC, K))) return st;
    if ((st = rgrow(ctx, &d->posRec, K))) return st;
    if ((st = rgrow(ctx, &d->sVer, K))) return st;
    if ((st = rgrow(ctx, &d->lamN, K))) return st;
    if ((st = rgrow(ctx, &d->rowOf, K))) return st;
    if ((st = rgrow(ctx, &d->lamF, K))) return st;
    int32_t **arrs[] = {&d->sItemA, &d->sItemB, &d->posKeep};
    for (int32_t **a : arrs) if ((st = rgrow(ctx, a, K))) return st;
    if ((st = rgrow(ctx, &d->posStart, K + 1))) return st;
    if ((st = rgrow(ctx, &d->sEnt, 2 * K))) return st;
    d->cap_contacts = cap;
    return LPE_OK;
}

static int rigid_alloc_bsum(lpe_ctx *ctx, RigidDev *d, long n) {
    int need = (int)(n / 1024 + 4);
    if (need <= d->cap_bsum && d->bsum) return LPE_OK;
    int st = rgrow(ctx, &d->bsum, (size_t)need);
    if (st) return st;
    d->cap_bsum = need;
    return LPE_OK;
}

// exclusive scan of n (device count nptr or host ncap) ints; start[n] = total
static int rscan(lpe_ctx *ctx, RigidDev *d, const int32_t *nptr, int ncap, const int32_t *cnt,
                 int32_t *start, int32_t *cursor, hipStream_t s = nullptr, int32_t *total_out = nullptr) {
    if (!s) s = ctx->stream;
    if (ncap <= RSCAN_SINGLE_MAX) {
        LPE_KERNEL(ctx, "k_rscan_single", k_rscan_single, dim3(1), dim3(RTPB), 0, s, nptr, ncap, cnt, start, cursor,
                   total_out);
        LPE_CHECK_LAUNCH(ctx, "rscan");
        return LPE_OK;
    }
    int st = rigid_alloc_bsum(ctx, d, ncap);
    if (st) return st;
    int nb = ncap / 1024 + 1;
    // <= 1,024 tiles: the tile prefix inside k_rscan_final (LPE_NO_RSCAN_FUSION=1: off)
    static const bool nofuse = getenv("LPE_NO_RSCAN_FUSION") != nullptr;
    const int fused = (nb <= 1024 && !nofuse) ? 1 : 0;
    LPE_KERNEL(ctx, "k_rscan_reduce", k_rscan_reduce, dim3(nb), dim3(RTPB), 0, s, nptr, ncap, cnt, d->bsum);
    if (!fused)
        LPE_KERNEL(ctx, "k_rscan_blocks", k_rscan_blocks, dim3(1), dim3(RTPB), 0, s, nptr, ncap, d->bsum, start);
    LPE_KERNEL(ctx, "k_rscan_final", k_rscan_final, dim3(nb), dim3(RTPB), 0, s, nptr, ncap, cnt, d->bsum, start, cursor,
               fused);
    if (total_out) {               // (a host-sized scan: the total is start[ncap])
        if (nptr) { ctx->err = "rscan: total_out needs a host-sized count"; return LPE_ERR_ARG; }
        LPE_HIP(ctx, hipMemcpyAsync(total_out, start + ncap, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    }
    LPE_CHECK_LAUNCH(ctx, "rscan");
    return LPE_OK;
}

extern "C" int lpe_rigid_upload(lpe_ctx *ctx, int nb, const lpe_body *bodies, int nverts,
                                const double *verts) {
    if (ctx) { rdev(ctx)->heavy_valid = false; rdev(ctx)->gen++; }
    if (!ctx || nb < 0 || nverts < 0 || (nb > 0 && !bodies) || (nverts > 0 && !verts))
        return LPE_ERR_ARG;
    // the portable sin / cos (lpe_trig.h) reduce exactly for |angle| below
    // LPE_TRIG_MAX_ARG (2^20 pi/2); the rotation system wraps every angle each
    // tick, so only an uploaded one can be larger: refuse it
    for (int i = 0; i < nb; i++)
        if (!(std::fabs(bodies[i].angle) < LPE_TRIG_MAX_ARG)) {
            ctx->err = "lpe_rigid_upload: a body angle is not finite or exceeds 2^20 * pi/2 rad (wrap it first)";
            return LPE_ERR_ARG;
        }
    (void)hipSetDevice(ctx->device);
    RigidDev *d = rdev(ctx);
    rigid_lag_off(ctx, d);
    if (!d->cfg_set) { lpe_rigid_config_default(&d->cfg); d->cfg_set = true; }
    static bool lds_attr = false;
    if (!lds_attr) {
        (void)hipFuncSetAttribute((const void *)k_pgs_flow, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k_pos_flow, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k_pgs_colour, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void *)k_pos_colour, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        // k_pair_colour also holds ~1 KB of static LDS
        (void)hipFuncSetAttribute((const void *)k_pair_colour, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
        (void)hipFuncSetAttribute((const void *)k_pgs_stripes, hipFuncAttributeMaxDynamicSharedMemorySize, STRIPE_LDS);
        (void)hipFuncSetAttribute((const void *)k_pos_stripes, hipFuncAttributeMaxDynamicSharedMemorySize, STRIPE_LDS);
        (void)hipGetLastError();   // a refused attribute must not surface at a later launch check
        lds_attr = true;
    }
    int st = rigid_alloc_bodies(ctx, d, std::max(nb, 1));
    if (st) return st;
    if (nverts > d->cap_verts || !d->verts) {
        if ((st = rgrow(ctx, &d->verts, 2 * (size_t)std::max(nverts, 1)))) return st;
        d->cap_verts = nverts;
    }
    d->nb = nb;
    d->nverts = nverts;
    hipStream_t s = ctx->stream;
    if (nb > 0) {
        for (int i = 0; i < nb; i++) {
            const lpe_body &b = bodies[i];
            if (!(b.flags & LPE_BODY_CIRCLE) && (b.vert_off < 0 || b.vert_cnt < 0 ||
                                                  b.vert_off + b.vert_cnt > nverts ||
                                                  b.vert_cnt > MAXV)) {
                ctx->err = "lpe_rigid_upload: polygon vertex range out of bounds (or > 32 vertices)";
                return LPE_ERR_ARG;
            }
        }
        // rank = position in entity-id order (pairs are ordered by eid)
        std::vector<int32_t> byRank(nb), rank(nb);
        for (int i = 0; i < nb; i++) byRank[i] = i;
        std::stable_sort(byRank.begin(), byRank.end(),
                         [&](int a, int b) { return bodies[a].eid < bodies[b].eid; });
        for (int r = 0; r < nb; r++) rank[byRank[r]] = r;
        LPE_HIP(ctx, hipMemcpyAsync(d->bodies, bodies, sizeof(lpe_body) * nb, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d->rank, rank.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d->byRank, byRank.data(), sizeof(int32_t) * nb, hipMemcpyHostToDevice, s));
        // broadphase cell: the largest rotation-bounded extent (2 x circumradius)
        // among bodies of at most 2 m (walls and the like go to the special list)
        double cell = 0.0;
        for (int i = 0; i < nb; i++) {
            const lpe_body &b = bodies[i];
            double R = 0.0;
            if (b.flags & LPE_BODY_CIRCLE) R = b.radius;
            else
                for (int v = 0; v < b.vert_cnt; v++) {
                    const double lx = verts[2 * (b.vert_off + v)], ly = verts[2 * (b.vert_off + v) + 1];
                    R = std::max(R, std::sqrt(lx * lx + ly * ly));
                }
            if (2.0 * R <= 2.0) cell = std::max(cell, 2.0 * R);
        }
        d->bp_cell = std::max(cell * 1.0001, 0.05);
        if ((st = rgrow(ctx, &d->bgList, (size_t)nb))) return st;
        if ((st = rgrow(ctx, &d->bgKey, (size_t)nb))) return st;
        if ((st = rgrow(ctx, &d->bgSpecial, (size_t)nb))) return st;
        if (nverts > 0)
            LPE_HIP(ctx, hipMemcpyAsync(d->verts, verts, sizeof(double) * 2 * nverts, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipStreamSynchronize(s));
    }
    if (d->cap_pairs == 0) {
        if ((st = rigid_alloc_pairs(ctx, d, std::max(16 * nb, 1024)))) return st;
        if ((st = rigid_alloc_contacts(ctx, d, std::max(64 * nb, 4096)))) return st;
    }
    return LPE_OK;
}

// per-item (rank, cnt) on the dependency bodies sItemA/sItemB of items
// [0, K) (device count kptr, host bound kcap) -> sVer
static int rigid_versions(lpe_ctx *ctx, RigidDev *d, const int32_t *kptr, int kcap) {
    hipStream_t s = ctx->stream;
    int nb = d->nb;
    LPE_HIP(ctx, hipMemsetAsync(d->sBCount, 0, sizeof(int32_t) * nb, s));
    LPE_KERNEL(ctx, "k_sched_count", k_sched_count, dim3(rblk(kcap)), dim3(RTPB), 0, s, kptr, d->sItemA, d->sItemB, d->sBCount);
    int st = rscan(ctx, d, nullptr, nb, d->sBCount, d->sBStart, d->sBCursor);
    if (st) return st;
    LPE_KERNEL(ctx, "k_sched_fill", k_sched_fill, dim3(rblk(kcap)), dim3(RTPB), 0, s, kptr, d->sItemA, d->sItemB, d->sBCursor, d->sEnt);
    LPE_KERNEL(ctx, "k_sched_rank", k_sched_rank, dim3(rblk(kcap)), dim3(RTPB), 0, s, kptr, d->sItemA, d->sItemB, d->sBStart, d->sEnt, d->sVer);
    LPE_CHECK_LAUNCH(ctx, "versions");
    return LPE_OK;
}

// broadphase (canonical) or upload of caller pairs, then narrowphase; syncs
// once to size the contact list
// Collision detection, part 1: broadphase (or the caller's pairs) and
// narrowphase on stream s, ending with the counts copied to hc (host) —
// nothing here waits for the host.
static int detect_launch(lpe_ctx *ctx, RigidDev *d, int np_in, const int32_t *pairs_in, hipStream_t s,
                         int32_t *hc, bool lagged = false) {
    const lpe_rigid_config &c = d->cfg;
    int nb = d->nb;
    // [0..3], [6] (counts[4], [5] belong to the solvers / gravity; [7]: solver fault, sticky)
    d->contacts_zeroed = false;
    if (pairs_in) {
        LPE_HIP(ctx, hipMemsetAsync(d->counts, 0, sizeof(int32_t) * 4, s));
        LPE_HIP(ctx, hipMemsetAsync(d->counts + 6, 0, sizeof(int32_t), s));
        LPE_HIP(ctx, hipMemsetAsync(d->counts + 11, 0, sizeof(int32_t), s));
        if (np_in > d->cap_pairs) {
            int st = rigid_alloc_pairs(ctx, d, np_in + 1024);
            if (st) return st;
        }
        if (np_in > 0)
            LPE_HIP(ctx, hipMemcpyAsync(d->pairs, pairs_in, sizeof(int32_t) * 2 * np_in, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d->counts, &np_in, sizeof(int32_t), hipMemcpyHostToDevice, s));
    } else {
        double lo = -c.boundaryBuffer, hi = -c.boundaryBuffer + (c.universeSize + 2 * c.boundaryBuffer);
        // grid over the universe plus 1 m (bodies the boundary system lets
        // stray further, or larger than a cell, are "special")
        const double org = -1.0, g = d->bp_cell > 0.0 ? d->bp_cell : 1.0;
        const long G = std::max(1L, (long)std::ceil((c.universeSize + 2.0) / g));
        if (G * G > (1L << 26)) {
            ctx->err = "rigid broadphase grid too large (universe / body size)";
            return LPE_ERR_CAPACITY;
        }
        const int cells = (int)(G * G);
        if (cells > d->cap_bgcells) {
            int st0 = rgrow(ctx, &d->bgCount, (size_t)cells + 1);
            if (!st0) st0 = rgrow(ctx, &d->bgStart, (size_t)cells + 1);
            if (!st0) st0 = rgrow(ctx, &d->bgCursor, (size_t)cells + 1);
            if (st0) return st0;
            d->cap_bgcells = cells;
        }
        LPE_KERNEL(ctx, "k_rb_prep", k_rb_prep, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, d->verts, lo, hi, d->aabb,
                   d->cand, d->counts, d->pcount, d->bgCount, cells, d->inContact);
        d->contacts_zeroed = true;
        LPE_KERNEL(ctx, "k_bg_key", k_bg_key, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->byRank, d->aabb, d->cand, org, g,
                   (int)G, d->bgKey, d->bgCount, d->bgSpecial, d->counts + 10);
        int st = rscan(ctx, d, nullptr, cells, d->bgCount, d->bgStart, d->bgCursor, s);
        if (st) return st;
        LPE_KERNEL(ctx, "k_bg_fill", k_bg_fill, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bgKey, d->bgCursor, d->bgList);
        LPE_KERNEL(ctx, "k_bg_pairs", k_bg_pairs, dim3((nb + BG_WAVES - 1) / BG_WAVES), dim3(RTPB), 0, s, nb, 0, d->byRank, d->bodies, d->aabb,
                   c.smallParticleThreshold, (int)G, d->bgKey, d->bgStart, d->bgList, d->bgSpecial, d->counts + 10,
                   d->pcount, d->pcursor, d->pairs, d->pairRankB, d->cap_pairs, d->counts + 6);
        // (the scan also leaves the pair count in counts[0])
        st = rscan(ctx, d, nullptr, nb, d->pcount, d->pstart, d->pcursor, s, d->counts);
        if (st) return st;
        LPE_KERNEL(ctx, "k_bg_pairs", k_bg_pairs, dim3((nb + BG_WAVES - 1) / BG_WAVES), dim3(RTPB), 0, s, nb, 1, d->byRank, d->bodies, d->aabb,
                   c.smallParticleThreshold, (int)G, d->bgKey, d->bgStart, d->bgList, d->bgSpecial, d->counts + 10,
                   d->pcount, d->pcursor, d->pairs, d->pairRankB, d->cap_pairs, d->counts + 6);
        LPE_KERNEL(ctx, "k_bp_sort", k_bp_sort, dim3((nb + RTPB / 64 - 1) / (RTPB / 64)), dim3(RTPB), 0, s, nb, d->pstart, d->pairs, d->pairRankB, d->cap_pairs);
    }
    LPE_KERNEL(ctx, "k_narrow", k_narrow, dim3(rblk(d->cap_pairs, 128)), dim3(128), 0, s, d->counts, d->cap_pairs, d->pairs, d->bodies, d->verts, d->cslots, d->ccount, d->counts);
    int st = rscan(ctx, d, d->counts, d->cap_pairs, d->ccount, d->cstart, nullptr, s);
    if (st) return st;
    if (lagged) {   // the compaction right away (capacity-bounded; the counts are checked later)
        LPE_KERNEL(ctx, "k_compact", k_compact, dim3(rblk(d->cap_pairs)), dim3(RTPB), 0, s, d->counts, d->cap_pairs,
                   d->cslots, d->ccount, d->cstart, d->contacts, d->cap_contacts, d->counts, hc);
        return LPE_OK;
    }
    LPE_HIP(ctx, hipMemcpyAsync(hc, d->counts, sizeof(int32_t) * 16, hipMemcpyDeviceToHost, s));
    return LPE_OK;
}

// counts[7]: bit 1 a dataflow (replay) solve made no progress, bit 2 a
// striped solver's workgroup waited ~0.2 s for a neighbour's hand-over, bit 64
// a k_wait_flag gave up
static const char *watchdog_msg(int bits) {
    if (bits & 64)
        return "world tick: a stream waited ~3 s for the context stream's boundary pass (k_wait_flag); the tick "
               "is wrong";
    if (bits & 2)
        return "striped rigid solver: a workgroup waited too long for its neighbour's hand-over (fewer "
               "co-resident workgroups than stripes, or CUs held by other work); that solve is wrong";
    return "rigid solver watchdog fired (a dataflow solve made no progress)";
}

// Part 2, once hc has arrived: capacity checks (1: the pair buffer
// overflowed and was grown, run part 1 again) and the contact compaction.
static int detect_finish(lpe_ctx *ctx, RigidDev *d, hipStream_t s, const int32_t *hc, int *retry) {
    *retry = 0;
    int np = hc[0];
    if (hc[7]) {
        ctx->err = watchdog_msg(hc[7]);
        return LPE_ERR_OVERFLOW;
    }
    if (hc[6] || np > d->cap_pairs) {   // pair buffer overflow: grow and redo
        *retry = 1;
        d->regrows++;
        return rigid_alloc_pairs(ctx, d, std::max(2 * d->cap_pairs, np + 1024));
    }
    if (hc[11]) {
        ctx->err = "narrowphase: a pair produced more contacts than a pair slot holds (MAXC)";
        return LPE_ERR_OVERFLOW;
    }
    int32_t ncv = 0;
    LPE_HIP(ctx, hipMemcpyAsync(&ncv, d->cstart + np, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipStreamSynchronize(s));
    if (ncv > d->cap_contacts) {
        d->regrows++;
        int st = rigid_alloc_contacts(ctx, d, ncv + 4096);
        if (st) return st;
    }
    LPE_KERNEL(ctx, "k_compact", k_compact, dim3(rblk(d->cap_pairs)), dim3(RTPB), 0, s, d->counts, d->cap_pairs,
               d->cslots, d->ccount, d->cstart, d->contacts, d->cap_contacts, d->counts, nullptr);
    LPE_CHECK_LAUNCH(ctx, "detect");
    d->last_np = np;
    d->last_nc = ncv;
    return LPE_OK;
}

static int rigid_detect(lpe_ctx *ctx, RigidDev *d, int np_in, const int32_t *pairs_in,
                        hipStream_t s = nullptr) {
    if (!s) s = ctx->stream;
    for (int attempt = 0; attempt < 4; attempt++) {
        int32_t hc[16];
        int st = detect_launch(ctx, d, np_in, pairs_in, s, hc);
        if (st) return st;
        LPE_HIP(ctx, hipStreamSynchronize(s));
        int retry = 0;
        st = detect_finish(ctx, d, s, hc, &retry);
        if (st || !retry) return st;
    }
    ctx->err = "rigid pair buffer kept overflowing";
    return LPE_ERR_OVERFLOW;
}

// colour: canonical mode (colour-major order for both solvers, see
// k_pair_colour); otherwise pgs_order (NULL = narrowphase order) for the PGS
// and narrowphase order for the position solver (reference-order replay)
// the canonical colouring of the pairs (k_pair_colour) on stream s
// The striped solver (canonical since round 3) or, with LPE_COLOUR_SOLVER=1,
// round 2's single-workgroup colour sweeps (a different sequential order:
// for measurements only, the oracle restates the striped one).
static bool striped() {
    static const bool old = getenv("LPE_COLOUR_SOLVER") != nullptr;
    return !old;
}
static StripeBufs *stripe_bufs(lpe_ctx *ctx, RigidDev *d) {
    StripeBufs *sb = (StripeBufs *)d->stripes;
    if (!sb) {
        sb = new StripeBufs();
        std::memset(sb, 0, sizeof(*sb));
        d->stripes = sb;
    }
    auto grow = [&](auto **p, size_t n) { return rgrow(ctx, p, n); };
    if (d->nb > d->cap_stripe_nb || !sb->bstripe) {
        const size_t N = (size_t)std::max(d->nb, 1);
        if (grow(&sb->bstripe, N) || grow(&sb->bpos, N) || grow(&sb->sbList, N) || grow(&sb->gvt, 3 * N) ||
            grow(&sb->gpos, 3 * N))
            return nullptr;
        // (epoch 0 never matches: the tagged hand-over's epochs start at sbase_pgs + 1 >= 17)
        if (hipMemset(sb->gvt, 0, sizeof(unsigned long long) * 3 * N) != hipSuccess) return nullptr;
        d->cap_stripe_nb = d->nb;
    }
    if (d->cap_pairs > d->cap_stripe_pairs || !sb->pgroup) {
        const size_t P = (size_t)std::max(d->cap_pairs, 1);
        if (grow(&sb->pgroup, P) || grow(&sb->pcolg, P) || grow(&sb->prank, P) || grow(&sb->prowoff, P) ||
            grow(&sb->glist, P) || grow(&sb->pflag, P) || grow(&sb->px, P) || grow(&sb->bred, 4 * (P / RTPB + 1)) ||
            grow(&sb->gla, P) || grow(&sb->glb, P) || grow(&sb->gln, P))
            return nullptr;
        d->cap_stripe_pairs = d->cap_pairs;
    }
    if (!sb->gstart) {
        if (grow(&sb->gstart, SGROUPS + 1) || grow(&sb->gcnt, (size_t)SGROUPS * SCOLS * 2 + SGROUPS) ||
            grow(&sb->stepIdx, (size_t)SGROUPS * SCOLS) || grow(&sb->stepPair, STEPS_MAX + 1) ||
            grow(&sb->stepRow, STEPS_MAX + 1) || grow(&sb->wgStep, 2 * STRIPES_MAX) ||
            grow(&sb->sbStart, STRIPES_MAX + 2) || grow(&sb->sflag, 2 * STRIPES_MAX))
            return nullptr;
        if (hipMemset(sb->sflag, 0, sizeof(uint32_t) * 2 * STRIPES_MAX) != hipSuccess) return nullptr;
    }
    return sb;
}

// The stripe count bound: k_pgs_stripes and k_pos_stripes run at the same
// time with S / 2 workgroups each, one per CU (their LDS), and hand data
// between workgroups with spin waits, so all S must be resident at once:
// S <= the device's CU count (256 on an MI355X: STRIPES_MAX binds; a smaller
// compute partition gets fewer, wider stripes).
// Cached per device (contexts on devices of different CU counts,
// e.g. another compute-partition mode, must not share one bound).
static int stripe_cap(lpe_ctx *ctx) {
    static std::atomic<int> caps[64];
    const int dev = ctx->device;
    int cap = (dev >= 0 && dev < 64) ? caps[dev].load(std::memory_order_relaxed) : 0;
    if (!cap) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 2;
        cap = std::min(STRIPES_MAX, cus) & ~1;
        if (dev >= 0 && dev < 64) caps[dev].store(cap, std::memory_order_relaxed);
    }
    return cap;
}

// stripes, groups, greedy colourings and the step layout on stream s
static int stripe_launch(lpe_ctx *ctx, RigidDev *d, hipStream_t s) {
    const int nb = d->nb;
    if (d->cap_pcol < d->cap_pairs || !d->pcol) {
        int st0 = rgrow(ctx, &d->pcol, (size_t)d->cap_pairs);
        if (!st0) st0 = rgrow(ctx, &d->cseg, (size_t)d->cap_pairs);
        if (st0) return st0;
        d->cap_pcol = d->cap_pairs;
    }
    StripeBufs *sb = stripe_bufs(ctx, d);
    if (!sb) return LPE_ERR_HIP;
    LPE_KERNEL(ctx, "k_stripe_pairs", k_stripe_pairs, dim3(rblk(d->cap_pairs)), dim3(RTPB), 0, s, d->counts,
               d->pairs, d->ccount, d->bodies, *sb);
    LPE_KERNEL(ctx, "k_stripe_setup", k_stripe_setup, dim3(1), dim3(SOLVE_TPB), sizeof(uint32_t) * 2 * ((nb + 31) / 32 + 1),
               s, nb, d->counts, d->pairs, d->bodies, *sb, d->counts, stripe_cap(ctx));
    LPE_KERNEL(ctx, "k_group_colour", k_group_colour, dim3(SGROUPS), dim3(RTPB), sizeof(unsigned long long) * (size_t)nb,
               s, d->counts, d->counts, d->pairs, d->ccount, *sb);
    LPE_KERNEL(ctx, "k_stripe_layout", k_stripe_layout, dim3(1), dim3(RTPB), 0, s, *sb, d->counts);
    LPE_KERNEL(ctx, "k_stripe_fill", k_stripe_fill, dim3(rblk(d->cap_pairs)), dim3(RTPB), 0, s, d->counts, d->ccount,
               d->cstart, *sb, d->pcol, d->cseg, d->order);
    LPE_CHECK_LAUNCH(ctx, "stripes");
    return LPE_OK;
}

static int colour_launch(lpe_ctx *ctx, RigidDev *d, hipStream_t s) {
    if (striped()) return stripe_launch(ctx, d, s);
    int nb = d->nb;
    if (d->cap_pcol < d->cap_pairs || !d->pcol) {
        int st0 = rgrow(ctx, &d->pcol, (size_t)d->cap_pairs);
        if (st0) return st0;
        st0 = rgrow(ctx, &d->cseg, (size_t)d->cap_pairs);
        if (st0) return st0;
        d->cap_pcol = d->cap_pairs;
    }
    if (!d->cbase) {
        int st0 = rgrow(ctx, &d->cbase, (size_t)MAX_COLOURS + 1);
        if (st0) return st0;
    }
    size_t lds = (2 * sizeof(unsigned long long) + 1) * (size_t)nb + 16;
    LPE_KERNEL(ctx, "k_pair_colour", k_pair_colour, dim3(1), dim3(SOLVE_TPB), lds, s, nb, d->counts, d->pairs, d->ccount, d->cstart, d->bodies, d->pcol, d->order, d->cseg, d->cbase, d->counts);
    return LPE_OK;
}

// ---- canonical-order solve (graph-coloured, see k_pair_colour), in three
// launches groups.  The position solver (position_solver.cpp:299-325) reads
// poses, masses and the narrowphase contacts, never a velocity; the PGS
// (contact_solver.cpp:449-543) writes only v and omega, and its rows take the
// lever arms from the poses BEFORE the position solver moves them
// (contact_solver.cpp:133-197).  So everything except the PGS sweeps is
// velocity independent and runs as soon as the contacts are coloured:
//   colour_prep  contact marks, inverse masses, PGS rows, position items
//   colour_pos   the position solver (one workgroup, poses in LDS)
//   colour_pgs   the velocities (final only after the fluid and gravity
//                systems have run) and the PGS sweeps
// The reference runs PGS then the position solver; the results are the same
// bits in any of these arrangements.
static size_t colour_lds_cap() { return 159 * 1024; }   // of a CU's 160 KB (the kernels use < 1 KB static)

// the colour-order position rows, carved from posRec's allocation
// (cap_contacts records of 88 bytes hold the arrays' 84 bytes a row)
static PosRows pos_rows(RigidDev *d) {
    static_assert(sizeof(PosRec) >= 4 * sizeof(double2) + sizeof(double) + sizeof(int2) + sizeof(int32_t),
                  "position rows must fit in posRec");
    const size_t K = (size_t)d->cap_contacts;
    PosRows r;
    double2 *base = (double2 *)d->posRec;
    r.n = base; r.c = base + K; r.m = base + 2 * K; r.i = base + 3 * K;
    r.py = (double *)(base + 4 * K);
    r.ab = (int2 *)(r.py + K);
    r.fl = (int32_t *)(r.ab + K);
    return r;
}

static int colour_prep(lpe_ctx *ctx, RigidDev *d, hipStream_t s) {
    const lpe_rigid_config &c = d->cfg;
    // (lagged detection: the count is on the device only, the grids cover the capacity)
    const int nb = d->nb, nc = d->lag ? d->cap_contacts : d->last_nc;
    int32_t *inPos = d->inContact + nb;
    d->contacts_zeroed = false;                   // (k_prep_bodies clears the marks)
    LPE_KERNEL(ctx, "k_prep_bodies", k_prep_bodies, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, d->imii,
               d->posState, d->inContact);
    LPE_KERNEL(ctx, "k_prep_items", k_prep_items, dim3(rblk(nc)), dim3(RTPB), 0, s, d->counts + 1, d->order,
               d->contacts, d->bodies, d->imii, d->posState, d->rowN, d->rowR, d->rowAB, d->rowM, d->sItemA, d->sItemB,
               pos_rows(d), d->inContact, inPos, c.baumgarte, c.slop, d->rowOf, d->rowC);
    LPE_CHECK_LAUNCH(ctx, "solver preparation");
    return LPE_OK;
}

static int colour_pos(lpe_ctx *ctx, RigidDev *d, hipStream_t s) {
    const lpe_rigid_config &c = d->cfg;
    const int nb = d->nb;
    if (striped()) {
        StripeBufs *sb = stripe_bufs(ctx, d);
        if (!sb) return LPE_ERR_HIP;
        const uint32_t base = d->sbase_pos;
        d->sbase_pos += (uint32_t)c.posIterations + 2;
        LPE_KERNEL(ctx, "k_pos_stripes", k_pos_stripes, dim3(STRIPES_MAX / 2), dim3(STPB), STRIPE_LDS, s, d->counts, *sb,
                   d->cseg, pos_rows(d), d->bodies, d->posState, d->inContact + nb, c.posIterations, base,
                   d->counts + 7);
        LPE_CHECK_LAUNCH(ctx, "position solver");
        return LPE_OK;
    }
    const size_t lds2 = sizeof(double) * 3 * (size_t)nb;
    LPE_KERNEL(ctx, "k_pos_colour", k_pos_colour, dim3(1), dim3(SOLVE_TPB), lds2, s, nb, d->counts, d->cbase, d->cseg, pos_rows(d), d->bodies, d->posState, d->inContact + nb, c.posIterations);
    LPE_CHECK_LAUNCH(ctx, "position solver");
    return LPE_OK;
}

// k_pgs_jacobi's blocks meet at a grid barrier every iteration,
// so all of them must be resident at once.  The most it may launch: its
// occupancy per CU times the CUs, less one CU per workgroup the position
// solver's stripe kernel (k_pos_stripes, up to stripe_cap / 2 workgroups of
// most of a CU's LDS) may hold beside it -- cached per device, at most
// JAC_BLOCKS_MAX.
static int jac_cap(lpe_ctx *ctx) {
    static std::atomic<int> caps[64];
    const int dev = ctx->device;
    int cap = (dev >= 0 && dev < 64) ? caps[dev].load(std::memory_order_relaxed) : 0;
    if (!cap) {
        int cus = 0, occ = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_pgs_jacobi, JAC_TPB, 0) != hipSuccess || occ <= 0)
            occ = 1;
        cap = std::max(1, std::min(JAC_BLOCKS_MAX, occ * (cus - stripe_cap(ctx) / 2)));
        if (dev >= 0 && dev < 64) caps[dev].store(cap, std::memory_order_relaxed);
    }
    return cap;
}

// the Jacobi solver's buffers (JacBufs), grown to nb bodies and nc contacts
static JacBufs jac_bufs(RigidDev *d) {
    const size_t nb = (size_t)d->cap_jac_nb;
    char *p = (char *)d->jac;
    JacBufs j;
    j.bar = (uint32_t *)p;
    j.cnt = (int32_t *)(p + 64);
    j.S0 = (long long *)(p + 64 + 8 * ((4 * nb + 7) / 8));
    j.S1 = j.S0 + 3 * nb;
    j.v0 = (float *)(j.S1 + 3 * nb);
    return j;
}
static size_t jac_zeroed_bytes(int nb) {           // bar, cnt, S0, S1: cleared before every launch
    return 64 + 8 * ((4 * (size_t)nb + 7) / 8) + 48 * (size_t)nb;
}
static int jac_launch(lpe_ctx *ctx, RigidDev *d, hipStream_t s) {
    const lpe_rigid_config &c = d->cfg;
    // (lagged detection: the counts are on the device only, the sizes are the capacities)
    const int nb = d->nb, nc = d->lag ? d->cap_contacts : d->last_nc;
    if (!d->jac || nb > d->cap_jac_nb) {
        if (d->jac) { LPE_HIP(ctx, hipStreamSynchronize(s)); (void)hipFree(d->jac); d->jac = nullptr; }
        const int cnb = std::max(nb, d->cap_jac_nb);
        LPE_HIP(ctx, hipMalloc(&d->jac, jac_zeroed_bytes(cnb) + 8 * ((12 * (size_t)cnb + 7) / 8)));
        d->cap_jac_nb = cnb;
    }
    LPE_HIP(ctx, hipMemsetAsync(d->jac, 0, jac_zeroed_bytes(d->cap_jac_nb), s));
    // blocks own at most JAC_CPB contacts each (their rows stay in LDS); in
    // lagged detection nc is the capacity, and a tick with more than
    // JAC_BLOCKS_MAX * JAC_CPB contacts raises the solver fault (counts[7])
    // (the grid barrier needs every block resident at once: at most what
    // the device holds beside the position solver's stripe workgroups, jac_cap)
    const int gmax = jac_cap(ctx);
    if (!d->lag && nc > gmax * JAC_CPB) {
        ctx->err = "rigid solver (Jacobi): more contacts than its co-resident blocks hold (" +
                   std::to_string(gmax) + " x JAC_CPB)";
        return LPE_ERR_CAPACITY;
    }
    const int G = std::max(1, std::min(gmax, (nc + JAC_CPB - 1) / JAC_CPB));
    LPE_KERNEL(ctx, "k_pgs_jacobi", k_pgs_jacobi, dim3(G), dim3(JAC_TPB), 0, s, nb, d->counts, d->counts + 1,
               d->ccount, d->cstart, d->rowOf, d->rowN, d->rowR, d->rowAB, d->rowM, c.pgsIterations,
               c.frictionCoeff, d->lamN, d->lamF, d->bodies, (const int32_t *)d->inContact, jac_bufs(d),
               d->counts + 7);
    LPE_CHECK_LAUNCH(ctx, "pgs (Jacobi)");
    d->lam_by_contact = true;
    return LPE_OK;
}

static int colour_pgs(lpe_ctx *ctx, RigidDev *d, hipStream_t s) {
    const lpe_rigid_config &c = d->cfg;
    const int nb = d->nb;
    if (c.pgsMode == LPE_PGS_JACOBI) return jac_launch(ctx, d, s);
    d->lam_by_contact = false;
    if (striped()) {
        StripeBufs *sb = stripe_bufs(ctx, d);
        if (!sb) return LPE_ERR_HIP;
        const uint32_t base = d->sbase_pgs;
        d->sbase_pgs += 2 * (uint32_t)c.pgsIterations + 4;      // (the tagged hand-over's epochs)
        LPE_KERNEL(ctx, "k_pgs_stripes", k_pgs_stripes, dim3(STRIPES_MAX / 2), dim3(STPB), STRIPE_LDS, s, d->counts, *sb,
                   d->cseg, d->rowN, d->rowR, d->rowC, d->rowAB, d->rowM, c.pgsIterations, c.frictionCoeff, d->lamN,
                   d->lamF, d->bodies, (const int32_t *)d->inContact, base, d->counts + 7);
        LPE_CHECK_LAUNCH(ctx, "pgs");
        return LPE_OK;
    }
    // (k_pgs_bodies and k_pgs_writeback run as the kernel's prologue / epilogue)
    const size_t lds = sizeof(float) * 3 * (size_t)nb;
    LPE_KERNEL(ctx, "k_pgs_colour", k_pgs_colour, dim3(1), dim3(SOLVE_TPB), lds, s, nb, d->counts, d->cbase, d->cseg, 0, d->rowN, d->rowR, d->rowAB, d->rowM, d->vel0, c.pgsIterations, c.frictionCoeff, d->lamN, d->lamF, d->bodies, (const int32_t *)d->inContact);
    LPE_CHECK_LAUNCH(ctx, "pgs");
    return LPE_OK;
}

static int solver_streams(lpe_ctx *ctx, RigidDev *d) {
    if (d->psolve) return LPE_OK;
    LPE_HIP(ctx, hipStreamCreateWithFlags(&d->psolve, hipStreamNonBlocking));
    LPE_HIP(ctx, hipEventCreateWithFlags(&d->evFork, hipEventDisableTiming));
    LPE_HIP(ctx, hipEventCreateWithFlags(&d->evJoin, hipEventDisableTiming));
    return LPE_OK;
}

static int solver_lds_check(lpe_ctx *ctx, RigidDev *d) {
    if ((size_t)d->nb * (3 * sizeof(double) + sizeof(int)) > 160 * 1024) {
        ctx->err = "rigid solver: too many bodies for the LDS-resident solve (max 5851)";
        return LPE_ERR_CAPACITY;
    }
    return LPE_OK;
}

// coloured: the colouring already ran (side stream)
static int rigid_solve(lpe_ctx *ctx, RigidDev *d, bool colour, const int32_t *pgs_order,
                       lpe_rigid_stats *stats) {
    hipStream_t s = ctx->stream;
    const lpe_rigid_config &c = d->cfg;
    int nb = d->nb, nc = d->last_nc;
    if (nc == 0) {                 // early out (rigid_body_collision.cpp:35-37)
        if (colour) {
            if (d->pcol && d->last_np > 0)
                LPE_HIP(ctx, hipMemsetAsync(d->pcol, 0xff, sizeof(int32_t) * d->last_np, s));
            LPE_HIP(ctx, hipMemsetAsync(d->counts + 8, 0, sizeof(int32_t), s));
        }
        return LPE_OK;
    }
    int st = solver_lds_check(ctx, d);
    if (st) return st;
    if (colour) {
        // canonical order: colour, prepare, then the two solvers concurrently
        // (one workgroup each) on the context stream and the solver stream
        st = colour_launch(ctx, d, s);
        if (!st) st = colour_prep(ctx, d, s);
        if (!st) st = solver_streams(ctx, d);
        if (st) return st;
        LPE_HIP(ctx, hipEventRecord(d->evFork, s));
        LPE_HIP(ctx, hipStreamWaitEvent(d->psolve, d->evFork, 0));
        st = colour_pos(ctx, d, d->psolve);
        if (st) return st;
        LPE_HIP(ctx, hipEventRecord(d->evJoin, d->psolve));
        st = colour_pgs(ctx, d, s);
        if (st) return st;
        LPE_HIP(ctx, hipStreamWaitEvent(s, d->evJoin, 0));
    } else {
        // caller-supplied order (reference replay): exact dataflow sweeps
        const int32_t *ord = nullptr;
        if (pgs_order) {
            LPE_HIP(ctx, hipMemcpyAsync(d->order, pgs_order, sizeof(int32_t) * nc, hipMemcpyHostToDevice, s));
            ord = d->order;
        }
        LPE_HIP(ctx, hipMemsetAsync(d->inContact, 0, sizeof(int32_t) * 2 * nb, s));
        LPE_KERNEL(ctx, "k_mark_contacts", k_mark_contacts, dim3(rblk(nc)), dim3(RTPB), 0, s, d->counts + 1, d->contacts, d->inContact);
        LPE_KERNEL(ctx, "k_pgs_bodies", k_pgs_bodies, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, d->vel0, d->imii, 3);
        LPE_KERNEL(ctx, "k_pgs_rows", k_pgs_rows, dim3(rblk(nc)), dim3(RTPB), 0, s, d->counts + 1, ord, d->contacts, d->bodies, d->imii, d->rowN, d->rowR, d->rowAB, d->rowM, d->sItemA, d->sItemB);
        int32_t *inPos = d->inContact + nb;
        st = rigid_versions(ctx, d, d->counts + 1, nc);
        if (st) return st;
        size_t lds = (sizeof(float) * 3 + sizeof(int)) * (size_t)nb;
        LPE_KERNEL(ctx, "k_pgs_flow", k_pgs_flow, dim3(1), dim3(SOLVE_TPB), lds, s, nb, d->counts + 1, d->rowN, d->rowR, d->rowAB, d->rowM, d->sVer, d->vel0, c.pgsIterations, c.frictionCoeff, d->lamN, d->lamF, d->counts + 7);
        LPE_KERNEL(ctx, "k_pgs_writeback", k_pgs_writeback, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, d->vel0, d->inContact);
        LPE_CHECK_LAUNCH(ctx, "pgs");
        // position solver in narrowphase order
        int32_t *keep = d->posKeep, *kstart = d->posStart;
        LPE_KERNEL(ctx, "k_pos_bodies", k_pos_bodies, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, d->posState);
        LPE_KERNEL(ctx, "k_pos_items", k_pos_items, dim3(rblk(nc)), dim3(RTPB), 0, s, d->counts + 1, (const int32_t *)nullptr, d->contacts, d->bodies, d->posState, keep);
        st = rscan(ctx, d, d->counts + 1, nc, keep, kstart, nullptr);
        if (st) return st;
        // kept-contact count -> counts[4]
        LPE_HIP(ctx, hipMemcpyAsync(d->counts + 4, kstart + nc, sizeof(int32_t), hipMemcpyDeviceToDevice, s));
        LPE_KERNEL(ctx, "k_pos_fill", k_pos_fill, dim3(rblk(nc)), dim3(RTPB), 0, s, d->counts + 1, (const int32_t *)nullptr, keep, kstart, d->contacts, d->posState, d->posRec, d->sItemA, d->sItemB, inPos, c.baumgarte, c.slop);
        st = rigid_versions(ctx, d, d->counts + 4, nc);
        if (st) return st;
        size_t lds2 = (sizeof(double) * 3 + sizeof(int)) * (size_t)nb;
        LPE_KERNEL(ctx, "k_pos_flow", k_pos_flow, dim3(1), dim3(SOLVE_TPB), lds2, s, nb, d->counts + 4, d->posRec, d->sVer, d->sItemA, d->sItemB, d->bodies, d->posState, inPos, c.posIterations, d->counts + 7);
        LPE_CHECK_LAUNCH(ctx, "position solver");
    }
    if (stats) {
        int32_t hc[16];
        LPE_HIP(ctx, hipMemcpyAsync(hc, d->counts, sizeof(int32_t) * 16, hipMemcpyDeviceToHost, s));
        LPE_HIP(ctx, hipStreamSynchronize(s));
        // colours of the canonical order (0: a caller-supplied order)
        stats->pgsLevels = colour ? hc[8] : 0;
        stats->posLevels = colour ? hc[8] : 0;
        stats->colourRounds = colour ? hc[9] : 0;
    }
    return LPE_OK;
}

static int rigid_step_impl(lpe_ctx *ctx, int np, const int32_t *pairs, int nc_order,
                           const int32_t *pgs_order, lpe_rigid_stats *stats) {
    if (!ctx) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    if (stats) std::memset(stats, 0, sizeof(*stats));
    if (d->nb <= 0) return LPE_OK;
    (void)hipSetDevice(ctx->device);
    int st = d->lag ? rigid_lag_drain(ctx, d) : LPE_OK;       // (a world tick's pending checks)
    if (st) return st;
    st = rigid_detect(ctx, d, np, pairs);
    if (st) return st;
    if (pgs_order && nc_order != d->last_nc) {
        ctx->err = "lpe_rigid_step_ordered: pgs_order length differs from the contact count";
        return LPE_ERR_ARG;
    }
    if (stats) { stats->pairs = d->last_np; stats->contacts = d->last_nc; }
    return rigid_solve(ctx, d, pairs == nullptr, pgs_order, stats);
}

extern "C" int lpe_rigid_reserve(lpe_ctx *ctx, int pairs, int contacts) {
    if (!ctx || pairs < 1 || contacts < 1) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    RigidDev *d = rdev(ctx);
    rigid_lag_off(ctx, d);
    if (d->side) LPE_HIP(ctx, hipStreamSynchronize(d->side));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    d->cap_pairs = 0;                     // re-allocated at exactly the requested sizes
    d->cap_contacts = 0;
    int st = rigid_alloc_pairs(ctx, d, pairs);
    if (!st) st = rigid_alloc_contacts(ctx, d, contacts);
    return st;
}

extern "C" int lpe_rigid_buffer_info(lpe_ctx *ctx, int *pairs, int *contacts, int *regrows) {
    if (!ctx) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    if (pairs) *pairs = d->cap_pairs;
    if (contacts) *contacts = d->cap_contacts;
    if (regrows) *regrows = d->regrows;
    return LPE_OK;
}

extern "C" int lpe_rigid_step(lpe_ctx *ctx, lpe_rigid_stats *stats) {
    return rigid_step_impl(ctx, 0, nullptr, 0, nullptr, stats);
}

// World tick (lpe_world.hip): collision detection and the pair colouring of
// RigidBodyCollisionSystem run on a side stream while the fluid step runs.
// Their inputs (poses, shapes, flags) are final once the boundary system's
// position clamp is applied (k_boundary_pos, at the start of the tick: the
// fluid step and gravity write only velocities); the solvers, which need the
// velocities, wait for the colouring on the context stream.
// ---- lagged detection checks (RigidDev::lag) ---------------------------
// The counts of one lagged detection (slot), once its copy has landed: an
// overflow of that tick fails loudly; counts past half a capacity schedule a
// growth for the next tick start.  wait = false: only if already complete.
static int rigid_lag_check(lpe_ctx *ctx, RigidDev *d, int slot, bool wait) {
    if (!d->hpend[slot]) return LPE_OK;
    if (wait) {
        LPE_HIP(ctx, hipEventSynchronize(d->evHc[slot]));
    } else {
        const hipError_t q = hipEventQuery(d->evHc[slot]);
        if (q == hipErrorNotReady) return LPE_OK;
        if (q != hipSuccess) { ctx->err = "hipEventQuery (lagged detection)"; return LPE_ERR_HIP; }
    }
    d->hpend[slot] = false;
    const int32_t *hc = d->hcr + 16 * slot;
    if (hc[7]) {
        ctx->err = watchdog_msg(hc[7]);
        return LPE_ERR_OVERFLOW;
    }
    if (hc[11]) {
        ctx->err = "narrowphase: a pair produced more contacts than a pair slot holds (MAXC)";
        return LPE_ERR_OVERFLOW;
    }
    // (hc[15]: the pairs the detection found; k_compact zeroed hc[0] of an
    // overflowing tick, which therefore solved nothing)
    if (hc[6] || hc[15] > d->cap_pairs || hc[14] > d->cap_contacts) {
        d->lag = false;
        ctx->err = "rigid pair / contact buffers overflowed in a tick checked after the fact (the counts grew "
                   "more than 4x within two ticks; that tick's contacts were dropped); reserve more with "
                   "lpe_rigid_reserve";
        return LPE_ERR_OVERFLOW;
    }
    d->last_np = hc[15];
    d->last_nc = hc[14];
    if (2 * hc[0] > d->cap_pairs) d->grow_pairs = std::max(d->grow_pairs, 4 * hc[0] + 1024);
    if (2 * hc[14] > d->cap_contacts) d->grow_contacts = std::max(d->grow_contacts, 4 * hc[14] + 4096);
    return LPE_OK;
}

// every pending check, oldest first (last_np / last_nc end as the newest tick's)
static int rigid_lag_drain(lpe_ctx *ctx, RigidDev *d) {
    int st = rigid_lag_check(ctx, d, (int)(d->htick & 1u), true);
    const int st2 = rigid_lag_check(ctx, d, (int)((d->htick + 1u) & 1u), true);
    return st ? st : st2;
}

// leave lagged mode (upload, reserve, config): the next detection is synchronous
static void rigid_lag_off(lpe_ctx *ctx, RigidDev *d) {
    if (d->hcr) (void)rigid_lag_drain(ctx, d);
    d->hpend[0] = d->hpend[1] = false;
    d->lag = d->lag_next = false;
    d->grow_pairs = d->grow_contacts = 0;
}

// Device waits need the waiting and the signalling streams' kernels to run
// at the same time.  Where dispatches are serialised (rocprofv3 counter
// collection, AMD_SERIALIZE_KERNEL, two streams on one hardware queue) the
// waiter would hold its queue until its watchdog: tsync_alloc probes once
// per context (a waiter on the context stream, its signal from the detection
// stream launched after it; ~6 ms watchdog) and falls back to the events.
static bool device_waits(const RigidDev *d) {
    static const bool ev = getenv("LPE_EVENT_WAITS") != nullptr;
    return !ev && d->devwait_ok;
}
static int tsync_alloc(lpe_ctx *ctx, RigidDev *d) {
    if (d->tsync) return LPE_OK;
    LPE_HIP(ctx, hipMalloc((void **)&d->tsync, sizeof(uint32_t) * 8));
    LPE_HIP(ctx, hipMemsetAsync(d->tsync, 0, sizeof(uint32_t) * 8, ctx->stream));
    d->tsyncTick = 0;
    if (d->side) {
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        LPE_KERNEL(ctx, "k_wait_flag", k_wait_flag, dim3(1), dim3(64), 0, ctx->stream, d->tsync + 6, 1u,
                   (int32_t *)(d->tsync + 7), 1u << 15, 1);
        LPE_KERNEL(ctx, "k_set_flag", k_set_flag, dim3(1), dim3(64), 0, d->side, d->tsync + 6, 1u);
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        LPE_HIP(ctx, hipStreamSynchronize(d->side));
        uint32_t probe[2] = {0, 0};
        LPE_HIP(ctx, hipMemcpy(probe, d->tsync + 6, sizeof(probe), hipMemcpyDeviceToHost));
        d->devwait_ok = probe[1] == 0;
    }
    return LPE_OK;
}
// stream `s` waits (a one-wave k_wait_flag) until the word reaches `want`
static int wait_flag(lpe_ctx *ctx, RigidDev *d, hipStream_t s, const uint32_t *flag, uint32_t want) {
    LPE_KERNEL(ctx, "k_wait_flag", k_wait_flag, dim3(1), dim3(64), 0, s, flag, want, d->counts + 7, 1u << 24, 64);
    return LPE_OK;
}
int rigid_tick_begin(lpe_ctx *ctx, bool on_main) {
    RigidDev *d = rdev(ctx);
    d->overlap_pending = false;
    d->colour_pending = false;
    d->bvgSignal = false;
    if (d->nb <= 0) return LPE_OK;
    const lpe_rigid_config &c = d->cfg;
    if (!d->side) {
        LPE_HIP(ctx, hipStreamCreateWithFlags(&d->side, hipStreamNonBlocking));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d->evStart, hipEventDisableTiming));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d->evDetect, hipEventDisableTiming));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d->evColour, hipEventDisableTiming));
        LPE_HIP(ctx, hipHostMalloc((void **)&d->hc, sizeof(int32_t) * 16, 0));
        LPE_HIP(ctx, hipHostMalloc((void **)&d->hcr, sizeof(int32_t) * 32, 0));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d->evHc[0], hipEventDisableTiming));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d->evHc[1], hipEventDisableTiming));
    }
    if (d->lag) {
        // the previous tick's counts if they are in (a growth they ask for
        // then happens before this tick's detection)
        int st = rigid_lag_check(ctx, d, (int)((d->htick + 1u) & 1u), false);
        if (st) return st;
    }
    if (d->grow_pairs > d->cap_pairs || d->grow_contacts > d->cap_contacts) {
        // (asked for by a check: nothing in flight may use the old buffers)
        int st = d->lag ? rigid_lag_drain(ctx, d) : LPE_OK;
        if (st) return st;
        LPE_HIP(ctx, hipStreamSynchronize(d->side));
        if (d->psolve) LPE_HIP(ctx, hipStreamSynchronize(d->psolve));
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (d->grow_pairs > d->cap_pairs && (st = rigid_alloc_pairs(ctx, d, d->grow_pairs))) return st;
        if (d->grow_contacts > d->cap_contacts && (st = rigid_alloc_contacts(ctx, d, d->grow_contacts)))
            return st;
        d->regrows++;
    }
    d->grow_pairs = d->grow_contacts = 0;
    if (d->lag_next) {                        // a synchronous tick left 4x headroom
        d->lag = true;
        d->lag_next = false;
    }
    hipStream_t s = ctx->stream;
    d->det = on_main ? s : d->side;
    static const bool evwaits = getenv("LPE_EVENT_WAITS") != nullptr;
    if (!evwaits) {
        int st = tsync_alloc(ctx, d);          // (the first time: the concurrency probe)
        if (st) return st;
        d->tsyncTick++;                        // (this tick's signals carry its number)
    }
    if (d->det != s && device_waits(d))         // (the detection's start: the clamp's last workgroup signals it)
        LPE_KERNEL(ctx, "k_boundary_pos", k_boundary_pos, dim3(rblk(d->nb)), dim3(RTPB), 0, s, d->nb, d->bodies,
                   c.marginPixels * c.metersPerPixel, c.universeSize, d->bbits, d->tsync, d->tsyncTick);
    else if (d->det != s)                      // (or its launch carries the event)
        LPE_KERNEL_SIGNAL(ctx, "k_boundary_pos", d->evStart, k_boundary_pos, dim3(rblk(d->nb)), dim3(RTPB), 0, s,
                          d->nb, d->bodies, c.marginPixels * c.metersPerPixel, c.universeSize, d->bbits,
                          (uint32_t *)nullptr, 0u);
    else
        LPE_KERNEL(ctx, "k_boundary_pos", k_boundary_pos, dim3(rblk(d->nb)), dim3(RTPB), 0, s, d->nb, d->bodies,
                   c.marginPixels * c.metersPerPixel, c.universeSize, d->bbits, (uint32_t *)nullptr, 0u);
    d->detect_launched = false;
    d->overlap_pending = true;
    return LPE_OK;
}

// The detection's launches on the side stream (after the boundary clamp).
// Issued from the fluid step's hook once its first sub-step is enqueued: the
// ~25 calls take the host ~150 us, and issued first they left the context
// stream without work for that long at every tick start.
static int rigid_tick_launch(lpe_ctx *ctx, RigidDev *d) {
    if (d->detect_launched) return LPE_OK;
    if (d->det != ctx->stream) {
        if (device_waits(d)) {
            int st = wait_flag(ctx, d, d->det, d->tsync + 2, d->tsyncTick);
            if (st) return st;
        } else {
            LPE_HIP(ctx, hipStreamWaitEvent(d->det, d->evStart, 0));
        }
    }
    if (d->lag) {
        // lagged: the compaction follows at once and the counts go to a ring
        // slot, checked when the slot comes round again (two ticks later)
        const int slot = (int)(d->htick & 1u);
        int st = rigid_lag_check(ctx, d, slot, true);
        if (st) return st;
        st = detect_launch(ctx, d, 0, nullptr, d->det, d->hcr + 16 * slot, true);
        if (st) return st;
        LPE_HIP(ctx, hipEventRecord(d->evHc[slot], d->det));
        d->hpend[slot] = true;
        d->htick++;
    } else {
        int st = detect_launch(ctx, d, 0, nullptr, d->det, d->hc);
        if (st) return st;
        LPE_HIP(ctx, hipEventRecord(d->evDetect, d->det));   // (the host waits on it: rigid_tick_detect)
    }
    d->detect_launched = true;
    return LPE_OK;
}

// Fluid-step hook, after each sub-step's forces are enqueued: the detection
// launches after sub-step 0, its host half and the colouring after sub-step
// 2 (the detection has finished on the device by then, so the host does not
// wait); step < 0: everything at once.
int rigid_tick_hook(lpe_ctx *ctx, int step) {
    RigidDev *d = rdev(ctx);
    if (d->nb <= 0 || !d->overlap_pending) return LPE_OK;
    int st = rigid_tick_launch(ctx, d);
    if (st) return st;
    if (step < 0 || step >= 2) st = rigid_tick_detect(ctx);
    return st;
}

// stream `s` waits for this tick's boundary/gravity pass (false: there is
// no device signal this tick; the caller waits on rigid_boundary_event)
int rigid_boundary_wait(lpe_ctx *ctx, hipStream_t s, bool *done) {
    RigidDev *d = rdev(ctx);
    *done = false;
    if (d->nb <= 0 || !d->bvgSignal || !device_waits(d)) return LPE_OK;
    *done = true;
    return wait_flag(ctx, d, s, d->tsync, d->tsyncTick);
}

// the event the world tick's boundary/gravity pass signalled this tick, or null
hipEvent_t rigid_boundary_event(lpe_ctx *ctx) {
    RigidDev *d = rdev(ctx);
    return d->nb > 0 && d->bvgSignal ? d->evBvg : nullptr;
}

// the boundary system's velocity part, at its place in the tick
int rigid_tick_boundary(lpe_ctx *ctx, bool gravity, double dt_state) {
    RigidDev *d = rdev(ctx);
    if (d->nb <= 0) return LPE_OK;
    const lpe_rigid_config &c = d->cfg;
    if (gravity) {   // the planetary-mass check (k_gravity_check) is queued before
        if (!d->evBvg) LPE_HIP(ctx, hipEventCreateWithFlags(&d->evBvg, hipEventDisableTiming));
        if (device_waits(d) && d->tsync)
            LPE_KERNEL(ctx, "k_boundary_vel_gravity", k_boundary_vel_gravity, dim3(rblk(d->nb)), dim3(RTPB), 0,
                       ctx->stream, d->nb, d->bodies, d->bbits, c.bounceDamping, c.maxSpeed, c.gravity, dt_state,
                       d->counts + 5, d->tsync, d->tsyncTick);
        else
            LPE_KERNEL_SIGNAL(ctx, "k_boundary_vel_gravity", d->evBvg, k_boundary_vel_gravity, dim3(rblk(d->nb)),
                              dim3(RTPB), 0, ctx->stream, d->nb, d->bodies, d->bbits, c.bounceDamping, c.maxSpeed,
                              c.gravity, dt_state, d->counts + 5, (uint32_t *)nullptr, 0u);
        d->bvgSignal = true;
        return LPE_OK;
    }
    LPE_KERNEL(ctx, "k_boundary_vel", k_boundary_vel, dim3(rblk(d->nb)), dim3(RTPB), 0, ctx->stream, d->nb,
               d->bodies, d->bbits, c.bounceDamping, c.maxSpeed);
    return LPE_OK;
}

// The host half of the detection (its counts decide whether the pair buffer
// must grow and how many contacts there are), then the colouring on the side
// stream.  The world tick calls this from inside the fluid step, after its
// first sub-steps are queued, so the host waits on the detection while the
// device is busy with the fluid and the colouring runs beside the rest of it.
int rigid_tick_detect(lpe_ctx *ctx) {
    RigidDev *d = rdev(ctx);
    if (d->nb <= 0 || d->colour_pending) return LPE_OK;
    if (!d->overlap_pending) {
        ctx->err = "rigid_tick_detect without rigid_tick_begin";
        return LPE_ERR_STATE;
    }
    int st0 = rigid_tick_launch(ctx, d);
    if (st0) return st0;
    d->overlap_pending = false;
    int st;
    if (d->lag) {
        // no host wait: the colouring and the preparation take the counts
        // from the device (an empty tick colours nothing and solves nothing)
        st = solver_streams(ctx, d);
        if (!st) st = solver_lds_check(ctx, d);
        if (!st) st = colour_launch(ctx, d, d->det);
        if (!st) st = colour_prep(ctx, d, d->det);
        if (st) return st;
        if (d->det != ctx->stream) LPE_HIP(ctx, hipEventRecord(d->evColour, d->det));
        d->colour_pending = true;
        return LPE_OK;
    }
    LPE_HIP(ctx, hipEventSynchronize(d->evDetect));
    int retry = 0;
    st = detect_finish(ctx, d, d->det, d->hc, &retry);
    if (st) return st;
    if (retry) {                     // the pair buffer grew: detect again (rare)
        st = rigid_detect(ctx, d, 0, nullptr, d->det);
        if (st) return st;
    }
    // the next ticks check their counts after the fact once the buffers have
    // 4x headroom (striped solver only); else grow them at the next tick start
    if (striped()) {
        if (4 * d->last_np <= d->cap_pairs && 4 * d->last_nc <= d->cap_contacts) {
            d->lag_next = true;
        } else {
            d->grow_pairs = std::max(d->cap_pairs, 4 * d->last_np + 1024);
            d->grow_contacts = std::max(d->cap_contacts, 4 * d->last_nc + 4096);
        }
    }
    st = solver_streams(ctx, d);
    if (st) return st;
    if (d->last_nc > 0) {
        // the velocity-independent preparation runs here, beside the fluid
        // step: colouring, contact marks, PGS rows, position items
        st = solver_lds_check(ctx, d);
        if (!st) st = colour_launch(ctx, d, d->det);
        if (!st) st = colour_prep(ctx, d, d->det);
        if (st) return st;
    }
    if (d->det != ctx->stream)
        LPE_HIP(ctx, hipEventRecord(d->evColour, d->det));   // everything on the side stream
    d->colour_pending = true;
    return LPE_OK;
}

int rigid_tick_finish(lpe_ctx *ctx) {
    RigidDev *d = rdev(ctx);
    if (d->nb <= 0) return LPE_OK;
    int st = rigid_tick_detect(ctx);          // (already done inside the fluid step)
    if (st) return st;
    d->colour_pending = false;
    hipStream_t s = ctx->stream;
    const bool joinColour = d->det != s;       // (detected on the context stream: in order already)
    if (!d->lag && d->last_nc == 0) {         // early out (rigid_body_collision.cpp:35-37)
        if (joinColour) LPE_HIP(ctx, hipStreamWaitEvent(s, d->evColour, 0));
        if (d->pcol && d->last_np > 0)
            LPE_HIP(ctx, hipMemsetAsync(d->pcol, 0xff, sizeof(int32_t) * d->last_np, s));
        LPE_HIP(ctx, hipMemsetAsync(d->counts + 8, 0, sizeof(int32_t), s));
        return LPE_OK;
    }
    // the two solvers, concurrently: the PGS after the fluid, boundary and
    // gravity systems set the velocities, the position solver beside it on
    // the detection stream (idle by now; the solver stream shares a hardware
    // queue with the next tick's prelaunch, which then delayed it).  (Run
    // during the fluid step instead, the one-workgroup position solver slows
    // the full-chip fluid kernels by more than it saves.)
    if (joinColour) LPE_HIP(ctx, hipStreamWaitEvent(s, d->evColour, 0));
    if (d->bvgSignal && joinColour) {
        // (the boundary/gravity pass is the context stream's last rigid work
        // before the solvers, and the side stream is past the colouring; a
        // detection on the context stream runs after that pass: recorded)
        if (device_waits(d)) {
            st = wait_flag(ctx, d, d->side, d->tsync, d->tsyncTick);
            if (st) return st;
        } else {
            LPE_HIP(ctx, hipStreamWaitEvent(d->side, d->evBvg, 0));
        }
    } else {
        LPE_HIP(ctx, hipEventRecord(d->evFork, s));
        LPE_HIP(ctx, hipStreamWaitEvent(d->side, d->evFork, 0));
    }
    d->bvgSignal = false;
    st = colour_pos(ctx, d, d->side);
    if (st) return st;
    LPE_HIP(ctx, hipEventRecord(d->evJoin, d->side));
    st = colour_pgs(ctx, d, s);
    if (st) return st;
    LPE_HIP(ctx, hipStreamWaitEvent(s, d->evJoin, 0));
    return LPE_OK;
}

extern "C" int lpe_rigid_step_ordered(lpe_ctx *ctx, int np, const int32_t *pairs, int nc_order,
                                      const int32_t *pgs_order, lpe_rigid_stats *stats) {
    if (!ctx || np < 0 || (np > 0 && !pairs)) return LPE_ERR_ARG;
    return rigid_step_impl(ctx, np, pairs ? pairs : (const int32_t *)"", nc_order, pgs_order, stats);
}

extern "C" int lpe_rigid_integrate(lpe_ctx *ctx, int systems, double dt_state, double dt_move) {
    if (!ctx) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    int nb = d->nb;
    if (nb <= 0) return LPE_OK;
    const lpe_rigid_config &c = d->cfg;
    hipStream_t s = ctx->stream;
    if (systems & 1)
        LPE_KERNEL(ctx, "k_boundary", k_boundary, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, c.marginPixels * c.metersPerPixel, c.universeSize, c.bounceDamping, c.maxSpeed);
    if (systems & (2 | 32)) {   // 32: planetary-mass check only (world tick)
        // gravity.cpp:43-51 scans every tick; its inputs (gravity view flags,
        // masses) change only by lpe_rigid_upload / lpe_rigid_set_config, so
        // the result is kept until then
        if (!d->heavy_valid) {
            LPE_HIP(ctx, hipMemsetAsync(d->counts + 5, 0, sizeof(int32_t), s));
            LPE_KERNEL(ctx, "k_gravity_check", k_gravity_check, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, c.planetaryMassThreshold, d->counts + 5);
            d->heavy_valid = true;
        }
    }
    if (systems & 2) {
        LPE_KERNEL(ctx, "k_gravity", k_gravity, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, c.gravity, dt_state, d->counts + 5);
    }
    if ((systems & (4 | 8 | 16)) == (4 | 8 | 16)) {
        LPE_KERNEL(ctx, "k_rotation_movement_sleep", k_rotation_movement_sleep, dim3(rblk(nb)), dim3(RTPB), 0, s, nb,
                   d->bodies, dt_state, c.angularDamping, c.maxAngularSpeed, dt_move, c.linearSleepThreshold,
                   c.angularSleepThreshold, c.sleepFramesThreshold);
        systems &= ~(4 | 8 | 16);
    }
    if (systems & 4)
        LPE_KERNEL(ctx, "k_rotation", k_rotation, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, dt_state, c.angularDamping, c.maxAngularSpeed);
    if (systems & 8)
        LPE_KERNEL(ctx, "k_movement", k_movement, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, dt_move);
    if (systems & 16)
        LPE_KERNEL(ctx, "k_sleep", k_sleep, dim3(rblk(nb)), dim3(RTPB), 0, s, nb, d->bodies, c.linearSleepThreshold, c.angularSleepThreshold, c.sleepFramesThreshold);
    LPE_CHECK_LAUNCH(ctx, "integrate");
    return LPE_OK;
}

extern "C" int lpe_rigid_download(lpe_ctx *ctx, lpe_body *bodies) {
    if (!ctx || !bodies) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    if (d->nb > 0)
        LPE_HIP(ctx, hipMemcpyAsync(bodies, d->bodies, sizeof(lpe_body) * d->nb, hipMemcpyDeviceToHost, ctx->stream));
    int32_t fault = 0;
    if (d->counts)
        LPE_HIP(ctx, hipMemcpyAsync(&fault, d->counts + 7, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (fault) {
        ctx->err = watchdog_msg(fault);
        return LPE_ERR_OVERFLOW;
    }
    return d->lag ? rigid_lag_drain(ctx, d) : LPE_OK;       // (the ticks checked after the fact)
}

extern "C" int lpe_rigid_download_contacts(lpe_ctx *ctx, int pair_cap, int32_t *pairs,
                                           int contact_cap, lpe_contact *contacts, int32_t *np,
                                           int32_t *nc) {
    if (!ctx) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    hipStream_t s = ctx->stream;
    if (d->lag) {                             // the last tick's counts (lagged checks)
        LPE_HIP(ctx, hipStreamSynchronize(s));
        int st = rigid_lag_drain(ctx, d);
        if (st) return st;
    }
    if (np) *np = d->last_np;
    if (nc) *nc = d->last_nc;
    if (pairs && d->last_np > 0)
        LPE_HIP(ctx, hipMemcpyAsync(pairs, d->pairs, sizeof(int2) * std::min(pair_cap, d->last_np), hipMemcpyDeviceToHost, s));
    if (contacts && d->last_nc > 0)
        LPE_HIP(ctx, hipMemcpyAsync(contacts, d->contacts, sizeof(lpe_contact) * std::min(contact_cap, d->last_nc), hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipStreamSynchronize(s));
    return LPE_OK;
}

extern "C" int lpe_rigid_download_impulses(lpe_ctx *ctx, int cap, float *lamN, float *lamF, int32_t *nc_out) {
    if (!ctx || cap < 0) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    hipStream_t s = ctx->stream;
    LPE_HIP(ctx, hipStreamSynchronize(s));
    if (d->lag) {
        int st = rigid_lag_drain(ctx, d);
        if (st) return st;
    }
    const int nc = d->last_nc;
    if (nc_out) *nc_out = nc;
    if (nc <= 0 || cap <= 0 || !d->lamN) return LPE_OK;
    // rows are in the solver's order: row t holds contact order[t] (the
    // Jacobi solver keeps them by contact)
    std::vector<int32_t> ord(nc);
    for (int t = 0; t < nc; t++) ord[t] = t;
    std::vector<float> ln(nc), lf(nc);
    if (!d->lam_by_contact)
        LPE_HIP(ctx, hipMemcpyAsync(ord.data(), d->order, sizeof(int32_t) * nc, hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipMemcpyAsync(ln.data(), d->lamN, sizeof(float) * nc, hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipMemcpyAsync(lf.data(), d->lamF, sizeof(float) * nc, hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipStreamSynchronize(s));
    for (int t = 0; t < nc; t++) {
        const int k = ord[t];
        if (k < 0 || k >= std::min(cap, nc)) continue;
        if (lamN) lamN[k] = ln[t];
        if (lamF) lamF[k] = lf[t];
    }
    return LPE_OK;
}

extern "C" int lpe_rigid_download_colours(lpe_ctx *ctx, int cap, int32_t *pair_colour, int32_t *ncolours) {
    if (!ctx || cap < 0) return LPE_ERR_ARG;
    RigidDev *d = rdev(ctx);
    hipStream_t s = ctx->stream;
    if (d->lag) {
        LPE_HIP(ctx, hipStreamSynchronize(s));
        int st = rigid_lag_drain(ctx, d);
        if (st) return st;
    }
    int32_t nc = 0;
    if (d->counts) LPE_HIP(ctx, hipMemcpyAsync(&nc, d->counts + 8, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (pair_colour && d->pcol && d->last_np > 0 && cap > 0)
        LPE_HIP(ctx, hipMemcpyAsync(pair_colour, d->pcol, sizeof(int32_t) * std::min(cap, d->last_np), hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipStreamSynchronize(s));
    if (ncolours) *ncolours = nc;
    return LPE_OK;
}
