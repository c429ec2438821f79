// lpe_sph.hip — SPH fluid step of the MI355X backend (Systems::FluidSystem).
//
// Replaces the 9 Metal kernels of src/systems/fluid/fluid_kernels.metal and the
// host orchestration of src/systems/fluid/fluid.cpp:582-1021 with a
// device-resident pipeline over particle state kept in cell-sorted order:
//
//   per sub-step (fluid.cpp:598-950):
//     k_kick_drift   velocityVerletHalf (metal:408-423) + bin key + histogram
//                    (wave-aggregated atomics) + per-block bbox partials
//                    (metal:446-514)
//     k_scan_*       exclusive scan of the bin histogram; the bbox finish
//                    (fluid.cpp:440-494) and the reference grid
//                    (fluid.cpp:717-752) are computed on device, no host sync
//     k_scatter      new slot per particle (wave-aggregated atomics)
//     k_rank_permute canonical order inside each bin + permutation of the
//                    state into the new sorted order
//     k_density      computeDensity (metal:246-307)
//     k_forces_couple computeForces (metal:312-403) + velocityVerletFinish
//                    (metal:428-441) + rigidFluidImpulseSolver (metal:679-924)
//                    + rigidFluidPositionSolver (metal:533-668), fused per particle
//   per tick:
//     k_rbin_*       rigids binned by AABB (rigids are frozen during the
//                    sub-steps, fluid.cpp:953-955): a particle tests only the
//                    rigids of its bin, in ascending rigid index
//     k_rigid_writeback  writeBackRigidBodies arithmetic (fluid.cpp:545-562)
//
// Bins are (reference 2h cell, h-sized quadrant).  The stencil walk visits the
// 3x3 reference cells row-major (metal:272-283) and each cell's quadrants
// row-major, ascending particle index inside a quadrant: the canonical order
// of oracle/sph_oracle.c.  Quadrants farther than h from the particle are
// skipped; they can only hold particles with r^2 >= h^2, which the reference
// discards (metal:291, :365), so the sums are unchanged bit for bit.
//
// The "not inserted" rule (metal:231-234: a particle in a cell outside the
// per-sub-step grid is in no cell list) is reproduced exactly: bins live on a
// fixed absolute grid and every stencil walk skips cells outside the
// reference grid [gridMin, gridMin + dim).
//
// Numerics: fp32, no FMA contraction (-ffp-contract=off), correctly rounded
// division and sqrt, tanh/pow via fp64 rounded once; with the canonical orders
// above the fluid state is bit-identical to the oracle.  The rigid
// accumulators (float atomics in the reference, metal:892-898) are exact
// fixed-point sums rounded once (sph_coupling.h): deterministic, and equal
// to the oracle's bit for bit.
#include <cstdlib>
#include "lpe_internal.h"
#include "sph_coupling.h"
#include "lpe_trace.h"
#include "lpe_transport.h"
#include <cmath>
#include <cstring>
#include <vector>
#include <algorithm>

namespace lpe {

static constexpr float PI_F = 3.14159265358979323846f;  // metal:17 evaluated in fp32
static constexpr int TPB = 256;
static constexpr int SCAN_ELEMS = 1024;   // elements per scan block (256 thr x 4)
static constexpr int MAX_KICK_BLOCKS = 2048;
static constexpr int NLIST_CAP = 128;     // neighbours kept per particle (column-major list)
static constexpr int NL_OFFS = 1 << 30;   // ncount flag: the list holds slot offsets k - s (else LDS indices)
static constexpr int FCAP = 1024;         // records of the forces pass's LDS image (k_forces_couple)

// kernel coefficients (metal:19-38), fp32
__device__ __forceinline__ float poly6Coeff2D(float h) {
    float h2 = h * h; float h4 = h2 * h2; float h8 = h4 * h4;
    return 4.0f / (PI_F * h8);
}
__device__ __forceinline__ float spikyCoeff2D(float h) {
    float h2 = h * h; float h4 = h2 * h2; float h5 = h4 * h;
    return -30.0f / (PI_F * h5);
}
__device__ __forceinline__ float viscLaplacianCoeff2D(float h) {
    float h2 = h * h; float h4 = h2 * h2; float h5 = h4 * h;
    return 40.0f / (PI_F * h5);
}

// ---------------------------------------------------------------------------
// wave helpers (wave64)
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Run-length aggregation of equal consecutive keys inside a wave.  Returns the
// lane that starts this lane's run; *runlen is set on run-start lanes.
__device__ __forceinline__ int wave_runs(uint32_t k, bool active, int *runlen, bool *is_start) {
    int lane = lane_id();
    uint32_t prev = __shfl_up(k, 1);
    int prev_active = __shfl_up((int)active, 1);
    bool st = active && (lane == 0 || prev != k || !prev_active);
    unsigned long long starts = __ballot(st);
    unsigned long long act = __ballot(active);
    unsigned long long stop = starts | ~act;
    unsigned long long above = (lane == 63) ? 0ull : (stop & (~0ull << (lane + 1)));
    int next = above ? __ffsll((long long)above) - 1 : 64;
    unsigned long long below = starts & ((lane == 63) ? ~0ull : ((1ull << (lane + 1)) - 1));
    int first = below ? 63 - __clzll(below) : lane;
    *runlen = next - lane;
    *is_start = st;
    return first;
}

// ---------------------------------------------------------------------------
// The kicked half-step state (x, y, vh after velocityVerletHalf) lives in
// scratch arrays (the S staging arrays x, y, vx, vy, dead inside a sub-step)
// until the permute copies it into the sorted records; P itself is rewritten
// only by the forces pass.  So the primary state is untouched until a
// sub-step's forces run: a sub-step prelaunched up to its density can be
// discarded at any time (sph_void_prelaunch).
struct KState { float *x, *y, *vhx, *vhy; };

// velocityVerletHalf (metal:408-423) of one particle from its state, and the
// bin key of the kicked position ((cell, quadrant) of the device grid)
__device__ __forceinline__ void kick_one(float x, float y, float vx, float vy, float ax, float ay, float dt,
                                         float hdt, float &px, float &py, float &hx, float &hy) {
    hx = vx + hdt * ax;
    hy = vy + hdt * ay;
    px = x + hx * dt;
    py = y + hy * dt;
}
__device__ __forceinline__ uint32_t bin_key(float px, float py, float eps, float cs, int ox, int oy, int W, int H,
                                            int32_t *__restrict__ status, int *okx = nullptr, int *oky = nullptr) {
    float tx = (px + eps) / cs, ty = (py + eps) / cs;
    int gx = (int)floorf(tx), gy = (int)floorf(ty);
    int qx = (int)floorf(2.0f * tx) - 2 * gx;
    int qy = (int)floorf(2.0f * ty) - 2 * gy;
    int kx = gx - ox, ky = gy - oy;
    if (kx < 0 || kx >= W || ky < 0 || ky >= H) {
        atomicOr(&status[ST_CAP_OVERFLOW], 1);
        kx = min(max(kx, 0), W - 1);
        ky = min(max(ky, 0), H - 1);
    }
    if (okx) { *okx = kx; *oky = ky; }
    return (((uint32_t)ky * (uint32_t)W + (uint32_t)kx) << 2) | (uint32_t)(qy * 2 + qx);
}
// the block's bbox partial (exact: min/max are order independent); every
// thread of the TPB-thread block calls it
__device__ __forceinline__ void bbox_partial(float mnx, float mxx, float mny, float mxy, float4 *__restrict__ out) {
    for (int off = 32; off > 0; off >>= 1) {
        mnx = fminf(mnx, __shfl_xor(mnx, off));
        mxx = fmaxf(mxx, __shfl_xor(mxx, off));
        mny = fminf(mny, __shfl_xor(mny, off));
        mxy = fmaxf(mxy, __shfl_xor(mxy, off));
    }
    __shared__ float4 wb[TPB / 64];
    if (lane_id() == 0) wb[threadIdx.x >> 6] = make_float4(mnx, mxx, mny, mxy);
    __syncthreads();
    if (threadIdx.x == 0) {
        float4 b = wb[0];
        for (int w = 1; w < TPB / 64; w++) {
            b.x = fminf(b.x, wb[w].x); b.y = fmaxf(b.y, wb[w].y);
            b.z = fminf(b.z, wb[w].z); b.w = fmaxf(b.w, wb[w].w);
        }
        *out = b;
    }
}

// Row totals for the next sub-step's scan (single domain): besides the bin
// histogram the kick counts the particles of every device-grid row, so that
// k_scan_rows scans a row per block with no tile-total pass.  Summed in LDS
// over 8 rows from a base row near the block's particles (a block's
// particles are a run of the sorted order: one or two rows), other rows
// directly.  The totals alternate between two buffers by the scan's parity
// (k_scan_rows clears the other one).
struct FastKick {
    int on;
    int32_t *rowtot;          // [H] particles per device row
    int32_t *bucket;          // [bins][BKT_CAP] particle ids by bin (k_bucket_permute), or null
    int32_t *ovf;             // the parity's overflow list: count, -, -, -, then (bin, id, arrival, -)
    int ovfcap;               // its entries (the particle capacity: it cannot overflow)
};

// The in-bin order without a scatter pass: the kick's atomic on its bin's
// count returns the particle's arrival index there, and the id is filed
// under the bin at that index (the first BKT_CAP of a bin).  Later arrivals
// go to an overflow list (bin, id, arrival) that k_scan_rows places at
// tmpId[start[bin] + arrival] once it has the bin's start; k_bucket_permute
// then ranks a particle among its bin's ids directly.  The list is
// double-buffered by the scan's parity (k_scan_rows clears the other one).
static constexpr int BKT_CAP = 32;
__device__ __forceinline__ void bucket_file(const FastKick &fk, uint32_t k, int a, int id,
                                            int32_t *__restrict__ status) {
    if (a < BKT_CAP) {
        fk.bucket[(size_t)k * BKT_CAP + a] = id;
    } else {
        const int e = atomicAdd(&fk.ovf[0], 1);
        if (e < fk.ovfcap) ((int4 *)(fk.ovf + 4))[e] = make_int4((int)k, id, a, 0);
        else atomicOr(&status[ST_BUCKET_OVERFLOW], 1);
    }
}

// x-slab decomposition (the slab section below): a slab rank's kick files
// the particles bound for a neighbour -- kicked into, or past, the
// SLAB_BAND cell columns along an edge -- as ghost records in that
// neighbour's send buffer.
static constexpr int SLAB_BAND = 2;                  // ghost cell columns each side of an edge
// ... in the reference cell-capacity mode: more, the cells the reference's
// literal loop reads on into past an over-full cell of the relevant columns
// (ref_cap_walk, metal:281-283): a cell of K > 64 particles reads
// ceil((K - 64) / 65) cells further.  The sender files SLAB_BAND_CAP columns
// plus that many for the largest cell seen so far (ST_MAX_OCC_TOTAL, one
// column of margin), at most SLAB_BAND_MAX, and tells the receiver in the
// wire header how many it sent (slab_band).
static constexpr int SLAB_BAND_CAP = 3;
static constexpr int SLAB_BAND_MAX = 8;
static constexpr uint32_t KEY_DEAD = 0xFFFFFFFFu;    // a slot the sub-step drops (no bin)
struct SlabKick {
    int on;
    const int32_t *edges;     // device [nranks + 1] edge cell columns
    int rank, hasL, hasR;
    int band;                 // ghost columns filed each side (SLAB_BAND, or SLAB_BAND_CAP at least)
    const int32_t *occ;       //   capped cells: the largest cell so far (ST_MAX_OCC_TOTAL), else null
    int32_t *rband;           //   [2]: the columns the left / right neighbour sent last (k_ghost_unpack)
    float *sL, *sR;           // send buffers: HDR header floats, then wcap records of GREC floats
    int wcap;
    const int32_t *nslot;     // k_kick_drift: the P slots in use
};
// the ghost columns this sub-step files each side (wave-uniform); every
// block that files records its band in the wire header's word [1] as
// SLAB_BAND_MAX - band by an atomic max, so the receiver learns the fewest
// columns any block sent completely (0, the cleared header: no block filed,
// the sender has no particle there -- all SLAB_BAND_MAX columns are empty)
__device__ __forceinline__ int slab_band(const SlabKick &sk) {
    if (!sk.occ) return sk.band;
    const int K = __builtin_amdgcn_readfirstlane(*sk.occ);
    const int extra = K > LPE_REF_MAX_PER_CELL ? (K - LPE_REF_MAX_PER_CELL + LPE_REF_MAX_PER_CELL) / 65 : 0;
    return min(SLAB_BAND_MAX, sk.band + extra);
}
__device__ __forceinline__ void slab_band_note(const SlabKick &sk, int band) {
    if (threadIdx.x != 0) return;
    if (sk.hasL) atomicMax((int *)sk.sL + 1, SLAB_BAND_MAX - band);
    if (sk.hasR) atomicMax((int *)sk.sR + 1, SLAB_BAND_MAX - band);
}
// wave-aggregated append of this lane's particle to the send buffers of the
// sides it is bound for (gx: its kicked bin's column, band: slab_band); every
// lane of the wave calls it
__device__ __forceinline__ void slab_file(const SlabKick &sk, int band, int cx0, int cx1, bool active, int gx, float px,
                                          float py, float vx, float vy, float hx, float hy, float ms, int id,
                                          int32_t *__restrict__ status) {
    const int lane = lane_id();
    for (int side = 0; side < 2; side++) {
        const bool go = active && (side == 0 ? (sk.hasL && gx < cx0 + band) : (sk.hasR && gx >= cx1 - band));
        const unsigned long long bal = __ballot(go);
        if (!bal) continue;
        float *buf = side == 0 ? sk.sL : sk.sR;
        const int leader = __ffsll((long long)bal) - 1;
        int b = 0;
        if (lane == leader) b = atomicAdd((int *)buf, __popcll(bal));
        b = __shfl(b, leader);
        if (!go) continue;
        const int k = b + __popcll(bal & ((1ull << lane) - 1ull));
        if (k < sk.wcap) {
            float4 *r = (float4 *)(buf + 4 + (size_t)k * 8);        // (HDR, GREC)
            r[0] = make_float4(px, py, vx, vy);
            r[1] = make_float4(hx, hy, ms, __int_as_float(id));
        } else {
            atomicOr(&status[ST_HALO_OVERFLOW], 1);
        }
    }
}
__device__ __forceinline__ void slab_cols(const SlabKick &sk, int &cx0, int &cx1) {
    cx0 = sk.hasL ? sk.edges[sk.rank] : -(1 << 29);
    cx1 = sk.hasR ? sk.edges[sk.rank + 1] : (1 << 29);
}

// The next sub-step's kick, fused into the forces pass of the current one
// (sub-steps 1..numSubSteps-1 of a single-domain tick): the finished state
// of a particle is exactly what k_kick_drift would read back from P.
struct KickNext {
    int on;
    float dt, hdt, eps, cs;
    int ox, oy, W, H;
    float *kx, *ky, *kvhx, *kvhy;     // KState
    uint32_t *key;
    int32_t *count;
    float4 *bboxPart;                 // one partial per forces block
    FastKick fk;                      // the next sub-step's one-pass sort (fk.on)
    SlabKick sk;                      // slab rank: the ghost records of the next sub-step
};

// k_kick_drift: velocityVerletHalf + bin key + histogram + bbox partials.
// first != 0: first sub-step of a tick; the gather set a = 0 (fluid.cpp:289-290).
__global__ void __launch_bounds__(TPB)
k_kick_drift(int n, float dt, float hdt, int first, int probe, float eps, float cs,
             int ox, int oy, int W, int H, PState P, KState K, uint32_t *__restrict__ key,
             int32_t *__restrict__ count, float4 *__restrict__ bboxPart,
             int32_t *__restrict__ status, FastKick fk, SlabKick sk) {
    if (fk.on && blockIdx.x == 0 && threadIdx.x == 0) status[ST_NOT_INSERTED] = 0;   // (k_scan_rows adds)
    float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
    const int stride = gridDim.x * TPB;
    const int iters = (n + stride - 1) / stride;
    // a slab rank: its P slots in use (sk.nslot), the dead ones (id -1) skipped
    const int nn = sk.on ? min(*sk.nslot, n) : n;
    int cx0 = 0, cx1 = 0, band = 0;
    if (sk.on) {
        slab_cols(sk, cx0, cx1);
        band = slab_band(sk);
        slab_band_note(sk, band);                           // (the receiver's reach)
    }
    for (int it = 0; it < iters; it++) {
        int i = it * stride + blockIdx.x * TPB + threadIdx.x;
        bool active = i < nn;
        uint32_t k = 0xFFFFFFFFu;
        float px = 0.f, py = 0.f, hx = 0.f, hy = 0.f, vx = 0.f, vy = 0.f, ms = 0.f;
        int id = -1, kx = 0;
        if (active && sk.on) {
            id = P.id[i];
            if (id < 0) {
                key[i] = KEY_DEAD;
                active = false;
            }
        }
        if (active) {
            if (probe) {
                px = P.x[i]; py = P.y[i];
            } else {
                vx = P.vx[i]; vy = P.vy[i];
                kick_one(P.x[i], P.y[i], vx, vy, first ? 0.f : P.ax[i], first ? 0.f : P.ay[i], dt, hdt,
                         px, py, hx, hy);
                K.vhx[i] = hx; K.vhy[i] = hy;
            }
            K.x[i] = px; K.y[i] = py;
            int ky;
            k = bin_key(px, py, eps, cs, ox, oy, W, H, status, &kx, &ky);
            key[i] = k;
            mnx = fminf(mnx, px); mxx = fmaxf(mxx, px);
            mny = fminf(mny, py); mxy = fmaxf(mxy, py);
            if (sk.on) ms = P.m[i];
        }
        if (sk.on) slab_file(sk, band, cx0, cx1, active, kx + ox, px, py, vx, vy, hx, hy, ms, id, status);
        int len; bool st;
        const int first = wave_runs(k, active, &len, &st);
        if (fk.on && fk.bucket) {
            int base = 0;
            if (st) base = atomicAdd(&count[k], len);
            base = __shfl(base, first);
            if (active) bucket_file(fk, k, base + lane_id() - first, P.id[i], status);
        } else if (st) {
            atomicAdd(&count[k], len);
        }
        if (fk.on) {                       // row totals: base row from the chunk's first particle
            __shared__ int ltab[8], lbase;
            const int row = active ? (int)((k >> 2) / (uint32_t)W) : -1;
            if (threadIdx.x < 8) ltab[threadIdx.x] = 0;
            if (threadIdx.x == 0) lbase = row - 3;
            __syncthreads();
            const int rowBase = lbase;
            (void)wave_runs((uint32_t)row, active, &len, &st);
            if (st) {
                const int t = row - rowBase;
                if (t >= 0 && t < 8) atomicAdd(&ltab[t], len);
                else atomicAdd(&fk.rowtot[row], len);
            }
            __syncthreads();
            if (threadIdx.x < 8 && ltab[threadIdx.x]) atomicAdd(&fk.rowtot[rowBase + threadIdx.x], ltab[threadIdx.x]);
            __syncthreads();
        }
    }
    bbox_partial(mnx, mxx, mny, mxy, bboxPart + blockIdx.x);
}

// ---------------------------------------------------------------------------
// the reference grid from the particle bbox (fluid.cpp:440-494, :717-752)
__device__ __forceinline__ GridParams grid_from_bbox(float minX, float maxX, float minY, float maxY, float cs) {
    if (minX > maxX) { float t = minX; minX = maxX; maxX = t; }
    if (minY > maxY) { float t = minY; minY = maxY; maxY = t; }
    minX -= 1e-6f;
    minY -= 1e-6f;
    GridParams g;
    g.cellSize = cs;
    g.gridMinX = (int)floorf(minX / cs);
    g.gridMinY = (int)floorf(minY / cs);
    g.gridMaxX = (int)floorf(maxX / cs);
    g.gridMaxY = (int)floorf(maxY / cs);
    g.gridDimX = g.gridMaxX - g.gridMinX + 1;
    g.gridDimY = g.gridMaxY - g.gridMinY + 1;
    if (g.gridDimX < 1) g.gridDimX = 1;
    if (g.gridDimY < 1) g.gridDimY = 1;
    return g;
}

// The reference grid clipped to the device grid [ox, ox + W) x [oy, oy + H).
// The device grid covers the particles' bbox with a margin (sph_plan_grid,
// lpe_sph_cover_box, grown by the lagged checks of sph_lag_service), so the
// clip is the identity in every sub-step the reference semantics hold.  A
// reference grid past it means a particle left the device grid (its bin was
// clamped to the edge by bin_key): the sub-step raises ST_CAP_OVERFLOW (the
// call fails with LPE_ERR_CAPACITY), and every walk, which clips to g, stays
// inside the bins that exist -- no access outside the grid's buffers.  A
// slab rank (slab != 0) clips only in y: its reference grid is the global
// one (every rank's bbox) while its device grid covers only its slab's
// columns and the ghost bands (lpe_sph_cover_box), and the reference
// cell-capacity mode's flat cell order needs the global columns -- the walks
// that could leave the device grid in x clip to it themselves (hood_spans,
// walk_ranges, ref_cap_walk / ref_cap_slow).
__device__ __forceinline__ GridParams clip_grid(GridParams g, int ox, int oy, int W, int H, int slab, bool *clipped) {
    const int x0 = slab ? g.gridMinX : max(g.gridMinX, ox), y0 = max(g.gridMinY, oy);
    const int x1 = slab ? g.gridMinX + g.gridDimX - 1 : min(g.gridMinX + g.gridDimX - 1, ox + W - 1);
    const int y1 = min(g.gridMinY + g.gridDimY - 1, oy + H - 1);
    const bool cx = x0 != g.gridMinX || x1 != g.gridMinX + g.gridDimX - 1;
    const bool cy = y0 != g.gridMinY || y1 != g.gridMinY + g.gridDimY - 1;
    *clipped = cx || cy;
    if (!cx && !cy) return g;
    g.gridMinX = x0; g.gridMinY = y0;
    g.gridMaxX = max(x1, x0); g.gridMaxY = max(y1, y0);
    g.gridDimX = g.gridMaxX - x0 + 1; g.gridDimY = g.gridMaxY - y0 + 1;
    return g;
}

// The sub-step's over-full reference cells (more than GPU_MAX_PER_CELL = 64,
// fluid.hpp:56), listed by the scan as absolute (cell x, cell y): in the
// reference cell-capacity mode a particle takes the literal capped walk only
// if one of its 3x3 cells is listed (ref_cap_near), so a sub-step with none
// costs the mode one uniform load per particle.  [0] = count (beyond
// OVL_CAP: every particle checks its cells' counts, ref_cap_slow), then
// pairs.  Two lists alternate by scan (the scan clears the next one).
static constexpr int OVL_CAP = 1024;
static constexpr int OVL_WORDS = 2 + 2 * OVL_CAP;
__device__ __forceinline__ void ovl_append(int32_t *__restrict__ ovl, int gx, int gy) {
    const int e = atomicAdd(&ovl[0], 1);
    if (e < OVL_CAP) { ovl[2 + 2 * e] = gx; ovl[3 + 2 * e] = gy; }
}

// ---------------------------------------------------------------------------
// scan
__device__ __forceinline__ int wave_incl_scan(int v) {
    int lane = lane_id();
    for (int off = 1; off < 64; off <<= 1) {
        int t = __shfl_up(v, off);
        if (lane >= off) v += t;
    }
    return v;
}

// block-wide exclusive scan of one int per thread (TPB threads); returns total
__device__ __forceinline__ int block_excl_scan(int v, int *total) {
    __shared__ int wsum[TPB / 64];
    int lane = lane_id(), w = threadIdx.x >> 6;
    int incl = wave_incl_scan(v);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int off = 0, tot = 0;
    for (int k = 0; k < TPB / 64; k++) { if (k < w) off += wsum[k]; tot += wsum[k]; }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}

__global__ void __launch_bounds__(TPB)
k_scan_reduce(int C, const int32_t *__restrict__ cnt, int32_t *__restrict__ bsum, int32_t *__restrict__ status,
              int32_t *__restrict__ ovl, int32_t *__restrict__ ovlNext) {
    if (status && blockIdx.x == 0 && threadIdx.x == 0) status[ST_NOT_INSERTED] = 0;   // (fused scan)
    if (ovl && blockIdx.x == 0 && threadIdx.x == 0) { ovl[0] = 0; ovlNext[0] = 0; }  // (k_scan_final appends)
    int base = blockIdx.x * SCAN_ELEMS;
    int s = 0;
    for (int k = 0; k < 4; k++) {
        int c = base + k * TPB + threadIdx.x;
        if (c < C) s += cnt[c];
    }
    int tot;
    (void)block_excl_scan(s, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// one block: scan the block sums; if gp != null, finish the bbox from the
// partials (fluid.cpp:440-494) and derive the reference grid (fluid.cpp:717-752)
__global__ void __launch_bounds__(TPB)
k_scan_blocks(int nb, int32_t *__restrict__ bsum, int32_t *__restrict__ start_last,
              const float4 *__restrict__ bboxPart, int nparts, float cs,
              GridParams *__restrict__ gp, int32_t *__restrict__ status,
              const float4 *__restrict__ bbG, int ox, int oy, int W, int H) {
    int carry = 0;
    for (int b0 = 0; b0 < nb; b0 += TPB) {
        int b = b0 + threadIdx.x;
        int v = (b < nb) ? bsum[b] : 0;
        int tot;
        int ex = block_excl_scan(v, &tot);
        if (b < nb) bsum[b] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *start_last = carry;
    if (!gp) return;
    float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
    if (bbG && threadIdx.x == 0) {
        // slab decomposition: the all-reduced bbox of every rank's particles
        // (stored as minX, minY, -maxX, -maxY for one MIN all-reduce)
        float4 b = *bbG;
        mnx = b.x; mny = b.y; mxx = -b.z; mxy = -b.w;
    }
    for (int p = threadIdx.x; p < (bbG ? 0 : nparts); p += TPB) {
        float4 b = bboxPart[p];
        mnx = fminf(mnx, b.x); mxx = fmaxf(mxx, b.y);
        mny = fminf(mny, b.z); mxy = fmaxf(mxy, b.w);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mnx = fminf(mnx, __shfl_xor(mnx, off));
        mxx = fmaxf(mxx, __shfl_xor(mxx, off));
        mny = fminf(mny, __shfl_xor(mny, off));
        mxy = fmaxf(mxy, __shfl_xor(mxy, off));
    }
    __shared__ float4 wb[TPB / 64];
    if (lane_id() == 0) wb[threadIdx.x >> 6] = make_float4(mnx, mxx, mny, mxy);
    __syncthreads();
    if (threadIdx.x == 0) {
        float4 b = wb[0];
        for (int w = 1; w < TPB / 64; w++) {
            b.x = fminf(b.x, wb[w].x); b.y = fmaxf(b.y, wb[w].y);
            b.z = fminf(b.z, wb[w].z); b.w = fmaxf(b.w, wb[w].w);
        }
        bool clipped;
        *gp = clip_grid(grid_from_bbox(b.x, b.y, b.z, b.w, cs), ox, oy, W, H, bbG != nullptr, &clipped);
        if (clipped) atomicOr(&status[ST_CAP_OVERFLOW], 2);
        status[ST_NOT_INSERTED] = 0;
    }
}

// final scan pass; one thread = 4 consecutive bins = one reference cell when
// the bins are the (cell, quadrant) bins of the fluid (do_stats).
// fused (the fluid hash, few tiles): bsum holds the raw tile totals and each
// block derives its own prefix, the total and the reference grid from the
// bbox partials itself (what k_scan_blocks computes once), block 0 storing
// gp and start[C] for the kernels after it: one launch fewer per sub-step
__global__ void __launch_bounds__(TPB)
k_scan_final(int C, int W, int ox, int oy, int32_t *__restrict__ cnt,
             const int32_t *__restrict__ bsum, int32_t *__restrict__ start,
             int32_t *__restrict__ cursor, GridParams *__restrict__ gp,
             int32_t *__restrict__ status, int do_stats, int fused, const float4 *__restrict__ bboxPart,
             int nparts, float gcs, const float4 *__restrict__ bbG, int32_t *__restrict__ ovl) {
    __shared__ int s_max, s_out, s_over;
    if (threadIdx.x == 0) { s_max = 0; s_out = 0; s_over = 0; }
    GridParams g{};
    int prefix = 0;
    if (fused) {
        const int nb = (C + SCAN_ELEMS - 1) / SCAN_ELEMS;
        int pre = 0, all = 0;
        for (int i = threadIdx.x; i < nb; i += TPB) {
            const int v = bsum[i];
            pre += i < (int)blockIdx.x ? v : 0;
            all += v;
        }
        float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
        if (bbG) {
            // slab decomposition: the all-reduced bbox of every rank's particles
            // (stored as minX, minY, -maxX, -maxY for one MIN all-reduce)
            const float4 b = *bbG;
            mnx = b.x; mny = b.y; mxx = -b.z; mxy = -b.w;
        } else if (fused == 1) {                  // (fused == 2: a plain prefix, no grid)
            for (int p = threadIdx.x; p < nparts; p += TPB) {
                const float4 b = bboxPart[p];
                mnx = fminf(mnx, b.x); mxx = fmaxf(mxx, b.y);
                mny = fminf(mny, b.z); mxy = fmaxf(mxy, b.w);
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            pre += __shfl_xor(pre, off);
            all += __shfl_xor(all, off);
            mnx = fminf(mnx, __shfl_xor(mnx, off));
            mxx = fmaxf(mxx, __shfl_xor(mxx, off));
            mny = fminf(mny, __shfl_xor(mny, off));
            mxy = fmaxf(mxy, __shfl_xor(mxy, off));
        }
        __shared__ int wp[TPB / 64], wa[TPB / 64];
        __shared__ float4 wb[TPB / 64];
        if (lane_id() == 0) {
            wp[threadIdx.x >> 6] = pre;
            wa[threadIdx.x >> 6] = all;
            wb[threadIdx.x >> 6] = make_float4(mnx, mxx, mny, mxy);
        }
        __syncthreads();
        float4 b = wb[0];
        pre = wp[0]; all = wa[0];
        for (int w = 1; w < TPB / 64; w++) {
            pre += wp[w]; all += wa[w];
            b.x = fminf(b.x, wb[w].x); b.y = fmaxf(b.y, wb[w].y);
            b.z = fminf(b.z, wb[w].z); b.w = fmaxf(b.w, wb[w].w);
        }
        bool clipped = false;
        if (fused == 1 || bbG)
            g = clip_grid(grid_from_bbox(b.x, b.y, b.z, b.w, gcs), ox, oy, W, C / (4 * W), bbG != nullptr, &clipped);
        prefix = pre;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (fused == 1) *gp = g;
            if (clipped) atomicOr(&status[ST_CAP_OVERFLOW], 2);
            start[C] = all;
        }
    } else {
        __syncthreads();
        if (do_stats) g = *gp;
        prefix = bsum[blockIdx.x];
    }
    int base = blockIdx.x * SCAN_ELEMS + threadIdx.x * 4;
    int v[4];
    int s = 0;
    for (int k = 0; k < 4; k++) {
        int c = base + k;
        v[k] = (c < C) ? cnt[c] : 0;
        s += v[k];
    }
    if (do_stats && s > 0) {
        int cell = base >> 2;
        int gx = cell % W + ox, gy = cell / W + oy;
        // the reference grid excludes gx > gridMax (no epsilon on the max side,
        // fluid.cpp:745-746 vs metal:224-226): those particles are "not inserted"
        bool in = gx >= g.gridMinX && gx < g.gridMinX + g.gridDimX &&
                  gy >= g.gridMinY && gy < g.gridMinY + g.gridDimY;
        if (in) atomicMax(&s_max, s); else atomicAdd(&s_out, s);
        if (in && s > LPE_REF_MAX_PER_CELL) {
            atomicAdd(&s_over, 1);
            if (ovl) ovl_append(ovl, gx, gy);
        }
    }
    int tot;
    int ex = block_excl_scan(s, &tot) + prefix;
    for (int k = 0; k < 4; k++) {
        int c = base + k;
        if (c < C) { start[c] = ex; cursor[c] = ex; cnt[c] = 0; }
        ex += v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_max) { atomicMax(&status[ST_MAX_OCC], s_max); atomicMax(&status[ST_MAX_OCC_TOTAL], s_max); }
        if (s_out) atomicAdd(&status[ST_NOT_INSERTED], s_out);
        if (s_over) { atomicAdd(&status[ST_OVER_CAP], s_over); atomicAdd(&status[ST_OVER_CAP_TOTAL], s_over); }
    }
}

// new slot per particle: slot = cursor[bin]++ (wave-aggregated)
__global__ void __launch_bounds__(TPB)
k_scatter(int n, const uint32_t *__restrict__ key, const int32_t *__restrict__ id,
          int32_t *__restrict__ cursor, int32_t *__restrict__ tmpId,
          int32_t *__restrict__ tmpOld, const int32_t *__restrict__ nptr) {
    int i = blockIdx.x * TPB + threadIdx.x;
    bool active = i < (nptr ? *nptr : n);
    uint32_t k = active ? key[i] : KEY_DEAD;
    active = active && k != KEY_DEAD;          // (slab rank: a dropped slot)
    int len; bool st;
    int first = wave_runs(k, active, &len, &st);
    int base = 0;
    if (st) base = atomicAdd(&cursor[k], len);
    base = __shfl(base, first);
    if (active) {
        int slot = base + (lane_id() - first);
        if ((unsigned)slot >= (unsigned)(nptr ? *nptr : n)) return;   // (never: the bins hold every particle)
        tmpId[slot] = id[i];
        tmpOld[slot] = i;
    }
}

// canonical order inside a bin (ascending particle id) + state permutation
// P -> sorted slots.  The neighbour loops read packed records: nbA = (x, y, m,
// -) written here; nbB = (vx, vy | rho, p/rho^2), first half written here,
// second half by k_density.
__global__ void __launch_bounds__(TPB)
k_rank_permute(int n, const uint32_t *__restrict__ key, const int32_t *__restrict__ start,
               const int32_t *__restrict__ tmpId, const int32_t *__restrict__ tmpOld,
               PState P, KState K, PState S, float4 *__restrict__ nbA, float2 *__restrict__ nbB,
               int probe, const int32_t *__restrict__ nptr, int32_t *__restrict__ refInv, int W,
               int32_t *__restrict__ clearCnt) {
    int s = blockIdx.x * TPB + threadIdx.x;
    if (s >= (nptr ? *nptr : n)) return;
    int o = tmpOld[s];
    int myid = tmpId[s];
    uint32_t k = key[o];
    int b = start[k], e = start[k + 1];
    int rank = 0;
    for (int j = b; j < e; j++) rank += (tmpId[j] < myid) ? 1 : 0;
    int d = b + rank;
    // .w: the bin's (cell row - oy) << 17 | (cell column - ox) << 2 | quadrant
    // (the density pass reads a slot's cell and quadrant row from it)
    const uint32_t cl = k >> 2, cyr = cl / (uint32_t)W, cxr = cl - cyr * (uint32_t)W;
    nbA[d] = make_float4(K.x[o], K.y[o], P.m[o], __int_as_float((int)((cyr << 17) | (cxr << 2) | (k & 3))));
    nbB[2 * d] = make_float2(P.vx[o], P.vy[o]);
    S.id[d] = myid;
    if (refInv) refInv[myid] = d;         // reference cell-capacity mode: id -> sorted slot
    if (!probe) { S.vhx[d] = K.vhx[o]; S.vhy[d] = K.vhy[o]; }
    if (clearCnt) clearCnt[k] = 0;  // (k_scan_rows leaves the counts for the next kick to find zeroed)
}

// k_scatter + k_rank_permute in one pass (single domain, the kick filed the
// ids by bin): thread o takes P slot o, ranks its id among its bin's ids
// (the bin's first BKT_CAP arrivals in the bucket, the rest in the overflow
// list) and writes the same records as k_rank_permute to slot start[bin] +
// rank.  Reads of P are coalesced; the writes land near o (a sub-step moves
// few particles to another bin).
__global__ void __launch_bounds__(TPB)
k_bucket_permute(int n, const int32_t *__restrict__ nptr, const uint32_t *__restrict__ key,
                 const int32_t *__restrict__ start, const int32_t *__restrict__ bucket,
                 const int32_t *__restrict__ tmpId, PState P, KState K, PState S, float4 *__restrict__ nbA,
                 float2 *__restrict__ nbB, int32_t *__restrict__ refInv, int W, int32_t *__restrict__ clearCnt,
                 int32_t *__restrict__ status) {
    const int o = blockIdx.x * TPB + threadIdx.x;
    if (o >= (nptr ? *nptr : n)) return;      // (slab rank: its own slots and the received ghosts)
    const uint32_t k = key[o];
    // the record's fields do not depend on the rank: loaded here, in flight
    // with the bin's bounds and filed ids
    const float kx = K.x[o], ky = K.y[o], pm = P.m[o], pvx = P.vx[o], pvy = P.vy[o];
    const float khx = K.vhx[o], khy = K.vhy[o];
    if (k == KEY_DEAD) return;                 // (slab rank: a slot the previous sub-step dropped)
    const int myid = P.id[o];
    const int b = start[k], nk = start[k + 1] - b;
    const int4 *bk = (const int4 *)(bucket + (size_t)k * BKT_CAP);
    int rank = 0;
    for (int j = 0; j < min(nk, BKT_CAP); j += 4) {
        const int4 q = bk[j >> 2];
        rank += (q.x < myid) + (j + 1 < nk && q.y < myid) + (j + 2 < nk && q.z < myid) + (j + 3 < nk && q.w < myid);
    }
    for (int j = b + BKT_CAP; j < b + nk; j++) rank += tmpId[j] < myid ? 1 : 0;   // (a full bin's later arrivals)
    if (rank >= nk) {              // (never: the bin's filed ids are its particles) fail loudly, write nothing
        atomicOr(&status[ST_BUCKET_OVERFLOW], 2);
        return;
    }
    const int d = b + rank;
    const uint32_t cl = k >> 2, cyr = cl / (uint32_t)W, cxr = cl - cyr * (uint32_t)W;
    nbA[d] = make_float4(kx, ky, pm, __int_as_float((int)((cyr << 17) | (cxr << 2) | (k & 3))));
    nbB[2 * d] = make_float2(pvx, pvy);
    S.id[d] = myid;
    if (refInv) refInv[myid] = d;
    S.vhx[d] = khx; S.vhy[d] = khy;
    clearCnt[k] = 0;
}

// ---------------------------------------------------------------------------
// k_scan_rows (single domain, FastKick): one launch replaces k_scan_reduce +
// k_scan_final.  One block per device-grid row.  Every block finishes the
// bbox and the reference grid from the kick's partials (as the fused
// k_scan_final) while its row's counts and the row totals below it are
// already in flight; rows outside the particles' rows +-2 (the device grid
// covers the universe in world mode and is mostly empty) only clear their
// entry of the other parity's row totals.  An active row's prefix is the sum
// of the kick's row totals of the active rows below it (no tile-total pass,
// no inter-block wait); its 4W bins are then scanned cell by cell into start
// and cursor with the reference-grid stats.  The counts are left for
// k_rank_permute to clear.  Bins outside the active rows are never read (the
// walks stay within a row of a particle's row; the last active row stores
// the end of its last bin).
static constexpr int SR_CELLS = 2 * TPB;   // cells a block loads before it knows its row is active
__global__ void __launch_bounds__(TPB)
k_scan_rows(int W, int H, int ox, int oy, float eps, const int32_t *__restrict__ cnt, int32_t *__restrict__ start,
            int32_t *__restrict__ cursor, const int32_t *__restrict__ rowtot, int32_t *__restrict__ rowtotNext,
            GridParams *__restrict__ gp, int32_t *__restrict__ status,
            const float4 *__restrict__ bboxPart, int nparts, float gcs, const int32_t *__restrict__ ovf,
            int ovfcap, int32_t *__restrict__ ovfNext, int32_t *__restrict__ tmpId, int32_t *__restrict__ ovl,
            int32_t *__restrict__ ovlNext, const float4 *__restrict__ bbG, int32_t *__restrict__ ntot, SlabKick sk) {
    const int r = (int)blockIdx.x;
    if (threadIdx.x == 0) rowtotNext[r] = 0;
    if (ovfNext && r == 0 && threadIdx.x == 0) ovfNext[0] = 0;
    if (ovlNext && r == 0 && threadIdx.x == 0) ovlNext[0] = 0;    // (the next scan's over-cap list)
    const int novf = ovf ? min(ovf[0], ovfcap) : 0;      // (in flight with the loads below)
    // everything the block needs is loaded up front (one round trip): the
    // row's first SR_CELLS cells, the row totals below it, the bbox partials
    int4 v[SR_CELLS / TPB];
#pragma unroll
    for (int u = 0; u < SR_CELLS / TPB; u++) {
        const int c = u * TPB + (int)threadIdx.x;
        v[u] = c < W ? *(const int4 *)(cnt + ((size_t)r * W + c) * 4) : make_int4(0, 0, 0, 0);
    }
    int pre = 0;
    for (int q = (int)threadIdx.x; q < r; q += TPB) pre += rowtot[q];     // (rows below the active ones hold 0)
    float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
    if (bbG) {                              // slab rank: every rank's particles (k_ghost_unpack)
        if (threadIdx.x == 0) { const float4 b = *bbG; mnx = b.x; mxx = b.y; mny = b.z; mxy = b.w; }
    } else {
        // (eight partials a thread in flight at once: the forces pass leaves
        // one per block, ~2,000 at the metric scene)
        for (int p0 = 0; p0 < nparts; p0 += 8 * TPB) {
            float4 bq[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int p = p0 + u * TPB + (int)threadIdx.x;
                bq[u] = p < nparts ? bboxPart[p] : make_float4(1e30f, -1e30f, 1e30f, -1e30f);
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                mnx = fminf(mnx, bq[u].x); mxx = fmaxf(mxx, bq[u].y);
                mny = fminf(mny, bq[u].z); mxy = fmaxf(mxy, bq[u].w);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        pre += __shfl_xor(pre, off);
        mnx = fminf(mnx, __shfl_xor(mnx, off));
        mxx = fmaxf(mxx, __shfl_xor(mxx, off));
        mny = fminf(mny, __shfl_xor(mny, off));
        mxy = fmaxf(mxy, __shfl_xor(mxy, off));
    }
    __shared__ float4 wb[TPB / 64];
    __shared__ int wsum[TPB / 64];
    __shared__ int s_max, s_out, s_over;
    if (lane_id() == 0) {
        wb[threadIdx.x >> 6] = make_float4(mnx, mxx, mny, mxy);
        wsum[threadIdx.x >> 6] = pre;
    }
    if (threadIdx.x == 0) { s_max = 0; s_out = 0; s_over = 0; }
    __syncthreads();
    float4 b = wb[0];
    pre = wsum[0];
    for (int w = 1; w < TPB / 64; w++) {
        b.x = fminf(b.x, wb[w].x); b.y = fmaxf(b.y, wb[w].y);
        b.z = fminf(b.z, wb[w].z); b.w = fmaxf(b.w, wb[w].w);
        pre += wsum[w];
    }
    bool clipped;
    const GridParams g = clip_grid(grid_from_bbox(b.x, b.y, b.z, b.w, gcs), ox, oy, W, H, bbG != nullptr, &clipped);
    // every particle's row is in [row(minY), row(maxY)] (bin_key's row is
    // monotone in y, and clamped to the device grid like these bounds); the
    // walks reach one row further, the reference cell-capacity walk stays
    // inside the reference grid
    const int ylo = min((int)floorf((b.z + eps) / gcs), g.gridMinY), yhi = max((int)floorf((b.w + eps) / gcs), g.gridMaxY);
    const int ry0 = max(min(max(ylo - oy, 0), H - 1) - 2, 0), ry1 = min(max(min(yhi - oy, H - 1), 0) + 2, H - 1);
    if (r < ry0 || r > ry1) return;
    if (r == ry0 && threadIdx.x == 0) {
        *gp = g;
        if (clipped) atomicOr(&status[ST_CAP_OVERFLOW], 2);
    }
    const int gy = r + oy;
    const bool rowIn = gy >= g.gridMinY && gy < g.gridMinY + g.gridDimY;
    // a slab rank's stats cover its own columns (the ghosts' are its neighbours')
    int ocx0 = -(1 << 29), ocx1 = 1 << 29;
    if (sk.on) slab_cols(sk, ocx0, ocx1);
    int tmax = 0, tout = 0, tover = 0;                 // this thread's cells' stats (reduced once at the end)
    for (int c0 = 0; c0 < W; c0 += TPB) {
        const int c = c0 + (int)threadIdx.x;
        const size_t base = ((size_t)r * W + c) * 4;
        int4 vv;
        if (c0 < SR_CELLS) {
            vv = v[0];
#pragma unroll
            for (int u = 1; u < SR_CELLS / TPB; u++) if (c0 == u * TPB) vv = v[u];
        } else {
            vv = c < W ? *(const int4 *)(cnt + base) : make_int4(0, 0, 0, 0);
        }
        const int sum = vv.x + vv.y + vv.z + vv.w;
        if (sum > 0) {
            // the reference grid excludes gx > gridMax (fluid.cpp:745-746 vs
            // metal:224-226): those particles are "not inserted"
            const int gx = c + ox;
            const bool in = rowIn && gx >= g.gridMinX && gx < g.gridMinX + g.gridDimX;
            const bool mine = gx >= ocx0 && gx < ocx1;
            if (!mine) {
            } else if (in) tmax = max(tmax, sum); else tout += sum;
            // (the over-full list covers a slab rank's ghost columns too: the
            // first ghost column's densities walk them)
            if (in && sum > LPE_REF_MAX_PER_CELL) {
                if (mine) tover++;
                if (ovl) ovl_append(ovl, gx, gy);
            }
        }
        int tot;
        int ex = block_excl_scan(sum, &tot) + pre;
        if (c < W) {
            const int4 st4 = make_int4(ex, ex + vv.x, ex + vv.x + vv.y, ex + vv.x + vv.y + vv.z);
            *(int4 *)(start + base) = st4;
            *(int4 *)(cursor + base) = st4;
        }
        pre += tot;
    }
    if (r == ry1 && threadIdx.x == 0) {
        start[(size_t)(r + 1) * W * 4] = pre;   // end of the last active bin
        if (ntot) *ntot = pre;                  // (slab rank: the sorted slots of the sub-step)
    }
    for (int off = 32; off > 0; off >>= 1) {
        tmax = max(tmax, __shfl_xor(tmax, off));
        tout += __shfl_xor(tout, off);
        tover += __shfl_xor(tover, off);
    }
    if (lane_id() == 0) {
        if (tmax) atomicMax(&s_max, tmax);
        if (tout) atomicAdd(&s_out, tout);
        if (tover) atomicAdd(&s_over, tover);
    }
    __syncthreads();
    if (novf > 0) {
        // the bucket's overflow entries of this row's bins to tmpId[start + arrival]
        // (k_bucket_permute reads a full bin's later arrivals there)
        const int4 *e = (const int4 *)(ovf + 4);
        for (int t = (int)threadIdx.x; t < novf; t += TPB) {
            const int4 v = e[t];
            if ((int)(((uint32_t)v.x >> 2) / (uint32_t)W) == r) tmpId[start[v.x] + v.z] = v.y;
        }
    }
    if (threadIdx.x == 0) {
        if (s_max) { atomicMax(&status[ST_MAX_OCC], s_max); atomicMax(&status[ST_MAX_OCC_TOTAL], s_max); }
        if (s_out) atomicAdd(&status[ST_NOT_INSERTED], s_out);
        if (s_over) { atomicAdd(&status[ST_OVER_CAP], s_over); atomicAdd(&status[ST_OVER_CAP_TOTAL], s_over); }
    }
}

// ---------------------------------------------------------------------------
// Canonical neighbour walk.  The reference visits the 3x3 reference cells of
// the particle row-major (metal:272-283); inside a cell our bins are the four
// h-quadrants row-major, ascending particle id inside a quadrant (the order of
// oracle/sph_oracle.c).  Only the quadrant columns/rows within `reach` (in
// quadrant units: 2h/cs widened by 0.2%) of the particle are walked; every
// quadrant left out holds only particles with r^2 >= h^2 in fp32, whose terms
// the reference discards (metal:291, :365), so the sums are unchanged bit for
// bit.  The walked quadrants always lie inside the particle's 3x3 cells, and
// cells outside the reference grid are skipped (not-inserted particles,
// metal:231-234).  Quadrants of one cell row and one cell are contiguous
// bins, so each (cell, quadrant row) is one contiguous slot range.
__device__ __forceinline__ int sel4(int4 v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// The walk issues every bin-boundary load of the (at most 3x3) cells up front
// and the candidate records U at a time, so a wave has many loads in flight
// (the loop is latency bound otherwise: one dependent L2 round trip per
// candidate).  ld(k, cy) loads candidate k's record (cy: the absolute cell
// row being walked), f(k, rec) consumes it; f is called in the canonical order.
// The candidate slot ranges of the walk in canonical order: f(b, e, cy) for
// each (cell, quadrant row) range [b, e) of absolute cell row cy.
template <class F>
__device__ __forceinline__ void walk_ranges(float xi, float yi, float eps, float cs, float reach,
                                            const GridParams &g, int W, int H, int ox, int oy,
                                            const int32_t *__restrict__ start, F f) {
    float u = 2.0f * ((xi + eps) / cs), v = 2.0f * ((yi + eps) / cs);
    int bx0 = (int)floorf(u - reach), bx1 = (int)floorf(u + reach);
    int by0 = (int)floorf(v - reach), by1 = (int)floorf(v + reach);
    // clipped to the reference grid and (a particle that left the device
    // grid raises ST_CAP_OVERFLOW in k_kick_drift) to the device grid
    int cxa = max(max(bx0 >> 1, g.gridMinX), ox);
    int cxb = min(min(bx1 >> 1, g.gridMinX + g.gridDimX - 1), ox + W - 1);
    int cya = max(max(by0 >> 1, g.gridMinY), oy);
    int cyb = min(min(by1 >> 1, g.gridMinY + g.gridDimY - 1), oy + H - 1);
    // every bin-boundary load of the (at most 3x3) cells is issued up front
    int4 q[3][3];
    int qn[3][3];
#pragma unroll
    for (int dy = 0; dy < 3; dy++)
#pragma unroll
        for (int dx = 0; dx < 3; dx++) {
            int cy = cya + dy, cx = cxa + dx;
            if (cy <= cyb && cx <= cxb) {
                int cbase = (((cy - oy) * W) + (cx - ox)) << 2;
                q[dy][dx] = *reinterpret_cast<const int4 *>(start + cbase);
                qn[dy][dx] = start[cbase + 4];
            } else {
                q[dy][dx] = make_int4(0, 0, 0, 0);
                qn[dy][dx] = 0;
            }
        }
#pragma unroll
    for (int dy = 0; dy < 3; dy++) {
        int cy = cya + dy;
        if (cy > cyb) break;
        int qya = max(by0 - 2 * cy, 0), qyb = min(by1 - 2 * cy, 1);
#pragma unroll
        for (int dx = 0; dx < 3; dx++) {
            int cx = cxa + dx;
            if (cx > cxb) break;
            int qxa = max(bx0 - 2 * cx, 0), qxb = min(bx1 - 2 * cx, 1);
            for (int qy = qya; qy <= qyb; qy++) {
                int i0 = qy * 2 + qxa, i1 = qy * 2 + qxb + 1;
                int b = sel4(q[dy][dx], i0);
                int e = (i1 == 4) ? qn[dy][dx] : sel4(q[dy][dx], i1);
                if (b < e) f(b, e, cy);
            }
        }
    }
}

// The walk over every candidate: the candidate records are loaded U at a time
// so a wave has many loads in flight (the loop is latency bound otherwise:
// one dependent L2 round trip per candidate).  ld(k, cy) loads candidate k's
// record (cy: the absolute cell row being walked), f(k, rec) consumes it; f
// is called once per candidate, in the canonical order.
template <int U, class L, class F>
__device__ __forceinline__ void walk_neighbours(float xi, float yi, float eps, float cs,
                                                float reach, const GridParams &g, int W, int H,
                                                int ox, int oy, const int32_t *__restrict__ start,
                                                L ld, F f) {
    walk_ranges(xi, yi, eps, cs, reach, g, W, H, ox, oy, start, [&](int b, int e, int cy) {
        for (int k = b; k < e; k += U) {
            decltype(ld(0, 0)) r[U];
#pragma unroll
            for (int j = 0; j < U; j++) r[j] = ld(min(k + j, e - 1), cy);
#pragma unroll
            for (int j = 0; j < U; j++)
                if (k + j < e) f(k + j, r[j]);
        }
    });
}

// XCD-aware block order: hardware block b runs on XCD b % 8; give each XCD a
// contiguous run of sorted slots so its L2 holds one spatial slab (and its
// halo) instead of the whole domain.  Launch xcd_grid(nb) blocks.
static constexpr int NXCD = 8;
__host__ __device__ __forceinline__ int xcd_grid(int nb) { return ((nb + NXCD - 1) / NXCD) * NXCD; }
__device__ __forceinline__ int xcd_block(int nb) {
    if ((int)blockIdx.x >= xcd_grid(nb)) return -1;   // (a grid sized for more blocks than are live)
    int per = (nb + NXCD - 1) / NXCD;
    int lb = (int)(blockIdx.x % NXCD) * per + (int)(blockIdx.x / NXCD);
    return lb < nb ? lb : -1;
}

// Chunked XCD order: runs of C consecutive blocks go to one XCD, the runs
// round robin over the XCDs (launch xcd_chunk_grid(nb, C) blocks).  A run's
// blocks share their halo rows in one L2, while a spatial cluster of heavy
// blocks longer than a run still spreads over several XCDs.
__host__ __device__ __forceinline__ int xcd_chunk_grid(int nb, int C) {
    return ((nb + NXCD * C - 1) / (NXCD * C)) * NXCD * C;
}
__device__ __forceinline__ int xcd_chunk_block(int nb, int C) {
    const int x = (int)(blockIdx.x % NXCD), k = (int)(blockIdx.x / NXCD);
    const int lb = (k / C) * (NXCD * C) + x * C + (k % C);
    return lb < nb ? lb : -1;
}

__device__ __forceinline__ float walk_reach(float h, float cs) {
    return (2.0f * h / cs) * 1.002f + 2e-3f;
}

// ---------------------------------------------------------------------------
// Reference cell-capacity mode (LPE_SPH_MODE_REF_CELL_CAP, include/lpe.h).
// The reference's grid buffer is, per reference cell c, 65 ints {count,
// indices[64]} (fluid.hpp:56-61), zeroed every sub-step (fluid.cpp:821-824):
// count is the cell's full population, indices its first 64 inserts
// (metal:237-240).  Our sorted slots ARE the canonical insertion order, so the
// buffer never needs to exist: its int at flat position 65 c + j is count(c)
// for j = 0, the id of the (j-1)-th slot of c for j - 1 < min(count, 64),
// else 0.  The readers loop k < count(c) over position 65 c + 1 + k
// unclamped (metal:281-283, :349-351), so past 64 they read the following
// cells' words, skipping values >= N.  A particle none of whose 3x3 cells
// exceeds 64 sees exactly its cells' members and takes the default walk
// (bit-identical); the others take this literal walk.
__device__ __forceinline__ int ref_cell_base(int c, const GridParams &g, int W, int ox, int oy) {
    const int cy = c / g.gridDimX, cx = c - cy * g.gridDimX;
    return (((cy + g.gridMinY - oy) * W) + (cx + g.gridMinX - ox)) << 2;
}

// does any of the particle's 3x3 reference cells hold more than 64?
__device__ __forceinline__ bool ref_cap_slow(float xi, float yi, float eps, const GridParams &g, int W, int ox,
                                             int oy, const int32_t *__restrict__ start) {
    const int cellX = (int)floorf((xi + eps) / g.cellSize) - g.gridMinX;
    const int cellY = (int)floorf((yi + eps) / g.cellSize) - g.gridMinY;
    bool over = false;
    for (int ny = -1; ny <= 1; ny++)
        for (int nx = -1; nx <= 1; nx++) {
            const int cx = cellX + nx, cy = cellY + ny;
            if (cx < 0 || cx >= g.gridDimX || cy < 0 || cy >= g.gridDimY) continue;
            if (cx + g.gridMinX < ox || cx + g.gridMinX >= ox + W) continue;   // (slab rank: no bins there)
            const int b = ref_cell_base(cy * g.gridDimX + cx, g, W, ox, oy);
            over |= start[b + 4] - start[b] > LPE_REF_MAX_PER_CELL;
        }
    return over;
}

// ref_cap_slow through the scan's over-cap list (ovl_append): gx, gy = the
// particle's absolute cell (its bin's, k_rank_permute's nbA.w)
__device__ __forceinline__ bool ref_cap_near(const int32_t *__restrict__ ovl, int gx, int gy, float xi, float yi,
                                             float eps, const GridParams &g, int W, int ox, int oy,
                                             const int32_t *__restrict__ start) {
    const int n = __builtin_amdgcn_readfirstlane(ovl[0]);
    if (n == 0) return false;
    if (n > OVL_CAP) return ref_cap_slow(xi, yi, eps, g, W, ox, oy, start);
    bool near = false;
    for (int k = 0; k < n; k++) {
        const int cx = ovl[2 + 2 * k], cy = ovl[3 + 2 * k];
        near |= abs(gx - cx) <= 1 && abs(gy - cy) <= 1;
    }
    return near;
}

// The reference's neighbour loop over its grid buffer (metal:272-291), in
// its order: for each of the 3x3 cells c (row-major, inside the reference
// grid) the words k < count(c) at flat position 65 c + 1 + k.  Words k < 64
// are the cell's first min(count, 64) members -- in canonical insertion
// order that is the contiguous slot range start(c) .. start(c) + min - 1,
// walked U records at a time; past 64 (an over-full cell) the loop reads on
// into the following cells' words: a count (read as an id), the next cell's
// first members, zeros of the memset buffer.  ld(slot) loads a record,
// f(slot, rec) consumes it, for every value read that is < n.
// On a slab rank (sk.on) the reference's buffer is the GLOBAL grid's, of
// which the rank holds its own columns and sk.band ghost columns each side
// (every particle of those cells): the cells the loop reads are the 3 x 3
// of the particle -- local for every particle whose density or forces the
// rank keeps (its own columns and the first ghost column each side, the
// "relevant" ones) -- and, past an over-full cell, the cells after it in
// the flat order: with SLAB_BAND_CAP ghost columns one more column is
// local; a read past that (a cell of more than 129, or the row wrap of the
// global grid's last column) raises ST_REF_SLAB for a relevant particle
// (the call fails: the rank cannot know the count of a cell it does not
// hold).  A value read as an id is a particle of the whole fluid (n = its
// global count); one that is not on the rank lies more than a column (2h)
// from every relevant particle, so its term is +0 / no neighbour: skipped,
// the sums unchanged.  nslot: the rank's sorted slots (refInv is validated
// against sid: stale entries of particles that left are never used).
template <int U, class L, class F>
__device__ void ref_cap_walk(float xi, float yi, float eps, const GridParams &g, int W, int ox, int oy,
                             const int32_t *__restrict__ start, const int32_t *__restrict__ sid,
                             const int32_t *__restrict__ refInv, int n, int32_t *__restrict__ status, L ld, F f,
                             const SlabKick &sk = SlabKick{}, int nslot = 0) {
    constexpr int CI = LPE_REF_MAX_PER_CELL + 1;
    const int cellX = (int)floorf((xi + eps) / g.cellSize) - g.gridMinX;
    const int cellY = (int)floorf((yi + eps) / g.cellSize) - g.gridMinY;
    const long C = (long)g.gridDimX * g.gridDimY;
    int lo = -(1 << 30), hi = 1 << 30;              // the rank's local columns (absolute)
    bool relevant = true;
    if (sk.on) {
        int cx0, cx1;
        slab_cols(sk, cx0, cx1);
        if (sk.hasL) lo = cx0 - sk.rband[0];
        if (sk.hasR) hi = cx1 + sk.rband[1] - 1;
        const int pc = cellX + g.gridMinX;
        relevant = pc >= cx0 - 1 && pc <= cx1;
    }
    // the bin base of reference cell (cx, cy) of the flat index
    auto base = [&](int cx, int cy) { return (((cy + g.gridMinY - oy) * W) + (cx + g.gridMinX - ox)) << 2; };
    for (int ny = -1; ny <= 1; ny++)
        for (int nx = -1; nx <= 1; nx++) {
            const int cx = cellX + nx, cy = cellY + ny;
            if (cx < 0 || cx >= g.gridDimX || cy < 0 || cy >= g.gridDimY) continue;
            if (cx + g.gridMinX < ox || cx + g.gridMinX >= ox + W) continue;   // (slab rank: no bins there)
            const int b0 = base(cx, cy);
            const int s0 = start[b0], count = start[b0 + 4] - s0;
            const int m = min(count, LPE_REF_MAX_PER_CELL);
            for (int k = 0; k < m; k += U) {
                decltype(ld(0)) r[U];
#pragma unroll
                for (int j = 0; j < U; j++) r[j] = ld(s0 + min(k + j, m - 1));
#pragma unroll
                for (int j = 0; j < U; j++)
                    if (k + j < m) f(s0 + k + j, r[j]);
            }
            if (count <= LPE_REF_MAX_PER_CELL) continue;
            // past the cell's 64 slots: words 65 (c + 1) + j of the cells after it
            long cc = (long)cy * g.gridDimX + cx + 1;
            int j = 0, ccx = cx + 1, ccy = cy, bb = 0, bcnt = 0;
            bool have = false;
            for (int k = CI - 1; k < count; k++) {
                int slot = -1, id = 0;
                if (cc >= C) {                                 // past the buffer: undefined
                    atomicOr(&status[ST_REF_UB], 1);
                } else {
                    if (!have) {
                        bool wrap = false;
                        if (ccx >= g.gridDimX) { ccx = 0; ccy++; wrap = true; }
                        const int col = ccx + g.gridMinX;
                        if (col < lo || col > hi) {             // (slab rank: a cell it does not hold)
                            if (relevant) atomicOr(&status[ST_REF_SLAB], wrap ? 2 : 1);
                            break;
                        }
                        bb = base(ccx, ccy);
                        bcnt = start[bb + 4] - start[bb];
                        have = true;
                    }
                    if (j == 0) id = bcnt;                                   // the next cell's count
                    else if (j - 1 < min(bcnt, LPE_REF_MAX_PER_CELL)) { slot = start[bb] + (j - 1); id = sid[slot]; }
                    // else 0: the memset buffer
                }
                if (++j == CI) { j = 0; cc++; ccx++; have = false; }
                if (id >= n) continue;
                if (slot < 0) {
                    slot = refInv[id];
                    if (sk.on && (slot < 0 || slot >= nslot || sid[slot] != id)) continue;   // (not on the rank)
                }
                f(slot, ld(slot));
            }
        }
}

// ---------------------------------------------------------------------------
// LDS-staged neighbourhoods.  A block owns HB consecutive sorted slots; in
// sorted order they cover one run of cells of one cell row, or the end of one
// row and the start of the next (unless the fluid is sparse).  Every record a
// walk of the block can touch then lies in <= 6 contiguous slot ranges ("row
// segments": rows cy-1..cy+1 of each run, one cell left and right of it).
// The block copies them into LDS with coalesced loads, together with the
// quadrant boundaries of every cell of those segments rebased to LDS offsets,
// so a walk reads nothing but LDS: the walk itself, and so every sum, is the
// canonical one.  The plan is computed by every wave from block-uniform loads
// (no serial section, one barrier).  A block whose neighbourhood does not fit
// walks global memory instead.
// Tile scheduling of the forces pass.  The rigid pile's tiles carry most of
// the coupling pairs (up to ~1400 against none for a median tile) and denser
// neighbour lists, so their blocks ended the launch 25-30 us after the median
// block, each wave alone on its SIMD (a round of 256 pairs takes ~5 us,
// latency-bound).  The density pass (same sub-step, same tiles) counts each
// particle's coupling pairs (the forces pass's AABB test on its rigid-bin
// candidates), finds the tile's quartiles of pairs over its slots, and files
// the tile by its total T:
//   T >= QUARTER_PAIRS: four part blocks (at most QUARTER_MAX tiles),
//   T >= HALF_PAIRS:    two part blocks  (at most HALF_MAX tiles),
//   T > 0:              one block, run whole (at most COUPLED_MAX tiles),
// a filing that finds its class full trying the next.  A part block takes
// the slots between two of the tile's pair quartiles (so the parts share the
// pairs, not the slots, evenly), stages the tile's image and runs its slots
// as a whole block would.  The forces grid is [quarters][halves][coupled]
// [every tile in order]: the costly blocks are dispatched first and the
// late-dispatched ones (beyond the resident blocks) are light tiles; a tile's
// own block exits when the tile was filed.  Every particle's arithmetic is
// the same (the fold order of its pairs is its own list's), so the results
// are bit-identical.  The lists alternate between two buffers by density
// pass; the forces pass that reads one clears the other's counts.  A filed
// block runs its tile only if the tile's flag holds its filing code and the
// list entry there is the tile (a stale entry is skipped: the tile's own
// block runs it), so every tile runs exactly once whatever the lists hold.
// LPE_NO_HEAVY=1: off (A/B).
static constexpr int QUARTER_PAIRS = 512, HALF_PAIRS = 256;
#ifndef LPE_QUARTER_MAX
#define LPE_QUARTER_MAX 128
#endif
#ifndef LPE_HALF_MAX
#define LPE_HALF_MAX 160
#endif
#ifndef LPE_COUPLED_MAX
#define LPE_COUPLED_MAX 160
#endif
static constexpr int QUARTER_MAX = LPE_QUARTER_MAX, HALF_MAX = LPE_HALF_MAX, COUPLED_MAX = LPE_COUPLED_MAX;
static constexpr int FILED_MAX = QUARTER_MAX + HALF_MAX + COUPLED_MAX;
// list: [0..2] the counts by class; then per filing code c (quarters c = 1 ..,
// halves c = QUARTER_MAX + 1 .., coupled c = QUARTER_MAX + HALF_MAX + 1 ..)
// two words at list[2 + 2c]: the tile, and its quartile slots (9 bits each)
static constexpr int HEAVY_WORDS = 4 + 2 * FILED_MAX;
struct HeavyOut {             // k_density<true>: where it files the heavy tiles
    int32_t *list;            //   [HEAVY_WORDS] of this pass's parity (null: off)
    int32_t *tile;            //   per tile: its list position + 1, or 0
    const int32_t *rbinStart; //   the rigid bins (candidates per bin)
    const float4 *rbinAabb;   //   and their AABBs in bin order (the pairs: AABB hits)
    float bcs;
    int bx0, by0, bW, bH;
    int qpairs, hpairs;       //   the classes' thresholds (QUARTER_PAIRS, HALF_PAIRS; LPE_HEAVY_Q / _H for A/B)
};
struct HeavyIn {              // k_forces_couple: the lists the density pass filed
    const int32_t *list;      //   (null: off)
    const int32_t *tile;
    int32_t *clearNext;       //   the other parity's list (its counts are cleared)
};
// the forces grid's filed blocks ahead of the tiles' own
static constexpr int QUARTER_BLOCKS = 4 * QUARTER_MAX, HALF_BLOCKS = 2 * HALF_MAX;
static constexpr int HEAVY_HEAD = QUARTER_BLOCKS + HALF_BLOCKS + COUPLED_MAX;

static constexpr int HB = 256;            // slots (threads) per staged block (4 waves: hood_stage)
static constexpr int HCAP = 1536;         // records staged per block (6 per thread)
static constexpr int HBND = 1280;         // staged cell boundaries per block (5 per thread)

// a sorted record's cell: its bin's (nbA.w, written by the permute), i.e.
// cell (floor((x + eps) / cs), floor((y + eps) / cs)) of its kicked position
// clamped to the device grid (bin_key) -- so a plan made from it never
// leaves the grid, even for a particle that did (ST_CAP_OVERFLOW)
__device__ __forceinline__ void bin_cell(const float4 &r, int ox, int oy, int &cx, int &cy) {
    const unsigned w = (unsigned)__float_as_int(r.w);
    cx = ox + (int)((w >> 2) & 0x7fffu);
    cy = oy + (int)(w >> 17);
}

struct Hood {
    bool ok;
    int nrun, cy0;            // runs (1 or 2: rows cy0, cy0 + 1)
    int L, NB;                // records, boundaries staged
    int ca[6], ss[6];         // per segment r * 3 + dy + 1: first cell column, first global slot
    int l[6], bb[6];          // LDS record offset; LDS offset of the first cell's boundaries
    int g0[6];                // global index of the first cell's first boundary
    int ncell[6];             // cells in the segment (0: none)
};

// the plan for slots [s0, s1) (s1 > s0); cells of the device grid [ox, ox+W) x [oy, oy+H)
__device__ __forceinline__ void hood_plan(Hood &hd, int s0, int s1, const float4 *__restrict__ nbA, float eps,
                                          float cs, int W, int H, int ox, int oy,
                                          const int32_t *__restrict__ start, int cap = HCAP, int bcap = HBND) {
    const float4 f = nbA[s0], l = nbA[s1 - 1];
    int cx0, cy0, cx1, cy1;
    bin_cell(f, ox, oy, cx0, cy0);
    bin_cell(l, ox, oy, cx1, cy1);
    int xa[2] = {cx0, 0}, xb[2] = {cx1, 0};
    hd.ok = true;
    hd.cy0 = cy0;
    if (cy1 == cy0) {
        hd.nrun = 1;
    } else if (cy1 == cy0 + 1 && cy1 - oy >= 0 && cy1 - oy < H) {
        // two runs: row cy0 from cx0 to the cell of the last slot before row
        // cy1, row cy1 from the cell of its first slot to cx1
        hd.nrun = 2;
        const int rs = start[((cy1 - oy) * W) << 2];        // first slot of row cy1 (> s0)
        const float4 e0 = nbA[rs - 1], b1 = nbA[rs];
        int t;
        bin_cell(e0, ox, oy, xb[0], t);
        bin_cell(b1, ox, oy, xa[1], t);
        xb[1] = cx1;
    } else {
        hd.ok = false;
        return;
    }
    int L = 0, NB = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
        const int r = i / 3, row = cy0 + r + (i % 3) - 1;
        const int ca = max(xa[r] - 1, ox), cb = min(xb[r] + 1, ox + W - 1);
        hd.l[i] = L;
        hd.bb[i] = NB;
        hd.ca[i] = ca;
        hd.ncell[i] = 0;
        hd.ss[i] = hd.g0[i] = 0;
        if (r < hd.nrun && row >= oy && row < oy + H && ca <= cb) {
            const int g0 = (((row - oy) * W) + ca - ox) << 2;
            const int ss = start[g0], se = start[((((row - oy) * W) + cb - ox) << 2) + 4];
            hd.ss[i] = ss;
            hd.g0[i] = g0;
            hd.ncell[i] = cb - ca + 1;
            L += se - ss;
            NB += 4 * (cb - ca + 1) + 1;                     // + the end sentinel
        }
    }
    hd.L = L;
    hd.NB = NB;
    hd.ok = L <= cap && NB <= bcap;
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glb_void_t;

// Copies the planned records and the cells' quadrant starts into LDS in one
// pass of asynchronous global -> LDS loads (global_load_lds: each lane's
// source address is its own, the destination the wave's base + lane * size):
// the records form one flat LDS array (segment i at l[i]), the boundaries
// another (segment i's cells at bb[i], 4 per cell + the segment end), kept
// as global slot numbers (a reader adds l[i] - ss[i]).  Every load of the
// block is in flight at once; the caller's __syncthreads() retires them.
// (Per-segment chunks of 64 instead of the flat index: fewer VALU per load
// but three times the SALU, measured slower.)
template <int NT = HB, int CAP = HCAP, int BCAP = HBND>
__device__ __forceinline__ void hood_stage(const Hood &hd, float4 *lrec, int *lbnd,
                                           const float4 *__restrict__ nbA,
                                           const int32_t *__restrict__ start, int s0) {
    const int wbase = threadIdx.x & ~63;
#pragma unroll
    for (int u = 0; u < CAP / NT; u++) {
        const int f0 = u * NT;
        if (f0 >= hd.L) break;
        const int f = f0 + threadIdx.x;
        int d = hd.ss[0] - hd.l[0];
#pragma unroll
        for (int i = 1; i < 6; i++)
            if (f >= hd.l[i]) d = hd.ss[i] - hd.l[i];
        const int src = f < hd.L ? f + d : s0;            // lanes past the end copy a valid record
        __builtin_amdgcn_global_load_lds((glb_void_t *)(nbA + src), (lds_void_t *)(lrec + f0 + wbase), 16, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < BCAP / NT; u++) {
        const int f0 = u * NT;
        if (f0 >= hd.NB) break;
        const int f = f0 + threadIdx.x;
        int d = hd.g0[0] - hd.bb[0];
#pragma unroll
        for (int i = 1; i < 6; i++)
            if (f >= hd.bb[i]) d = hd.g0[i] - hd.bb[i];
        const int src = f < hd.NB ? f + d : 0;
        __builtin_amdgcn_global_load_lds((glb_void_t *)(start + src), (lds_void_t *)(lbnd + f0 + wbase), 4, 0, 0);
    }
}

// min and max of v (0 <= v < 65536) over the wave, as wave-uniform values
// (every lane active): one xor-shuffle tree on the pair (v, 65535 - v)
typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void wave_minmax(int v, int &mn, int &mx) {
    ushort2v p = {(unsigned short)v, (unsigned short)(0xffff - v)};
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        unsigned u = __builtin_bit_cast(unsigned, p);
        unsigned o = (unsigned)__shfl_xor((int)u, m);
        p = __builtin_elementwise_max(p, __builtin_bit_cast(ushort2v, o));
    }
    mx = __builtin_amdgcn_readfirstlane((int)p.x);
    mn = __builtin_amdgcn_readfirstlane(0xffff - (int)p.y);
}

// The canonical walk over the staged neighbourhood, as one contiguous LDS
// span per cell row: from the first walked quadrant of the row's first cell
// to the end of the last walked quadrant of its last cell.  Slots are
// cell-major and quadrant-major inside a cell, so the span visits the walked
// candidates (walk_ranges) in the canonical order; the quadrants in between
// that the walk skips lie outside the reach box (more than h * 1.002 away in
// x or y), so their r^2 >= h^2: they add +0 to a density sum and are never
// neighbours.  Rows the particle does not reach get empty spans.  Span r
// covers LDS records [b[r], e[r]); shift[r] maps an LDS index to its slot.
// The quadrant ranges come from u = 2 (x + eps) / cs by a multiply with the
// rounded reciprocal, widened by a bound on its error (|u| 2^-20 + 1e-5 covers
// the product's rounding against the correctly rounded quotient): the walk is
// then a superset of walk_ranges' quadrants, which is bit-identical (every
// extra quadrant lies beyond h * 1.002, its terms are +0 and never
// neighbours), and costs no division.  A quadrant column of the superset is
// at most one past the exact one, so it stays inside the staged cells.
__device__ __forceinline__ void hood_spans(const Hood &hd, const int *lbnd, float xi, float yi, float eps,
                                           float cs, float reach, int cyp, const GridParams &g, int b[3],
                                           int e[3], int shift[3], int gx0, int gx1) {
    const float rcs = 2.0f / cs;
    const float u = (xi + eps) * rcs, v = (yi + eps) * rcs;
    const float wu = reach + fabsf(u) * 0x1p-20f + 1e-5f, wv = reach + fabsf(v) * 0x1p-20f + 1e-5f;
    const int bx0 = (int)floorf(u - wu), bx1 = (int)floorf(u + wu);
    const int by0 = (int)floorf(v - wv), by1 = (int)floorf(v + wv);
    // (and to the device grid's columns [gx0, gx1]: a slab rank's reference
    // grid is the global one, wider than its device grid)
    const int cxa = max(max(bx0 >> 1, g.gridMinX), gx0), cxb = min(min(bx1 >> 1, g.gridMinX + g.gridDimX - 1), gx1);
    const int cya = max(by0 >> 1, g.gridMinY), cyb = min(by1 >> 1, g.gridMinY + g.gridDimY - 1);
    const int r3 = (cyp == hd.cy0) ? 0 : 3;
    const int qa = max(bx0 - 2 * cxa, 0), qb = min(bx1 - 2 * cxb, 1);
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const int cy = cyp - 1 + r;
        b[r] = e[r] = shift[r] = 0;
        if (cy < cya || cy > cyb || cxa > cxb) continue;
        const int i = r3 + r;                                 // segment of this cell row
        const int qya = max(by0 - 2 * cy, 0), qyb = min(by1 - 2 * cy, 1);
        const int *c0 = lbnd + hd.bb[i] + 4 * (cxa - hd.ca[i]);
        const int *c1 = lbnd + hd.bb[i] + 4 * (cxb - hd.ca[i]);
        const int rebase = hd.l[i] - hd.ss[i];               // global slot -> LDS index
        b[r] = c0[qya * 2 + qa] + rebase;
        e[r] = c1[qyb * 2 + qb + 1] + rebase;                 // [4] is the next cell's start
        shift[r] = -rebase;
    }
}

// computeDensity (metal:246-307), one thread per sorted slot, HB slots per
// block with the neighbourhood staged in LDS.  NL: also write the neighbours
// of the forces pass (r^2 < h^2, not itself: metal:360-366) in the canonical
// walk order as int16 slot offsets k - s, eight to a uint4, column-major
// [NLIST_CAP / 8][nstride]: each thread collects eight offsets in its 16-byte
// LDS slot and writes them with one 16-byte store.  More than NLIST_CAP
// neighbours: ncount > NLIST_CAP and the forces pass walks the bins.
// fplans (NL only): the block's plan, for the forces pass to stage the same
// image; when that image fits the forces pass's LDS (L <= FCAP) the list
// holds LDS indices of the image instead of slot offsets, except for the
// particles whose list came from a global walk (ncount's NL_OFFS bit).
template <bool NL>
__global__ void __launch_bounds__(HB)
k_density(int n, const int32_t *__restrict__ nptr, int nstride, float h, float eps, float stiffness,
          float restDensity, int W, int H, int ox, int oy, const GridParams *__restrict__ gp,
          const int32_t *__restrict__ start, const float4 *__restrict__ nbA, float2 *__restrict__ nbB,
          float *__restrict__ rho, float *__restrict__ pr, uint4 *__restrict__ nlist,
          int32_t *__restrict__ ncount, int32_t *__restrict__ status, const int32_t *__restrict__ sid,
          const int32_t *__restrict__ refInv, const int32_t *__restrict__ ovl, Hood *__restrict__ fplans,
          HeavyOut ho, SlabKick sk, int nref) {
    __shared__ float4 lrec[HCAP + 4];                     // + 4: the span walk reads up to 3 past a span
    __shared__ int hcand[5];                              // (NL, ho.list: the waves' coupling pairs; quartiles)
    __shared__ int lbnd[HBND];
    __shared__ uint4 lnl[NL ? 2 * HB : 1];                // per thread: a ring of two groups of 8 entries
    // (a slab rank's grid is sized by its slot capacity: the XCD runs are laid
    // out over the slots in use, so every XCD gets its share)
    const int lb = xcd_block(((nptr ? min(*nptr, n) : n) + HB - 1) / HB);
    if (lb < 0) return;                                   // whole block idle
    const int nn = nptr ? *nptr : n;
    const int s0 = lb * HB, s1 = min(s0 + HB, nn);
    if (s0 >= s1) return;
    const int dtb = NL ? lb : 4096;           // (trace builds: the tile's stamp slots; the tick's pass only)
    (void)dtb;
    DTRCLR();
    DTR(0);
    DTRHW();
    const GridParams g = *gp;
    const float cs = g.cellSize;
    // the tile filing's candidate range (HeavyOut), loaded before the walk so
    // that its latency hides behind it
    int hk0 = 0, hk1 = 0;
    if (NL && ho.list && s0 + (int)threadIdx.x < s1) {
        const float4 m0 = nbA[s0 + threadIdx.x];
        const float fbx = fminf(fmaxf(floorf(m0.x / ho.bcs) - (float)ho.bx0, 0.f), (float)(ho.bW - 1));
        const float fby = fminf(fmaxf(floorf(m0.y / ho.bcs) - (float)ho.by0, 0.f), (float)(ho.bH - 1));
        const int bin = (int)fby * ho.bW + (int)fbx;
        hk0 = ho.rbinStart[bin]; hk1 = ho.rbinStart[bin + 1];
    }
    __shared__ Hood hd;                                   // (LDS: the walks index it per lane)
    {
        Hood p;
        hood_plan(p, s0, s1, nbA, eps, cs, W, H, ox, oy, start);
        if (p.ok) hood_stage(p, lrec, lbnd, nbA, start, s0);
        if (threadIdx.x == 0) {
            hd = p;
            if (NL && fplans) fplans[lb] = p;
            hcand[4] = 0;
        }
    }
    __syncthreads();
    DTR(1);
    DTRSET(6, hd.L);
    // the list as LDS indices of the forces pass's image (block-uniform)
    const bool lidx = NL && fplans && hd.ok && hd.L <= FCAP;
    // every lane stays to the end (the span walk's trip counts are wave
    // reductions); lanes past the block's last slot walk nothing
    const int s = s0 + threadIdx.x;
    const bool live = s < s1;
    const int sl = live ? s : s1 - 1;
    if (!hd.ok && threadIdx.x == 0) atomicAdd(&status[ST_STAGE_FALLBACK], 1);
    const float4 me = nbA[sl];
    const float xi = me.x, yi = me.y;
    const int cyp = oy + (int)((unsigned)__float_as_int(me.w) >> 17);   // the bin's cell row (k_rank_permute)
    const float h2 = h * h;
    const float poly6 = poly6Coeff2D(h);
    const float reach = walk_reach(h, cs);
    float acc = 0.0f;
    int cnt = 0;
    int16_t *ring = reinterpret_cast<int16_t *>(&lnl[NL ? 2 * threadIdx.x : 0]);
    // the ring's group g, as one 16-byte word
    auto group = [&](int g) { return lnl[NL ? 2 * threadIdx.x + (g & 1) : 0]; };
    // one candidate: r^2 < h^2 adds m * poly6 (h^2 - r^2)^3; otherwise +0,
    // which leaves the non-negative sum unchanged bit for bit
    auto term = [&](const float4 &o, bool valid) {
        const float dx = xi - o.x, dy = yi - o.y;
        const float r2 = dx * dx + dy * dy;
        const float diff = h2 - r2;
        const float w = poly6 * diff * diff * diff;
        const float t = o.z * w;
        const bool in = valid && r2 < h2;
        acc += in ? t : 0.0f;
        return in;
    };
    // the same sum without the neighbour test: max(h^2 - r^2, 0) is h^2 - r^2
    // inside and +0 outside, where the term is then m * (+0) = +0
    auto term0 = [&](const float4 &o, bool valid) {
        const float dx = xi - o.x, dy = yi - o.y;
        const float r2 = dx * dx + dy * dy;
        const float diff = fmaxf(h2 - r2, 0.0f);
        const float t = o.z * (poly6 * diff * diff * diff);
        acc += valid ? t : 0.0f;
    };
    // a neighbour for the forces pass (its image index or slot offset k - s)
    auto emit = [&](int code, bool ok) {
        if (cnt < NLIST_CAP && ok) {
            ring[cnt & 15] = (int16_t)code;
            if ((cnt & 7) == 7) nlist[(size_t)(cnt >> 3) * nstride + s] = group(cnt >> 3);
        } else {
            cnt = NLIST_CAP;                              // overflow: forces walks the bins
        }
        cnt++;
    };
    // reference cell-capacity mode, an over-full cell in reach: the
    // reference's literal loop (the list in its order; past the list's
    // capacity the forces pass walks the same way)
    const bool slow = live && refInv &&
                      ref_cap_near(ovl, ox + (int)((__float_as_int(me.w) >> 2) & 0x7fff), cyp, xi, yi, eps, g, W, ox,
                                   oy, start);
    if (hd.ok) {
        // one span per cell row (hood_spans), the non-empty ones first; four
        // candidates per trip, trip counts wave-uniform: unmasked trips up to
        // the wave's shortest span, masked ones up to its longest.  LDS reads
        // at immediate offsets.
        int sb[3], se[3], sh[3];
        hood_spans(hd, lbnd, xi, yi, eps, cs, reach, cyp, g, sb, se, sh, ox, ox + W - 1);
#pragma unroll
        for (int r = 0; r < 3; r++)
            if (!live || slow) sb[r] = se[r] = 0;
#pragma unroll
        for (int pass = 0; pass < 2; pass++)
#pragma unroll
            for (int r = 0; r < 2; r++)
                if (se[r] == sb[r]) {
                    sb[r] = sb[r + 1]; se[r] = se[r + 1]; sh[r] = sh[r + 1];
                    sb[r + 1] = se[r + 1] = 0;
                }
        int selfL[3];                                     // the particle's own LDS index, per span
#pragma unroll
        for (int r = 0; r < 3; r++) selfL[r] = s - sh[r];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const int b = sb[r], len = se[r] - b;
            int lmin, lmax;
            wave_minmax(len, lmin, lmax);
            if (lmax == 0) break;                         // (later spans are empty too)
            // (the list without branches per candidate: every candidate's code
            // is written to the ring at cnt, which advances only for a
            // neighbour -- a trip adds at most 4 < 8, so the group it
            // completes is flushed after the trip, before the ring comes
            // round to it again)
            auto trip = [&](int t, bool masked) {
                const int a = min(b + t, HCAP);           // past every span: reads the pad, masked
                float4 o[4];
#pragma unroll
                for (int j = 0; j < 4; j++) o[j] = lrec[a + j];
                const int c0 = cnt;
                // the trip's first code (image index or slot offset); a slot
                // offset outside int16 overflows the list, for the whole trip
                const int cb = lidx ? b + t : b + t + sh[r] - s;
                const int lim = (lidx || (cb >= -32768 && cb + 3 <= 32767)) ? NLIST_CAP : 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const bool valid = !masked || t + j < len;
                    if (NL) {
                        const bool in = term(o[j], valid);
                        ring[cnt & 15] = (int16_t)(cb + j);
                        cnt += (in && b + t + j != selfL[r]) ? 1 : 0;            // (not itself: metal:360-366)
                    } else {
                        term0(o[j], valid);
                    }
                }
                // past the list's capacity (or a slot offset outside int16):
                // the forces pass walks the bins -- the same count as capping
                // each neighbour, cnt = cnt < lim ? cnt + 1 : NLIST_CAP + 1,
                // since a trip adds at most 4 and only a trip with
                // neighbours can overflow (without exec-mask branches per
                // candidate)
                if (NL && cnt != c0 && cnt > lim) cnt = NLIST_CAP + 1;
                if (NL && (cnt >> 3) != (c0 >> 3) && cnt <= NLIST_CAP)
                    nlist[(size_t)(c0 >> 3) * nstride + s] = group(c0 >> 3);
            };
            int t = 0;
            for (; t + 4 <= lmin; t += 4) trip(t, false);
            for (; t < lmax; t += 4) trip(t, true);
        }
    } else if (live && !slow) {
        walk_neighbours<4>(xi, yi, eps, cs, reach, g, W, H, ox, oy, start,
                           [&](int k, int) { return nbA[k]; },
                           [&](int k, const float4 &o) {
                               if (term(o, true) && NL && k != s)
                                   emit(k - s, k - s >= -32768 && k - s <= 32767);
                           });
    }
    if (slow) {
        // (the neighbour list in the literal order, repeats included: the
        // forces pass then sums exactly what the reference's loop visits)
        ref_cap_walk<4>(xi, yi, eps, g, W, ox, oy, start, sid, refInv, sk.on ? nref : nn, status,
                        [&](int k) { return nbA[k]; },
                        [&](int k, const float4 &o) {
                            if (term(o, true) && NL && k != s) emit(k - s, k - s >= -32768 && k - s <= 32767);
                        },
                        sk, nn);
    }
    DTRMAX(2, wall_clock64());
    DTRMAX(5, (unsigned long long)cnt);
    if (NL && ho.list) {
        // the tile's rigid-bin candidates (the forces pass's coupling work):
        // a heavy or coupled tile is filed for the forces pass (HeavyOut)
        int c = 0;
        if (live) {
            const int k0 = hk0, k1 = hk1;
            for (int k = k0; k < k1; k += 4) {           // (the forces pass's phase-0 test, counted)
                float4 bb[4];
#pragma unroll
                for (int u = 0; u < 4; u++) bb[u] = ho.rbinAabb[min(k + u, k1 - 1)];
#pragma unroll
                for (int u = 0; u < 4; u++) c += (k + u < k1 && aabb_holds(bb[u], xi, yi)) ? 1 : 0;
            }
        }
        int inc = c;                                     // the pairs of the block's slots up to this one
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(inc, off);
            if (lane_id() >= off) inc += v;
        }
        const int w = threadIdx.x >> 6;
        if (lane_id() == 63) hcand[w] = inc;
        __syncthreads();
        for (int u = 0; u < w; u++) inc += hcand[u];
        const int T = hcand[0] + hcand[1] + hcand[2] + hcand[3];
        // the quartiles: the slot after the one whose pairs reach j T / 4
        for (int j = 1; j < 4; j++)
            if (c && (inc - c) * 4 < j * T && j * T <= inc * 4)
                atomicOr(&hcand[4], ((int)threadIdx.x + 1) << (9 * (j - 1)));
        __syncthreads();
        if (threadIdx.x == 0) {
            int code = 0;
            if (T >= ho.qpairs) {
                const int t = atomicAdd(&ho.list[0], 1);
                if (t < QUARTER_MAX) code = 1 + t;
            }
            if (!code && T >= ho.hpairs) {
                const int t = atomicAdd(&ho.list[1], 1);
                if (t < HALF_MAX) code = QUARTER_MAX + 1 + t;
            }
            if (!code && T > 0) {
                const int t = atomicAdd(&ho.list[2], 1);
                if (t < COUPLED_MAX) code = QUARTER_MAX + HALF_MAX + 1 + t;
            }
            if (code) {
                ho.list[2 + 2 * code] = lb;
                ho.list[3 + 2 * code] = hcand[4];
            }
            ho.tile[lb] = code;
        }
    }
    DTR(3);
    if (!live) return;
    if (NL) {
        if (cnt <= NLIST_CAP && (cnt & 7)) nlist[(size_t)(cnt >> 3) * nstride + s] = group(cnt >> 3);
        ncount[s] = cnt | ((!lidx || slow) ? NL_OFFS : 0);
    }
    float pres = stiffness * (acc - restDensity);
    if (pres < 0.f) pres = 0.f;
    rho[s] = acc;
    pr[s] = pres;
    nbB[2 * s + 1] = make_float2(acc, pres / (acc * acc));   // the p_j / rho_j^2 of metal:370
    DTRMAX(4, wall_clock64());
}

// ---------------------------------------------------------------------------
// Pure density pass with two particles per lane (lpe_sph_probe_density and
// the density microbench: computeDensity, metal:246-307, without the
// forces pass's neighbour list).  A block of DT_NT threads owns DT_TILE =
// 2 DT_NT consecutive sorted slots and stages their neighbourhood once
// (hood_plan / hood_stage, as k_density); lane t takes slots s0 + 2t and
// s0 + 2t + 1.  The pair walks ONE set of row spans: per cell row, the union
// of its two particles' spans.  A superset of a particle's canonical walk, in
// canonical order, leaves its sum unchanged bit for bit: the extra candidates
// lie beyond h * 1.002 in x or y (skipped quadrants, later or earlier cells
// of the row), so max(h^2 - r^2, 0) = +0, m * +0 = +0 and acc + 0 = acc.  So
// every LDS record read serves both particles, and the two sums advance in
// one packed fp32 pipe (v_pk_add_f32 / v_pk_mul_f32 round lane-wise exactly
// like the scalar ops; no FMA contraction).  A pair that straddles the tile's
// two row runs walks its particles one after the other, the other one parked
// at +inf (r^2 = inf: its terms are +0).
static constexpr int DT_NT = 256;
static constexpr int DT_TILE = 2 * DT_NT;
static constexpr int DT_CAP = 2048;       // records staged per tile (32 KB of LDS)
static constexpr int DT_BND = 1536;       // cell boundaries staged per tile (6 KB)

typedef float f2v __attribute__((ext_vector_type(2)));

// one canonical pass over <= 3 row spans for the lane's two particles
// (X, Y): four records per trip, trip counts wave-uniform (unmasked up to the
// wave's shortest span, masked - mass forced to +0 - up to its longest)
__device__ __forceinline__ void pair_pass(int sb[3], int se[3], const float4 *lrec, f2v X, f2v Y, float h2,
                                          float poly6, f2v &acc) {
#pragma unroll
    for (int pass = 0; pass < 2; pass++)
#pragma unroll
        for (int r = 0; r < 2; r++)
            if (se[r] == sb[r]) {
                sb[r] = sb[r + 1]; se[r] = se[r + 1];
                sb[r + 1] = se[r + 1] = 0;
            }
    const f2v H2 = {h2, h2}, P6 = {poly6, poly6}, Z = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const int b = sb[r], len = se[r] - b;
        int lmin, lmax;
        wave_minmax(len, lmin, lmax);
        if (lmax == 0) break;
        auto trip = [&](int t, bool masked) {
            const int a = min(b + t, DT_CAP);
            float4 o[4];
#pragma unroll
            for (int j = 0; j < 4; j++) o[j] = lrec[a + j];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float m = (!masked || t + j < len) ? o[j].z : 0.0f;
                const f2v dx = X - o[j].x, dy = Y - o[j].y;
                const f2v r2 = dx * dx + dy * dy;
                const f2v diff = __builtin_elementwise_max(H2 - r2, Z);
                const f2v w = P6 * diff * diff * diff;
                acc += m * w;
            }
        };
        int t = 0;
        for (; t + 4 <= lmin; t += 4) trip(t, false);
        for (; t < lmax; t += 4) trip(t, true);
    }
}

// The lane's two slots of tile [s0, s1) (staged in lrec / lbnd per hd):
// their densities, or the global walk when the neighbourhood did not fit
__device__ __forceinline__ f2v pair_tile(const Hood &hd, const float4 *lrec, const int *lbnd, int s0, int s1,
                                         int pair, float h, float eps, const GridParams &g, int W, int H, int ox, int oy,
                                         const int32_t *__restrict__ start, const float4 *__restrict__ nbA,
                                         int32_t *__restrict__ status) {
    const float cs = g.cellSize;
    const int sa = s0 + 2 * pair, sb = sa + 1;
    const bool la = sa < s1, lv = sb < s1;
    const float4 pa = nbA[la ? sa : s1 - 1];
    const float4 pb = nbA[lv ? sb : s1 - 1];
    const float h2 = h * h;
    const float poly6 = poly6Coeff2D(h);
    const float reach = walk_reach(h, cs);
    const float INF = __builtin_inff();
    f2v acc = {0.0f, 0.0f};
    if (hd.ok) {
        const int cya = oy + (int)((unsigned)__float_as_int(pa.w) >> 17);   // the bin's cell row (k_rank_permute)
        const int cyb = oy + (int)((unsigned)__float_as_int(pb.w) >> 17);
        int Ab[3], Ae[3], Bb[3], Be[3], sh[3];
        hood_spans(hd, lbnd, pa.x, pa.y, eps, cs, reach, cya, g, Ab, Ae, sh, ox, ox + W - 1);
        hood_spans(hd, lbnd, pb.x, pb.y, eps, cs, reach, cyb, g, Bb, Be, sh, ox, ox + W - 1);
        const bool strad = la && lv && cya != cyb;           // one pair per tile at most
#pragma unroll
        for (int r = 0; r < 3; r++) {
            if (!la) Ab[r] = Ae[r] = 0;
            if (!lv) Bb[r] = Be[r] = 0;
        }
        int Pb[3], Pe[3];
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const bool ea = Ae[r] == Ab[r], eb = Be[r] == Bb[r];
            if (strad) {
                Pb[r] = Ab[r]; Pe[r] = Ae[r];
            } else {
                Pb[r] = ea ? Bb[r] : (eb ? Ab[r] : min(Ab[r], Bb[r]));
                Pe[r] = ea ? Be[r] : (eb ? Ae[r] : max(Ae[r], Be[r]));
            }
        }
        const f2v X = {pa.x, strad ? INF : pb.x}, Y = {pa.y, pb.y};
        pair_pass(Pb, Pe, lrec, X, Y, h2, poly6, acc);
        if (__any(strad)) {
#pragma unroll
            for (int r = 0; r < 3; r++) {
                Pb[r] = strad ? Bb[r] : 0;
                Pe[r] = strad ? Be[r] : 0;
            }
            const f2v X2 = {INF, pb.x};
            pair_pass(Pb, Pe, lrec, X2, Y, h2, poly6, acc);
        }
    } else {
        if (threadIdx.x == 0) atomicAdd(&status[ST_STAGE_FALLBACK], 1);
        auto one = [&](const float4 &me, float &out) {
            walk_neighbours<4>(me.x, me.y, eps, cs, reach, g, W, H, ox, oy, start,
                               [&](int k, int) { return nbA[k]; },
                               [&](int, const float4 &o) {
                                   const float dx = me.x - o.x, dy = me.y - o.y;
                                   const float r2 = dx * dx + dy * dy;
                                   const float diff = fmaxf(h2 - r2, 0.0f);
                                   out += o.z * (poly6 * diff * diff * diff);
                               });
        };
        float ra = 0.0f, rb = 0.0f;
        if (la) one(pa, ra);
        if (lv) one(pb, rb);
        acc = f2v{ra, rb};
    }
    return acc;
}

// density / pressure / nbB write-back of one slot (metal:299-306)
__device__ __forceinline__ void density_out(int s, float a, float stiffness, float restDensity,
                                            float *__restrict__ rho, float *__restrict__ pr,
                                            float2 *__restrict__ nbB) {
    float pres = stiffness * (a - restDensity);
    if (pres < 0.f) pres = 0.f;
    rho[s] = a;
    pr[s] = pres;
    if (nbB) nbB[2 * s + 1] = make_float2(a, pres / (a * a));   // the p_j / rho_j^2 of metal:370
}

// A plan (sizeof(Hood) bytes) copied global -> LDS by wave 0, asynchronously
// (global_load_lds, one dword per lane; retired by the next barrier)
static constexpr int HOOD_WORDS = (int)(sizeof(Hood) / 4);
static_assert(sizeof(Hood) % 4 == 0 && HOOD_WORDS <= 64, "a plan is at most one wave of dwords");
__device__ __forceinline__ void hood_fetch(const Hood *__restrict__ plans, int t, int *dst) {
    if (threadIdx.x < HOOD_WORDS) {
        const int *src = reinterpret_cast<const int *>(plans + t) + threadIdx.x;
        __builtin_amdgcn_global_load_lds((glb_void_t *)src, (lds_void_t *)dst, 4, 0, 0);
    }
}

// One tile per block.  The tile's staging plan comes precomputed
// (k_density_plan, fetched into LDS by wave 0) instead of being derived by
// every lane.  Lanes are grouped by the quadrant row of their pair's first
// particle (upper quadrants first): a pair's span lengths depend mostly on
// which q-row of its cell it sits in (one q-row of the row above vs of the
// row below), so grouping them keeps a wave's lanes on equal trip counts
// (fewer masked trips).  Results go to the pair's own slots, so the lane
// order changes nothing in the sums.
__global__ void __launch_bounds__(DT_NT)
k_density_pair(int n, const int32_t *__restrict__ nptr, float h, float eps, float stiffness, float restDensity,
               int W, int H, int ox, int oy, const GridParams *__restrict__ gp, const int32_t *__restrict__ start,
               const float4 *__restrict__ nbA, float2 *__restrict__ nbB, float *__restrict__ rho,
               float *__restrict__ pr, int32_t *__restrict__ status, const Hood *__restrict__ plans) {
    __shared__ float4 lrec[DT_CAP + 4];                   // + 4: a trip reads up to 3 past a span
    __shared__ int lbnd[DT_BND];
    __shared__ int hraw[64];
    __shared__ int nup[DT_NT / 64];
    const int lb = xcd_block((n + DT_TILE - 1) / DT_TILE);
    if (lb < 0) return;
    const int nn = nptr ? *nptr : n;
    const int s0 = lb * DT_TILE, s1 = min(s0 + DT_TILE, nn);
    if (s0 >= s1) return;
    const GridParams g = *gp;
    hood_fetch(plans, lb, hraw);
    // the pair's quadrant row: bit 1 of the bin's quadrant (nbA.w, k_rank_permute)
    const int sp = s0 + 2 * (int)threadIdx.x;
    const int up = (sp < s1) ? ((__float_as_int(nbA[sp].w) & 2) ? 0 : 1) : 0;
    const unsigned long long bal = __ballot(up);
    const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
    const int below = __popcll(bal & ((1ull << lane) - 1));
    if (lane == 0) nup[wv] = __popcll(bal);
    __syncthreads();                                      // the plan, nup
    const Hood &hd = *reinterpret_cast<const Hood *>(hraw);
    if (hd.ok) hood_stage<DT_NT, DT_CAP, DT_BND>(hd, lrec, lbnd, nbA, start, s0);
    int ubefore = 0, utot = 0;
#pragma unroll
    for (int w = 0; w < DT_NT / 64; w++) {
        ubefore += (w < wv) ? nup[w] : 0;
        utot += nup[w];
    }
    // lane position of this pair: upper pairs first, each group in tile order
    const int pos = up ? (ubefore + below) : (utot + (wv * 64 + lane - ubefore - below));
    __shared__ short perm[DT_NT];
    perm[pos] = (short)threadIdx.x;
    __syncthreads();                                      // staged records, perm
    const int pair = perm[threadIdx.x];
    const f2v acc = pair_tile(hd, lrec, lbnd, s0, s1, pair, h, eps, g, W, H, ox, oy, start, nbA, status);
    const int sa = s0 + 2 * pair;
    if (sa + 1 < s1 && !nbB) {
        // the pure pass (nbB null: computeDensity's outputs only, 8 B per
        // particle): the pair's two densities and pressures as one 8-B store each
        float p0 = stiffness * (acc.x - restDensity), p1 = stiffness * (acc.y - restDensity);
        if (p0 < 0.f) p0 = 0.f;
        if (p1 < 0.f) p1 = 0.f;
        *(float2 *)(rho + sa) = make_float2(acc.x, acc.y);
        *(float2 *)(pr + sa) = make_float2(p0, p1);
        return;
    }
    if (sa < s1) density_out(sa, acc.x, stiffness, restDensity, rho, pr, nbB);
    if (sa + 1 < s1) density_out(sa + 1, acc.y, stiffness, restDensity, rho, pr, nbB);
}

// The tiles' staging plans, one thread per tile (the persistent pass reads
// them a tile ahead instead of computing them between its walks).  nrun = -1:
// an empty tile (the sharded slot count ended before it).
__global__ void __launch_bounds__(TPB)
k_density_plan(int n, const int32_t *__restrict__ nptr, float eps, int W, int H, int ox, int oy,
               const GridParams *__restrict__ gp, const int32_t *__restrict__ start,
               const float4 *__restrict__ nbA, Hood *__restrict__ plans) {
    const int t = blockIdx.x * TPB + threadIdx.x;
    if (t >= (n + DT_TILE - 1) / DT_TILE) return;
    const int nn = nptr ? *nptr : n;
    const int s0 = t * DT_TILE, s1 = min(s0 + DT_TILE, nn);
    Hood p;
    if (s0 >= s1) {
        p.ok = false;
        p.nrun = -1;
    } else {
        hood_plan(p, s0, s1, nbA, eps, gp->cellSize, W, H, ox, oy, start, DT_CAP, DT_BND);
        if (!p.ok) p.nrun = 0;                            // (left unset on the >2-run early out)
    }
    plans[t] = p;
}


struct SphStepParams {
    const int32_t *nptr;      // slab decomposition: device slot count (owned + ghosts), else null
    SlabKick own;             // slab decomposition (own.on): the edges that decide which slots are owned
    int nstride;              // neighbour-list stride (allocated slots)
    int n, W, H, ox, oy;
    float h, eps, dt, hdt;
    float viscosity, minDist, minDens;
    int diag;                 // count diagnostics into status (lpe_sph_diag)
    const int32_t *refInv;    // reference cell-capacity mode: id -> slot (else null)
    const int32_t *ovl;       //   and the sub-step's over-cap cells (ovl_append)
    int nblk, chunk;          // forces pass: logical blocks, blocks per XCD run (0: plain order)
    int32_t *mergePre;        // sub-step 0 after a prelaunch: its stats to merge into status (else null)
    int nref;                 // slab rank: the whole fluid's particle count (ref_cap_walk's id bound)
    int shortDiv;             // the pair term's thresholds keep its operands in range (pair_term)
};

// computeForces + velocityVerletFinish + impulse + push-out; reads the sorted
// records, writes P.  The block is the density pass's block (same HB slots,
// same plan, fplans): it stages the records of that neighbourhood -- both
// of every slot, 32 B -- as an LDS image of at most FCAP records, and the
// neighbour list (LDS indices, k_density) gathers from it without leaving the
// CU.  A block whose neighbourhood is larger, and a particle whose list came
// from a global walk (NL_OFFS), gather from global memory by slot offsets.
// After the fluid loop the image's LDS is reused for the coupling's
// per-block pair list (CouplePool).
#ifndef LPE_FORCES_MINW
#define LPE_FORCES_MINW 4
#endif
struct FRec { float4 a, b; };        // nbA (x, y, m, -), nbB (vx, vy, rho, p / rho^2)
static constexpr int PAIR_CAP = 1024;
// the prelaunched sub-step's stats (pre) into the step's (st), resetting the
// step stats first (what k_merge_prestats did as its own launch): one thread
// of the first forces pass, atomics where the pass itself adds to a slot
__device__ __forceinline__ void merge_prestats_dev(int32_t *__restrict__ st, int32_t *__restrict__ pre) {
    st[ST_MAX_OCC] = pre[ST_MAX_OCC];
    st[ST_OVER_CAP] = pre[ST_OVER_CAP];
    st[ST_REF_UB] = pre[ST_REF_UB];
    st[ST_NOT_INSERTED] = pre[ST_NOT_INSERTED];
    atomicOr(&st[ST_CAP_OVERFLOW], pre[ST_CAP_OVERFLOW]);
    atomicOr(&st[ST_BUCKET_OVERFLOW], pre[ST_BUCKET_OVERFLOW]);
    atomicAdd(&st[ST_STAGE_FALLBACK], pre[ST_STAGE_FALLBACK]);
    atomicAdd(&st[ST_FORCES_GLOBAL], pre[ST_FORCES_GLOBAL]);
    // (a slab rank's prelaunched sub-step 0 ran its exchange: its failures and maxima too)
    atomicOr(&st[ST_HALO_OVERFLOW], pre[ST_HALO_OVERFLOW]);
    atomicOr(&st[ST_HALO_DRIFT], pre[ST_HALO_DRIFT]);
    atomicOr(&st[ST_SLAB_CAPACITY], pre[ST_SLAB_CAPACITY]);
    atomicOr(&st[ST_LIST_OVERFLOW], pre[ST_LIST_OVERFLOW]);
    atomicOr(&st[ST_REF_SLAB], pre[ST_REF_SLAB]);
    atomicMax(&st[ST_RX_GHOST_L], pre[ST_RX_GHOST_L]);
    atomicMax(&st[ST_RX_GHOST_R], pre[ST_RX_GHOST_R]);
    atomicMax(&st[ST_SLOT_PEAK], pre[ST_SLOT_PEAK]);
    atomicAdd(&st[ST_OVER_CAP_TOTAL], pre[ST_OVER_CAP_TOTAL]);
    atomicMax(&st[ST_MAX_OCC_TOTAL], pre[ST_MAX_OCC_TOTAL]);
    for (int k = 0; k < ST_COUNT; k++) pre[k] = 0;
}
// the same as its own launch (the capped-cell mode: there the forces pass
// itself may raise ST_REF_UB, which the in-pass merge's plain store of
// that slot could erase)
__global__ void k_merge_prestats(int32_t *__restrict__ st, int32_t *__restrict__ pre) {
    if (blockIdx.x == 0 && threadIdx.x == 0) merge_prestats_dev(st, pre);
}

// One neighbour j != i of computeForces (metal:352-399): false when the
// reference skips it, else its force terms (the caller adds them in list
// order: sumFx += fx, sumFy += fy).
// The correctly rounded fp32 quotient and square root of the pair term
// without the general sequences' range handling.  The compiler's x / y is
// v_div_scale(y), v_rcp, v_div_scale(x), three Newton / remainder fma pairs,
// v_div_fmas, v_div_fixup; its sqrtf scales inputs below 2^-96, takes
// v_sqrt and picks the correctly rounded neighbour by two fma residuals, and
// passes zero / inf through a class test.  For the pair term's operands --
// r^2 >= minDistanceThreshold (1e-14) > 2^-96; r >= 1e-7 and rho_j >= 1e-12
// normal with normal reciprocals; numerators zero or far above 2^-100; the
// quotients normal or zero -- every scaling step is the identity and the fixups
// return their input, so these shortened sequences compute the same values
// bit for bit (the sub-step / tick parity tests run through them).
__device__ __forceinline__ float div_inrange(float x, float y) {
    float r = __builtin_amdgcn_rcpf(y);
    const float e = __builtin_fmaf(-y, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    float q = x * r;
    float rem = __builtin_fmaf(-y, q, x);
    q = __builtin_fmaf(rem, r, q);
    rem = __builtin_fmaf(-y, q, x);
    return __builtin_fmaf(rem, r, q);
}
__device__ __forceinline__ float sqrt_inrange(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1), sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    float r = (0.0f >= rm) ? sm : s;
    r = (0.0f < rp) ? sp : r;
    return r;
}

struct PairOwn { float xi, yi, vxi, vyi, pti; bool ok; };
struct PairConst { float h_ij, h_ij2, spF, lapC, visc, minDist, minDens; };
template <bool SHORT>
__device__ __forceinline__ bool pair_term(const PairOwn &o, const PairConst &k, const float4 &oa, const float4 &ob,
                                          float &fx, float &fy) {
    const float dx = o.xi - oa.x, dy = o.yi - oa.y;
    const float r2 = dx * dx + dy * dy;
    if (r2 < k.minDist) return false;
    if (r2 >= k.h_ij2) return false;
    const float r = SHORT ? sqrt_inrange(r2) : sqrtf(r2);
    const float rhoj = ob.z;
    if (rhoj < k.minDens || !o.ok) return false;
    const float mj = oa.z;
    const float term = o.pti + ob.w;
    const float diff = (k.h_ij - r);
    const float wSpiky = k.spF * (diff * diff);
    const float rx = SHORT ? div_inrange(dx, r) : dx / r, ry = SHORT ? div_inrange(dy, r) : dy / r;
    const float fxPress = -mj * term * wSpiky;
    fx = fxPress * rx;
    fy = fxPress * ry;
    const float vx_ij = o.vxi - ob.x, vy_ij = o.vyi - ob.y;
    const float wVisc = k.lapC * diff;
    const float fVisc = k.visc * mj * (SHORT ? div_inrange(wVisc, rhoj) : wVisc / rhoj);
    fx -= fVisc * vx_ij;
    fy -= fVisc * vy_ij;
    return true;
}

// the coupling's per-block arrays, laid over the image once the fluid loop is done
struct CouplePool {
    PairTerm term[PAIR_CAP];
    CoupleIn in[HB];
    unsigned char flag[PAIR_CAP];
};
static_assert(sizeof(CouplePool) <= sizeof(float4) * 2 * FCAP, "the coupling pool fits the forces image");

// SHORT: the pair term's shortened quotients and square root (SphStepParams
// shortDiv: the thresholds keep their operands in range); else the general ones
template <bool SHORT>
__global__ void __launch_bounds__(HB, LPE_FORCES_MINW)
k_forces_couple(SphStepParams sp, CoupleParams cp, const GridParams *__restrict__ gp,
                const int32_t *__restrict__ start, PState S, const float4 *__restrict__ nbA,
                const float4 *__restrict__ nbB, const float *__restrict__ pr,
                const uint4 *__restrict__ nlist, const int32_t *__restrict__ ncount, PState P,
                const lpe_gpu_rigid *__restrict__ rig, const float4 *__restrict__ raabb,
                const int32_t *__restrict__ rbinStart, const int32_t *__restrict__ rbinList,
                const float4 *__restrict__ rbinAabb,
                unsigned long long *__restrict__ acq,
                int32_t *__restrict__ status, KickNext kn, const Hood *__restrict__ fplans, HeavyIn hv) {
    // plain block order (blocks go round robin over the XCDs): the costly
    // blocks, the particles in and around the rigid pile, are one spatial
    // run that an XCD-contiguous mapping (xcd_block) would put on one XCD.
    // With tile scheduling (HeavyIn) the grid is [heavy parts][coupled][tiles].
    const int nq = hv.list ? HEAVY_HEAD : 0;
    const int bq = (int)blockIdx.x;
    int slo = 0, shi = HB;                    // the block's slots of its tile: [s0 + slo, s0 + shi)
    int lb, pb;                               // the tile; the block's bbox partial slot
    if (bq < nq) {
        int code, part, nparts;
        if (bq < QUARTER_BLOCKS) {
            code = 1 + bq / 4; part = bq % 4; nparts = 4;
        } else if (bq < QUARTER_BLOCKS + HALF_BLOCKS) {
            code = QUARTER_MAX + 1 + (bq - QUARTER_BLOCKS) / 2; part = (bq - QUARTER_BLOCKS) % 2; nparts = 2;
        } else {
            code = QUARTER_MAX + HALF_MAX + 1 + (bq - QUARTER_BLOCKS - HALF_BLOCKS); part = 0; nparts = 1;
        }
        pb = sp.nblk + bq;
        lb = hv.list[2 + 2 * code];
        if (lb < 0 || lb >= sp.nblk || hv.tile[lb] != code) {     // (no such tile this sub-step)
            if (kn.on && threadIdx.x == 0) kn.bboxPart[pb] = make_float4(1e30f, -1e30f, 1e30f, -1e30f);
            return;
        }
        if (nparts > 1) {
            const int qs = hv.list[3 + 2 * code];
            const int step = 4 / nparts;      // the part's quartile bounds j0 = step part, j1 = j0 + step
            const int j0 = step * part, j1 = j0 + step;
            slo = j0 == 0 ? 0 : (qs >> (9 * (j0 - 1))) & 511;
            shi = j1 == 4 ? HB : (qs >> (9 * (j1 - 1))) & 511;
        }
    } else {
        lb = sp.chunk > 0 ? xcd_chunk_block(sp.nblk, sp.chunk) : bq - nq;
        if (lb < 0) return;                   // (padding of the chunked grid)
        pb = lb;
    }
    const int ftb = pb;                       // (trace builds: the block's stamp slots, cleared per launch)
    (void)ftb;
    FTRCLR();
    if (bq >= nq && lb == 0 && threadIdx.x == 0) {
        if (sp.mergePre) merge_prestats_dev(status, sp.mergePre);
        if (kn.on && kn.fk.on) status[ST_NOT_INSERTED] = 0;       // (k_scan_rows adds)
        if (hv.clearNext) {                   // (the next density pass's lists)
            hv.clearNext[0] = 0; hv.clearNext[1] = 0; hv.clearNext[2] = 0;
        }
    }
    const int nn = sp.nptr ? *sp.nptr : sp.n;
    const int s0 = lb * HB, s1 = min(s0 + HB, nn);
    if (s0 >= s1 || (bq >= nq && hv.list && hv.tile[lb] > 0 && hv.list[2 + 2 * hv.tile[lb]] == lb)) {
        // (past the slots in use, or a tile a filed block runs)
        if (kn.on && threadIdx.x == 0) kn.bboxPart[pb] = make_float4(1e30f, -1e30f, 1e30f, -1e30f);
        return;
    }
    FTR(0);
    FTRHW();
    // the image: records [0, FCAP) nbA, [FCAP, 2 FCAP) nbB; then the CouplePool
    __shared__ float4 fimg[2 * FCAP];
    __shared__ int hraw[64];
    __shared__ int pRig[PAIR_CAP];
    __shared__ unsigned char pOwn[PAIR_CAP];
    __shared__ int pCount;
    CouplePool &pool = *reinterpret_cast<CouplePool *>(fimg);
    // the coupling's constants in LDS (read where the pair math uses them):
    // held in SGPRs across the kernel they spilled into VGPR lanes
    __shared__ CoupleParams s_cp;
    if (threadIdx.x == 0) { pCount = 0; s_cp = cp; }
    if (fplans) hood_fetch(fplans, lb, hraw);
    const GridParams g = *gp;
    const float cs = g.cellSize;
    // every lane stays to the end (the coupling pairs are shared by the
    // block); lanes past the last slot and ghost slots only join the barriers
    const int s = s0 + slo + (int)threadIdx.x;
    bool live = s < s1 && (int)threadIdx.x < shi - slo;
    const int out = s;                        // P slot written (P is kept in the sorted order)
    const int sl = live ? s : s0;
    const float4 meA = nbA[sl], meB = nbB[sl];
    int ocx0 = 0, ocx1 = 0;
    if (sp.own.on) {
        // a slab rank owns the slots whose bin column lies in its slab; the
        // others are neighbours only, and their slots end here (dead: no
        // bin in the next hash, id -1 for the next tick's kick)
        slab_cols(sp.own, ocx0, ocx1);
        const int gx = sp.ox + ((__float_as_int(meA.w) >> 2) & 0x7fff);
        if (live && !(gx >= ocx0 && gx < ocx1)) {
            live = false;
            P.id[s] = -1;
            if (kn.on) kn.key[s] = KEY_DEAD;
        }
    }
    const float xi = meA.x, yi = meA.y;
    const float vxi = meB.x, vyi = meB.y;
    const float rhoi = meB.z;
    const float pi = pr[sl];
    const float hi = sp.h;
    // all particles carry h = smoothingLength (fluid.cpp:287-292): the pair
    // smoothing length and its kernel coefficients are per-launch constants
    const float hj = sp.h;
    const float h_ij = 0.5f * (hi + hj);
    const float h_ij2 = h_ij * h_ij;
    const float spF = spikyCoeff2D(h_ij);
    const float lapC = viscLaplacianCoeff2D(h_ij);
    const float pti = meB.w;                      // pi / (rhoi * rhoi)
    const bool rhoi_ok = !(rhoi < sp.minDens);
    float sumFx = 0.f, sumFy = 0.f;
    // one neighbour j != i (metal:352-399)
    const PairOwn me{xi, yi, vxi, vyi, pti, rhoi_ok};
    const PairConst pk{h_ij, h_ij2, spF, lapC, sp.viscosity, sp.minDist, sp.minDens};
    auto pair = [&](const float4 &oa, const float4 &ob) {
        float fx, fy;
        if (pair_term<SHORT>(me, pk, oa, ob, fx, fy)) {
            sumFx += fx;
            sumFy += fy;
        }
    };
    const int craw = live ? ncount[s] : 0;
    const int cnt = craw & ~NL_OFFS;
    const bool offs = (craw & NL_OFFS) != 0;      // the list holds slot offsets (else image indices)
    // the neighbour list's first two words, in flight during the staging
    const size_t ns = (size_t)sp.nstride;
    uint4 gA = make_uint4(0u, 0u, 0u, 0u), gB = gA;
    if (cnt > 0 && cnt <= NLIST_CAP) gA = nlist[s];   // entries 0-7
    if (cnt > 8 && cnt <= NLIST_CAP) gB = nlist[ns + s];   // entries 8-15
    __syncthreads();                                  // (the plan, pCount)
    const Hood &hd = *reinterpret_cast<const Hood *>(hraw);
    const bool img = fplans && hd.ok && hd.L <= FCAP;   // (block-uniform; k_density's lidx)
    if (img) {
        // the image, one pass of asynchronous global -> LDS copies (retired
        // by the barrier after phase 0)
        const int wbase = threadIdx.x & ~63;
#pragma unroll
        for (int u = 0; u < FCAP / HB; u++) {
            const int f0 = u * HB;
            if (f0 >= hd.L) break;
            const int f = f0 + threadIdx.x;
            int d = hd.ss[0] - hd.l[0];
#pragma unroll
            for (int i = 1; i < 6; i++)
                if (f >= hd.l[i]) d = hd.ss[i] - hd.l[i];
            const int src = f < hd.L ? f + d : s0;        // lanes past the end copy a valid record
            __builtin_amdgcn_global_load_lds((glb_void_t *)(nbA + src), (lds_void_t *)(fimg + f0 + wbase), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((glb_void_t *)(nbB + src), (lds_void_t *)(fimg + FCAP + f0 + wbase), 16,
                                             0, 0);
        }
    } else if (fplans && threadIdx.x == 0) {
        atomicAdd(&status[ST_FORCES_GLOBAL], 1);
    }
    // ---- coupling, phase 0: the rigid candidates (positions only) --------
    // (impulse solver only if R > 0, fluid.cpp:910; push-out always).  The
    // (particle, rigid) pairs whose AABB test passes are few and clustered
    // (particles in and around the rigid pile), so they are spread over the
    // block: each wave appends its particles' pairs to the block's list (one
    // LDS atomic per wave; a particle's pairs stay consecutive, in candidate
    // = ascending rigid order); after the fluid loop every thread computes
    // pairs' geometry (couple_geom), then their impulse halves (couple_imp,
    // which need the finished velocities), round robin, and each particle
    // folds its own pairs in order.  A block with more than PAIR_CAP pairs
    // couples per thread instead (couple_both, the same arithmetic).
    const int lane = (int)threadIdx.x & 63;
    int nh = 0, off = 0;
    {
        int k0 = 0, k1 = 0;
        if (cp.nr > 0 && live) {
            float fbx = fminf(fmaxf(floorf(xi / cp.bcs) - (float)cp.bx0, 0.f), (float)(cp.bW - 1));
            float fby = fminf(fmaxf(floorf(yi / cp.bcs) - (float)cp.by0, 0.f), (float)(cp.bH - 1));
            int bin = (int)fby * cp.bW + (int)fbx;
            k0 = rbinStart[bin]; k1 = rbinStart[bin + 1];
            if (sp.diag && k1 > k0) atomicAdd(&status[ST_RIGID_CAND], k1 - k0);
        }
        // AABB hits among the bin's candidates (bin-ordered AABBs, 8 loads in
        // flight); the first 64 candidates' hits kept as a mask
        unsigned long long hitm = 0ull;
        for (int k = k0; k < k1; k += 8) {
            float4 bb[8];
#pragma unroll
            for (int u = 0; u < 8; u++) bb[u] = rbinAabb[min(k + u, k1 - 1)];
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (k + u < k1 && aabb_holds(bb[u], xi, yi)) {
                    nh++;
                    if (k + u - k0 < 64) hitm |= 1ull << (k + u - k0);
                }
        }
        // the wave's run of the block list
        int incl = nh;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d) incl += v;
        }
        const int wtot = __shfl(incl, 63);
        int wbase = 0;
        if (lane == 0 && wtot > 0) wbase = atomicAdd(&pCount, wtot);
        off = __shfl(wbase, 0) + incl - nh;
        if (nh > 0 && off + nh <= PAIR_CAP) {
            int q = off;
            for (unsigned long long m = hitm; m; m &= m - 1ull, q++) {
                pRig[q] = rbinList[k0 + __ffsll((long long)m) - 1];
                pOwn[q] = (unsigned char)threadIdx.x;
            }
            for (int k = k0 + 64; k < k1; k++)             // (a bin of more than 64 candidates)
                if (aabb_holds(rbinAabb[k], xi, yi)) { pRig[q] = rbinList[k]; pOwn[q] = (unsigned char)threadIdx.x; q++; }
        }
    }
    if (sp.diag && live) {
        atomicAdd(&status[ST_NEIGH], cnt);
        if (cnt > NLIST_CAP) atomicAdd(&status[ST_NL_OVERFLOW], 1);
    }
    __syncthreads();                                  // (the image, the block's pair list)
    FTR(1);
    FTRMAX(7, img ? hd.L : 100000 + (fplans ? hd.L : 0));
    if (!live) {
    } else if (cnt > NLIST_CAP && sp.refInv &&
               ref_cap_near(sp.ovl, sp.ox + (int)((__float_as_int(meA.w) >> 2) & 0x7fff),
                            sp.oy + (int)((unsigned)__float_as_int(meA.w) >> 17), xi, yi, sp.eps, g, sp.W, sp.ox,
                            sp.oy, start)) {
        // reference cell-capacity mode, the literal loop's neighbours past the
        // list's capacity: the loop itself (metal:345-351; nbrID == globalID
        // is skipped)
        ref_cap_walk<4>(xi, yi, sp.eps, g, sp.W, sp.ox, sp.oy, start, S.id, sp.refInv,
                        sp.own.on ? sp.nref : sp.n, status,
                        [&](int k) { return FRec{nbA[k], nbB[k]}; },
                        [&](int k, const FRec &o) { if (k != s) pair(o.a, o.b); }, sp.own, nn);
    } else if (cnt <= NLIST_CAP) {
        // the density pass's list: the r^2 < h^2 neighbours in canonical
        // order, so the heavy pair math runs only on real neighbours.
        // Software-pipelined in quads: the records of the next quad (and the
        // list word after the next) are in flight while a quad is computed.
        const int jend = cnt;
        struct Quad { FRec r[4]; };
        // records of list entries j .. j+3 held by words (wa, wb) of a list group
        auto quad = [&](uint32_t wa, uint32_t wb, int j) {
            const uint32_t w2[4] = {wa & 0xffffu, wa >> 16, wb & 0xffffu, wb >> 16};
            Quad q;
            if (!offs) {                              // image indices
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = j + u < jend ? (int)w2[u] : 0;
                    q.r[u] = FRec{fimg[k], fimg[FCAP + k]};
                }
            } else {                                  // slot offsets (past the end: itself, unused)
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = s + (j + u < jend ? (int)(int16_t)w2[u] : 0);
                    q.r[u] = FRec{nbA[k], nbB[k]};
                }
            }
            return q;
        };
        Quad cur = quad(gA.x, gA.y, 0);
        for (int j = 0; j < jend; j += 8) {
            const Quad nxt = quad(gA.z, gA.w, j + 4);   // entries j+4 .. j+7
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (j + u < jend) pair(cur.r[u].a, cur.r[u].b);
            cur = quad(gB.x, gB.y, j + 8);            // entries j+8 .. j+11
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (j + 4 + u < jend) pair(nxt.r[u].a, nxt.r[u].b);
            gA = gB;
            if (j + 16 < jend) gB = nlist[(size_t)((j >> 3) + 2) * ns + s];   // entries j+16 .. j+23
        }
    } else {
        walk_neighbours<4>(xi, yi, sp.eps, cs, walk_reach(hi, cs), g, sp.W, sp.H, sp.ox, sp.oy, start,
                           [&](int k, int) { return FRec{nbA[k], nbB[k]}; },
                           [&](int k, const FRec &o) { if (k != s) pair(o.a, o.b); });
    }
    FTRMAX(5, wall_clock64());
    CoupleState st;
    st.x = xi; st.y = yi;
    st.vhx = S.vhx[sl]; st.vhy = S.vhy[sl];
    st.ax = sumFx; st.ay = sumFy;
    // velocityVerletFinish (metal:428-441)
    st.vx = st.vhx + sp.hdt * st.ax;
    st.vy = st.vhy + sp.hdt * st.ay;
    st.mass = meA.z; st.rho = rhoi; st.p = pi;
    const CoupleParams &cpl = s_cp;
    const float4 *rc = raabb + cpl.nr;                 // the compact records (k_rig_couple)
    const int total = pCount;                         // (block-uniform: final since the barrier)
    if (total > PAIR_CAP) {
        if (live) {
            const float fbx = fminf(fmaxf(floorf(st.x / cpl.bcs) - (float)cpl.bx0, 0.f), (float)(cpl.bW - 1));
            const float fby = fminf(fmaxf(floorf(st.y / cpl.bcs) - (float)cpl.by0, 0.f), (float)(cpl.bH - 1));
            const int bin = (int)fby * cpl.bW + (int)fbx;
            couple_both(st, cpl, sp.dt, cpl.nr > 0, rc, rbinAabb, rbinList, rbinStart[bin], rbinStart[bin + 1], acq,
                        status);
        }
    } else {
        CoupleAcc a;
        if (total > 0) {
            __syncthreads();                          // (every read of the image done: the pool replaces it)
            // the particle's coupling inputs (pow only for a particle with hits)
            pool.in[threadIdx.x] = couple_in(st, cpl, cpl.nr > 0 && nh > 0);
            __syncthreads();
            FTR(6);
            FTR2SET(5, total);
            // ---- the pairs (geometry and impulse in one pass: the
            // velocities are final), round robin
            for (int q = threadIdx.x; q < total; q += HB) {
                PairTerm t;
                pool.flag[q] = (unsigned char)couple_pair(pool.in[pOwn[q]], cpl, sp.dt, true, rc, pRig[q], acq,
                                                          status, t, FTR_PAIRS());
                pool.term[q] = t;
            }
            __syncthreads();
            FTR(2);
            if (live)
                for (int q = off; q < off + nh; q++) a.fold(pool.term[q], pool.flag[q]);
        }
        if (live) couple_finish(st, cpl, a);
    }
    FTR(4);
    if (live) {
        // a sub-step that kicks the next one (kn.on) leaves only what the next
        // hash reads from P (velocity, mass, id: the kicked position and
        // half-step velocity go to the K scratch below); x, y, vh and a are
        // written by the tick's last sub-step
        if (!kn.on) {
            P.x[out] = st.x; P.y[out] = st.y;
            P.vhx[out] = st.vhx; P.vhy[out] = st.vhy;
            P.ax[out] = st.ax; P.ay[out] = st.ay;
        }
        P.vx[out] = st.vx; P.vy[out] = st.vy;
        P.m[out] = st.mass; P.id[out] = S.id[s];
    }
    if (kn.on) {            // the next sub-step's k_kick_drift for this particle (block-uniform)
        float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
        uint32_t k = 0xFFFFFFFFu;
        int ky = 0;
        // the next scan's row totals (FastKick), summed in LDS over the 8 rows
        // around the row of the block's first slot in the current order
        __shared__ int ltab[8];
        int rowBase = 0;
        if (kn.fk.on) {
            if (threadIdx.x < 8) ltab[threadIdx.x] = 0;
            rowBase = (__float_as_int(nbA[s0].w) >> 17) - 3;
        }
        float px = 0.f, py = 0.f, hx = 0.f, hy = 0.f;
        int kx = 0;
        if (live) {
            kick_one(st.x, st.y, st.vx, st.vy, st.ax, st.ay, kn.dt, kn.hdt, px, py, hx, hy);
            kn.kvhx[out] = hx; kn.kvhy[out] = hy;
            kn.kx[out] = px; kn.ky[out] = py;
            k = bin_key(px, py, kn.eps, kn.cs, kn.ox, kn.oy, kn.W, kn.H, status, &kx, &ky);
            kn.key[out] = k;
            mnx = mxx = px;
            mny = mxy = py;
        }
        if (kn.sk.on) {                                // (the whole wave: ballots)
            const int band = slab_band(kn.sk);
            slab_band_note(kn.sk, band);               // (the receiver's reach)
            slab_file(kn.sk, band, ocx0, ocx1, live, kx + kn.ox, px, py, st.vx, st.vy, hx, hy, st.mass, S.id[sl],
                      status);
        }
        int len; bool stt;
        const int first = wave_runs(k, live, &len, &stt);
        if (kn.fk.on && kn.fk.bucket) {
            int base = 0;
            if (stt) base = atomicAdd(&kn.count[k], len);
            base = __shfl(base, first);
            if (live) bucket_file(kn.fk, k, base + lane_id() - first, S.id[s], status);
        } else if (stt) {
            atomicAdd(&kn.count[k], len);
        }
        if (kn.fk.on) {
            __syncthreads();                               // (ltab zeroed)
            (void)wave_runs(live ? (uint32_t)ky : 0xFFFFFFFFu, live, &len, &stt);
            if (stt) {
                const int t = ky - rowBase;
                if (t >= 0 && t < 8) atomicAdd(&ltab[t], len);
                else atomicAdd(&kn.fk.rowtot[ky], len);
            }
        }
        bbox_partial(mnx, mxx, mny, mxy, kn.bboxPart + pb);   // (a block barrier)
        if (kn.fk.on && threadIdx.x < 8) {
            const int v = ltab[threadIdx.x];
            if (v) atomicAdd(&kn.fk.rowtot[rowBase + threadIdx.x], v);
        }
    }
    FTR(3);
}

// ---------------------------------------------------------------------------
// x-slab decomposition.  Rank r owns the particles whose
// reference-cell column gx = floor((x + eps) / cs) -- the column of their
// grid bin -- lies in [cx0, cx1) = [edges[r], edges[r + 1]) (cell columns;
// the first and last slab are open-ended), judged anew from the kicked
// position at every sub-step.  Per sub-step:
//   kick (k_kick_drift, or the previous forces pass): every particle the rank
//     owned is kicked and hashed; those within SLAB_BAND columns of an edge,
//     or past it, are also filed as ghost records for that neighbour
//     (kicked position, velocity, half-step velocity, mass, global id:
//     everything a particle carries between sub-steps);
//   k_bbox_reduce: the rank's bbox record; transport exchange: the ghost
//     records with both neighbours, and every rank's bbox record (the
//     reference grid is the global one: the "not inserted" rule, the stats);
//   k_ghost_unpack: the received ghosts after the rank's own slots (keys,
//     histogram, bucket: the single-domain one-pass hash), the global bbox;
//   k_scan_rows + k_bucket_permute: every local particle in canonical order
//     (ascending global id inside a bin: every sum is the single domain's,
//     bit for bit);
//   density over all local slots; forces, finish, coupling and the next kick
//     on the owned slots only.  A slot is owned iff its bin's column lies in
//     [cx0, cx1): a ghost that crossed an edge is adopted by the rank it
//     crossed into, and the sender marks the particle's slot dead (id = -1,
//     key KEY_DEAD) -- ownership moves inside the sub-step, with no
//     migration pass and no host synchronisation.
// Why SLAB_BAND = 2 columns: an owned particle's neighbours lie in its 3 x 3
// cells (columns cx0 - 1 .. cx1), theirs in columns cx0 - 2 .. cx1 + 1, all
// present locally, so every ghost density the forces pass reads is computed
// from its owner's neighbours in its owner's order.  A particle kicked more
// than a slab away would be owned by no rank: the receiver's check
// (ST_HALO_DRIFT) fails the step loudly.  Once per tick the rigid
// accumulators are all-reduced (exact int64 limbs); every `rebalance` ticks
// the inner edges move a column towards equal counts (k_slab_hist ->
// all-reduce -> k_slab_rebalance, identically on every rank).
static constexpr int GREC = 8;    // floats per ghost record: x, y, vx, vy, vhx, vhy, m, id
static constexpr int HDR = 4;     // header floats of a wire buffer ([0]: record count, int)
static constexpr int SLAB_OPEN = 1 << 29;   // the open ends' edge columns (-/+)
static constexpr int SLAB_MINW = 8;         // narrowest slab (columns) the rebalancing leaves

struct Shard {
    int nranks = 1, rank = 0, hasL = 0, hasR = 0;
    int wcap = 0;                  // ghost records per direction (the wire: HDR + wcap records)
    int rebalance = 0;             // ticks between edge moves (0: fixed edges)
    long ticks = 0;
    int n0 = 0;                    // particles uploaded
    int mv = 0;                    // columns an inner edge may move from its initial one
    std::vector<int> e0;           // initial edges (columns), host
    int32_t *edges = nullptr;      // device [nranks + 1]: the current edges
    int32_t *edges0 = nullptr;     // device [nranks + 1]: the initial ones (the rebalancing's range)
    int32_t *cnt = nullptr;        // device: [0], [1] slots in use (sorted counts, by parity), [2] the
                                   //   hash's input slots (own + received)
    int cur = 0;                   // host: the parity of the committed slot count (P's layout)
    float *sL = nullptr, *sR = nullptr, *rL = nullptr, *rR = nullptr;   // wire buffers
    float4 *bbAll = nullptr;       // [nranks] every rank's bbox record (minX, minY, -maxX, -maxY)
    float4 *bbG = nullptr;         // the global bbox (minX, maxX, minY, maxY)
    float *hist = nullptr;         // rebalancing: owned particles per universe column
    int hcol0 = 0, hcols = 0;
    int nglobal = 0;               // the whole fluid's particle count (lpe_sph_set_global_count)
};

static int sh_nglobal(const SphDev &d) { return d.shard ? d.shard->nglobal : 0; }
static void slab_clip_cols(const SphDev &d, long &gx0, long &gx1) {
    if (!d.shard) return;
    const Shard &h = *d.shard;
    const long m = h.mv + SLAB_BAND_MAX + 8;
    if (h.hasL) gx0 = std::max<long>(gx0, h.e0[h.rank] - m);
    if (h.hasR) gx1 = std::min<long>(gx1, h.e0[h.rank + 1] + m);
}

// the rank's bbox record from the kick's block partials
__global__ void __launch_bounds__(TPB)
k_bbox_reduce(const float4 *__restrict__ part, int nparts, float4 *__restrict__ out) {
    float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
    for (int p = threadIdx.x; p < nparts; p += TPB) {
        float4 b = part[p];
        mnx = fminf(mnx, b.x); mxx = fmaxf(mxx, b.y);
        mny = fminf(mny, b.z); mxy = fmaxf(mxy, b.w);
    }
    for (int off = 32; off > 0; off >>= 1) {
        mnx = fminf(mnx, __shfl_xor(mnx, off));
        mxx = fmaxf(mxx, __shfl_xor(mxx, off));
        mny = fminf(mny, __shfl_xor(mny, off));
        mxy = fmaxf(mxy, __shfl_xor(mxy, off));
    }
    __shared__ float4 wb[TPB / 64];
    if (lane_id() == 0) wb[threadIdx.x >> 6] = make_float4(mnx, mxx, mny, mxy);
    __syncthreads();
    if (threadIdx.x == 0) {
        float4 b = wb[0];
        for (int w = 1; w < TPB / 64; w++) {
            b.x = fminf(b.x, wb[w].x); b.y = fmaxf(b.y, wb[w].y);
            b.z = fminf(b.z, wb[w].z); b.w = fmaxf(b.w, wb[w].w);
        }
        *out = make_float4(b.x, b.z, -b.y, -b.w);     // every component reduces by MIN
    }
}

// The received ghosts -> slots [nslot, nslot + gL + gR) after the rank's own
// (left ones first), with the kick's bin key, histogram, bucket filing and
// row totals; the global bbox from every rank's record; the send headers
// cleared for the next sub-step (the transport is done with them).
__global__ void __launch_bounds__(TPB)
k_ghost_unpack(const float *__restrict__ rL, const float *__restrict__ rR, int wcap, float *__restrict__ sL,
               float *__restrict__ sR, const float4 *__restrict__ bbAll, int nranks, float4 *__restrict__ bbG,
               const int32_t *__restrict__ nslot, int32_t *__restrict__ nin, int cap_slots, SlabKick sk, PState P,
               KState K, uint32_t *__restrict__ key, int32_t *__restrict__ count, FastKick fk, float eps, float cs,
               int ox, int oy, int W, int H, int32_t *__restrict__ status) {
    const int t = blockIdx.x * TPB + threadIdx.x;
    const int gL = rL ? min(*(const int *)rL, wcap) : 0, gR = rR ? min(*(const int *)rR, wcap) : 0;
    const int base = *nslot;
    const int room = max(cap_slots - base, 0);
    if (t == 0) {
        float4 b = bbAll[0];
        for (int r = 1; r < nranks; r++) {
            const float4 q = bbAll[r];
            b.x = fminf(b.x, q.x); b.y = fminf(b.y, q.y); b.z = fminf(b.z, q.z); b.w = fminf(b.w, q.w);
        }
        *bbG = make_float4(b.x, -b.z, b.y, -b.w);
        *nin = base + min(gL + gR, room);
        if (gL + gR > room) atomicOr(&status[ST_SLAB_CAPACITY], 1);
        // the columns each neighbour sent (the literal capped walk's reach)
        sk.rband[0] = rL ? SLAB_BAND_MAX - ((const int *)rL)[1] : 0;
        sk.rband[1] = rR ? SLAB_BAND_MAX - ((const int *)rR)[1] : 0;
        atomicMax(&status[ST_SLOT_PEAK], base + gL + gR);
        atomicMax(&status[ST_RX_GHOST_L], rL ? *(const int *)rL : 0);
        atomicMax(&status[ST_RX_GHOST_R], rR ? *(const int *)rR : 0);
        if (sL) { ((int *)sL)[0] = 0; ((int *)sL)[1] = 0; }
        if (sR) { ((int *)sR)[0] = 0; ((int *)sR)[1] = 0; }
    }
    const bool active = t < gL + gR && t < room;
    uint32_t k = KEY_DEAD;
    int id = 0, ky = 0;
    if (active) {
        const float4 *src = (const float4 *)(t < gL ? rL + HDR + (size_t)t * GREC : rR + HDR + (size_t)(t - gL) * GREC);
        const float4 a = src[0], b = src[1];
        const int slot = base + t;
        id = __float_as_int(b.w);
        K.x[slot] = a.x; K.y[slot] = a.y; P.vx[slot] = a.z; P.vy[slot] = a.w;
        K.vhx[slot] = b.x; K.vhy[slot] = b.y; P.m[slot] = b.z; P.id[slot] = id;
        int kx;
        k = bin_key(a.x, a.y, eps, cs, ox, oy, W, H, status, &kx, &ky);
        key[slot] = k;
        // a ghost beyond this slab's far edge would be owned by no rank
        int cx0, cx1;
        slab_cols(sk, cx0, cx1);
        const int gx = kx + ox;
        if ((t < gL && gx >= cx1) || (t >= gL && gx < cx0)) atomicOr(&status[ST_HALO_DRIFT], 1);
    }
    int len; bool st;
    const int first = wave_runs(k, active, &len, &st);
    if (fk.on && fk.bucket) {
        int b0 = 0;
        if (st) b0 = atomicAdd(&count[k], len);
        b0 = __shfl(b0, first);
        if (active) bucket_file(fk, k, b0 + lane_id() - first, id, status);
    } else if (st) {
        atomicAdd(&count[k], len);
    }
    if (fk.on && active) atomicAdd(&fk.rowtot[ky], 1);
}

// Rebalancing: the owned particles per universe column (sorted order:
// consecutive slots share columns, so one atomic per run of a wave)
__global__ void __launch_bounds__(TPB)
k_slab_hist(int n, const int32_t *__restrict__ nslot, const float *__restrict__ x, const int32_t *__restrict__ id,
            float eps, float cs, int col0, int ncols, float *__restrict__ hist) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    const bool active = i < *nslot && i < n && id[i] >= 0;
    int c = 0;
    if (active) c = min(max((int)floorf((x[i] + eps) / cs) - col0, 0), ncols - 1);
    int len; bool st;
    (void)wave_runs(active ? (uint32_t)c : KEY_DEAD, active, &len, &st);
    if (st) atomicAdd(&hist[c], (float)len);
}

// One block: the inner edges move one column towards equal counts (the
// all-reduced histogram is the same on every rank, so are the edges), inside
// [edges0 - mv, edges0 + mv] and at least SLAB_MINW columns apart; a
// neighbourhood within 1 % of the mean count (or half the edge column's
// count) stays put.  Clears the histogram for the next time.
__global__ void __launch_bounds__(TPB)
k_slab_rebalance(float *__restrict__ hist, int ncols, int col0, int32_t *__restrict__ edges,
                 const int32_t *__restrict__ edges0, int nranks, int mv) {
    __shared__ float wsum[TPB / 64];
    __shared__ float s_tot;
    auto block_sum = [&](float v) {
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        __syncthreads();
        if (lane_id() == 0) wsum[threadIdx.x >> 6] = v;
        __syncthreads();
        float tot = 0.f;
        for (int w = 0; w < TPB / 64; w++) tot += wsum[w];
        return tot;
    };
    float part = 0.f;
    for (int c = threadIdx.x; c < ncols; c += TPB) part += hist[c];
    const float total = block_sum(part);
    if (threadIdx.x == 0) s_tot = total;
    for (int j = 1; j < nranks; j++) {
        const int e = edges[j];
        float lp = 0.f;
        for (int c = threadIdx.x; c < min(e - col0, ncols); c += TPB) lp += hist[c];
        const float left = block_sum(lp);
        if (threadIdx.x == 0) {
            const float target = s_tot * (float)j / (float)nranks;
            const float colc = (e - col0 >= 0 && e - col0 < ncols) ? hist[e - col0] : 0.f;
            const float tol = fmaxf(0.01f * s_tot / (float)nranks, 0.5f * colc);
            int ne = e;
            if (left < target - tol) ne = e + 1;
            else if (left > target + tol) ne = e - 1;
            ne = min(max(ne, edges0[j] - mv), edges0[j] + mv);
            if (j > 1) ne = max(ne, edges[j - 1] + SLAB_MINW);
            if (j + 1 < nranks) ne = min(ne, edges[j + 1] - SLAB_MINW);
            edges[j] = ne;
        }
        __syncthreads();
    }
    for (int c = threadIdx.x; c < ncols; c += TPB) hist[c] = 0.f;
}


// ---------------------------------------------------------------------------
// rigid binning (once per tick)
__device__ __forceinline__ int bin_of(float v, float bcs, int b0, int nb) {
    float t = floorf(v / bcs) - (float)b0;
    t = fminf(fmaxf(t, 0.f), (float)(nb - 1));
    return (int)t;
}
// compact AABBs of the coupling rigids: (minX, maxX, minY, maxY)
// and their compact coupling records (sph_coupling.h RigC), nr after them
__global__ void k_rig_couple(int nr, const lpe_gpu_rigid *__restrict__ rig, float maxSafeVelocitySq,
                             float4 *__restrict__ aabb) {
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr) return;
    rig_couple_one(rig[r], r, nr, maxSafeVelocitySq, aabb);
}

// one wave per rigid, lanes stride over the bins its AABB covers (a wall
// covers thousands of 0.25 m bins; a thread per rigid serialises on it)
__global__ void k_rbin_count(int nr, const lpe_gpu_rigid *__restrict__ rig, float bcs,
                             int bx0, int by0, int bW, int bH, int32_t *__restrict__ cnt) {
    int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    if (r >= nr) return;
    const lpe_gpu_rigid &b = rig[r];
    int x0 = bin_of(b.minX, bcs, bx0, bW), x1 = bin_of(b.maxX, bcs, bx0, bW);
    int y0 = bin_of(b.minY, bcs, by0, bH), y1 = bin_of(b.maxY, bcs, by0, bH);
    int w = x1 - x0 + 1, tot = w * (y1 - y0 + 1);
    for (int k = lane; k < tot; k += 64) atomicAdd(&cnt[(y0 + k / w) * bW + x0 + k % w], 1);
}
__global__ void k_rbin_fill(int nr, const lpe_gpu_rigid *__restrict__ rig, float bcs,
                            int bx0, int by0, int bW, int bH, int32_t *__restrict__ cursor,
                            int32_t *__restrict__ list, int cap, int32_t *__restrict__ status) {
    int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    if (r >= nr) return;
    const lpe_gpu_rigid &b = rig[r];
    int x0 = bin_of(b.minX, bcs, bx0, bW), x1 = bin_of(b.maxX, bcs, bx0, bW);
    int y0 = bin_of(b.minY, bcs, by0, bH), y1 = bin_of(b.maxY, bcs, by0, bH);
    int w = x1 - x0 + 1, tot = w * (y1 - y0 + 1);
    for (int k = lane; k < tot; k += 64) {
        int slot = atomicAdd(&cursor[(y0 + k / w) * bW + x0 + k % w], 1);
        if (slot < cap) list[slot] = r;
        else atomicOr(&status[ST_LIST_OVERFLOW], 1);
    }
}
// each bin's list -> ascending rigid index (indices in a list are distinct):
// one wave per bin, an entry's place is the number of smaller indices (bins
// of more than 64 entries: one lane, insertion sort); then the entries'
// AABBs in list order (the coupling's candidate walk reads them contiguously
// instead of through the index)
static constexpr int RBS_WAVES = 4;                        // bins per 256-thread block
__global__ void __launch_bounds__(256)
k_rbin_sort(int B, int32_t *__restrict__ start, int32_t *__restrict__ list, int cap,
            const float4 *__restrict__ aabb, float4 *__restrict__ baabb, int32_t *__restrict__ count,
            int32_t *__restrict__ st, int32_t *__restrict__ pre) {
    // (the tick's first forces pass follows: the prelaunched sub-step's stats
    // merged here, k_merge_prestats' work without its launch)
    if (pre && blockIdx.x == 0 && threadIdx.x == 0) merge_prestats_dev(st, pre);
    const int b = blockIdx.x * RBS_WAVES + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (b >= B) return;                                     // (whole wave)
    if (lane == 0) count[b] = 0;                            // the next build's histogram (consumed by the scan)
    const int s = min(start[b], cap), e = min(start[b + 1], cap), n = e - s;
    if (n <= 0) return;
    if (n > 64) {
        if (lane == 0) {
            for (int k = s + 1; k < e; k++) {
                int v = list[k];
                int j = k - 1;
                while (j >= s && list[j] > v) { list[j + 1] = list[j]; j--; }
                list[j + 1] = v;
            }
            for (int k = s; k < e; k++) baabb[k] = aabb[list[k]];
        }
        return;
    }
    const int v = lane < n ? list[s + lane] : 0x7fffffff;
    int rank = 0;
    for (int j = 0; j < n; j++) rank += __shfl(v, j) < v ? 1 : 0;
    if (lane < n) {
        list[s + rank] = v;
        baabb[s + rank] = aabb[v];
    }
}

// writeBackRigidBodies arithmetic (fluid.cpp:545-562), once per tick: the
// exact sums rounded to fp32 (kept in accum_out for download), then zeroed
__global__ void k_rigid_writeback(int nr, lpe_gpu_rigid *__restrict__ rig,
                                  unsigned long long *__restrict__ acq, float *__restrict__ accum_out,
                                  float damping, const int32_t *__restrict__ coupleBody,
                                  lpe_body *__restrict__ bodies) {
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr) return;
    lpe_gpu_rigid &rb = rig[r];
    unsigned long long *a = acq + (size_t)r * (3 * XACC_LIMBS);
    const float fx = xacc_round(a), fy = xacc_round(a + XACC_LIMBS), tq = xacc_round(a + 2 * XACC_LIMBS);
    for (int k = 0; k < 3 * XACC_LIMBS; k++) a[k] = 0ull;
    accum_out[3 * r] = fx; accum_out[3 * r + 1] = fy; accum_out[3 * r + 2] = tq;
    float invMass = (rb.mass > 1e-12f) ? (1.f / rb.mass) : 0.f;
    float invInertia = (rb.inertia > 1e-12f) ? (1.f / rb.inertia) : 0.f;
    rb.vx += fx * invMass;
    rb.vy += fy * invMass;
    rb.vx *= damping;
    rb.vy *= damping;
    rb.omega += tq * invInertia;
    rb.omega *= damping;
    rb.accumFx = 0.f; rb.accumFy = 0.f; rb.accumTorque = 0.f;
    if (bodies) {   // world tick: the velocities straight back to the coupled bodies (fluid.cpp:564-579)
        lpe_body &b = bodies[coupleBody[r]];
        if (b.flags & LPE_BODY_HAS_VEL) { b.vx = rb.vx; b.vy = rb.vy; }
        if (b.flags & LPE_BODY_HAS_ANGVEL) b.omega = rb.omega;
    }
}

// reference cell index (metal:224-236) of each particle, written at its id
__global__ void k_ref_cells(int n, float eps, const float *__restrict__ x,
                            const float *__restrict__ y, const int32_t *__restrict__ id,
                            const GridParams *__restrict__ gp, int32_t *__restrict__ out) {
    int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    const GridParams g = *gp;
    int gx = (int)floorf((x[i] + eps) / g.cellSize);
    int gy = (int)floorf((y[i] + eps) / g.cellSize);
    int cx = gx - g.gridMinX, cy = gy - g.gridMinY;
    out[id[i]] = (cx < 0 || cx >= g.gridDimX || cy < 0 || cy >= g.gridDimY) ? -1
                                                                             : cy * g.gridDimX + cx;
}

struct Fields6 { const float *src[6]; float *dst[6]; };

// scatter sorted-order arrays back to gather order (for downloads)
__global__ void k_unpermute(int n, const int32_t *__restrict__ id, int nf, Fields6 f) {
    int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= n) return;
    int d = id[i];
    for (int k = 0; k < nf; k++) f.dst[k][d] = f.src[k][i];
}

// download of a slab rank's owned particles (P slots with an id), in no
// particular order: x, y, vx, vy, rho, p and the id to staging arrays (ids
// null: only their count)
__global__ void k_slab_gather_owned(int n, const int32_t *__restrict__ nslot, PState P,
                                    const float *__restrict__ rho, const float *__restrict__ pr, Fields6 f,
                                    int32_t *__restrict__ ids, int32_t *__restrict__ cnt) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    const bool live = i < n && i < *nslot && P.id[i] >= 0;
    const unsigned long long m = __ballot(live);
    if (!m) return;
    const int lane = lane_id(), leader = __ffsll((long long)m) - 1;
    int b = 0;
    if (lane == leader) b = atomicAdd(cnt, __popcll(m));
    if (!ids) return;
    b = __shfl(b, leader);
    if (!live) return;
    const int d = b + __popcll(m & ((1ull << lane) - 1ull));
    f.dst[0][d] = P.x[i]; f.dst[1][d] = P.y[i]; f.dst[2][d] = P.vx[i]; f.dst[3][d] = P.vy[i];
    f.dst[4][d] = rho[i]; f.dst[5][d] = pr[i];
    ids[d] = P.id[i];
}


}  // namespace lpe

using namespace lpe;

// ===========================================================================
// host side
static inline int nblk(long n, int t = TPB) { return (int)((n + t - 1) / t); }
// the rigid bin list buffer: cap ints, then cap float4 AABBs (16-B aligned)
static inline size_t rbin_list_pad(int cap) { return ((sizeof(int32_t) * (size_t)cap + 15) / 16) * 16; }
static inline size_t rbin_bytes(int cap) { return rbin_list_pad(cap) + sizeof(float4) * (size_t)cap; }
static inline float4 *rbin_aabb(const SphDev &d) {
    return d.rbinList ? (float4 *)((char *)d.rbinList + rbin_list_pad(d.cap_rlist)) : nullptr;
}
static inline int nblk1(long n, int t = TPB) { return std::max(1, nblk(n, t)); }   // never an empty grid
// ints per parity of the grid hash's overflow list (header + one int4 per particle slot)
static inline size_t ovf_words(const SphDev &d) { return 4 + 4 * (size_t)std::max(d.cap_n, 1); }

// the id -> slot map of the reference cell-capacity mode, or null (mode off)
static inline int32_t *sph_ref_inv(const SphDev &d) {
    return (d.mode & LPE_SPH_MODE_REF_CELL_CAP) ? d.refInv : nullptr;
}

// per-step stats (max occupancy, over-capacity cells, undefined reads)
static int sph_reset_step_stats(lpe_ctx *ctx, hipStream_t s, int32_t *status) {
    LPE_HIP(ctx, hipMemsetAsync(status + ST_MAX_OCC, 0, sizeof(int32_t), s));
    LPE_HIP(ctx, hipMemsetAsync(status + ST_OVER_CAP, 0, 2 * sizeof(int32_t), s));
    return LPE_OK;
}

// the kicked-state scratch (the S staging arrays, dead inside a sub-step)
static inline KState sph_kstate(const SphDev &d) { return KState{d.S.x, d.S.y, d.S.vx, d.S.vy}; }

// A pending prelaunch (sph_prelaunch) only wrote scratch: voiding it orders
// the context stream after it (its buffers are reused next) and forgets it.
static int sph_void_prelaunch(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    if (!d.pre) return LPE_OK;
    d.pre = false;
    LPE_HIP(ctx, hipStreamWaitEvent(ctx->stream, d.preDone, 0));
    return LPE_OK;
}
// order the context stream after a pending prelaunch, which stays valid
// (downloads stage through arrays the prelaunched sub-step no longer needs)
static int sph_join_prelaunch(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    if (d.pre) LPE_HIP(ctx, hipStreamWaitEvent(ctx->stream, d.preDone, 0));
    return LPE_OK;
}

static void pstate_free(PState &p) {
    void *ptrs[] = {p.x, p.y, p.vx, p.vy, p.vhx, p.vhy, p.ax, p.ay, p.m, p.id};
    for (void *q : ptrs) if (q) (void)hipFree(q);
    p = PState();
}

static void shard_free(Shard *h) {
    if (!h) return;
    void *ptrs[] = {h->edges, h->edges0, h->cnt, h->sL, h->sR, h->rL, h->rR, h->bbAll, h->bbG, h->hist};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    delete h;
}

static void sph_free(SphDev &d) {
    if (d.pside) (void)hipStreamSynchronize(d.pside);   // a prelaunch may still use the buffers
    d.pre = false;
    shard_free(d.shard);
    d.shard = nullptr;
    pstate_free(d.P);
    pstate_free(d.S);
    void *ptrs[] = {d.ovl, d.rho, d.pr, d.rhoN, d.prN, d.nbA, d.nbB, d.nlist, d.ncount, d.key, d.tmpId, d.tmpOld, d.refInv, d.stage, d.count, d.start, d.cursor,
                    d.rowtot, d.bucket, d.bovf,
                    d.blocksum, d.bboxPart, d.gp, d.status, d.rig, d.raabb, d.accum, d.acq, d.rbinStart, d.rgrid, d.rmax,
                    d.rbinList, d.rbinCount, d.coupleBody, d.plans, d.fplans, d.heavy, d.tileHeavy};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    for (int k = 0; k < 2; k++)
        if (d.lpend[k] && d.evLag[k]) (void)hipEventSynchronize(d.evLag[k]);
    if (d.hlag) (void)hipHostFree(d.hlag);
    hipEvent_t evs[] = {d.preReady, d.preDone, d.fbgDone, d.evLag[0], d.evLag[1]};
    for (hipEvent_t e : evs) if (e) (void)hipEventDestroy(e);
    if (d.pside) (void)hipStreamDestroy(d.pside);
    d = SphDev();
}

extern "C" int lpe_abi_version(void) { return LPE_ABI_VERSION; }

extern "C" int lpe_device_count(int *count) {
    if (!count) return LPE_ERR_ARG;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return LPE_OK;
}

// Hardware queues.  A context runs four streams (fluid step,
// prelaunch, detection, position solver); HIP maps streams round robin onto
// GPU_MAX_HW_QUEUES queues, 4 by default, one per stream of a context.  Round
// 4's load-time constructor raised it to 8 when unset; round 6 measured more
// than 4 queues running every kernel ~2x slower on MI355X / ROCm 7.2 (810
// against 453 ticks/s, profiles/r06/hwq/sweep.txt), so the library leaves it
// alone; lpe_hw_queues reports the value in effect.
static const int g_hwq_set_by_lib = 0;

extern "C" int lpe_hw_queues(int *queues, int *set_by_library) {
    if (!queues) return LPE_ERR_ARG;
    const char *v = std::getenv("GPU_MAX_HW_QUEUES");
    *queues = (v && std::atoi(v) > 0) ? std::atoi(v) : 4;
    if (set_by_library) *set_by_library = g_hwq_set_by_lib;
    return LPE_OK;
}

extern "C" int lpe_create(int device, lpe_ctx **out) {
    if (!out) return LPE_ERR_ARG;
    *out = nullptr;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) return LPE_ERR_NO_DEVICE;
    if (device < 0 || device >= c) return LPE_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return LPE_ERR_HIP;
    lpe_ctx *ctx = new lpe_ctx();
    ctx->device = device;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return LPE_ERR_HIP;
    }
    lpe_fluid_config_default(&ctx->sph.cfg);
    *out = ctx;
    return LPE_OK;
}

extern "C" int lpe_destroy(lpe_ctx *ctx) {
    if (!ctx) return LPE_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    sph_free(ctx->sph);
    delete ctx->transport;
    ctx->transport = nullptr;
    lpe_rigid_destroy_internal(ctx);
    lpe_bh_destroy_internal(ctx);
    lpe_timer_destroy_internal(ctx);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return LPE_OK;
}

extern "C" const char *lpe_last_error(const lpe_ctx *ctx) {
    return ctx ? ctx->err.c_str() : "null context";
}

extern "C" int lpe_sync(lpe_ctx *ctx) {
    if (!ctx) return LPE_ERR_ARG;
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LPE_OK;
}

extern "C" int lpe_fluid_config_default(lpe_fluid_config *c) {
    if (!c) return LPE_ERR_ARG;
    std::memset(c, 0, sizeof(*c));
    c->gravity = 9.81f; c->restDensity = 0.5f; c->stiffness = 200.0f; c->viscosity = 0.03f;
    c->positionSolver.safetyMargin = 0.001f; c->positionSolver.relaxFactor = 0.9f;
    c->positionSolver.maxCorrection = 0.1f; c->positionSolver.maxVelocityUpdate = 1.0f;
    c->positionSolver.minSafeDistance = 1e-10f; c->positionSolver.velocityDamping = 0.3f;
    c->positionSolver.minPositionChange = 1e-6f;
    c->impulseSolver.maxForce = 0.15f; c->impulseSolver.maxTorque = 0.03f;
    c->impulseSolver.fluidForceScale = 100.0f; c->impulseSolver.fluidForceMax = 50000.0f;
    c->impulseSolver.buoyancyStrength = 0.2f; c->impulseSolver.viscosityScale = 0.05f;
    c->impulseSolver.depthScale = 0.04f; c->impulseSolver.depthTransitionRate = 2.0f;
    c->impulseSolver.depthEstimateScale = 10.0f; c->impulseSolver.pressureForceRatio = 1.0f;
    c->impulseSolver.viscousForceRatio = 0.3f; c->impulseSolver.angularDampingThreshold = 0.5f;
    c->impulseSolver.angularDampingFactor = 0.005f; c->impulseSolver.maxSafeVelocitySq = 80.0f;
    c->impulseSolver.minPenetration = 1e-6f; c->impulseSolver.minRelVelocity = 1e-6f;
    c->gridConfig.gridEpsilon = 1e-6f; c->gridConfig.smoothingLength = 0.05f;
    c->gridConfig.boundaryOffset = 0.001f;
    c->numericalConfig.minDistanceThreshold = 1e-14f;
    c->numericalConfig.minDensityThreshold = 1e-12f;
    c->numericalConfig.minTimestep = 1e-10f; c->numericalConfig.fallbackTimestep = 1e-4f;
    c->dampingFactor = 1.0f; c->numSubSteps = 10; c->threadsPerGroup = 256;
    return LPE_OK;
}

extern "C" int lpe_sph_set_config(lpe_ctx *ctx, const lpe_fluid_config *cfg) {
    if (!ctx || !cfg) return LPE_ERR_ARG;
    if (cfg->numSubSteps < 0) return LPE_ERR_ARG;
    int st = sph_void_prelaunch(ctx);
    if (st) return st;
    ctx->sph.cfg = *cfg;
    ctx->sph.cfg_set = true;
    ctx->sph.rig_dirty = true;
    return LPE_OK;
}

// cellSize = 2 * max(0.05, max_i h_i), h_i = smoothingLength (fluid.cpp:724-737)
static float ref_cell_size(const lpe_fluid_config &c) {
    float maxH = 0.05f;
    if (c.gridConfig.smoothingLength > maxH) maxH = c.gridConfig.smoothingLength;
    return 2.f * maxH;
}

// absolute device grid [gx0, gx1] x [gy0, gy1] (reference cells)
static int sph_set_grid(lpe_ctx *ctx, int gx0, int gy0, int gx1, int gy1) {
    SphDev &d = ctx->sph;
    if (d.pside) LPE_HIP(ctx, hipStreamSynchronize(d.pside));   // the bins may be re-allocated
    d.pre = false;
    const long nW = (long)gx1 - gx0 + 1, nH = (long)gy1 - gy0 + 1;
    long C = 4L * nW * nH;
    // (a sorted record's bin keeps its cell row and column in 15 bits each:
    // bin_cell); the grid in use stays as it was
    if (C > (1L << 29) || nW >= (1 << 15) || nH >= (1 << 15) || nW < 1 || nH < 1) {
        ctx->err = "device grid too large (the fluid spans more than 32767 cells, or 2^27 cells in all)";
        return LPE_ERR_CAPACITY;
    }
    d.ox = gx0; d.oy = gy0;
    d.W = (int)nW; d.H = (int)nH;
    if (C > d.cap_cells) {
        void *old[] = {d.count, d.start, d.cursor, d.blocksum};
        for (void *p : old) if (p) (void)hipFree(p);
        d.count = d.start = d.cursor = d.blocksum = nullptr;
        LPE_HIP(ctx, hipMalloc((void **)&d.count, sizeof(int32_t) * C));
        LPE_HIP(ctx, hipMalloc((void **)&d.start, sizeof(int32_t) * (C + 1)));
        LPE_HIP(ctx, hipMalloc((void **)&d.cursor, sizeof(int32_t) * C));
        LPE_HIP(ctx, hipMalloc((void **)&d.blocksum, sizeof(int32_t) * (C / SCAN_ELEMS + 2)));
        d.cap_cells = (int)C;
    }
    if (d.H > d.cap_rows || !d.rowtot) {
        if (d.rowtot) (void)hipFree(d.rowtot);
        d.rowtot = nullptr;
        LPE_HIP(ctx, hipMalloc((void **)&d.rowtot, sizeof(int32_t) * 2 * (size_t)d.H));
        d.cap_rows = d.H;
    }
    // the in-bin id bucket (k_bucket_permute) for grids up to 2^25 bins (4 GiB;
    // LPE_NO_BUCKET=1: off, the scatter + rank pass)
    static const bool noBucket = getenv("LPE_NO_BUCKET") != nullptr;
    if (!noBucket && C <= (1L << 25) && C > d.cap_bucket) {
        if (d.bucket) (void)hipFree(d.bucket);
        d.bucket = nullptr;
        d.cap_bucket = 0;
        LPE_HIP(ctx, hipMalloc((void **)&d.bucket, sizeof(int32_t) * BKT_CAP * (size_t)C));
        d.cap_bucket = C;
    }
    if (d.bovf) LPE_HIP(ctx, hipMemsetAsync(d.bovf, 0, sizeof(int32_t) * 2 * ovf_words(d), ctx->stream));
    LPE_HIP(ctx, hipMemsetAsync(d.count, 0, sizeof(int32_t) * C, ctx->stream));
    LPE_HIP(ctx, hipMemsetAsync(d.rowtot, 0, sizeof(int32_t) * 2 * (size_t)d.cap_rows, ctx->stream));
    d.fast_armed = false;
    d.fast_bucket = false;
    d.rig_dirty = true;    // the coupling bins span the device grid
    return LPE_OK;
}

// absolute device grid covering the particle bbox with a generous margin
static int sph_plan_grid(lpe_ctx *ctx, const float *x, const float *y, int n) {
    SphDev &d = ctx->sph;
    float cs = ref_cell_size(d.cfg);
    float mnx = 1e30f, mxx = -1e30f, mny = 1e30f, mxy = -1e30f;
    for (int i = 0; i < n; i++) {
        mnx = std::min(mnx, x[i]); mxx = std::max(mxx, x[i]);
        mny = std::min(mny, y[i]); mxy = std::max(mxy, y[i]);
    }
    if (n == 0) { mnx = mny = 0.f; mxx = mxy = 1.f; }
    // margin: 25% of the extent on every side, at least 64 cells
    float ex = std::max(mxx - mnx, mxy - mny);
    int pad = std::max(64, (int)(0.25f * ex / cs) + 8);
    d.cs = cs;
    return sph_set_grid(ctx, (int)std::floor(mnx / cs) - pad, (int)std::floor(mny / cs) - pad,
                        (int)std::floor(mxx / cs) + pad, (int)std::floor(mxy / cs) + pad);
}

// A slab rank only ever holds particles near its slab: its edges move at
// most mv columns (rebalancing), its ghosts lie SLAB_BAND columns beyond
// them, a kicked particle a fraction of a column further -- so its device
// grid covers the wanted cells only that far past its inner edges
// (slab_clip_cols).

// the device grid grown to cover the cells [gx0, gx1] x [gy0, gy1] (the
// union with the grid in use); recentre: if that union would be more than
// four times the wanted area, the wanted cells alone (a fluid drifting far
// from where it started leaves the old cells empty)
static int sph_cover_cells(lpe_ctx *ctx, long gx0, long gy0, long gx1, long gy1, bool recentre) {
    SphDev &d = ctx->sph;
    slab_clip_cols(d, gx0, gx1);
    if (gx1 < gx0) gx1 = gx0;
    long ux0 = std::min<long>(d.ox, gx0), uy0 = std::min<long>(d.oy, gy0);
    long ux1 = std::max<long>(d.ox + d.W - 1, gx1), uy1 = std::max<long>(d.oy + d.H - 1, gy1);
    if (ux0 == d.ox && uy0 == d.oy && ux1 == d.ox + d.W - 1 && uy1 == d.oy + d.H - 1) return LPE_OK;
    if (recentre && (ux1 - ux0 + 1) * (uy1 - uy0 + 1) > 4 * (gx1 - gx0 + 1) * (gy1 - gy0 + 1)) {
        ux0 = gx0; uy0 = gy0; ux1 = gx1; uy1 = gy1;
    }
    const long lim = 1L << 20;     // (sph_set_grid refuses more than 32767 cells a side)
    if (ux0 < -lim || uy0 < -lim || ux1 > lim || uy1 > lim) {
        ctx->err = "device grid too large (the fluid spans more than 32767 cells, or 2^27 cells in all)";
        return LPE_ERR_CAPACITY;
    }
    return sph_set_grid(ctx, (int)ux0, (int)uy0, (int)ux1, (int)uy1);
}

// grow the device grid to cover [x0, x1] x [y0, y1] (world mode: the
// universe the boundary system keeps every body and particle in)
int lpe_sph_cover_box(lpe_ctx *ctx, double x0, double y0, double x1, double y1) {
    SphDev &d = ctx->sph;
    if (d.cs <= 0.f || (d.n <= 0 && !d.shard)) return LPE_OK;
    const double cs = d.cs;
    return sph_cover_cells(ctx, (long)std::floor(x0 / cs) - 4, (long)std::floor(y0 / cs) - 4,
                           (long)std::floor(x1 / cs) + 4, (long)std::floor(y1 / cs) + 4, false);
}

static int pstate_alloc(lpe_ctx *ctx, PState &p, size_t N, bool with_a) {
    float **fl[] = {&p.x, &p.y, &p.vx, &p.vy, &p.vhx, &p.vhy, &p.m};
    for (float **q : fl) LPE_HIP(ctx, hipMalloc((void **)q, sizeof(float) * N));
    if (with_a) {
        LPE_HIP(ctx, hipMalloc((void **)&p.ax, sizeof(float) * N));
        LPE_HIP(ctx, hipMalloc((void **)&p.ay, sizeof(float) * N));
    }
    LPE_HIP(ctx, hipMalloc((void **)&p.id, sizeof(int32_t) * N));
    return LPE_OK;
}

// slots per particle array: n (single domain); a slab rank's owned particles
// and received ghosts, with room for its owned count to grow (slab_cap)
static long slab_cap(const Shard &h, int n) { return 2L * n + 4L * h.wcap + 4096; }
static int sph_realloc_slots(lpe_ctx *ctx, int n);
static int sph_alloc_particles(lpe_ctx *ctx, int n) {
    SphDev &d = ctx->sph;
    Shard *h = d.shard;
    if (h) {
        const long want = slab_cap(*h, n);
        if (want > (1L << 30)) { ctx->err = "slab capacity too large"; return LPE_ERR_CAPACITY; }
        n = (int)want;
    }
    if (n <= d.cap_n && d.P.x) return LPE_OK;
    return sph_realloc_slots(ctx, n);
}
// every per-slot array for n slots (the particle state P, rho and pr are
// freed like the scratch: sph_grow_slots detaches them first to keep them)
static int sph_realloc_slots(lpe_ctx *ctx, int n) {
    SphDev &d = ctx->sph;
    pstate_free(d.P);
    pstate_free(d.S);
    void *ptrs[] = {d.rho, d.pr, d.nbA, d.nbB, d.nlist, d.ncount, d.key, d.tmpId, d.tmpOld, d.bboxPart, d.refInv,
                    d.stage, d.rhoN, d.prN, d.fplans};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    size_t N = (size_t)std::max(n, 1);
    int st = pstate_alloc(ctx, d.P, N, true);
    if (st) return st;
    st = pstate_alloc(ctx, d.S, N, false);
    if (st) return st;
    LPE_HIP(ctx, hipMalloc((void **)&d.rho, sizeof(float) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.pr, sizeof(float) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.rhoN, sizeof(float) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.prN, sizeof(float) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.nbA, sizeof(float4) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.nbB, sizeof(float4) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.nlist, sizeof(uint4) * N * (NLIST_CAP / 8)));
    LPE_HIP(ctx, hipMalloc((void **)&d.ncount, sizeof(int32_t) * N));
    LPE_HIP(ctx, hipMalloc(&d.fplans, sizeof(Hood) * ((N + HB - 1) / HB)));
    LPE_HIP(ctx, hipMalloc((void **)&d.key, sizeof(uint32_t) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.tmpId, sizeof(int32_t) * N));
    LPE_HIP(ctx, hipMalloc((void **)&d.tmpOld, sizeof(int32_t) * N));
    // (id -> sorted slot: a slab rank's ids are the whole fluid's, lpe_sph_set_global_count)
    LPE_HIP(ctx, hipMalloc((void **)&d.refInv, sizeof(int32_t) * std::max(N, (size_t)std::max(sh_nglobal(d), 0))));
    LPE_HIP(ctx, hipMalloc((void **)&d.stage, sizeof(float) * N));
    // the grid hash's overflow lists (one entry per particle at most; both counts start at 0)
    if (d.bovf) (void)hipFree(d.bovf);
    d.bovf = nullptr;
    LPE_HIP(ctx, hipMalloc((void **)&d.bovf, sizeof(int32_t) * 2 * (4 + 4 * N)));
    LPE_HIP(ctx, hipMemsetAsync(d.bovf, 0, sizeof(int32_t) * 2 * (4 + 4 * N), ctx->stream));

    // bbox partials: the kick's blocks, or the forces pass's when it kicks the next sub-step
    LPE_HIP(ctx, hipMalloc((void **)&d.bboxPart, sizeof(float4) * std::max<size_t>(MAX_KICK_BLOCKS,
                                                                                    (N + HB - 1) / HB + HEAVY_HEAD)));
    // heavy tiles of the forces pass: two lists by parity, a flag per tile
    if (d.heavy) (void)hipFree(d.heavy);
    if (d.tileHeavy) (void)hipFree(d.tileHeavy);
    d.heavy = d.tileHeavy = nullptr;
    LPE_HIP(ctx, hipMalloc((void **)&d.heavy, sizeof(int32_t) * 2 * HEAVY_WORDS));
    LPE_HIP(ctx, hipMemsetAsync(d.heavy, 0, sizeof(int32_t) * 2 * HEAVY_WORDS, ctx->stream));
    LPE_HIP(ctx, hipMalloc((void **)&d.tileHeavy, sizeof(int32_t) * ((N + HB - 1) / HB)));
    LPE_HIP(ctx, hipMemsetAsync(d.tileHeavy, 0, sizeof(int32_t) * ((N + HB - 1) / HB), ctx->stream));
    d.cap_n = n;
    if (!d.ovl) {
        LPE_HIP(ctx, hipMalloc((void **)&d.ovl, sizeof(int32_t) * 2 * OVL_WORDS));
        LPE_HIP(ctx, hipMemsetAsync(d.ovl, 0, sizeof(int32_t) * 2 * OVL_WORDS, ctx->stream));
        d.ovl_cur = d.ovl_pre = d.ovl;
    }
    if (!d.gp) {
        LPE_HIP(ctx, hipMalloc((void **)&d.gp, 2 * sizeof(GridParams)));
        LPE_HIP(ctx, hipMalloc((void **)&d.status, sizeof(int32_t) * 2 * ST_COUNT));
        LPE_HIP(ctx, hipMemsetAsync(d.gp, 0, 2 * sizeof(GridParams), ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.status, 0, sizeof(int32_t) * 2 * ST_COUNT, ctx->stream));
    }
    d.gp_cur = d.gp;
    d.stat_cur = d.status;
    return LPE_OK;
}

static void sph_lag_reset(lpe_ctx *ctx);
extern "C" int lpe_sph_upload(lpe_ctx *ctx, int n, const float *x, const float *y,
                              const float *vx, const float *vy, const float *mass,
                              const float *density, const float *pressure) {
    if (!ctx || n < 0) return LPE_ERR_ARG;
    if (n > 0 && (!x || !y || !vx || !vy || !mass)) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    SphDev &d = ctx->sph;
    if (d.pside) LPE_HIP(ctx, hipStreamSynchronize(d.pside));   // buffers may be re-allocated
    d.pre = false;
    sph_lag_reset(ctx);                                          // (the records of the old state)
    int st = sph_alloc_particles(ctx, n);
    if (st) return st;
    d.n = n;
    if (d.shard) {
        // a slab rank's kernels run over its slot capacity, bounded by the
        // device counts (Shard::cnt): n owned slots to start with
        d.n = d.cap_n;
        d.shard->n0 = n;
        d.shard->cur = 0;
        const int32_t c3[3] = {n, 0, 0};
        LPE_HIP(ctx, hipMemcpy(d.shard->cnt, c3, sizeof(c3), hipMemcpyHostToDevice));
    }
    d.rig_dirty = true;
    st = sph_plan_grid(ctx, x, y, n);
    if (st) return st;
    size_t B = sizeof(float) * (size_t)n;
    hipStream_t s = ctx->stream;
    if (n > 0) {
        std::vector<int32_t> ids(n);
        for (int i = 0; i < n; i++) ids[i] = i;
        LPE_HIP(ctx, hipMemcpyAsync(d.P.x, x, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.y, y, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.vx, vx, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.vy, vy, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.m, mass, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.vhx, vx, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.vhy, vy, B, hipMemcpyHostToDevice, s));
        LPE_HIP(ctx, hipMemsetAsync(d.P.ax, 0, B, s));
        LPE_HIP(ctx, hipMemsetAsync(d.P.ay, 0, B, s));
        LPE_HIP(ctx, hipMemcpyAsync(d.P.id, ids.data(), sizeof(int32_t) * n,
                                    hipMemcpyHostToDevice, s));
        // density / pressure are carried from the ECS (fluid.cpp:294-295); they
        // are recomputed before any use, and are stored in P's slot order
        if (density) LPE_HIP(ctx, hipMemcpyAsync(d.rho, density, B, hipMemcpyHostToDevice, s));
        else LPE_HIP(ctx, hipMemsetAsync(d.rho, 0, B, s));
        if (pressure) LPE_HIP(ctx, hipMemcpyAsync(d.pr, pressure, B, hipMemcpyHostToDevice, s));
        else LPE_HIP(ctx, hipMemsetAsync(d.pr, 0, B, s));
        LPE_HIP(ctx, hipStreamSynchronize(s));
    }
    LPE_HIP(ctx, hipMemsetAsync(d.status, 0, sizeof(int32_t) * ST_COUNT, s));
    d.upload_gen++;
    return LPE_OK;
}

int sph_alloc_rigids(lpe_ctx *ctx, int n) {
    SphDev &d = ctx->sph;
    if (n <= d.cap_nr && d.rig) return LPE_OK;
    const size_t R = (size_t)std::max(n, 1);
    void *ptrs[] = {d.rig, d.accum, d.acq};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    d.rig = nullptr; d.accum = nullptr; d.acq = nullptr;
    LPE_HIP(ctx, hipMalloc((void **)&d.rig, sizeof(lpe_gpu_rigid) * R));
    LPE_HIP(ctx, hipMalloc((void **)&d.accum, sizeof(float) * 3 * R));
    LPE_HIP(ctx, hipMalloc((void **)&d.acq, sizeof(unsigned long long) * 3 * XACC_LIMBS * R));
    LPE_HIP(ctx, hipMemsetAsync(d.accum, 0, sizeof(float) * 3 * R, ctx->stream));
    LPE_HIP(ctx, hipMemsetAsync(d.acq, 0, sizeof(unsigned long long) * 3 * XACC_LIMBS * R, ctx->stream));
    d.cap_nr = (int)R;
    return LPE_OK;
}

extern "C" int lpe_sph_upload_rigids(lpe_ctx *ctx, int r, const lpe_gpu_rigid *rigids) {
    if (!ctx || r < 0 || (r > 0 && !rigids)) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    SphDev &d = ctx->sph;
    int st = sph_alloc_rigids(ctx, r);
    if (st) return st;
    d.nr = r;
    if (r > 0) {
        std::vector<lpe_gpu_rigid> tmp(rigids, rigids + r);
        for (auto &b : tmp) b.accumFx = b.accumFy = b.accumTorque = 0.f;
        LPE_HIP(ctx, hipMemcpyAsync(d.rig, tmp.data(), sizeof(lpe_gpu_rigid) * r,
                                    hipMemcpyHostToDevice, ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.accum, 0, sizeof(float) * 3 * r, ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.acq, 0, sizeof(unsigned long long) * 3 * XACC_LIMBS * r, ctx->stream));
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    d.rig_dirty = true;
    return LPE_OK;
}

static void sph_couple_params(const SphDev &d, CoupleParams &cp) {
    const lpe_fluid_config &c = d.cfg;
    cp.gravity = c.gravity; cp.restDensity = c.restDensity; cp.viscosity = c.viscosity;
    cp.maxForce = c.impulseSolver.maxForce; cp.maxTorque = c.impulseSolver.maxTorque;
    cp.viscosityScale = c.impulseSolver.viscosityScale; cp.depthScale = c.impulseSolver.depthScale;
    cp.depthTransitionRate = c.impulseSolver.depthTransitionRate;
    cp.pressureForceRatio = c.impulseSolver.pressureForceRatio;
    cp.viscousForceRatio = c.impulseSolver.viscousForceRatio;
    cp.angDampThr = c.impulseSolver.angularDampingThreshold;
    cp.angDampFactor = c.impulseSolver.angularDampingFactor;
    cp.depthEstimateScale = c.impulseSolver.depthEstimateScale;
    cp.maxSafeVelocitySq = c.impulseSolver.maxSafeVelocitySq;
    cp.minPenetration = c.impulseSolver.minPenetration;
    cp.minRelVelocity = c.impulseSolver.minRelVelocity;
    cp.fluidForceScale = c.impulseSolver.fluidForceScale;
    cp.fluidForceMax = c.impulseSolver.fluidForceMax;
    cp.buoyancyStrength = c.impulseSolver.buoyancyStrength;
    cp.safetyMargin = c.positionSolver.safetyMargin;
    cp.relaxFactor = c.positionSolver.relaxFactor;
    cp.minSafeDistance = c.positionSolver.minSafeDistance;
    cp.minPositionChange = c.positionSolver.minPositionChange;
    cp.maxCorrection = c.positionSolver.maxCorrection;
    cp.boundaryOffset = c.gridConfig.boundaryOffset;
    cp.bx0 = d.bx0; cp.by0 = d.by0; cp.bW = d.bW; cp.bH = d.bH; cp.bcs = d.bcs;
    cp.nr = d.nr;
}

// exclusive scan of C counts into start/cursor (and, for the fluid bins, the
// bbox finish + reference grid)
static int sph_scan(lpe_ctx *ctx, int C, int32_t *cnt, int32_t *start, int32_t *cursor,
                    int32_t *bsum, int nparts, bool fluid, const float4 *bbG = nullptr) {
    SphDev &d = ctx->sph;
    int nb = (C + SCAN_ELEMS - 1) / SCAN_ELEMS;
    hipStream_t s = ctx->stream;
    // the fluid hash with few tiles: k_scan_blocks' work folded into every
    // k_scan_final block (LPE_NO_SCAN_FUSION=1: off)
    // (the rigid bins too, as a plain prefix: no grid, no stats)
    static const bool nofuse = getenv("LPE_NO_SCAN_FUSION") != nullptr;
    const bool fused = nb <= 1024 && !nofuse;
    int32_t *ovl = fluid ? d.ovl + (size_t)(d.ovlIdx & 1) * OVL_WORDS : nullptr;
    int32_t *ovlNext = fluid ? d.ovl + (size_t)((d.ovlIdx + 1) & 1) * OVL_WORDS : nullptr;
    LPE_KERNEL(ctx, "k_scan_reduce", k_scan_reduce, dim3(nb), dim3(TPB), 0, s, C, cnt, bsum,
               fused && fluid ? d.stat_cur : (int32_t *)nullptr, ovl, ovlNext);
    if (!fused)
        LPE_KERNEL(ctx, "k_scan_blocks", k_scan_blocks, dim3(1), dim3(TPB), 0, s, nb, bsum, start + C, d.bboxPart,
                   nparts, d.cs, fluid ? d.gp_cur : (GridParams *)nullptr, d.stat_cur, bbG, d.ox, d.oy, d.W, d.H);
    LPE_KERNEL(ctx, "k_scan_final", k_scan_final, dim3(nb), dim3(TPB), 0, s, C, d.W, d.ox, d.oy, cnt, bsum,
               start, cursor, d.gp_cur, d.stat_cur, fluid ? 1 : 0, fused ? (fluid ? 1 : 2) : 0, (const float4 *)d.bboxPart,
               nparts, d.cs, bbG, ovl);
    LPE_CHECK_LAUNCH(ctx, "scan");
    if (fluid) {
        d.ovl_cur = ovl;
        d.ovlIdx++;
    }
    return LPE_OK;
}

// the compact coupling records of nr rigids (k_rig_couple's output; the world
// tick's gather writes them itself, rig_coupled)
float4 *sph_rig_records(lpe_ctx *ctx, int nr) {
    SphDev &d = ctx->sph;
    if (nr > d.cap_raabb || !d.raabb) {
        if (d.raabb) (void)hipFree(d.raabb);
        d.raabb = nullptr;
        d.cap_raabb = 0;
        if (hipMalloc((void **)&d.raabb, sizeof(float4) * (size_t)std::max(nr, 1) * (1 + RIGC_F4)) != hipSuccess) {
            ctx->err = "hipMalloc (rigid coupling records)";
            return nullptr;
        }
        d.cap_raabb = std::max(nr, 1);
    }
    return d.raabb;
}

// pre: the prelaunched sub-step's stats to merge (k_rbin_sort does it; *merged set)
static int sph_build_rigid_bins(lpe_ctx *ctx, int32_t *pre = nullptr, bool *merged = nullptr) {
    SphDev &d = ctx->sph;
    if (merged) *merged = false;
    if (d.nr <= 0 || !d.rig_dirty) return LPE_OK;
    // bin grid over the fluid device grid extent; bins of 0.25 m (>= 2h cells)
    d.bcs = std::max(0.25f, d.cs);
    d.bx0 = (int)std::floor(d.ox * d.cs / d.bcs) - 1;
    d.by0 = (int)std::floor(d.oy * d.cs / d.bcs) - 1;
    d.bW = (int)std::ceil(d.W * d.cs / d.bcs) + 3;
    d.bH = (int)std::ceil(d.H * d.cs / d.bcs) + 3;
    int B = d.bW * d.bH;
    int nbs = (B + SCAN_ELEMS - 1) / SCAN_ELEMS;
    if (B > d.cap_rbins) {
        if (d.rbinStart) (void)hipFree(d.rbinStart);
        if (d.rbinCount) (void)hipFree(d.rbinCount);
        LPE_HIP(ctx, hipMalloc((void **)&d.rbinStart, sizeof(int32_t) * (B + 1)));
        LPE_HIP(ctx, hipMalloc((void **)&d.rbinCount, sizeof(int32_t) * ((size_t)B * 2 + nbs + 4)));
        d.cap_rbins = B;
        d.rbin_zero = 0;
    }
    hipStream_t s = ctx->stream;
    if (!sph_rig_records(ctx, d.nr)) return LPE_ERR_HIP;
    if (!d.rig_coupled)
        LPE_KERNEL(ctx, "k_rig_couple", k_rig_couple, dim3(nblk(d.nr, 128)), dim3(128), 0, s, d.nr, d.rig,
                   d.cfg.impulseSolver.maxSafeVelocitySq, d.raabb);
    d.rig_coupled = false;
    if (B > d.rbin_zero)   // else the previous build's k_rbin_sort left counts [0, B) zeroed
        LPE_HIP(ctx, hipMemsetAsync(d.rbinCount, 0, sizeof(int32_t) * B, s));
    d.rbin_zero = 0;
    LPE_KERNEL(ctx, "k_rbin_count", k_rbin_count, dim3(nblk(d.nr, 4)), dim3(256), 0, s, d.nr, d.rig, d.bcs,
                       d.bx0, d.by0, d.bW, d.bH, d.rbinCount);
    int32_t *cursor = d.rbinCount + B;
    int st = sph_scan(ctx, B, d.rbinCount, d.rbinStart, cursor, d.rbinCount + 2 * B, 0, false);
    if (st) return st;
    // list length: a host-known bound (world mode, no sync) or read back once
    int total = d.rlist_bound;
    if (total <= 0) {
        LPE_HIP(ctx, hipMemcpyAsync(&total, d.rbinStart + B, sizeof(int), hipMemcpyDeviceToHost, s));
        LPE_HIP(ctx, hipStreamSynchronize(s));
    }
    if (total > d.cap_rlist || !d.rbinList) {
        if (d.rbinList) (void)hipFree(d.rbinList);
        // the list, then its entries' AABBs (float4, bin order: rbin_aabb)
        LPE_HIP(ctx, hipMalloc((void **)&d.rbinList, rbin_bytes(std::max(total, 1))));
        d.cap_rlist = std::max(total, 1);
    }
    d.rlist_len = total;
    LPE_KERNEL(ctx, "k_rbin_fill", k_rbin_fill, dim3(nblk(d.nr, 4)), dim3(256), 0, s, d.nr, d.rig, d.bcs,
                       d.bx0, d.by0, d.bW, d.bH, cursor, d.rbinList, d.cap_rlist, d.status);
    LPE_KERNEL(ctx, "k_rbin_sort", k_rbin_sort, dim3((B + RBS_WAVES - 1) / RBS_WAVES), dim3(256), 0, s, B, d.rbinStart, d.rbinList, d.cap_rlist,
               d.raabb, rbin_aabb(d), d.rbinCount, d.status, pre);
    if (merged) *merged = pre != nullptr;
    LPE_CHECK_LAUNCH(ctx, "rbin");
    d.rbin_zero = B;
    d.rig_dirty = false;
    return LPE_OK;
}

// The one-launch scan (k_scan_rows; LPE_NO_ROW_SCAN=1: off on a single
// domain, a slab rank always uses it): the kick that prepares it records the
// row totals (FastKick) into the buffer of the scan's parity.
static bool sph_rowscan_ok(const SphDev &d) {
    static const bool off = getenv("LPE_NO_ROW_SCAN") != nullptr;
    return (d.shard || !off) && d.rowtot && d.n > 0;
}
// the armed kick's FastKick again (the slab's ghost unpack files into the
// same histogram, bucket and row totals), without re-arming
static FastKick sph_fastkick_current(const SphDev &d) {
    FastKick fk{};
    if (!d.fast_armed) return fk;
    fk.on = 1;
    fk.rowtot = d.rowtot + (size_t)(d.fastIdx & 1) * d.cap_rows;
    if (d.fast_bucket) {
        fk.bucket = d.bucket;
        fk.ovf = d.bovf + (size_t)(d.fastIdx & 1) * ovf_words(d);
        fk.ovfcap = d.cap_n;
    }
    return fk;
}
static FastKick sph_fastkick(lpe_ctx *ctx, bool on) {
    SphDev &d = ctx->sph;
    FastKick fk{};
    fk.on = on ? 1 : 0;
    const bool bucket = on && d.bucket && d.bovf && d.cap_bucket >= 4L * d.W * d.H;
    if (on) {
        fk.rowtot = d.rowtot + (size_t)(d.fastIdx & 1) * d.cap_rows;
        if (bucket) {
            fk.bucket = d.bucket;
            fk.ovf = d.bovf + (size_t)(d.fastIdx & 1) * ovf_words(d);
            fk.ovfcap = d.cap_n;
        }
        // a kick whose scan never ran (an error in between) left its totals
        if (d.fast_armed) {
            (void)hipMemsetAsync(fk.rowtot, 0, sizeof(int32_t) * (size_t)d.cap_rows, ctx->stream);
            if (d.bovf)
                (void)hipMemsetAsync(d.bovf + (size_t)(d.fastIdx & 1) * ovf_words(d), 0, sizeof(int32_t), ctx->stream);
        }
    }
    d.fast_armed = on;
    d.fast_bucket = bucket;
    return fk;
}

// the sort after a kick: the scan (the reference grid and its stats), then
// the permutation into the new sorted order.  Slab rank: bbG the global
// bbox, ntot where the sorted count goes, nin the input slots (own +
// received), sk its edges (the stats cover its own columns).
static int sph_hash_sort(lpe_ctx *ctx, int kb, bool probe, const float4 *bbG, int32_t *ntot, const int32_t *nin,
                         SlabKick sk) {
    SphDev &d = ctx->sph;
    hipStream_t s = ctx->stream;
    int32_t *clear = nullptr;
    const int par = (int)(d.fastIdx & 1);
    const bool bucket = d.fast_armed && d.fast_bucket && !probe;
    if (d.fast_armed && !probe) {
        // one launch for the scan (the counts are cleared by the permute)
        LPE_KERNEL(ctx, "k_scan_rows", k_scan_rows, dim3(d.H), dim3(TPB), 0, s, d.W, d.H, d.ox, d.oy,
                   d.cfg.gridConfig.gridEpsilon, d.count, d.start, d.cursor, d.rowtot + (size_t)par * d.cap_rows,
                   d.rowtot + (size_t)(1 - par) * d.cap_rows, d.gp_cur, d.stat_cur, (const float4 *)d.bboxPart, kb,
                   d.cs, bucket ? d.bovf + (size_t)par * ovf_words(d) : (const int32_t *)nullptr, d.cap_n,
                   d.bovf ? d.bovf + (size_t)(1 - par) * ovf_words(d) : (int32_t *)nullptr, d.tmpId,
                   d.ovl + (size_t)(d.ovlIdx & 1) * OVL_WORDS, d.ovl + (size_t)((d.ovlIdx + 1) & 1) * OVL_WORDS,
                   bbG, ntot, sk);
        LPE_CHECK_LAUNCH(ctx, "k_scan_rows");
        d.ovl_cur = d.ovl + (size_t)(d.ovlIdx & 1) * OVL_WORDS;
        d.ovlIdx++;
        d.fastIdx++;
        clear = d.count;
    } else {
        if (sk.on) { ctx->err = "slab rank: the grid hash needs the row scan"; return LPE_ERR_STATE; }
        int st = sph_scan(ctx, 4 * d.W * d.H, d.count, d.start, d.cursor, d.blocksum, kb, true);
        if (st) return st;
    }
    d.fast_armed = false;
    d.fast_bucket = false;
    if (bucket) {
        LPE_KERNEL(ctx, "k_bucket_permute", k_bucket_permute, dim3(nblk(d.n)), dim3(TPB), 0, s, d.n, nin, d.key,
                   d.start, d.bucket, d.tmpId, d.P, sph_kstate(d), d.S, d.nbA,
                   (float2 *)d.nbB, sph_ref_inv(d), d.W, clear, d.stat_cur);
        LPE_CHECK_LAUNCH(ctx, "hash");
        return LPE_OK;
    }
    LPE_KERNEL(ctx, "k_scatter", k_scatter, dim3(nblk(d.n)), dim3(TPB), 0, s, d.n, d.key, d.P.id, d.cursor,
                       d.tmpId, d.tmpOld, nin);
    LPE_KERNEL(ctx, "k_rank_permute", k_rank_permute, dim3(nblk(d.n)), dim3(TPB), 0, s, d.n, d.key, d.start,
                       d.tmpId, d.tmpOld, d.P, sph_kstate(d), d.S, d.nbA, (float2 *)d.nbB, probe ? 1 : 0,
                       (const int32_t *)ntot, sph_ref_inv(d), d.W, clear);
    LPE_CHECK_LAUNCH(ctx, "hash");
    return LPE_OK;
}


static int sph_hash_slab(lpe_ctx *ctx, float subDt, float halfDt, bool first, int kicked);
static int status_error(lpe_ctx *ctx, const int32_t *status);

// one grid hash: kick (unless probe) + histogram + scan + scatter + rank/permute
// kicked > 0: the previous forces pass already kicked this sub-step (KickNext)
// and left `kicked` bbox partials.  A slab rank's hash (sph_hash_slab) adds
// the exchange between the kick and the scan.
static int sph_hash(lpe_ctx *ctx, float subDt, float halfDt, bool first, bool probe, int kicked = 0) {
    SphDev &d = ctx->sph;
    if (d.shard && !probe) return sph_hash_slab(ctx, subDt, halfDt, first, kicked);
    hipStream_t s = ctx->stream;
    int kb = kicked;
    if (!kicked) {
        kb = std::min(MAX_KICK_BLOCKS, std::max(1, nblk(d.n)));
        const FastKick fk = sph_fastkick(ctx, !probe && sph_rowscan_ok(d));
        LPE_KERNEL(ctx, "k_kick_drift", k_kick_drift, dim3(kb), dim3(TPB), 0, s, d.n, subDt, halfDt,
                   first ? 1 : 0, probe ? 1 : 0, d.cfg.gridConfig.gridEpsilon, d.cs, d.ox,
                   d.oy, d.W, d.H, d.P, sph_kstate(d), d.key, d.count, d.bboxPart, d.stat_cur, fk, SlabKick{});
        LPE_CHECK_LAUNCH(ctx, "k_kick_drift");
    }
    return sph_hash_sort(ctx, kb, probe, nullptr, nullptr, nullptr, SlabKick{});
}

// density over n slots (nptr: device count of the sharded sub-step); nl:
// also the neighbour lists of the forces pass (the tick), else density only
// (the probe / microbench)
static int sph_cu_count(lpe_ctx *ctx) {
    static int cus = 0;
    if (!cus) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess || v <= 0)
            v = 256;
        cus = v;
    }
    return cus;
}

// the density pass's block plans for the forces pass's LDS image
// (LPE_FORCES_NOIMG=1: none -- both passes fall back to slot-offset lists and
// global gathers, for A/B measurements)
static Hood *sph_fplans(SphDev &d) {
    static const bool off = getenv("LPE_FORCES_NOIMG") != nullptr;
    return off ? nullptr : (Hood *)d.fplans;
}

// heavy tiles of the forces pass (HeavyOut / HeavyIn): with at least
// HEAVY_MIN_RIGIDS coupling rigids and their bins, in plain block order
// (LPE_NO_HEAVY=1: off).  A handful of rigids -- the four walls of a dam
// break -- never make a tile heavy, and the part blocks' empty launches and
// the count in the density pass would only cost there.
static constexpr int HEAVY_MIN_RIGIDS = 64;
static bool sph_heavy_on(const SphDev &d) {
    static const bool off = getenv("LPE_NO_HEAVY") != nullptr;
    static const bool chunked = getenv("LPE_FORCES_CHUNK") != nullptr && atoi(getenv("LPE_FORCES_CHUNK")) > 0;
    return !off && !chunked && d.nr >= HEAVY_MIN_RIGIDS && d.rbinStart && d.heavy && d.tileHeavy;
}

static SlabKick slab_kick(const SphDev &d);
static int sph_density(lpe_ctx *ctx, int n, const int32_t *nptr, float *rho, float *pr, bool nl = true) {
    SphDev &d = ctx->sph;
    const lpe_fluid_config &c = d.cfg;
    static const bool v1 = getenv("LPE_DENSITY_V1") != nullptr;   // A/B switch: the one-particle-per-lane pass
    const int ntiles = (n + DT_TILE - 1) / DT_TILE;
    if (!nl && !v1 && !sph_ref_inv(d)) {
        if ((size_t)ntiles > d.cap_plans) {
            if (d.plans) (void)hipFree(d.plans);
            d.plans = nullptr;
            d.cap_plans = 0;
            LPE_HIP(ctx, hipMalloc(&d.plans, sizeof(Hood) * (size_t)ntiles));
            d.cap_plans = (size_t)ntiles;
        }
        LPE_KERNEL(ctx, "k_density_plan", k_density_plan, dim3(nblk(ntiles)), dim3(TPB), 0, ctx->stream, n, nptr,
                   c.gridConfig.gridEpsilon, d.W, d.H, d.ox, d.oy, d.gp_cur, d.start, d.nbA, (Hood *)d.plans);
        LPE_KERNEL(ctx, "k_density", k_density_pair, dim3(xcd_grid(ntiles)), dim3(DT_NT), 0, ctx->stream, n, nptr,
                   c.gridConfig.smoothingLength, c.gridConfig.gridEpsilon, c.stiffness, c.restDensity, d.W, d.H,
                   d.ox, d.oy, d.gp_cur, d.start, d.nbA, (float2 *)nullptr, rho, pr, d.stat_cur,
                   (const Hood *)d.plans);
    }
    else if (nl) {
        HeavyOut ho{};
        if (sph_heavy_on(d)) {
            d.heavyCur ^= 1;                          // (this pass's list; the forces pass reads it)
            ho.list = d.heavy + (size_t)d.heavyCur * HEAVY_WORDS;
            ho.tile = d.tileHeavy;
            ho.rbinStart = d.rbinStart;
            ho.rbinAabb = rbin_aabb(d);
            ho.bcs = d.bcs; ho.bx0 = d.bx0; ho.by0 = d.by0; ho.bW = d.bW; ho.bH = d.bH;
            // read per pass (the overflow parity test changes them between contexts)
            const char *qs = getenv("LPE_HEAVY_Q"), *hs = getenv("LPE_HEAVY_H");
            ho.qpairs = qs ? std::max(1, std::atoi(qs)) : QUARTER_PAIRS;
            ho.hpairs = hs ? std::max(1, std::atoi(hs)) : HALF_PAIRS;
        }
        LPE_KERNEL(ctx, "k_density", k_density<true>, dim3(xcd_grid(nblk(n, HB))), dim3(HB), 0, ctx->stream, n,
                   nptr, d.cap_n, c.gridConfig.smoothingLength, c.gridConfig.gridEpsilon, c.stiffness,
                   c.restDensity, d.W, d.H, d.ox, d.oy, d.gp_cur, d.start, d.nbA, (float2 *)d.nbB,
                   rho, pr, d.nlist, d.ncount, d.stat_cur, d.S.id, sph_ref_inv(d), d.ovl_cur, sph_fplans(d), ho,
                   slab_kick(d), d.shard ? d.shard->nglobal : 0);
    } else
        LPE_KERNEL(ctx, "k_density", k_density<false>, dim3(xcd_grid(nblk(n, HB))), dim3(HB), 0, ctx->stream, n,
                   nptr, d.cap_n, c.gridConfig.smoothingLength, c.gridConfig.gridEpsilon, c.stiffness,
                   c.restDensity, d.W, d.H, d.ox, d.oy, d.gp_cur, d.start, d.nbA, (float2 *)d.nbB,
                   rho, pr, d.nlist, d.ncount, d.stat_cur, d.S.id, sph_ref_inv(d), d.ovl_cur, (Hood *)nullptr,
                   HeavyOut{}, slab_kick(d), d.shard ? d.shard->nglobal : 0);
    LPE_CHECK_LAUNCH(ctx, "k_density");
    return LPE_OK;
}

// ---- x-slab decomposition (host side of the kernels above) -------------
const int32_t *sph_slab_slots(lpe_ctx *ctx) {
    const Shard *h = ctx->sph.shard;
    return h ? h->cnt + h->cur : nullptr;
}

static size_t wire_bytes(int wcap) { return sizeof(float) * (HDR + (size_t)wcap * GREC); }

// the slab rank's edges and send buffers for the kernels (nslot: the
// committed slot count, P's layout)
static SlabKick slab_kick(const SphDev &d) {
    SlabKick sk{};
    const Shard *h = d.shard;
    if (!h) return sk;
    sk.on = 1;
    sk.edges = h->edges;
    sk.rank = h->rank; sk.hasL = h->hasL; sk.hasR = h->hasR;
    const bool capped = (d.mode & LPE_SPH_MODE_REF_CELL_CAP) != 0;
    sk.band = capped ? SLAB_BAND_CAP : SLAB_BAND;
    sk.occ = capped ? d.status + ST_MAX_OCC_TOTAL : nullptr;
    sk.rband = h->cnt + 4;
    sk.sL = h->sL; sk.sR = h->sR; sk.wcap = h->wcap;
    sk.nslot = h->cnt + h->cur;
    return sk;
}
// where the hash in flight puts its sorted count (the density and forces
// passes' slot count), or null on a single domain
static const int32_t *slab_sorted(const SphDev &d) {
    return d.shard ? d.shard->cnt + (1 - d.shard->cur) : nullptr;
}

// A slab rank's grid hash: the kick (unless the previous forces pass did it;
// either files the ghost records), its bbox record, the exchange, the
// received ghosts, then the sort of every local slot.  The sorted count goes
// to cnt[1 - cur], committed (cur flipped) when the forces pass that reads
// it is launched, so a voided prelaunch leaves P's count as it was.
static int sph_hash_slab(lpe_ctx *ctx, float subDt, float halfDt, bool first, int kicked) {
    SphDev &d = ctx->sph;
    Shard &h = *d.shard;
    hipStream_t s = ctx->stream;
    if (!ctx->transport) {
        ctx->err = "slab decomposition without a transport (lpe_mg_init_rccl / lpe_mg_loopback_run)";
        return LPE_ERR_STATE;
    }
    if (!sph_rowscan_ok(d)) { ctx->err = "slab rank without particle arrays"; return LPE_ERR_STATE; }
    const float eps = d.cfg.gridConfig.gridEpsilon;
    int kb = kicked;
    if (!kicked) {
        kb = std::min(MAX_KICK_BLOCKS, std::max(1, nblk(d.n)));
        const FastKick fk = sph_fastkick(ctx, true);
        LPE_KERNEL(ctx, "k_kick_drift", k_kick_drift, dim3(kb), dim3(TPB), 0, s, d.n, subDt, halfDt,
                   first ? 1 : 0, 0, eps, d.cs, d.ox, d.oy, d.W, d.H, d.P, sph_kstate(d), d.key, d.count,
                   d.bboxPart, d.stat_cur, fk, slab_kick(d));
        LPE_CHECK_LAUNCH(ctx, "k_kick_drift");
    }
    LPE_KERNEL(ctx, "k_bbox_reduce", k_bbox_reduce, dim3(1), dim3(TPB), 0, s, d.bboxPart, kb, h.bbAll + h.rank);
    LPE_CHECK_LAUNCH(ctx, "k_bbox_reduce");
    // (one rank has no peer to exchange with; LPE_SLAB_FORCE_XCHG=1 calls the
    // transport anyway -- a probe of its per-call cost)
    static const bool force = getenv("LPE_SLAB_FORCE_XCHG") != nullptr;
    if (h.nranks > 1 || force) {
        int st = ctx->transport->exchange(ctx, h.hasL ? h.sL : nullptr, h.hasR ? h.sR : nullptr,
                                          h.hasL ? h.rL : nullptr, h.hasR ? h.rR : nullptr, wire_bytes(h.wcap), HDR,
                                          GREC, h.bbAll);
        if (st) return st;
    }
    LPE_KERNEL(ctx, "k_ghost_unpack", k_ghost_unpack, dim3(nblk1(2L * h.wcap)), dim3(TPB), 0, s,
               h.hasL ? h.rL : (const float *)nullptr, h.hasR ? h.rR : (const float *)nullptr, h.wcap,
               h.hasL ? h.sL : (float *)nullptr, h.hasR ? h.sR : (float *)nullptr, (const float4 *)h.bbAll, h.nranks,
               h.bbG, (const int32_t *)(h.cnt + h.cur), h.cnt + 2, d.cap_n, slab_kick(d), d.P, sph_kstate(d), d.key,
               d.count, sph_fastkick_current(d), eps, d.cs, d.ox, d.oy, d.W, d.H, d.stat_cur);
    LPE_CHECK_LAUNCH(ctx, "k_ghost_unpack");
    return sph_hash_sort(ctx, kb, false, h.bbG, h.cnt + (1 - h.cur), h.cnt + 2, slab_kick(d));
}

// Every `rebalance` ticks (after a fluid step): the owned particles per
// column, all-reduced, and the inner edges moved a column towards equal
// counts -- the same arithmetic on the same histogram on every rank.
static int slab_rebalance(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    Shard &h = *d.shard;
    h.ticks++;
    if (h.rebalance <= 0 || h.nranks < 2 || h.ticks % h.rebalance) return LPE_OK;
    hipStream_t s = ctx->stream;
    LPE_KERNEL(ctx, "k_slab_hist", k_slab_hist, dim3(nblk1(d.n)), dim3(TPB), 0, s, d.n,
               (const int32_t *)(h.cnt + h.cur), (const float *)d.P.x, (const int32_t *)d.P.id,
               d.cfg.gridConfig.gridEpsilon, d.cs, h.hcol0, h.hcols, h.hist);
    LPE_CHECK_LAUNCH(ctx, "k_slab_hist");
    int st = ctx->transport->allreduce(ctx, h.hist, h.hcols, 0);
    if (st) return st;
    LPE_KERNEL(ctx, "k_slab_rebalance", k_slab_rebalance, dim3(1), dim3(TPB), 0, s, h.hist, h.hcols, h.hcol0,
               h.edges, (const int32_t *)h.edges0, h.nranks, h.mv);
    LPE_CHECK_LAUNCH(ctx, "k_slab_rebalance");
    return LPE_OK;
}

// World tick (lpe_world.hip): sub-step 0's kick-drift, grid hash and density
// of the NEXT tick read only the fluid state, which is final once this tick's
// fluid boundary/gravity kernel has run; they are launched on a side stream
// then, so they run while the rigid solvers (one CU each) run, and that
// tick's lpe_sph_step starts at the forces (a slab rank's sub-step 0
// exchange runs on the side stream too, ordered after every exchange and
// reduction of the tick on the context stream).  The side stream is a plain one: a
// CU-masked queue (round 1 kept 16 CUs free for the solvers) cost a third of
// the tick rate on MI355X (396 vs 554 ticks/s on the settled metric scene),
// while the solvers start promptly without it.
int sph_prelaunch(lpe_ctx *ctx, double dt_tick, const std::function<int(hipStream_t)> &first, hipEvent_t ready,
                  bool devwait) {
    SphDev &d = ctx->sph;
    d.pre = false;
    if (d.n <= 0 || !d.P.x) return LPE_OK;
    if (!d.pside) {
        // default priority.  (LPE_PSIDE_PRIO=1: the lowest, so that the
        // solvers' workgroups would be dispatched first -- measured: the
        // tick rate halves, 344 against 740 ticks/s on the settled metric
        // scene, profiles/r04/prelaunch_priority_ab.txt)
        static const char *pp = getenv("LPE_PSIDE_PRIO");
        int least = 0, greatest = 0;
        if (pp && std::atoi(pp) != 0 && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
            LPE_HIP(ctx, hipStreamCreateWithPriority(&d.pside, hipStreamNonBlocking, least));
        else
            LPE_HIP(ctx, hipStreamCreateWithFlags(&d.pside, hipStreamNonBlocking));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d.preReady, hipEventDisableTiming));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d.preDone, hipEventDisableTiming));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d.fbgDone, hipEventDisableTiming));
    }
    bool waited = false;
    if (devwait) {
        int st = rigid_boundary_wait(ctx, d.pside, &waited);
        if (st) return st;
    }
    if (!waited) {
        if (!ready) {
            LPE_HIP(ctx, hipEventRecord(d.preReady, ctx->stream));
            ready = d.preReady;
        }
        LPE_HIP(ctx, hipStreamWaitEvent(d.pside, ready, 0));
    }
    if (first) {
        const int st0 = first(d.pside);
        if (st0) {
            (void)hipStreamSynchronize(d.pside);
            return st0;
        }
        LPE_HIP(ctx, hipEventRecord(d.fbgDone, d.pside));
    }
    const lpe_fluid_config &c = d.cfg;
    const float subDt = (float)dt_tick / (float)c.numSubSteps;
    const float halfDt = 0.5f * subDt;
    hipStream_t main = ctx->stream;
    // the hash / density helpers launch on ctx->stream and write gp_cur /
    // stat_cur: here the side stream and the prelaunch's own slots
    ctx->stream = d.pside;
    d.gp_cur = d.gp + 1;
    d.stat_cur = d.status + ST_COUNT;
    int st = hipMemsetAsync(d.stat_cur, 0, sizeof(int32_t) * ST_COUNT, d.pside) == hipSuccess ? LPE_OK : LPE_ERR_HIP;
    if (!st) st = sph_hash(ctx, subDt, halfDt, true, false);
    if (!st) st = sph_density(ctx, d.n, slab_sorted(d), d.rhoN, d.prN);   // P-order rho / p stay the tick's
    d.ovl_pre = d.ovl_cur;
    ctx->stream = main;
    d.gp_cur = d.gp;
    d.stat_cur = d.status;
    // recorded even after a failed launch, so whoever voids it waits on
    // everything that reached the side stream
    const bool rec = hipEventRecord(d.preDone, d.pside) == hipSuccess;
    if (st || !rec) {
        (void)hipStreamSynchronize(d.pside);
        ctx->err = st ? ctx->err : "hipEventRecord (prelaunch)";
        return st ? st : LPE_ERR_HIP;
    }
    d.pre = true;
    d.pre_dt = dt_tick;
    return LPE_OK;
}

// ---- lagged checks of the fluid step (SphDev::hlag) ---------------------
// Every lpe_sph_step call (and every world tick of a slab rank) ends with one
// small launch that copies the last sub-step's reference grid (the bbox of
// the particles, in cells; a slab rank's is the global one), the status words
// and the slots in use into a pinned ring slot.  The next call's end reads the
// previous record if it has landed, and the record two calls back (waiting
// for it: the host runs at most two calls ahead), and then
//   - fails with the status error the record shows (off-grid, slab slots,
//     halo...), two calls after the fact at most, as the rigid path's lagged
//     checks do; lpe_sph_download reports it too;
//   - grows the device grid when the bbox, widened by a margin that covers
//     four calls of its observed drift (16 cells at least), leaves it: the
//     reference regrows its grid to the bbox every sub-step
//     (fluid.cpp:740-755); here the bins are re-planned at a call boundary,
//     where no kernel holds them (each sub-step re-sorts from its kicked
//     positions, so the results do not depend on the device grid);
//   - grows a slab rank's slots (keeping its state) when the most slots a
//     sub-step wanted passes half of them.
static constexpr int LAG_WORDS = 32;     // [0, 7) GridParams, [8, 8 + ST_COUNT) status, [30] slots in use
static_assert(sizeof(GridParams) == 7 * sizeof(int32_t) && 8 + ST_COUNT <= 30, "lag record layout");

__global__ void __launch_bounds__(64)
k_lag_record(const GridParams *__restrict__ gp, const int32_t *__restrict__ status,
             const int32_t *__restrict__ slots, int32_t *__restrict__ out) {
    const int t = threadIdx.x;
    if (t < 7) out[t] = ((const int32_t *)gp)[t];
    if (t < ST_COUNT) out[8 + t] = status[t];
    if (t == 0) out[30] = slots ? *slots : 0;
}

// a slab rank's slots grown to `want`, keeping the particle state (P in its
// sorted order, rho, pr); everything else is per-sub-step scratch
static int sph_grow_slots(lpe_ctx *ctx, long want) {
    SphDev &d = ctx->sph;
    if (want > (1L << 30)) { ctx->err = "slab capacity too large"; return LPE_ERR_CAPACITY; }
    if (d.pside) LPE_HIP(ctx, hipStreamSynchronize(d.pside));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    d.pre = false;
    const size_t old = (size_t)d.cap_n;
    PState keep = d.P;
    float *rho = d.rho, *pr = d.pr;
    d.P = PState();
    d.rho = d.pr = nullptr;
    int st = sph_realloc_slots(ctx, (int)want);
    if (!st) {
        float *src[] = {keep.x, keep.y, keep.vx, keep.vy, keep.vhx, keep.vhy, keep.ax, keep.ay, keep.m, rho, pr};
        float *dst[] = {d.P.x, d.P.y, d.P.vx, d.P.vy, d.P.vhx, d.P.vhy, d.P.ax, d.P.ay, d.P.m, d.rho, d.pr};
        for (int k = 0; k < 11 && !st; k++)
            if (hipMemcpyAsync(dst[k], src[k], sizeof(float) * old, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess)
                st = LPE_ERR_HIP;
        if (!st && hipMemcpyAsync(d.P.id, keep.id, sizeof(int32_t) * old, hipMemcpyDeviceToDevice, ctx->stream) !=
                       hipSuccess)
            st = LPE_ERR_HIP;
        if (!st && hipStreamSynchronize(ctx->stream) != hipSuccess) st = LPE_ERR_HIP;
        if (st) ctx->err = "slab slot growth: copying the particle state";
    }
    pstate_free(keep);
    if (rho) (void)hipFree(rho);
    if (pr) (void)hipFree(pr);
    if (st) return st;
    d.n = d.cap_n;                 // (a slab rank's kernels run over its slot capacity)
    d.slot_regrows++;
    return LPE_OK;
}

// one record (slot), once it has landed (wait = false: only if it has)
static int sph_lag_check(lpe_ctx *ctx, int slot, bool wait, unsigned tick) {
    SphDev &d = ctx->sph;
    if (!d.lpend[slot]) return LPE_OK;
    if (wait) {
        LPE_HIP(ctx, hipEventSynchronize(d.evLag[slot]));
    } else {
        const hipError_t q = hipEventQuery(d.evLag[slot]);
        if (q == hipErrorNotReady) return LPE_OK;
        if (q != hipSuccess) { ctx->err = "hipEventQuery (lagged fluid check)"; return LPE_ERR_HIP; }
    }
    d.lpend[slot] = false;
    const int32_t *w = d.hlag + (size_t)LAG_WORDS * slot;
    int st = status_error(ctx, w + 8);
    if (st) return st;
    GridParams g;
    std::memcpy(&g, w, sizeof(g));
    if (d.n <= 0 && !d.shard) return LPE_OK;
    if (g.gridDimX <= 0 || g.gridDimY <= 0 || g.cellSize != d.cs) return LPE_OK;   // (no sub-step recorded)
    const long box[4] = {g.gridMinX, g.gridMinY, g.gridMinX + g.gridDimX - 1L, g.gridMinY + g.gridDimY - 1L};
    // the bbox's drift per call since the previous sample (outward only)
    long rate = 0;
    if (d.lag_prev && tick > d.lag_box_tick) {
        const long span = (long)(tick - d.lag_box_tick);
        const long out = std::max(std::max(d.lag_box[0] - box[0], d.lag_box[1] - box[1]),
                                  std::max(box[2] - d.lag_box[2], box[3] - d.lag_box[3]));
        rate = (std::max(out, 0L) + span - 1) / span;
    }
    if (!d.lag_prev || tick > d.lag_box_tick) {
        for (int k = 0; k < 4; k++) d.lag_box[k] = (int)box[k];
        d.lag_box_tick = tick;
        d.lag_prev = true;
    }
    const long m = 16 + 6 * rate;
    long wx0 = box[0] - m, wy0 = box[1] - m, wx1 = box[2] + m, wy1 = box[3] + m;
    slab_clip_cols(d, wx0, wx1);
    if (wx0 < d.ox || wy0 < d.oy || wx1 > d.ox + d.W - 1 || wy1 > d.oy + d.H - 1) {
        const long ex = std::max(box[2] - box[0], box[3] - box[1]);
        const long M = std::max(std::max(2 * m, 64L), ex / 4);
        if (d.pside) LPE_HIP(ctx, hipStreamSynchronize(d.pside));
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));   // (nothing in flight may hold the bins)
        st = sph_cover_cells(ctx, box[0] - M, box[1] - M, box[2] + M, box[3] + M, true);
        if (st) return st;
        d.grid_regrows++;
    }
    if (d.shard) {
        const long peak = std::max(w[8 + ST_SLOT_PEAK], w[30]);
        if (2 * peak > d.cap_n) {
            st = sph_grow_slots(ctx, std::max(2L * d.cap_n, 4 * peak + 4096));
            if (st) return st;
        }
    }
    return LPE_OK;
}

// the end of a call: the pending records, then this call's
static int sph_lag_service(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    if (!d.status || !d.gp) return LPE_OK;
    if (!d.hlag) {
        LPE_HIP(ctx, hipHostMalloc((void **)&d.hlag, sizeof(int32_t) * 2 * LAG_WORDS, 0));
        std::memset(d.hlag, 0, sizeof(int32_t) * 2 * LAG_WORDS);
        LPE_HIP(ctx, hipEventCreateWithFlags(&d.evLag[0], hipEventDisableTiming));
        LPE_HIP(ctx, hipEventCreateWithFlags(&d.evLag[1], hipEventDisableTiming));
    }
    const int slot = (int)(d.ltick & 1u);
    // the older record (this slot's, two calls back: waited for), then the previous one if it is in
    int st = sph_lag_check(ctx, slot, true, d.ltick - 2);
    if (!st) st = sph_lag_check(ctx, 1 - slot, false, d.ltick - 1);
    if (st) return st;
    LPE_KERNEL(ctx, "k_lag_record", k_lag_record, dim3(1), dim3(64), 0, ctx->stream, (const GridParams *)d.gp,
               (const int32_t *)d.status, sph_slab_slots(ctx), d.hlag + (size_t)LAG_WORDS * slot);
    LPE_CHECK_LAUNCH(ctx, "k_lag_record");
    LPE_HIP(ctx, hipEventRecord(d.evLag[slot], ctx->stream));
    d.lpend[slot] = true;
    d.ltick++;
    return LPE_OK;
}

// every pending record (an upload or a reconfiguration starts afresh)
static void sph_lag_reset(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    for (int k = 0; k < 2; k++)
        if (d.lpend[k] && d.evLag[k]) (void)hipEventSynchronize(d.evLag[k]);
    d.lpend[0] = d.lpend[1] = false;
    d.lag_prev = false;
}

extern "C" int lpe_sph_step(lpe_ctx *ctx, double dt_tick) {
    return sph_step_hooked(ctx, dt_tick, nullptr);
}

int sph_step_hooked(lpe_ctx *ctx, double dt_tick, int (*hook)(lpe_ctx *, int)) {
    if (!ctx) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (d.n <= 0 && !d.shard) return LPE_OK;  // fluid.cpp:969-972 (a slab rank joins the exchanges)
    if (!d.P.x) return LPE_ERR_STATE;
    (void)hipSetDevice(ctx->device);
    const lpe_fluid_config &c = d.cfg;
    float dt = (float)dt_tick;                       // fluid.cpp:592
    float subDt = dt / (float)c.numSubSteps;         // fluid.cpp:593
    float halfDt = 0.5f * subDt;
    hipStream_t s = ctx->stream;
    // sub-step 0 up to the forces already launched (sph_prelaunch)?  One for
    // another time step is discarded (it never touched P; on a slab rank every
    // rank must discard it alike: it joined an exchange)
    if (d.pre && d.pre_dt != dt_tick) {
        int st0 = sph_void_prelaunch(ctx);
        if (st0) return st0;
    }
    const bool pre = d.pre;
    d.pre = false;
    if (pre) {
        std::swap(d.rho, d.rhoN);                     // sub-step 0's density is the prelaunch's
        std::swap(d.pr, d.prN);
        LPE_HIP(ctx, hipStreamWaitEvent(s, d.preDone, 0));
    }
    bool merged = false;
    int st = sph_build_rigid_bins(ctx, pre ? d.status + ST_COUNT : nullptr, &merged);
    if (st) return st;
    if (pre) {
        // (k_rbin_sort, or else the first forces pass, resets the step stats
        // and merges the prelaunch's: sp.mergePre)
    } else {
        st = sph_reset_step_stats(ctx, s, d.status);
        if (st) return st;
    }
    SphStepParams sp;
    sp.n = d.n; sp.W = d.W; sp.H = d.H; sp.ox = d.ox; sp.oy = d.oy;
    sp.h = c.gridConfig.smoothingLength; sp.eps = c.gridConfig.gridEpsilon;
    sp.dt = subDt; sp.hdt = halfDt;
    sp.viscosity = c.viscosity;
    sp.minDist = c.numericalConfig.minDistanceThreshold;
    sp.minDens = c.numericalConfig.minDensityThreshold;
    {
        // the shortened quotients / square root of pair_term need r^2 >= 2^-60
        // (r >= 2^-30), rho_j >= 2^-60 and wVisc / rho_j <= lapC h / minDens far
        // below 2^90 (the general sequences' scaling thresholds); positions
        // 0 or of magnitude >= 2^-76 m keep the differences' numerators above
        // 2^-100 (any scene: the boundary keeps particles >= its margin inside)
        const double h = c.gridConfig.smoothingLength;
        const double lapC = 40.0 / (3.14159265358979 * std::pow(h, 5.0));   // (viscLaplacianCoeff2D)
        sp.shortDiv = sp.minDist >= 0x1p-60f && sp.minDens >= 0x1p-60f && h > 0.0 && h < 1e3 &&
                      lapC * h / sp.minDens < 0x1p80;
    }
    sp.diag = d.diag;
    sp.refInv = sph_ref_inv(d);
    sp.nptr = nullptr;
    sp.own = slab_kick(d);            // (on a slab rank: the slots it owns)
    sp.nref = sh_nglobal(d);
    sp.nstride = d.cap_n;
    Shard *sh = d.shard;
    if (sh && !ctx->transport) {
        ctx->err = "slab decomposition without a transport (lpe_mg_init_rccl / lpe_mg_loopback_run)";
        return LPE_ERR_STATE;
    }
    CoupleParams cp;
    sph_couple_params(d, cp);
    // each forces pass but the last also kicks the next sub-step (KickNext),
    // so its hash starts at the scan (slab ranks: at the bbox all-reduce);
    // LPE_NO_KICK_FUSION=1: off
    static const bool nofuse = getenv("LPE_NO_KICK_FUSION") != nullptr;
    const bool fuse = !nofuse;
    const int fblocks = nblk1(sp.n, HB);
    // forces blocks in XCD runs of LPE_FORCES_CHUNK blocks (0: plain order)
    static const int fchunk = [] {
        const char *e = getenv("LPE_FORCES_CHUNK");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    sp.nblk = fblocks;
    sp.chunk = fchunk;
    // tile scheduling: the filed blocks head the grid and leave their own bbox
    // partials after the tiles' (the scan reads fblocks + HEAVY_HEAD)
    const bool heavy = sph_heavy_on(d) && fchunk == 0;
    const int nq = heavy ? HEAVY_HEAD : 0;
    const int fgrid = (fchunk > 0 ? xcd_chunk_grid(fblocks, fchunk) : fblocks) + nq;
    int kicked = 0;
    for (int step = 0; step < c.numSubSteps; step++) {
        if (step == 0 && pre) {
            st = LPE_OK;                              // waited for above
        } else {
            st = sph_hash(ctx, subDt, halfDt, step == 0, false, kicked);
            if (st) return st;
            st = sph_density(ctx, d.n, slab_sorted(d), d.rho, d.pr);
        }
        if (st) return st;
        sp.nptr = slab_sorted(d);                     // (slab rank: the hash's sorted count)
        KickNext kn{};
        kn.on = fuse && step + 1 < c.numSubSteps;
        if (kn.on) {
            kn.dt = subDt; kn.hdt = halfDt; kn.eps = c.gridConfig.gridEpsilon; kn.cs = d.cs;
            kn.ox = d.ox; kn.oy = d.oy; kn.W = d.W; kn.H = d.H;
            const KState K = sph_kstate(d);
            kn.kx = K.x; kn.ky = K.y; kn.kvhx = K.vhx; kn.kvhy = K.vhy;
            kn.key = d.key; kn.count = d.count; kn.bboxPart = d.bboxPart;
            kn.fk = sph_fastkick(ctx, sph_rowscan_ok(d));
            kn.sk = slab_kick(d);
        }
        kicked = kn.on ? fblocks + nq : 0;
        sp.mergePre = (step == 0 && pre && !merged) ? d.status + ST_COUNT : nullptr;
        if (sp.mergePre && sp.refInv) {
            LPE_KERNEL(ctx, "k_merge_prestats", k_merge_prestats, dim3(1), dim3(64), 0, s, d.status, sp.mergePre);
            sp.mergePre = nullptr;
        }
        sp.ovl = (step == 0 && pre) ? d.ovl_pre : d.ovl_cur;
        const HeavyIn hv = heavy ? HeavyIn{d.heavy + (size_t)d.heavyCur * HEAVY_WORDS, d.tileHeavy,
                                           d.heavy + (size_t)(1 - d.heavyCur) * HEAVY_WORDS}
                                 : HeavyIn{};
        const GridParams *gpf = (step == 0 && pre) ? d.gp + 1 : d.gp;
        if (sp.shortDiv)
            LPE_KERNEL(ctx, "k_forces_couple", k_forces_couple<true>, dim3(fgrid), dim3(HB), 0, s, sp, cp, gpf,
                       d.start, d.S, d.nbA, d.nbB, d.pr, d.nlist, d.ncount, d.P, d.rig, d.raabb, d.rbinStart,
                       d.rbinList, rbin_aabb(d), d.acq, d.status, kn, (const Hood *)sph_fplans(d), hv);
        else
            LPE_KERNEL(ctx, "k_forces_couple", k_forces_couple<false>, dim3(fgrid), dim3(HB), 0, s, sp, cp, gpf,
                       d.start, d.S, d.nbA, d.nbB, d.pr, d.nlist, d.ncount, d.P, d.rig, d.raabb, d.rbinStart,
                       d.rbinList, rbin_aabb(d), d.acq, d.status, kn, (const Hood *)sph_fplans(d), hv);
        LPE_CHECK_LAUNCH(ctx, "k_forces_couple");
        if (sh) sh->cur = 1 - sh->cur;               // P's slots are now the ones this pass wrote
        if (hook) {                                  // (lpe_world_tick: the rigid detection)
            st = hook(ctx, step);
            if (st) return st;
        }
    }
    if (hook) {                                      // after the sub-steps: whatever is still pending
        st = hook(ctx, -1);
        if (st) return st;
    }
    if (d.nr > 0) {
        // slab decomposition: every rank holds its particles' share of the
        // fluid->rigid impulses; the rigids are replicated, so the shares are
        // summed before the write-back (fluid.cpp:545-562): the exact limbs
        // add as int64, so the result is the single domain's bit for bit
        if (sh) {
            st = ctx->transport->allreduce_i64(ctx, (long long *)d.acq, 3 * XACC_LIMBS * d.nr);
            if (st) return st;
        }
        LPE_KERNEL(ctx, "k_rigid_writeback", k_rigid_writeback, dim3(nblk(d.nr, 128)), dim3(128), 0, s, d.nr, d.rig,
                           d.acq, d.accum, c.dampingFactor, (const int32_t *)d.coupleBody, d.wb_bodies);
        LPE_CHECK_LAUNCH(ctx, "k_rigid_writeback");
    }
    if (sh) {
        st = slab_rebalance(ctx);
        if (st) return st;
    }
    // (a world tick's single-domain grid covers the universe, lpe_sph_cover_box)
    if (!hook || sh) return sph_lag_service(ctx);
    return LPE_OK;
}

// gather-order download of up to 6 sorted-order fields keyed by `id`; the S
// arrays (dead between sub-steps) are the staging buffers
static int sph_unpermute_download(lpe_ctx *ctx, const int32_t *id, int nf, const float **src,
                                  float **host) {
    SphDev &d = ctx->sph;
    hipStream_t s = ctx->stream;
    // staging: arrays a pending prelaunch no longer needs (it keeps S.vhx,
    // S.vhy, S.id, the records and the bins)
    int st0 = sph_join_prelaunch(ctx);
    if (st0) return st0;
    float *stage[6] = {d.S.x, d.S.y, d.S.vx, d.S.vy, d.S.m, d.stage};
    Fields6 f{};
    for (int k = 0; k < nf; k++) { f.src[k] = src[k]; f.dst[k] = stage[k]; }
    LPE_KERNEL(ctx, "k_unpermute", k_unpermute, dim3(nblk(d.n)), dim3(TPB), 0, s, d.n, id, nf, f);
    LPE_CHECK_LAUNCH(ctx, "k_unpermute");
    for (int k = 0; k < nf; k++)
        if (host[k])
            LPE_HIP(ctx, hipMemcpyAsync(host[k], stage[k], sizeof(float) * d.n,
                                        hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipStreamSynchronize(s));
    return LPE_OK;
}

static int check_status(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    if (!d.status) return LPE_OK;
    int32_t status[ST_COUNT];
    LPE_HIP(ctx, hipMemcpy(status, d.status, sizeof(status), hipMemcpyDeviceToHost));
    return status_error(ctx, status);
}

static int status_error(lpe_ctx *ctx, const int32_t *status) {
    if (status[ST_CAP_OVERFLOW]) {
        ctx->err = "a fluid particle left the device grid (it moved further than the grid's margin between two "
                   "lagged checks; lpe_sph_set_domain can cover the region the fluid reaches)";
        return LPE_ERR_CAPACITY;
    }
    if (status[ST_LIST_OVERFLOW]) {
        ctx->err = "the rigid coupling bin list overflowed its capacity bound";
        return LPE_ERR_OVERFLOW;
    }
    if (status[ST_BUCKET_OVERFLOW]) {
        ctx->err = "the grid hash's in-bin sort lost a particle (bucket overflow list or rank check)";
        return LPE_ERR_OVERFLOW;
    }
    if (status[ST_HALO_DRIFT]) {
        ctx->err = "slab decomposition: a particle was kicked past its neighbour's slab (it would belong to no "
                   "rank; slabs must be wider than a sub-step's drift)";
        return LPE_ERR_OVERFLOW;
    }
    if (status[ST_SLAB_CAPACITY]) {
        ctx->err = "slab decomposition: the rank's own and received particles outgrew its slots";
        return LPE_ERR_CAPACITY;
    }
    if (status[ST_XACC_RANGE]) {
        ctx->err = "a rigid coupling force left the exact accumulator's range (|f| >= 2^64 or not finite)";
        return LPE_ERR_OVERFLOW;
    }
    if (status[ST_REF_SLAB]) {
        ctx->err = std::string("slab decomposition, reference cell-capacity mode: the reference's loop read past an "
                               "over-full cell into a cell the rank does not hold (") +
                   ((status[ST_REF_SLAB] & 1) ? "a cell of more than 129 particles at the ghost band's edge" : "") +
                   ((status[ST_REF_SLAB] & 3) == 3 ? "; " : "") +
                   ((status[ST_REF_SLAB] & 2) ? "the global grid's row wrap: an over-full cell in its last column" : "") +
                   ")";
        return LPE_ERR_CAPACITY;
    }
    if (status[ST_HALO_OVERFLOW]) {
        ctx->err = "slab decomposition: more ghost records than wire_cap along a slab edge in a sub-step (raise "
                   "wire_cap of lpe_sph_set_slab)";
        return LPE_ERR_OVERFLOW;
    }
    return LPE_OK;
}

extern "C" int lpe_sph_download(lpe_ctx *ctx, float *x, float *y, float *vx, float *vy,
                                float *density, float *pressure) {
    if (!ctx) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (d.shard) {
        ctx->err = "slab decomposition: the ranks hold global ids, use lpe_sph_download_owned";
        return LPE_ERR_STATE;
    }
    if (d.n > 0) {
        const float *src[6] = {d.P.x, d.P.y, d.P.vx, d.P.vy, d.rho, d.pr};
        float *dst[6] = {x, y, vx, vy, density, pressure};
        int st = sph_unpermute_download(ctx, d.P.id, 6, src, dst);
        if (st) return st;
    }
    return check_status(ctx);
}

extern "C" int lpe_sph_download_aux(lpe_ctx *ctx, float *vxHalf, float *vyHalf, float *ax,
                                    float *ay) {
    if (!ctx) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (d.shard) { ctx->err = "slab decomposition: use lpe_sph_download_owned"; return LPE_ERR_STATE; }
    if (d.n <= 0) return LPE_OK;
    const float *src[4] = {d.P.vhx, d.P.vhy, d.P.ax, d.P.ay};
    float *dst[4] = {vxHalf, vyHalf, ax, ay};
    return sph_unpermute_download(ctx, d.P.id, 4, src, dst);
}

extern "C" int lpe_sph_download_rigids(lpe_ctx *ctx, lpe_gpu_rigid *rigids, float *accum) {
    if (!ctx) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    hipStream_t s = ctx->stream;
    if (d.nr > 0) {
        if (rigids)
            LPE_HIP(ctx, hipMemcpyAsync(rigids, d.rig, sizeof(lpe_gpu_rigid) * d.nr,
                                        hipMemcpyDeviceToHost, s));
        if (accum)
            LPE_HIP(ctx, hipMemcpyAsync(accum, d.accum, sizeof(float) * 3 * d.nr,
                                        hipMemcpyDeviceToHost, s));
    }
    LPE_HIP(ctx, hipStreamSynchronize(s));
    return LPE_OK;
}

extern "C" int lpe_sph_get_stats(lpe_ctx *ctx, lpe_sph_stats *out) {
    if (!ctx || !out) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    std::memset(out, 0, sizeof(*out));
    if (!d.status) return LPE_OK;
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int32_t status[ST_COUNT];
    GridParams g;
    LPE_HIP(ctx, hipMemcpy(status, d.status, sizeof(status), hipMemcpyDeviceToHost));
    LPE_HIP(ctx, hipMemcpy(&g, d.gp, sizeof(g), hipMemcpyDeviceToHost));
    out->maxCellOccupancy = status[ST_MAX_OCC];
    out->notInserted = status[ST_NOT_INSERTED];
    out->capacityOverflow = status[ST_CAP_OVERFLOW];
    out->listOverflow = status[ST_LIST_OVERFLOW];
    out->gridDimX = g.gridDimX; out->gridDimY = g.gridDimY;
    out->gridMinX = g.gridMinX; out->gridMinY = g.gridMinY;
    out->cellSize = g.cellSize;
    out->nlistOverflow = status[ST_NL_OVERFLOW];
    out->rigidCandidates = status[ST_RIGID_CAND];
    out->neighbours = status[ST_NEIGH];
    out->stageFallback = status[ST_STAGE_FALLBACK];
    out->forcesGlobal = status[ST_FORCES_GLOBAL];
    out->overCapCells = status[ST_OVER_CAP];
    out->refUndefined = status[ST_REF_UB];
    out->overCapCellsTotal = status[ST_OVER_CAP_TOTAL];
    out->maxCellOccupancyTotal = status[ST_MAX_OCC_TOTAL];
    out->gridRegrows = (int32_t)d.grid_regrows;
    out->slotRegrows = (int32_t)d.slot_regrows;
    out->deviceGrid[0] = d.ox; out->deviceGrid[1] = d.oy; out->deviceGrid[2] = d.W; out->deviceGrid[3] = d.H;
    out->haloWire[0] = (d.shard && d.shard->hasL) ? d.shard->wcap : 0;
    out->haloWire[1] = (d.shard && d.shard->hasR) ? d.shard->wcap : 0;
    if (d.shard) {
        Shard &h = *d.shard;
        int32_t c2[2] = {0, 0};
        LPE_HIP(ctx, hipMemsetAsync(h.cnt + 3, 0, sizeof(int32_t), ctx->stream));
        LPE_KERNEL(ctx, "k_slab_gather_owned", k_slab_gather_owned, dim3(nblk1(d.n)), dim3(TPB), 0, ctx->stream,
                   d.n, (const int32_t *)(h.cnt + h.cur), d.P, (const float *)d.rho, (const float *)d.pr, Fields6{},
                   (int32_t *)nullptr, h.cnt + 3);
        LPE_HIP(ctx, hipMemcpyAsync(&c2[0], h.cnt + 3, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
        LPE_HIP(ctx, hipMemcpyAsync(&c2[1], h.cnt + h.cur, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        out->slabOwned = c2[0];
        out->slabSlots = c2[1];
        out->ghostsIn[0] = status[ST_RX_GHOST_L];
        out->ghostsIn[1] = status[ST_RX_GHOST_R];
    }
    return LPE_OK;
}

extern "C" int lpe_sph_set_mode(lpe_ctx *ctx, int flags) {
    if (!ctx || (flags & ~(LPE_SPH_MODE_REF_CELL_CAP | LPE_SPH_MODE_PROBE_TICK_PASS))) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if ((flags & LPE_SPH_MODE_REF_CELL_CAP) && d.shard && d.shard->nglobal <= 0) {
        ctx->err = "slab rank: the reference cell-capacity mode needs the whole fluid's particle count "
                   "(lpe_sph_set_global_count) and a wire sized for SLAB_BAND_CAP ghost columns";
        return LPE_ERR_STATE;
    }
    // (every rank of a slab group sets the same mode at the same point: the
    // band it files ghosts in follows it, slab_kick)
    int st = sph_void_prelaunch(ctx);        // a prelaunched sub-step ran in the old mode
    if (st) return st;
    d.mode = flags;
    return LPE_OK;
}

extern "C" int lpe_sph_diag(lpe_ctx *ctx, int on) {
    if (!ctx) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    d.diag = on ? 1 : 0;
    if (d.status) {
        LPE_HIP(ctx, hipMemsetAsync(d.status + ST_NL_OVERFLOW, 0, sizeof(int32_t) * 4, ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.status + ST_OVER_CAP_TOTAL, 0, sizeof(int32_t) * 2, ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.status + ST_RX_GHOST_L, 0, sizeof(int32_t) * 2, ctx->stream));
    }
    return LPE_OK;
}

int lpe_sph_hash_current(lpe_ctx *ctx) {
    SphDev &d = ctx->sph;
    if (d.shard) { ctx->err = "not on a slab rank (its slots hold ghosts)"; return LPE_ERR_STATE; }
    if (d.n <= 0) return LPE_OK;
    int st = sph_void_prelaunch(ctx);           // the probe's hash reuses the prelaunch's buffers
    if (st) return st;
    st = sph_reset_step_stats(ctx, ctx->stream, d.status);
    if (st) return st;
    return sph_hash(ctx, 0.f, 0.f, false, true);
}

extern "C" int lpe_sph_probe_cells(lpe_ctx *ctx, int32_t *cell_index, lpe_sph_stats *stats) {
    if (!ctx || !cell_index) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (d.shard) { ctx->err = "not on a slab rank (its slots hold ghosts)"; return LPE_ERR_STATE; }
    if (d.n <= 0) return LPE_OK;
    (void)hipSetDevice(ctx->device);
    int st = sph_void_prelaunch(ctx);           // the probe's hash reuses the prelaunch's buffers
    if (st) return st;
    st = sph_reset_step_stats(ctx, ctx->stream, d.status);
    if (st) return st;
    st = sph_hash(ctx, 0.f, 0.f, false, true);
    if (st) return st;
    LPE_KERNEL(ctx, "k_ref_cells", k_ref_cells, dim3(nblk(d.n)), dim3(TPB), 0, ctx->stream, d.n,
                       d.cfg.gridConfig.gridEpsilon, d.P.x, d.P.y, d.P.id, d.gp, d.tmpId);
    LPE_CHECK_LAUNCH(ctx, "k_ref_cells");
    LPE_HIP(ctx, hipMemcpyAsync(cell_index, d.tmpId, sizeof(int32_t) * d.n, hipMemcpyDeviceToHost,
                                ctx->stream));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (stats) return lpe_sph_get_stats(ctx, stats);
    return LPE_OK;
}

extern "C" int lpe_sph_probe_density(lpe_ctx *ctx, float *density, float *pressure) {
    if (!ctx) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (d.shard) { ctx->err = "not on a slab rank (its slots hold ghosts)"; return LPE_ERR_STATE; }
    if (d.n <= 0) return LPE_OK;
    (void)hipSetDevice(ctx->device);
    int st = sph_void_prelaunch(ctx);           // the probe's hash reuses the prelaunch's buffers
    if (st) return st;
    st = sph_reset_step_stats(ctx, ctx->stream, d.status);
    if (st) return st;
    st = sph_hash(ctx, 0.f, 0.f, false, true);
    if (st) return st;
    // the pure pass (computeDensity's outputs), or with LPE_SPH_MODE_PROBE_TICK_PASS the tick's
    // pass (which also writes the forces pass's neighbour lists)
    st = sph_density(ctx, d.n, nullptr, d.rho, d.pr, (d.mode & LPE_SPH_MODE_PROBE_TICK_PASS) != 0);
    if (st) return st;
    // rho/p are in S slot order here; S.x.. are the unpermute staging buffers,
    // so keep S.id aside in tmpOld first
    LPE_HIP(ctx, hipMemcpyAsync(d.tmpOld, d.S.id, sizeof(int32_t) * d.n, hipMemcpyDeviceToDevice,
                                ctx->stream));
    const float *src[2] = {d.rho, d.pr};
    float *dst[2] = {density, pressure};
    return sph_unpermute_download(ctx, d.tmpOld, 2, src, dst);
}

// ---- slab decomposition: configuration and owned-particle I/O -----------
extern "C" int lpe_sph_set_slab(lpe_ctx *ctx, int nranks, int rank, const float *edges, int wire_cap,
                                int rebalance) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || !edges || wire_cap < 1 || rebalance < 0)
        return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    SphDev &d = ctx->sph;
    if (d.mode & LPE_SPH_MODE_REF_CELL_CAP) {
        ctx->err = "the reference cell-capacity mode is single-domain only (not on a slab rank)";
        return LPE_ERR_STATE;
    }
    if (!d.cfg_set) {
        ctx->err = "lpe_sph_set_slab: set the fluid config first (the edges are reference-cell columns)";
        return LPE_ERR_STATE;
    }
    const float cs = ref_cell_size(d.cfg);
    std::vector<int> e(nranks + 1);
    e[0] = -SLAB_OPEN;
    e[nranks] = SLAB_OPEN;
    int minw = 1 << 20;
    for (int j = 1; j < nranks; j++) {
        const double q = (double)edges[j] / cs;
        const double c = std::nearbyint(q);
        if (!(std::fabs(q - c) < 1e-3) || std::fabs(c) > 1e8) {
            ctx->err = "lpe_sph_set_slab: inner edges must lie on reference-cell boundaries (multiples of 2h)";
            return LPE_ERR_ARG;
        }
        e[j] = (int)c;
        if (j > 1) {
            if (e[j] - e[j - 1] < SLAB_MINW) {
                ctx->err = "lpe_sph_set_slab: inner slabs must be at least 8 reference cells wide";
                return LPE_ERR_ARG;
            }
            minw = std::min(minw, e[j] - e[j - 1]);
        }
    }
    if (d.pside) LPE_HIP(ctx, hipStreamSynchronize(d.pside));
    d.pre = false;
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    shard_free(d.shard);
    d.shard = nullptr;
    d.cap_n = 0;                // the particle arrays are re-sized (slots for ghosts and growth) by the upload
    Shard *h = new Shard();
    d.shard = h;
    h->nranks = nranks; h->rank = rank;
    h->hasL = rank > 0 ? 1 : 0;
    h->hasR = rank < nranks - 1 ? 1 : 0;
    h->wcap = wire_cap;
    h->rebalance = nranks > 1 ? rebalance : 0;
    h->e0 = e;
    h->mv = h->rebalance ? std::max(SLAB_MINW, std::min(minw / 4, 1024)) : 0;
    const size_t E = sizeof(int32_t) * (size_t)(nranks + 1);
    LPE_HIP(ctx, hipMalloc((void **)&h->edges, E));
    LPE_HIP(ctx, hipMalloc((void **)&h->edges0, E));
    LPE_HIP(ctx, hipMemcpy(h->edges, e.data(), E, hipMemcpyHostToDevice));
    LPE_HIP(ctx, hipMemcpy(h->edges0, e.data(), E, hipMemcpyHostToDevice));
    // [0], [1] slots by parity, [2] the hash's input slots, [3] scratch, [4], [5] the ghost columns received
    LPE_HIP(ctx, hipMalloc((void **)&h->cnt, sizeof(int32_t) * 8));
    LPE_HIP(ctx, hipMemset(h->cnt, 0, sizeof(int32_t) * 8));
    float **wb[] = {&h->sL, &h->sR, &h->rL, &h->rR};
    for (float **q : wb) {
        LPE_HIP(ctx, hipMalloc((void **)q, wire_bytes(wire_cap)));
        LPE_HIP(ctx, hipMemset(*q, 0, sizeof(float) * HDR));
    }
    LPE_HIP(ctx, hipMalloc((void **)&h->bbAll, sizeof(float4) * (size_t)nranks));
    LPE_HIP(ctx, hipMalloc((void **)&h->bbG, sizeof(float4)));
    if (h->rebalance) {
        h->hcol0 = e[1] - h->mv - 2;
        h->hcols = e[nranks - 1] + h->mv + 2 - h->hcol0 + 1;
        LPE_HIP(ctx, hipMalloc((void **)&h->hist, sizeof(float) * (size_t)h->hcols));
        LPE_HIP(ctx, hipMemset(h->hist, 0, sizeof(float) * (size_t)h->hcols));
    }
    return LPE_OK;
}

extern "C" int lpe_sph_slab_info(lpe_ctx *ctx, int cap, int32_t *edges, int *nranks, int *move) {
    if (!ctx || cap < 0) return LPE_ERR_ARG;
    const Shard *h = ctx->sph.shard;
    if (nranks) *nranks = h ? h->nranks : 0;
    if (move) *move = h ? h->mv : 0;
    if (!h) return LPE_OK;
    if (edges && cap >= h->nranks + 1) {
        LPE_HIP(ctx, hipMemcpyAsync(edges, h->edges, sizeof(int32_t) * (size_t)(h->nranks + 1),
                                    hipMemcpyDeviceToHost, ctx->stream));
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    return LPE_OK;
}

extern "C" int lpe_sph_set_ids(lpe_ctx *ctx, int n, const int32_t *ids) {
    if (!ctx || n < 0 || (n > 0 && !ids)) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (n != (d.shard ? d.shard->n0 : d.n)) return LPE_ERR_ARG;
    if (n == 0) return LPE_OK;
    int st = sph_void_prelaunch(ctx);          // it sorted by the old ids
    if (st) return st;
    LPE_HIP(ctx, hipMemcpyAsync(d.P.id, ids, sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LPE_OK;
}

extern "C" int lpe_sph_set_global_count(lpe_ctx *ctx, int n_global) {
    if (!ctx || n_global < 0) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    if (!d.shard) { ctx->err = "lpe_sph_set_global_count: not a slab rank (lpe_sph_set_slab)"; return LPE_ERR_STATE; }
    int st = sph_void_prelaunch(ctx);
    if (st) return st;
    d.shard->nglobal = n_global;
    if (d.P.x && n_global > d.cap_n) {          // refInv holds an entry per particle id
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (d.refInv) (void)hipFree(d.refInv);
        d.refInv = nullptr;
        LPE_HIP(ctx, hipMalloc((void **)&d.refInv, sizeof(int32_t) * (size_t)n_global));
    }
    if (d.refInv)
        LPE_HIP(ctx, hipMemsetAsync(d.refInv, 0xff, sizeof(int32_t) * (size_t)std::max(n_global, d.cap_n), ctx->stream));
    return LPE_OK;
}

extern "C" int lpe_sph_download_owned(lpe_ctx *ctx, int cap, float *x, float *y, float *vx, float *vy,
                                      float *density, float *pressure, int32_t *ids, int *n_out) {
    if (!ctx || !n_out || cap < 0) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    hipStream_t s = ctx->stream;
    if (d.shard) {
        // the owned slots (id >= 0) gathered into the staging arrays a pending
        // prelaunch no longer needs (as sph_unpermute_download), ids to tmpOld
        Shard &h = *d.shard;
        *n_out = 0;
        if (!d.P.x) return LPE_OK;
        int st0 = sph_join_prelaunch(ctx);
        if (st0) return st0;
        LPE_HIP(ctx, hipMemsetAsync(h.cnt + 3, 0, sizeof(int32_t), s));
        Fields6 f{};
        float *stage[6] = {d.S.x, d.S.y, d.S.vx, d.S.vy, d.S.m, d.stage};
        for (int k = 0; k < 6; k++) f.dst[k] = stage[k];
        LPE_KERNEL(ctx, "k_slab_gather_owned", k_slab_gather_owned, dim3(nblk1(d.n)), dim3(TPB), 0, s, d.n,
                   (const int32_t *)(h.cnt + h.cur), d.P, (const float *)d.rho, (const float *)d.pr, f, d.tmpOld,
                   h.cnt + 3);
        LPE_CHECK_LAUNCH(ctx, "k_slab_gather_owned");
        int32_t m = 0;
        LPE_HIP(ctx, hipMemcpyAsync(&m, h.cnt + 3, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        LPE_HIP(ctx, hipStreamSynchronize(s));
        *n_out = m;
        if (m > cap) return LPE_ERR_CAPACITY;
        float *dst[6] = {x, y, vx, vy, density, pressure};
        for (int k = 0; k < 6; k++)
            if (dst[k] && m) LPE_HIP(ctx, hipMemcpyAsync(dst[k], stage[k], sizeof(float) * m, hipMemcpyDeviceToHost, s));
        if (ids && m) LPE_HIP(ctx, hipMemcpyAsync(ids, d.tmpOld, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s));
        LPE_HIP(ctx, hipStreamSynchronize(s));
        return check_status(ctx);
    }
    *n_out = d.n;
    if (d.n > cap) return LPE_ERR_CAPACITY;
    int st0 = sph_join_prelaunch(ctx);
    if (st0) return st0;
    const size_t B = sizeof(float) * (size_t)d.n;
    if (d.n > 0) {
        const float *src[6] = {d.P.x, d.P.y, d.P.vx, d.P.vy, d.rho, d.pr};
        float *dst[6] = {x, y, vx, vy, density, pressure};
        for (int k = 0; k < 6; k++)
            if (dst[k]) LPE_HIP(ctx, hipMemcpyAsync(dst[k], src[k], B, hipMemcpyDeviceToHost, s));
        if (ids) LPE_HIP(ctx, hipMemcpyAsync(ids, d.P.id, sizeof(int32_t) * d.n, hipMemcpyDeviceToHost, s));
    }
    LPE_HIP(ctx, hipStreamSynchronize(s));
    return check_status(ctx);
}

extern "C" int lpe_sph_set_domain(lpe_ctx *ctx, double x0, double y0, double x1, double y1) {
    if (!ctx || !(x1 >= x0) || !(y1 >= y0)) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    if (ctx->sph.cs <= 0.f) return LPE_ERR_STATE;     // after lpe_sph_upload
    return lpe_sph_cover_box(ctx, x0, y0, x1, y1);
}
