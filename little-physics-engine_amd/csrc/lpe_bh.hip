// lpe_bh.hip — Barnes-Hut gravity on the device.
//
// Replaces BarnesHutSystem::update (src/systems/barnes_hut.cpp:50-295).  The
// reference inserts the bodies one by one into a point-region quadtree and
// folds each internal node's centre of mass incrementally, in insertion
// order (:171-177), then walks the tree recursively for every body (:240-294).
// Both are order-dependent in fp64, so the device reproduces the orders, not
// just the mathematics:
//
//  - The tree is built level by level.  At level L the inserted bodies are
//    held sorted by (node, insertion index); one thread per node of the level
//    replays that node's insertion sequence through the reference's state
//    machine (empty -> store the body; leaf -> subdivide, re-insert the old
//    occupant, insert the new one; internal -> fold and route down), so the
//    node's mass, centre of mass, "all small" flag and occupant are the
//    reference's bit for bit, including the occupant counted twice when a
//    leaf is split (:162-168 re-inserts it through the internal branch).  The
//    bodies routed to a child keep their insertion order: a stable radix sort
//    by child node id gives the next level's segments.
//  - The force walk is one thread per body, stackless over parent links, in
//    the reference's child order nw, ne, sw, se, accumulating vel += a * dt in
//    the same sequence as the recursion.
//
// Every level is a handful of launches plus one 8-byte read-back (the number
// of nodes and of routed bodies sizes the next level), so the build is
// O(depth) round trips; the work per level is O(N) except the sequential
// fold of each node, which is the reference's own dependency chain.  fp64
// throughout, no FMA contraction (Makefile), IEEE division and square root.
#include "lpe_internal.h"
#include "rigid_dev.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>

namespace lpe {

struct BhNode {
    double mass, cx, cy;          // totalMass, centerOfMassX/Y
    double bx, by, size;          // boundaryX/Y, boundarySize
    int32_t single;               // occupant body (-1: entt::null)
    int32_t child;                // first child (nw, ne, sw, se contiguous), -1: none
    int32_t parent;               // -1 at the root
    int32_t flags;                // BH_LEAF | BH_SMALL | digit << 2
};
static_assert(sizeof(BhNode) == 64, "one node per 64 B");

enum { BH_LEAF = 1, BH_SMALL = 2 };
static constexpr int32_t BH_DROP = INT_MAX;    // sort key of a body that left the tree

struct BhDev {
    int n = 0, cap = 0;
    double *x = nullptr, *y = nullptr, *vx = nullptr, *vy = nullptr, *m = nullptr;
    uint8_t *hv = nullptr;
    // bodies of the current level: keys (node ids) and values (body ids), ping-pong
    int32_t *key[2] = {nullptr, nullptr}, *val[2] = {nullptr, nullptr};
    uint8_t *route = nullptr;
    int32_t *segB = nullptr, *segE = nullptr;   // per node of the level: member range
    int segCap = 0;
    BhNode *nodes = nullptr;
    long ncap = 0;
    int32_t *cnt = nullptr;                     // [0] node count, [1] routed bodies, [2] any big mass
    int32_t *hcnt = nullptr;                    // pinned copy
    void *tmp = nullptr;
    size_t tmpBytes = 0;
    lpe_bh_stats last{};
    // BarnesHutSystem inside lpe_world_tick (lpe_world_set_barnes_hut)
    bool w_on = true;                           // the reference always runs the system (sim.cpp:111)
    bool w_cfg_set = false;                     // else: defaults + the rigid config's universe
    lpe_bh_config w_cfg{};
    std::vector<int32_t> w_order_user;          // insertion order given by the host (empty: default)
    int32_t *w_order = nullptr;                 // device: body index per inserted body
    int w_n = 0, w_cap = 0;
    bool w_valid = false, w_active = false, w_fluid_heavy = false;
    unsigned w_rgen = ~0u, w_sgen = ~0u;
};

// ---- kernels ---------------------------------------------------------------

__global__ void k_bh_masscheck(int n, const double *__restrict__ m, double thr, int32_t *cnt) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && m[i] >= thr) cnt[2] = 1;                   // (:60-67; benign same-value race)
}

// root and level-0 keys: the bodies inside [0, U)^2 (buildTree :122-127)
__global__ void k_bh_root(int n, const double *__restrict__ x, const double *__restrict__ y, double U,
                          int32_t *__restrict__ key, int32_t *__restrict__ val, BhNode *nodes, int32_t *cnt) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        BhNode r;
        r.mass = r.cx = r.cy = 0.0;
        r.bx = 0.0;
        r.by = 0.0;
        r.size = U;
        r.single = -1;
        r.child = -1;
        r.parent = -1;
        r.flags = BH_LEAF | BH_SMALL;
        nodes[0] = r;
        cnt[0] = 1;
    }
    if (i >= n) return;
    const bool in = x[i] >= 0.0 && x[i] < U && y[i] >= 0.0 && y[i] < U;
    key[i] = in ? 0 : BH_DROP;
    val[i] = i;
    if (in) atomicAdd(&cnt[1], 1);
}

// member range of every node of the level: keys are sorted, [0, A) active
__global__ void k_bh_segs(int A, int base, const int32_t *__restrict__ key, int32_t *__restrict__ segB,
                          int32_t *__restrict__ segE) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A) return;
    const int c = key[k];
    if (k == 0 || key[k - 1] != c) segB[c - base] = k;
    if (k == A - 1 || key[k + 1] != c) segE[c - base] = k + 1;
}

__device__ __forceinline__ void bh_fold(BhNode &nd, double x, double y, double m, double thr) {
    const double nt = nd.mass + m;                          // (:172-182)
    nd.cx = (nd.cx * nd.mass + x * m) / nt;
    nd.cy = (nd.cy * nd.mass + y * m) / nt;
    nd.mass = nt;
    if (m >= thr) nd.flags &= ~BH_SMALL;
}

// lane i's double (i wave-uniform): two v_readlane, no LDS round trip
__device__ __forceinline__ double bh_lane(double v, int i) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)u, i);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), i);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// one wave per node of the level: the node's insertion sequence through
// insertParticle's state machine (:143-196); route[k] = 1 where member k is
// passed on to a child (the child itself is found by k_bh_route).  The
// sequence is one dependent chain in fp64, so the lanes only fetch: each
// round gathers 64 members' (id, x, y, m) at once and every lane replays
// them in order from its registers (wave-uniform state), so the chain pays
// one gather latency per 64 members instead of one per member.
__global__ __launch_bounds__(64) void k_bh_fold(int base, int nlev, const int32_t *__restrict__ segB,
                                                const int32_t *__restrict__ segE, const int32_t *__restrict__ val,
                                                const double *__restrict__ x, const double *__restrict__ y,
                                                const double *__restrict__ m, double thr,
                                                BhNode *__restrict__ nodes, uint8_t *__restrict__ route,
                                                int32_t *cnt) {
    const int j = blockIdx.x;
    if (j >= nlev) return;
    const int lane = threadIdx.x;
    const int id = base + j;
    BhNode nd = nodes[id];
    const int b = segB[j], e = segE[j];
    int occK = -1;                                          // position of the occupant in the segment
    int lateOcc = -1;                                       // occupant routed after its round was written
    for (int k0 = b; k0 < e; k0 += 64) {
        const int nk = min(64, e - k0);
        int p = 0;
        double px = 0.0, py = 0.0, pm = 0.0;
        if (lane < nk) {
            p = val[k0 + lane];
            px = x[p];
            py = y[p];
            pm = m[p];
        }
        uint64_t rmask = 0;                                 // route bits of this round (uniform)
        for (int i = 0; i < nk; i++) {
            const int qp = __builtin_amdgcn_readlane(p, i);
            const double qx = bh_lane(px, i), qy = bh_lane(py, i), qm = bh_lane(pm, i);
            const int k = k0 + i;
            if (nd.mass == 0.0) {                           // empty: store (:144-154)
                nd.mass = qm;
                nd.cx = qx;
                nd.cy = qy;
                nd.single = qp;
                occK = k;
                if (qm >= thr) nd.flags &= ~BH_SMALL;
                rmask &= ~(1ull << i);
                continue;
            }
            if (nd.flags & BH_LEAF) {                       // split (:157-169)
                nd.flags &= ~BH_LEAF;
                const int o = nd.single;
                bh_fold(nd, x[o], y[o], m[o], thr);         // the occupant again, via the internal branch
                if (occK >= k0) rmask |= 1ull << (occK - k0);
                else lateOcc = occK;
            }
            bh_fold(nd, qx, qy, qm, thr);
            rmask |= 1ull << i;
        }
        if (lane < nk) route[k0 + lane] = (uint8_t)((rmask >> lane) & 1);
    }
    if (lateOcc >= 0) {                                     // after this wave's earlier store of 0 landed
        __threadfence();
        if (lane == 0) route[lateOcc] = 1;
    }
    if (lane != 0) return;
    if (!(nd.flags & BH_LEAF)) {                            // subdivide (:199-238)
        const int c = atomicAdd(&cnt[0], 4);
        nd.child = c;
        const double half = nd.size * 0.5, bx = nd.bx, by = nd.by;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            BhNode ch;
            ch.mass = ch.cx = ch.cy = 0.0;
            ch.bx = (q & 1) ? bx + half : bx;
            ch.by = (q & 2) ? by + half : by;
            ch.size = half;
            ch.single = -1;
            ch.child = -1;
            ch.parent = id;
            ch.flags = BH_LEAF | BH_SMALL | (q << 2);
            nodes[c + q] = ch;
        }
    }
    nodes[id] = nd;
}

// the child of every routed member (getQuadrant, then the child's contains
// test at the top of insertParticle, :139-141): its node id, else dropped
__global__ void k_bh_route(int A, const int32_t *__restrict__ key, const int32_t *__restrict__ val,
                           const uint8_t *__restrict__ route, const double *__restrict__ x,
                           const double *__restrict__ y, const BhNode *__restrict__ nodes,
                           int32_t *__restrict__ keyOut, int32_t *cnt) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A) return;
    int out = BH_DROP;
    if (route[k]) {
        const BhNode &nd = nodes[key[k]];
        const int p = val[k];
        const double px = x[p], py = y[p];
        const double midX = nd.bx + nd.size * 0.5, midY = nd.by + nd.size * 0.5;
        const int q = (px < midX) ? ((py < midY) ? 0 : 2) : ((py < midY) ? 1 : 3);
        const BhNode &ch = nodes[nd.child + q];
        if (px >= ch.bx && px < ch.bx + ch.size && py >= ch.by && py < ch.by + ch.size) {
            out = nd.child + q;
            atomicAdd(&cnt[1], 1);
        }
    }
    keyOut[k] = out;
}

// calculateForce (:240-294) for every body with a velocity: the recursion
// as a stackless walk (children nw, ne, sw, se are contiguous; after a
// subtree, the next sibling or the parent's next sibling)
__global__ void k_bh_force(int n, const double *__restrict__ x, const double *__restrict__ y,
                           const double *__restrict__ m, const uint8_t *__restrict__ hv,
                           double *__restrict__ vx, double *__restrict__ vy, const BhNode *__restrict__ nodes,
                           double theta, double thr, double soft, double G, double dt) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n || !hv[p]) return;
    const double px = x[p], py = y[p], pm = m[p];
    const double soft2 = soft * soft;
    const double thetaSq = theta * theta;
    double wx = vx[p], wy = vy[p];
    int cur = 0;
    while (true) {
        const BhNode nd = nodes[cur];
        bool down = false;
        if (nd.mass != 0.0 && !((nd.flags & BH_SMALL) && thr > 0.0)) {
            const double dx = nd.cx - px;
            const double dy = nd.cy - py;
            const double distSq = dx * dx + dy * dy + soft2;
            const double dist = sqrt(distSq);
            const double sizeSq = nd.size * nd.size;
            const bool leaf = nd.flags & BH_LEAF;
            if (leaf || (sizeSq / distSq < thetaSq)) {
                if (!(leaf && nd.single == p)) {
                    const double f = G * nd.mass * pm / distSq;
                    const double inv = f / (pm * dist);
                    const double ax = dx * inv;
                    const double ay = dy * inv;
                    wx += ax * dt;
                    wy += ay * dt;
                }
            } else {
                down = true;
            }
        }
        if (down) {
            cur = nd.child;
            continue;
        }
        // next sibling, climbing while this was a last child
        int c = cur, fl = nd.flags;
        while (c != 0 && (fl >> 2) == 3) {
            c = nodes[c].parent;
            fl = nodes[c].flags;
        }
        if (c == 0) break;
        cur = c + 1;
    }
    vx[p] = wx;
    vy[p] = wy;
}

// the world's bodies in insertion order -> the Barnes-Hut arrays
__global__ void k_bh_gather(int n, const int32_t *__restrict__ order, const lpe_body *__restrict__ bodies,
                            double *__restrict__ x, double *__restrict__ y, double *__restrict__ vx,
                            double *__restrict__ vy, double *__restrict__ m, uint8_t *__restrict__ hv) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const lpe_body &b = bodies[order[k]];
    x[k] = b.x; y[k] = b.y; vx[k] = b.vx; vy[k] = b.vy; m[k] = b.mass;
    hv[k] = (b.flags & LPE_BODY_HAS_VEL) ? 1 : 0;
}
__global__ void k_bh_scatter(int n, const int32_t *__restrict__ order, const double *__restrict__ vx,
                             const double *__restrict__ vy, const uint8_t *__restrict__ hv,
                             lpe_body *__restrict__ bodies) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || !hv[k]) return;
    lpe_body &b = bodies[order[k]];
    b.vx = vx[k];
    b.vy = vy[k];
}

// ---- host ------------------------------------------------------------------

static inline int bblk(long n, int t = 256) { return (int)std::max<long>(1, (n + t - 1) / t); }

// the body / tree buffers (the world-tick settings and order stay)
static void bh_free(BhDev &d) {
    for (void *p : {(void *)d.x, (void *)d.y, (void *)d.vx, (void *)d.vy, (void *)d.m, (void *)d.hv,
                    (void *)d.key[0], (void *)d.key[1], (void *)d.val[0], (void *)d.val[1], (void *)d.route,
                    (void *)d.segB, (void *)d.segE, (void *)d.nodes, (void *)d.cnt, d.tmp})
        if (p) (void)hipFree(p);
    if (d.hcnt) (void)hipHostFree(d.hcnt);
    d.x = d.y = d.vx = d.vy = d.m = nullptr;
    d.hv = d.route = nullptr;
    d.key[0] = d.key[1] = d.val[0] = d.val[1] = nullptr;
    d.segB = d.segE = nullptr;
    d.nodes = nullptr;
    d.cnt = d.hcnt = nullptr;
    d.tmp = nullptr;
    d.n = d.cap = d.segCap = 0;
    d.ncap = 0;
    d.tmpBytes = 0;
}

static BhDev &bh_dev(lpe_ctx *ctx) {
    if (!ctx->bh) ctx->bh = new BhDev();
    return *(BhDev *)ctx->bh;
}

static int bh_alloc(lpe_ctx *ctx, BhDev &d, int n) {
    if (n <= d.cap && d.x) return LPE_OK;
    (void)hipStreamSynchronize(ctx->stream);
    bh_free(d);
    const size_t N = (size_t)std::max(n, 1);
    LPE_HIP(ctx, hipMalloc(&d.x, sizeof(double) * N));
    LPE_HIP(ctx, hipMalloc(&d.y, sizeof(double) * N));
    LPE_HIP(ctx, hipMalloc(&d.vx, sizeof(double) * N));
    LPE_HIP(ctx, hipMalloc(&d.vy, sizeof(double) * N));
    LPE_HIP(ctx, hipMalloc(&d.m, sizeof(double) * N));
    LPE_HIP(ctx, hipMalloc(&d.hv, N));
    LPE_HIP(ctx, hipMalloc(&d.route, N));
    for (int i = 0; i < 2; i++) {
        LPE_HIP(ctx, hipMalloc(&d.key[i], sizeof(int32_t) * N));
        LPE_HIP(ctx, hipMalloc(&d.val[i], sizeof(int32_t) * N));
    }
    LPE_HIP(ctx, hipMalloc(&d.cnt, sizeof(int32_t) * 4));
    LPE_HIP(ctx, hipHostMalloc(&d.hcnt, sizeof(int32_t) * 4, hipHostMallocDefault));
    size_t tb = 0;
    LPE_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, d.key[0], d.key[1], d.val[0], d.val[1], (int)N,
                                                    0, 31, ctx->stream));
    LPE_HIP(ctx, hipMalloc(&d.tmp, tb));
    d.tmpBytes = tb;
    d.cap = (int)N;
    return LPE_OK;
}

static int bh_grow_nodes(lpe_ctx *ctx, BhDev &d, long want) {
    if (want <= d.ncap) return LPE_OK;
    long nc = std::max(want, 2 * d.ncap);
    BhNode *p = nullptr;
    LPE_HIP(ctx, hipMalloc(&p, sizeof(BhNode) * (size_t)nc));
    if (d.nodes) {
        LPE_HIP(ctx, hipMemcpyAsync(p, d.nodes, sizeof(BhNode) * (size_t)d.ncap, hipMemcpyDeviceToDevice,
                                    ctx->stream));
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        (void)hipFree(d.nodes);
    }
    d.nodes = p;
    d.ncap = nc;
    return LPE_OK;
}

static int bh_grow_segs(lpe_ctx *ctx, BhDev &d, int want) {
    if (want <= d.segCap) return LPE_OK;
    int nc = std::max(want, 2 * d.segCap);
    if (d.segB) (void)hipFree(d.segB);
    if (d.segE) (void)hipFree(d.segE);
    d.segB = d.segE = nullptr;
    LPE_HIP(ctx, hipMalloc(&d.segB, sizeof(int32_t) * (size_t)nc));
    LPE_HIP(ctx, hipMalloc(&d.segE, sizeof(int32_t) * (size_t)nc));
    d.segCap = nc;
    return LPE_OK;
}

static int bh_readback(lpe_ctx *ctx, BhDev &d) {
    LPE_HIP(ctx, hipMemcpyAsync(d.hcnt, d.cnt, sizeof(int32_t) * 4, hipMemcpyDeviceToHost, ctx->stream));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LPE_OK;
}

}  // namespace lpe

using namespace lpe;

int lpe_bh_destroy_internal(lpe_ctx *ctx) {
    if (!ctx->bh) return LPE_OK;
    (void)hipStreamSynchronize(ctx->stream);
    BhDev *d = (BhDev *)ctx->bh;
    bh_free(*d);
    if (d->w_order) (void)hipFree(d->w_order);
    delete d;
    ctx->bh = nullptr;
    return LPE_OK;
}

extern "C" int lpe_bh_config_default(lpe_bh_config *c) {
    if (!c) return LPE_ERR_ARG;
    c->theta = 0.5;                   // barnes_hut.hpp:21
    c->small_mass_threshold = 1e3;    // barnes_hut.hpp:24
    c->universe_size = 0.0;
    c->softener = 0.0;
    c->G = 6.674e-11;                 // constants.cpp:8
    return LPE_OK;
}

extern "C" int lpe_bh_upload(lpe_ctx *ctx, int n, const double *x, const double *y, const double *vx,
                             const double *vy, const double *mass, const uint8_t *has_vel) {
    if (!ctx || n < 0 || (n > 0 && (!x || !y || !vx || !vy || !mass))) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    BhDev &d = bh_dev(ctx);
    int st = bh_alloc(ctx, d, n);
    if (st) return st;
    d.n = n;
    if (n == 0) return LPE_OK;
    const size_t b = sizeof(double) * (size_t)n;
    LPE_HIP(ctx, hipMemcpyAsync(d.x, x, b, hipMemcpyHostToDevice, ctx->stream));
    LPE_HIP(ctx, hipMemcpyAsync(d.y, y, b, hipMemcpyHostToDevice, ctx->stream));
    LPE_HIP(ctx, hipMemcpyAsync(d.vx, vx, b, hipMemcpyHostToDevice, ctx->stream));
    LPE_HIP(ctx, hipMemcpyAsync(d.vy, vy, b, hipMemcpyHostToDevice, ctx->stream));
    LPE_HIP(ctx, hipMemcpyAsync(d.m, mass, b, hipMemcpyHostToDevice, ctx->stream));
    if (has_vel)
        LPE_HIP(ctx, hipMemcpyAsync(d.hv, has_vel, (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    else
        LPE_HIP(ctx, hipMemsetAsync(d.hv, 1, (size_t)n, ctx->stream));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LPE_OK;
}

// One update on the bodies in the BhDev arrays (n = d.n); check_small: the
// small-mass early exit on the device (the world path decides it itself)
static int bh_run(lpe_ctx *ctx, BhDev &d, const lpe_bh_config *cfg, double dt, lpe_bh_stats *stats,
                  bool check_small) {
    hipStream_t s = ctx->stream;
    d.last = lpe_bh_stats{};
    if (stats) *stats = d.last;
    const int n = d.n;
    if (n == 0) return LPE_OK;
    const double thr = cfg->small_mass_threshold;
    LPE_HIP(ctx, hipMemsetAsync(d.cnt, 0, sizeof(int32_t) * 4, s));
    if (thr > 0.0 && check_small) {                         // early exit (:55-71)
        LPE_KERNEL(ctx, "k_bh_masscheck", k_bh_masscheck, dim3(bblk(n)), dim3(256), 0, s, n, d.m, thr, d.cnt);
        LPE_CHECK_LAUNCH(ctx, "k_bh_masscheck");
        int st = bh_readback(ctx, d);
        if (st) return st;
        if (!d.hcnt[2]) {
            d.last.skipped = 1;
            if (stats) *stats = d.last;
            return LPE_OK;
        }
    }
    int st = bh_grow_nodes(ctx, d, 1 + 4L * n);
    if (st) return st;
    LPE_KERNEL(ctx, "k_bh_root", k_bh_root, dim3(bblk(n)), dim3(256), 0, s, n, d.x, d.y, cfg->universe_size,
               d.key[0], d.val[0], d.nodes, d.cnt);
    LPE_CHECK_LAUNCH(ctx, "k_bh_root");
    if ((st = bh_readback(ctx, d))) return st;
    d.last.inserted = d.hcnt[1];
    int A = n;                          // bodies in the key/value arrays (dropped ones sort last)
    int active = d.hcnt[1];
    long base = 0, end = 1;             // node ids of the current level
    int level = 0, cur = 0;
    while (active > 0) {
        if (level > LPE_BH_MAX_DEPTH) {
            ctx->err = "lpe_bh_step: quadtree deeper than LPE_BH_MAX_DEPTH";
            return LPE_ERR_OVERFLOW;
        }
        d.last.depth = level;
        size_t tb = d.tmpBytes;
        LPE_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(d.tmp, tb, d.key[cur], d.key[cur ^ 1], d.val[cur],
                                                        d.val[cur ^ 1], A, 0, 31, s));
        cur ^= 1;
        A = active;                     // the dropped bodies are past the end now
        const int nlev = (int)(end - base);
        if ((st = bh_grow_segs(ctx, d, nlev))) return st;
        if ((st = bh_grow_nodes(ctx, d, end + 4L * nlev))) return st;
        LPE_HIP(ctx, hipMemsetAsync(d.segB, 0, sizeof(int32_t) * (size_t)nlev, s));
        LPE_HIP(ctx, hipMemsetAsync(d.segE, 0, sizeof(int32_t) * (size_t)nlev, s));
        LPE_KERNEL(ctx, "k_bh_segs", k_bh_segs, dim3(bblk(A)), dim3(256), 0, s, A, (int)base, d.key[cur], d.segB,
                   d.segE);
        LPE_KERNEL(ctx, "k_bh_fold", k_bh_fold, dim3(std::max(1, nlev)), dim3(64), 0, s, (int)base, nlev, d.segB,
                   d.segE, d.val[cur], d.x, d.y, d.m, thr, d.nodes, d.route, d.cnt);
        LPE_HIP(ctx, hipMemsetAsync(d.cnt + 1, 0, sizeof(int32_t), s));
        LPE_KERNEL(ctx, "k_bh_route", k_bh_route, dim3(bblk(A)), dim3(256), 0, s, A, d.key[cur], d.val[cur],
                   d.route, d.x, d.y, d.nodes, d.key[cur], d.cnt);
        LPE_CHECK_LAUNCH(ctx, "barnes-hut level");
        if ((st = bh_readback(ctx, d))) return st;
        active = d.hcnt[1];
        base = end;
        end = d.hcnt[0];
        level++;
    }
    d.last.nodes = (int32_t)end;
    LPE_KERNEL(ctx, "k_bh_force", k_bh_force, dim3(bblk(n, 128)), dim3(128), 0, s, n, d.x, d.y, d.m, d.hv, d.vx,
               d.vy, d.nodes, cfg->theta, thr, cfg->softener, cfg->G, dt);
    LPE_CHECK_LAUNCH(ctx, "k_bh_force");
    LPE_HIP(ctx, hipStreamSynchronize(s));
    if (stats) *stats = d.last;
    return LPE_OK;
}

extern "C" int lpe_bh_step(lpe_ctx *ctx, const lpe_bh_config *cfg, double dt, lpe_bh_stats *stats) {
    if (!ctx || !cfg) return LPE_ERR_ARG;
    if (!ctx->bh) return LPE_ERR_STATE;
    (void)hipSetDevice(ctx->device);
    return bh_run(ctx, *(BhDev *)ctx->bh, cfg, dt, stats, true);
}

extern "C" int lpe_bh_download(lpe_ctx *ctx, double *vx, double *vy) {
    if (!ctx || !vx || !vy) return LPE_ERR_ARG;
    if (!ctx->bh) return LPE_ERR_STATE;
    (void)hipSetDevice(ctx->device);
    BhDev &d = *(BhDev *)ctx->bh;
    if (d.n == 0) return LPE_OK;
    LPE_HIP(ctx, hipMemcpyAsync(vx, d.vx, sizeof(double) * (size_t)d.n, hipMemcpyDeviceToHost, ctx->stream));
    LPE_HIP(ctx, hipMemcpyAsync(vy, d.vy, sizeof(double) * (size_t)d.n, hipMemcpyDeviceToHost, ctx->stream));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return LPE_OK;
}

extern "C" int lpe_world_set_barnes_hut(lpe_ctx *ctx, int enable, const lpe_bh_config *cfg, int n,
                                        const int32_t *order) {
    if (!ctx || n < 0 || (n > 0 && !order)) return LPE_ERR_ARG;
    BhDev &d = bh_dev(ctx);
    d.w_on = enable != 0;
    d.w_cfg_set = cfg != nullptr;
    if (cfg) d.w_cfg = *cfg;
    d.w_order_user.assign(order, order + n);
    d.w_valid = false;
    return LPE_OK;
}

// BarnesHutSystem::update inside the world tick.  The early exit and the
// insertion order depend only on masses and component flags, which change
// only by an upload or a config change: decided once (one read-back) and
// cached.  Fluid particles are entities with Position + Mass too; a world
// whose fluid would make the system act fails loudly (its velocities live
// in fp32 on the device: strict mode runs it through lpe_bh_step).
int bh_world_prepare(lpe_ctx *ctx) {
    BhDev &d = bh_dev(ctx);
    if (!d.w_on) return LPE_OK;
    RigidDev *rd = (RigidDev *)ctx->rigid;
    SphDev &sd = ctx->sph;
    const int nb = rd ? rd->nb : 0;
    lpe_bh_config cfg;
    if (d.w_cfg_set) cfg = d.w_cfg;
    else {
        lpe_bh_config_default(&cfg);
        cfg.universe_size = rd ? rd->cfg.universeSize : 0.0;
    }
    const unsigned rgen = rd ? rd->gen : 0u;
    if (!d.w_valid || d.w_rgen != rgen || d.w_sgen != sd.upload_gen) {
        // the reads below see the bodies and the fluid masses after every
        // kernel queued so far (k_forces_couple rewrites P.m in sorted order)
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        std::vector<lpe_body> hb(nb);
        if (nb) {
            LPE_HIP(ctx, hipMemcpyAsync(hb.data(), rd->bodies, sizeof(lpe_body) * nb, hipMemcpyDeviceToHost,
                                        ctx->stream));
        }
        const bool fluid_m = sd.n > 0 && !sd.shard && sd.P.m;
        std::vector<float> fm(fluid_m ? sd.n : 0);
        if (fluid_m) {
            LPE_HIP(ctx, hipMemcpyAsync(fm.data(), sd.P.m, sizeof(float) * sd.n, hipMemcpyDeviceToHost,
                                        ctx->stream));
        }
        LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
        const double thr = cfg.small_mass_threshold;
        auto inserted = [](const lpe_body &b) {
            return (b.flags & LPE_BODY_HAS_MASS) && !(b.flags & LPE_BODY_BOUNDARY);
        };
        std::vector<int32_t> ord;
        if (!d.w_order_user.empty()) {
            for (int32_t i : d.w_order_user) {
                if (i < 0 || i >= nb || !inserted(hb[i])) {
                    ctx->err = "lpe_world_set_barnes_hut: order names a body without Mass or with Boundary";
                    return LPE_ERR_ARG;
                }
                ord.push_back(i);
            }
        } else {
            for (int i = nb - 1; i >= 0; i--)          // EnTT views iterate newest first
                if (inserted(hb[i])) ord.push_back(i);
        }
        bool heavy = thr <= 0.0;
        for (int i : ord) heavy = heavy || hb[i].mass >= thr;
        bool fheavy = false;
        for (float v : fm) fheavy = fheavy || thr <= 0.0 || (double)v >= thr;
        int st = bh_alloc(ctx, d, std::max((int)ord.size(), 1));
        if (st) return st;
        if ((int)ord.size() > d.w_cap) {
            if (d.w_order) (void)hipFree(d.w_order);
            d.w_order = nullptr;
            LPE_HIP(ctx, hipMalloc(&d.w_order, sizeof(int32_t) * std::max<size_t>(ord.size(), 1)));
            d.w_cap = (int)ord.size();
        }
        if (!ord.empty())
            LPE_HIP(ctx, hipMemcpy(d.w_order, ord.data(), sizeof(int32_t) * ord.size(), hipMemcpyHostToDevice));
        d.w_n = (int)ord.size();
        d.w_active = heavy || fheavy;
        d.w_fluid_heavy = sd.n > 0 || sd.shard;
        d.w_rgen = rgen;
        d.w_sgen = sd.upload_gen;
        d.w_valid = true;
    }
    if (d.w_active && d.w_fluid_heavy) {
        ctx->err = "Barnes-Hut would act on a world with fluid particles: run it in strict mode (lpe_bh_step)";
        return LPE_ERR_STATE;
    }
    return LPE_OK;
}

int bh_world_tick(lpe_ctx *ctx, double dt_state) {
    BhDev &d = bh_dev(ctx);
    if (!d.w_on) return LPE_OK;
    int st0 = bh_world_prepare(ctx);
    if (st0) return st0;
    if (!d.w_active) return LPE_OK;
    RigidDev *rd = (RigidDev *)ctx->rigid;
    lpe_bh_config cfg;
    if (d.w_cfg_set) cfg = d.w_cfg;
    else {
        lpe_bh_config_default(&cfg);
        cfg.universe_size = rd ? rd->cfg.universeSize : 0.0;
    }
    if (d.w_n == 0) return LPE_OK;
    int st = bh_alloc(ctx, d, d.w_n);
    if (st) return st;
    d.n = d.w_n;
    hipStream_t s = ctx->stream;
    LPE_KERNEL(ctx, "k_bh_gather", k_bh_gather, dim3(bblk(d.n)), dim3(256), 0, s, d.n, d.w_order, rd->bodies, d.x,
               d.y, d.vx, d.vy, d.m, d.hv);
    st = bh_run(ctx, d, &cfg, dt_state, nullptr, false);
    if (st) return st;
    LPE_KERNEL(ctx, "k_bh_scatter", k_bh_scatter, dim3(bblk(d.n)), dim3(256), 0, s, d.n, d.w_order, d.vx, d.vy,
               d.hv, rd->bodies);
    LPE_CHECK_LAUNCH(ctx, "world barnes-hut");
    return LPE_OK;
}
