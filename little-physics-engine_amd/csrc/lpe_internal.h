// lpe_internal.h — shared internals of the HIP backend (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include <utility>
#include <functional>
#include "../../include/lpe.h"

namespace lpe {

// Device mirror of the reference's per-sub-step grid (fluid.cpp:737-752)
// plus the absolute device grid the counting sort runs on.
struct GridParams {
    float cellSize;        // 2 * max(0.05, h)                   fluid.cpp:724-737
    int gridMinX, gridMinY; // reference grid origin (cells)      fluid.cpp:743-744
    int gridMaxX, gridMaxY; // floor(max/cs)                      fluid.cpp:745-746
    int gridDimX, gridDimY; // max-min+1 clamped to >= 1          fluid.cpp:748-751
};

// Particle state in cell-sorted order (SoA fp32).  `id` is the gather index
// of the particle (the reference's particle index i, fluid.cpp:268-299).
struct PState {
    float *x = nullptr, *y = nullptr, *vx = nullptr, *vy = nullptr;
    float *vhx = nullptr, *vhy = nullptr, *ax = nullptr, *ay = nullptr;
    float *m = nullptr;
    int32_t *id = nullptr;
};

struct Shard;

struct SphDev {
    int n = 0, cap_n = 0;
    PState P;                     // primary state (sorted order of the last sub-step)
    PState S;                     // permutation target of the current sub-step
    float *rho = nullptr, *pr = nullptr;  // in S/P slot order
    float *rhoN = nullptr, *prN = nullptr;// the prelaunched sub-step's (swapped in when it is consumed)
    float4 *nbA = nullptr;        // sorted neighbour records (x, y, m, -)
    float4 *nbB = nullptr;        // (vx, vy, rho, p / rho^2)
    uint4 *nlist = nullptr;       // per-slot neighbour list (int16, 8 per uint4), [cap/8][cap_n]: LDS indices of
                                  // the forces pass's image, or slot offsets k - s (ncount's NL_OFFS bit)
    void *fplans = nullptr;       // the density pass's block plans (Hood), for the forces pass's image
    float *rgrid = nullptr;       // renderer density grid, two W*H buffers (lpe_render_density)
    size_t cap_rgrid = 0;
    uint32_t *rmax = nullptr;     // renderer: max of the blurred grid (float bits)
    int32_t *ncount = nullptr;    // neighbours found (> cap: forces walks the bins)
    // counting-sort grid hash over (2h cell, h quadrant) bins
    uint32_t *key = nullptr;      // bin of each P slot
    int32_t *tmpId = nullptr;     // scatter output: particle id per new slot
    int32_t *tmpOld = nullptr;    // scatter output: old P slot per new slot
    int32_t *count = nullptr;     // per bin
    int32_t *start = nullptr;     // nbins+1
    int32_t *cursor = nullptr;    // nbins
    int32_t *blocksum = nullptr;  // scan partials
    float4 *bboxPart = nullptr;   // per-block bbox partials (minX, maxX, minY, maxY)
    int cap_cells = 0;
    // absolute device grid: origin (cells) and dims, fixed per upload
    int ox = 0, oy = 0, W = 0, H = 0;
    float cs = 0.1f;
    GridParams *gp = nullptr;     // device copy of the reference grid; [1]: the prelaunched sub-step's
    int32_t *status = nullptr;    // [ST_COUNT] flags / stats; [ST_COUNT..2 ST_COUNT): the prelaunch's
    GridParams *gp_cur = nullptr; // where the hash / density launches write (gp, or gp + 1 in sph_prelaunch)
    int32_t *stat_cur = nullptr;  // likewise status / status + ST_COUNT
    float *stage = nullptr;       // download staging (with S.x, S.y, S.vx, S.vy, S.m)
    // rigid coupling
    int nr = 0, cap_nr = 0;
    lpe_gpu_rigid *rig = nullptr;
    float *accum = nullptr;       // [3R] the last tick's accumulators (rounded, before the write-back)
    unsigned long long *acq = nullptr;  // [3R][XACC_LIMBS] exact running sums (sph_coupling.h)
    int32_t *rbinStart = nullptr; // rigid bins (absolute grid of bin size bcs)
    int32_t *rbinList = nullptr;
    int32_t *rbinCount = nullptr;
    int rbin_zero = 0;            // rbinCount[0, rbin_zero) is zero (left so by k_rbin_sort)
    int cap_rbins = 0, cap_rlist = 0;
    float4 *raabb = nullptr;      // coupling rigids' AABBs (minX, maxX, minY, maxY), per tick
    int cap_raabb = 0;
    int bx0 = 0, by0 = 0, bW = 0, bH = 0;
    float bcs = 0.25f;
    int rlist_len = 0;
    int rlist_bound = 0;          // > 0: capacity bound of the bin list (no host sync)
    int32_t *coupleBody = nullptr;// world mode: body index of each coupling rigid
    int couple_n = 0, cap_couple = 0;
    bool fluid_heavy = false;     // a fluid mass >= planetaryMassThreshold
    lpe_fluid_config cfg{};
    bool cfg_set = false;
    bool rig_dirty = true;
    bool rig_coupled = false;     // the coupling records were written by the world gather (skip k_rig_couple)
    // world tick: sub-step 0's kick/hash/density of the next tick, launched on
    // a side stream while the rigid solvers run (sph_prelaunch).  It writes
    // only scratch (kicked state, bins, sorted records, gp[1], status[1]),
    // never P, so it can be voided at any time (sph_void_prelaunch) and may
    // outlive the lpe_world_tick call that launched it
    hipStream_t pside = nullptr;
    hipEvent_t preReady = nullptr, preDone = nullptr, fbgDone = nullptr;
    lpe_body *wb_bodies = nullptr;   // world tick: k_rigid_writeback also scatters to these (coupleBody)
    bool pre = false;
    double pre_dt = 0.0;
    int diag = 0;                 // count the ST_NL_OVERFLOW / ST_RIGID_CAND / ST_NEIGH stats
    int mode = 0;                 // LPE_SPH_MODE_* (lpe_sph_set_mode)
    int32_t *refInv = nullptr;    // reference cell-capacity mode: sorted slot of each particle id
    void *plans = nullptr;        // pure density pass: per-tile staging plans (lpe_sph.hip Hood)
    unsigned upload_gen = 0;      // bumped by every lpe_sph_upload (world Barnes-Hut cache)
    size_t cap_plans = 0;
    struct Shard *shard = nullptr;// x-slab decomposition state (lpe_sph_set_slab), else single domain
    // one-launch scan (lpe_sph.hip k_scan_rows): the kick's row totals by parity
    int32_t *rowtot = nullptr;    // [2][cap_rows] particles per device row
    int cap_rows = 0;
    long fastIdx = 0;             // row scans launched (parity)
    bool fast_armed = false;      // the pending kick recorded the row totals
    // in-bin order without a scatter pass (lpe_sph.hip k_bucket_permute): the
    // kick files each particle id under its bin (BKT_CAP per bin, the rest in
    // an overflow list by parity)
    int32_t *bucket = nullptr;    // [cap_bucket][BKT_CAP] ids by bin, arrival order
    long cap_bucket = 0;          // bins the bucket covers (0: off, the scatter path)
    int32_t *bovf = nullptr;      // [2][OVF_WORDS]: count, then (bin, id) pairs
    bool fast_bucket = false;     // the pending kick filed the ids
    // over-full reference cells of a sub-step (lpe_sph.hip ovl_append), two
    // lists alternating by scan: the capped-cell mode's per-particle test
    int32_t *ovl = nullptr;       // [2][OVL_WORDS]
    long ovlIdx = 0;              // scans that wrote a list (parity)
    const int32_t *ovl_cur = nullptr;   // the last hash's list
    const int32_t *ovl_pre = nullptr;   // the prelaunched sub-step's
    // the forces pass's tile scheduling (lpe_sph.hip HeavyOut / HeavyIn)
    int32_t *heavy = nullptr;     // [2][HEAVY_WORDS]: counts, filed tiles -- by density pass parity
    int32_t *tileHeavy = nullptr; // per tile: its filing code, or 0
    int heavyCur = 0;             // the parity the last density pass filed into
    // lagged checks of the fluid step (lpe_sph.hip sph_lag_service), the
    // pattern of RigidDev::lag: every call of an SPH-only or slab-rank step
    // leaves its last sub-step's reference grid (the particles' bbox), the
    // status words and a slab rank's slots in use in a pinned ring slot; the
    // host reads a slot when it comes round (two calls later) or at once if it
    // has landed.  An error a slot shows fails the call that reads it; a bbox
    // nearing the device grid's edge grows (or recentres) the grid, a slab
    // rank nearing its slot capacity grows the slots, before the next call.
    int32_t *hlag = nullptr;      // pinned [2][LAG_WORDS]
    hipEvent_t evLag[2] = {nullptr, nullptr};
    bool lpend[2] = {false, false};
    unsigned ltick = 0;           // records issued
    bool lag_prev = false;        // a previous bbox sample (the drift rate)
    int lag_box[4] = {0, 0, 0, 0};// its cells: minX, minY, maxX, maxY
    unsigned lag_box_tick = 0;
    long grid_regrows = 0, slot_regrows = 0;
};

// status slots
enum StatusSlot {
    ST_CAP_OVERFLOW = 0,
    ST_MAX_OCC = 1,
    ST_NOT_INSERTED = 2,
    ST_LIST_OVERFLOW = 3,
    ST_NL_OVERFLOW = 4,     // diag: particles whose neighbour list overflowed (forces walk the bins)
    ST_RIGID_CAND = 5,      // diag: rigid candidates tested by the coupling (sum over particles)
    ST_NEIGH = 6,           // diag: neighbours (r < h) found by the density pass (sum)
    ST_STAGE_FALLBACK = 7,  // staged density blocks whose neighbourhood did not fit LDS
    ST_HALO_OVERFLOW = 8,   // slab decomposition: a ghost / migrant buffer overflowed
    ST_HALO_DRIFT = 9,      // slab decomposition: an owned particle beyond the halo's reach
    ST_XACC_RANGE = 10,     // a rigid coupling force outside the exact accumulator's range (|f| >= 2^64)
    ST_OVER_CAP = 11,       // reference cells over GPU_MAX_PER_CELL, summed over the tick's sub-steps
    ST_REF_UB = 12,         // reference cell-capacity mode read past the last cell (undefined in the reference)
    ST_OVER_CAP_TOTAL = 13, // ST_OVER_CAP summed since the last lpe_sph_diag call (bench windows)
    ST_MAX_OCC_TOTAL = 14,  // ST_MAX_OCC maximum since the last lpe_sph_diag call
    ST_BUCKET_OVERFLOW = 15,// the in-bin sort's overflow list overflowed (a tick's sort is wrong: fails loudly)
    ST_RX_GHOST_L = 16,     // slab decomposition: most ghosts the left / right neighbour packed for this
    ST_RX_GHOST_R = 17,     //   rank in a sub-step of the current tick (sizes the next tick's exchange)
    ST_SLAB_CAPACITY = 18,  // slab decomposition: the received ghosts did not fit the rank's slots
    ST_FORCES_GLOBAL = 19,  // forces blocks whose neighbourhood did not fit the LDS image (global gathers)
    ST_SLOT_PEAK = 20,      // slab decomposition: most slots a sub-step's hash wanted (own + received ghosts)
    ST_REF_SLAB = 21,       // slab rank, reference cell-capacity mode: the literal loop needed a cell it does not hold
    ST_COUNT = 22
};

}  // namespace lpe

namespace lpe {
// Optional per-kernel HIP-event timing on the context's stream (bench.py uses
// it for the live roofline numbers).  Event pairs are recorded around each
// launch of a named kernel and resolved at lpe_timing_read().
struct KernelTimer {
    int on = 0;                   // 0 off, 1 every kernel, 2 the hot kernels only
    bool wants(const char *name) const;
    std::vector<std::string> names;
    std::vector<std::vector<std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::vector<double> total_ms;
    std::vector<long> calls;
    std::vector<hipEvent_t> pool;
    int slot(const char *name);
    hipEvent_t get();
};
}  // namespace lpe

namespace lpe { struct Transport; }

struct lpe_ctx {
    lpe::Transport *transport = nullptr;   // slab decomposition (lpe_transport.hip)
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    lpe::SphDev sph;
    void *rigid = nullptr;  // lpe::RigidDev*, owned by lpe_rigid.hip
    void *bh = nullptr;     // lpe::BhDev*, owned by lpe_bh.hip (Barnes-Hut)
    lpe::KernelTimer timer;
};

// Records a start event before and a stop event after `launch` when timing is on.
// Launch a kernel on the context stream; with timing on, the launch carries
// start/stop events that the runtime stamps at the dispatch's own begin and
// end (hipExtLaunchKernelGGL), i.e. the kernel's execution time, not the gap
// between two markers on the stream.
#define LPE_KERNEL(ctx, name, kernel, grid, block, shmem, stream, ...)                   \
    do {                                                                                 \
        if ((ctx)->timer.on && (ctx)->timer.wants(name)) {                               \
            int ts_ = (ctx)->timer.slot(name);                                           \
            hipEvent_t e0_ = (ctx)->timer.get(), e1_ = (ctx)->timer.get();               \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, e0_, e1_, 0,       \
                                  __VA_ARGS__);                                          \
            (ctx)->timer.pending[ts_].push_back({e0_, e1_});                             \
        } else {                                                                         \
            hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);         \
        }                                                                                \
    } while (0)

// Launch a kernel and signal `ev` at its end, on the dispatch's own
// completion signal (hipExtLaunchKernelGGL's stop event) instead of a marker
// packet after it: a recorded event holds the stream ~4 us at that boundary,
// the carried one ~1.5 us (profiles/r06/probe/gap_probe.txt).  With the
// kernel timed, or LPE_EVENT_RECORDS=1 (A/B): the launch, then a record.
inline bool lpe_event_records() {
    static const bool on = getenv("LPE_EVENT_RECORDS") != nullptr;
    return on;
}
#define LPE_KERNEL_SIGNAL(ctx, name, ev, kernel, grid, block, shmem, stream, ...)        \
    do {                                                                                 \
        if (((ctx)->timer.on && (ctx)->timer.wants(name)) || lpe_event_records()) {      \
            LPE_KERNEL(ctx, name, kernel, grid, block, shmem, stream, __VA_ARGS__);      \
            LPE_HIP(ctx, hipEventRecord(ev, stream));                                    \
        } else {                                                                         \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, nullptr, ev, 0,    \
                                  __VA_ARGS__);                                          \
        }                                                                                \
    } while (0)

#define LPE_HIP(ctx, call)                                                       \
    do {                                                                         \
        hipError_t e_ = (call);                                                  \
        if (e_ != hipSuccess) {                                                  \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);      \
            return LPE_ERR_HIP;                                                  \
        }                                                                        \
    } while (0)

#define LPE_CHECK_LAUNCH(ctx, name)                                              \
    do {                                                                         \
        hipError_t e_ = hipGetLastError();                                       \
        if (e_ != hipSuccess) {                                                  \
            (ctx)->err = std::string("launch ") + name + ": " + hipGetErrorString(e_); \
            return LPE_ERR_HIP;                                                  \
        }                                                                        \
    } while (0)

template <typename T>
static inline int lpe_grow(lpe_ctx *ctx, T **p, int *cap, long want, long elems_alloc) {
    if (want <= *cap && *p) return LPE_OK;
    if (*p) { (void)hipFree(*p); *p = nullptr; }
    hipError_t e = hipMalloc((void **)p, sizeof(T) * (size_t)(elems_alloc > 0 ? elems_alloc : 1));
    if (e != hipSuccess) { ctx->err = std::string("hipMalloc: ") + hipGetErrorString(e); return LPE_ERR_HIP; }
    *cap = (int)want;
    return LPE_OK;
}

int lpe_rigid_destroy_internal(lpe_ctx *ctx);
// world tick: rigid collision detection overlapped with the fluid step (lpe_rigid.hip)
int rigid_tick_begin(lpe_ctx *ctx, bool on_main = false);   // on_main: detect on the context stream
int rigid_tick_boundary(lpe_ctx *ctx, bool gravity = false, double dt_state = 0.0);   // + BasicGravity fused
int rigid_tick_detect(lpe_ctx *ctx);   // host half of the detection + colouring launch
int rigid_tick_hook(lpe_ctx *ctx, int step);   // fluid-step hook (after each sub-step's forces)
int rigid_tick_finish(lpe_ctx *ctx);
// lpe_sph_step with a host callback after the forces of sub-step `after`
int sph_step_hooked(lpe_ctx *ctx, double dt_tick, int (*hook)(lpe_ctx *, int));
float4 *sph_rig_records(lpe_ctx *ctx, int nr);   // the coupling records buffer (nr rigids)
// first (optional): launched on the side stream ahead of the prelaunch (the
// tick's own fluid boundary / gravity pass); fbgDone is recorded after it
// ready: an event the context stream has signalled after its last work the
// prelaunch depends on (null: one is recorded here)
// (devwait: the side stream waits on the rigid boundary pass's device signal
// when there is one this tick, rigid_boundary_wait)
int sph_prelaunch(lpe_ctx *ctx, double dt_tick, const std::function<int(hipStream_t)> &first = {},
                  hipEvent_t ready = nullptr, bool devwait = false);
hipEvent_t rigid_boundary_event(lpe_ctx *ctx);
int rigid_boundary_wait(lpe_ctx *ctx, hipStream_t s, bool *done);
int lpe_sph_cover_box(lpe_ctx *ctx, double x0, double y0, double x1, double y1);
// a slab rank's P slots in use (device count; ids -1 mark dropped slots), else null
const int32_t *sph_slab_slots(lpe_ctx *ctx);
// coupling rigids' device arrays (rig, accum, acq) for n rigids (grow-only)
int sph_alloc_rigids(lpe_ctx *ctx, int n);
// sort the CURRENT particle positions into the bins (no integration): the
// state of lpe_sph_probe_* and of the renderer's density grid
int lpe_sph_hash_current(lpe_ctx *ctx);
int lpe_timer_destroy_internal(lpe_ctx *ctx);
int lpe_bh_destroy_internal(lpe_ctx *ctx);
// BarnesHutSystem inside lpe_world_tick (lpe_bh.hip): on the rigid context's
// bodies, between the collision system and rotation (sim.cpp:107-114)
int bh_world_tick(lpe_ctx *ctx, double dt_state);
// its early-exit decision and fluid guard (cached per upload / config change):
// lpe_world_tick calls it before queuing any work, so a world the system
// cannot run fails before the tick starts
int bh_world_prepare(lpe_ctx *ctx);
