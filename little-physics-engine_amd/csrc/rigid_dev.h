// rigid_dev.h — device state of the rigid path (shared by lpe_rigid.hip and
// lpe_world.hip).  Not part of the ABI.
#pragma once
#include "lpe_internal.h"

namespace lpe {

static constexpr int RTPB = 256;
static constexpr int MAXC = 36;        // contacts per pair slot (poly-poly <= nB + 3)
static constexpr int EPA_MAX = 104;    // EPA polygon: 3 + 100 insertions + 1
static constexpr int CLIP_MAX = 40;    // clip output <= nB + 3
static constexpr int MAXV = 32;        // polygon vertex cap of the device narrowphase
static constexpr int SOLVE_TPB = 1024;

// one position-solver item, packed (the fields of solvePositionConstraint,
// position_solver.cpp:201-297, that do not change during the solve)
struct PosRec {
    double nx, ny, corr, px, py, invMA, invMB, invIA, invIB;
    int32_t a, b;
    int32_t flags;       // 1 skipped, 2 A rotates, 4 B rotates
    int32_t pad;
};

struct RigidDev {
    int nb = 0, cap_nb = 0;
    lpe_body *bodies = nullptr;
    double *verts = nullptr;
    int nverts = 0, cap_verts = 0;
    int32_t *rank = nullptr, *byRank = nullptr;
    double4 *aabb = nullptr;
    int32_t *cand = nullptr;
    // pairs
    int32_t *pcount = nullptr, *pstart = nullptr, *pcursor = nullptr;
    int2 *pairs = nullptr;
    int32_t *pairRankB = nullptr;
    int cap_pairs = 0;
    // contacts
    lpe_contact *cslots = nullptr;
    int32_t *ccount = nullptr, *cstart = nullptr;
    lpe_contact *contacts = nullptr;
    int cap_contacts = 0;
    // scan partials
    int32_t *bsum = nullptr;
    int cap_bsum = 0;
    // PGS / position solver
    int32_t *order = nullptr;                 // PGS visiting order (contact indices)
    float4 *rowN = nullptr;                   // dirX, dirY, effN, effF
    float4 *rowR = nullptr;                   // rxA, ryA, rxB, ryB
    int2 *rowAB = nullptr;                    // body indices (-1 = static)
    float *vel0 = nullptr;                    // float3 per body (PGS load)
    float *imii = nullptr;                    // float2 per body (invMass, invInertia)
    int32_t *inContact = nullptr;             // per body flags
    float4 *rowM = nullptr;                   // imA, iiA, imB, iiB
    float4 *rowC = nullptr;                   // canonical path: the lever arms' crosses with the normal (A, B)
                                              // and the friction direction (A, B) -- k_pgs_stripes
    float *lamN = nullptr, *lamF = nullptr;   // accumulated impulses per contact
    int32_t *rowOf = nullptr;                 // canonical path: the PGS row of each contact (inverse of order)
    double *posState = nullptr;               // per body: invM, invI, flags (pos solver)
    PosRec *posRec = nullptr;                 // position-solver items
    int32_t *posKeep = nullptr, *posStart = nullptr;
    // dataflow versions (shared by both solvers)
    int32_t *sItemA = nullptr, *sItemB = nullptr;    // dependency bodies per item (-1 none)
    int4 *sVer = nullptr;                            // rank/cnt on A, rank/cnt on B
    int32_t *sBCount = nullptr, *sBStart = nullptr, *sBCursor = nullptr, *sEnt = nullptr;
    int32_t *counts = nullptr;                // [0]=np [1]=nc [4]=npos [5]=heavy [6]=pair overflow [14]=contacts found
    bool detect_launched = false;             // this tick's detection is on the side stream
    bool heavy_valid = false;                 // counts[5] holds the planetary-mass check of the bodies
    unsigned gen = 0;                         // bumped by every upload / config change (world Barnes-Hut cache)
                                              // (masses and flags change only by upload / config)
                                              // [7]=solver fault [8]=colours [9]=colouring rounds
                                              // [10]=special broadphase bodies [11]=contact truncation
    int32_t *pcol = nullptr;                  // colour per pair (canonical order)
    int2 *cseg = nullptr;                     // (row start, rows) per coloured pair, colour-major
    int32_t *cbase = nullptr;                 // first cseg entry of each colour (+ end)
    int cap_pcol = 0;
    // uniform-grid broadphase: bodies whose AABB fits a cell are keyed by the
    // cell of their AABB min corner; the rest ("special": walls, bodies off
    // the grid) are tested against every candidate
    double bp_cell = 0.0;                     // cell size (largest bounded body extent)
    int32_t *bgCount = nullptr, *bgStart = nullptr, *bgCursor = nullptr;   // per cell
    int32_t *bgList = nullptr, *bgKey = nullptr, *bgSpecial = nullptr;      // per body (rank)
    long cap_bgcells = 0;
    lpe_rigid_config cfg{};
    bool cfg_set = false;
    int last_np = 0, last_nc = 0;
    int regrows = 0;                          // detections redone / contact buffer grown (lpe_rigid_buffer_info)
    // world tick: collision detection and colouring run on a side stream
    // while the fluid step runs (rigid_tick_begin / rigid_tick_finish)
    int32_t *bbits = nullptr;                 // per body: boundary bounce bits of the tick
    int32_t *hc = nullptr;                    // pinned: detection counts read by the host
    hipStream_t side = nullptr;
    // the stream the tick's detection and colouring run on: `side` beside a
    // fluid step, the context stream in a world without fluid (nothing to
    // overlap with: the side stream's joins would only add cross-queue
    // packets to the serial path)
    hipStream_t det = nullptr;
    hipEvent_t evStart = nullptr, evDetect = nullptr, evColour = nullptr;
    bool overlap_pending = false;             // detection queued on the side stream
    bool colour_pending = false;              // ... finished by the host, colouring queued
    // world tick, lagged detection check (rigid_tick_launch): once a
    // synchronous detection left 4x headroom in the pair and contact buffers,
    // the detections run without a host wait -- the stages take their sizes
    // from the device counts and capacity-sized grids, and the host checks
    // each tick's counts (copied to hcr[slot]) when it reuses the slot two
    // ticks later, or at a download.  Counts past half the capacity grow the
    // buffers at the next tick start; an overflow (more than 4x growth within
    // two ticks) fails loudly (LPE_ERR_OVERFLOW).  counts[14] = contacts found.
    bool lag = false, lag_next = false;
    bool contacts_zeroed = false;       // k_rb_prep of this detection zeroed inContact (colour_prep skips its memset)
    int32_t *hcr = nullptr;                   // pinned [2][16]
    hipEvent_t evHc[2] = {nullptr, nullptr};
    bool hpend[2] = {false, false};
    unsigned htick = 0;                       // detections issued in lagged mode
    int grow_pairs = 0, grow_contacts = 0;    // capacities wanted at the next tick start
    // striped solver buffers (lpe_rigid.hip StripeBufs, allocated on first use)
    void *stripes = nullptr;
    int cap_stripe_nb = 0, cap_stripe_pairs = 0;
    uint32_t sbase_pgs = 16, sbase_pos = 16;  // hand-over flag epochs of the two solvers
    // opt-in Jacobi contact solver (lpe_rigid.hip JacBufs, allocated on first use)
    void *jac = nullptr;
    int cap_jac_nb = 0;
    bool lam_by_contact = false;              // the last solve's lamN / lamF are by contact (Jacobi), not by row
    // the position solver runs beside the PGS on its own stream (rigid_solve)
    hipStream_t psolve = nullptr;
    hipEvent_t evFork = nullptr, evJoin = nullptr;
    // the world tick's boundary/gravity pass signals evBvg itself (its launch
    // carries the event); the position solver's fork and the next tick's
    // prelaunch wait on it instead of recording their own (bvgSignal: this tick)
    hipEvent_t evBvg = nullptr;
    bool bvgSignal = false;
    // device-side waits (default; LPE_EVENT_WAITS=1: the events above): the
    // boundary passes' last workgroup stores the tick number into a word that
    // a one-wave kernel on the waiting stream polls, so no stream holds a
    // blocked barrier packet during the fluid step (profiles/r06/events/).
    // tsync: [0] boundary/gravity done, [1] its arrivals, [2] clamp done, [3] its arrivals
    uint32_t *tsync = nullptr;
    uint32_t tsyncTick = 0;
    bool devwait_ok = false;              // (tsync_alloc's probe: kernels of two streams run together)
};


RigidDev *rigid_dev(lpe_ctx *ctx);

}  // namespace lpe
