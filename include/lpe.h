/*
 * lpe.h — C ABI of the MI355X-native per-tick physics backend.
 *
 * This is the drop-in boundary for the hot path of little-physics-engine
 * (reference snapshot 2025-05-23).  The reference has no C ABI: its device
 * objects are C++ members of Systems::FluidSystem (include/systems/fluid/
 * fluid.hpp:328-355) and its rigid path is a chain of static C++ functions
 * (src/systems/rigid/rigid_body_collision.cpp:24-50).  Every entry point
 * below names the reference code it replaces.  The C++ host mirror in
 * little-physics-engine_amd/host/ (Systems::FluidSystem,
 * Systems::RigidBodyCollisionSystem, ...) gathers the ECS into these plain
 * arrays and calls through here, exactly where the reference called Metal or
 * its CPU solvers.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Host arrays are caller-owned and only
 *    borrowed for the duration of a call.  Device buffers belong to lpe_ctx
 *    and are grow-only (like FluidSystem::initBuffersIfNeeded,
 *    fluid.cpp:170-248).
 *  - Every function returns an int status, LPE_OK (0) on success.  No C++
 *    exception crosses this boundary.  lpe_last_error() gives a message.
 *  - One HIP stream per context; a context is not re-entrant.
 *  - y points down (gravity is +y), SI units, as in the reference.
 */
#ifndef LPE_H
#define LPE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LPE_ABI_VERSION 2

enum lpe_status {
    LPE_OK = 0,
    LPE_ERR_HIP = 1,        /* a HIP runtime call failed                       */
    LPE_ERR_ARG = 2,        /* bad argument (null pointer, negative count ...) */
    LPE_ERR_STATE = 3,      /* call out of order (e.g. tick before upload)     */
    LPE_ERR_CAPACITY = 4,   /* a particle left the device grid capacity        */
    LPE_ERR_OVERFLOW = 5,   /* a per-particle/per-pair fixed list overflowed   */
    LPE_ERR_NO_DEVICE = 6   /* no HIP device (reference: fluid.cpp:97-100)     */
};

/* Reference: GPU_MAX_PER_CELL (fluid.hpp:56) and GPU_POLYGON_MAX_VERTS
 * (fluid.hpp:93).  The HIP grid hash is a counting sort with no per-cell cap;
 * the cap is only reported (max occupancy) so scenes can be checked against
 * the reference's limit. */
#define LPE_REF_MAX_PER_CELL 64
#define LPE_MAX_POLY_VERTS 16

/* ------------------------------------------------------------------------ */
/* Fluid configuration: field-for-field mirror of Systems::FluidConfig       */
/* (include/systems/fluid/fluid.hpp:131-200); defaults via                   */
/* lpe_fluid_config_default().                                               */
/* ------------------------------------------------------------------------ */
typedef struct lpe_fluid_config {
    float gravity;            /* 9.81  (used only by the coupling solver)   */
    float restDensity;        /* 0.5                                          */
    float stiffness;          /* 200                                          */
    float viscosity;          /* 0.03                                         */
    struct {                  /* fluid.hpp:140-148                            */
        float safetyMargin;       /* 0.001 */
        float relaxFactor;        /* 0.9   */
        float maxCorrection;      /* 0.1   */
        float maxVelocityUpdate;  /* 1.0   (read but unused, as reference)    */
        float minSafeDistance;    /* 1e-10 */
        float velocityDamping;    /* 0.3   (read but unused, as reference)    */
        float minPositionChange;  /* 1e-6  */
    } positionSolver;
    struct {                  /* fluid.hpp:151-179                            */
        float maxForce;               /* 0.15  */
        float maxTorque;              /* 0.03  */
        float fluidForceScale;        /* 100   */
        float fluidForceMax;          /* 5e4   */
        float buoyancyStrength;       /* 0.2   */
        float viscosityScale;         /* 0.05  */
        float depthScale;             /* 0.04  */
        float depthTransitionRate;    /* 2.0   */
        float depthEstimateScale;     /* 10.0  */
        float pressureForceRatio;     /* 1.0   */
        float viscousForceRatio;      /* 0.3   */
        float angularDampingThreshold;/* 0.5   */
        float angularDampingFactor;   /* 0.005 */
        float maxSafeVelocitySq;      /* 80    */
        float minPenetration;         /* 1e-6  */
        float minRelVelocity;         /* 1e-6  */
    } impulseSolver;
    struct {                  /* fluid.hpp:182-186                            */
        float gridEpsilon;        /* 1e-6  */
        float smoothingLength;    /* 0.05  */
        float boundaryOffset;     /* 0.001 */
    } gridConfig;
    struct {                  /* fluid.hpp:189-194                            */
        float minDistanceThreshold;   /* 1e-14 */
        float minDensityThreshold;    /* 1e-12 */
        float minTimestep;            /* 1e-10 */
        float fallbackTimestep;       /* 1e-4  */
    } numericalConfig;
    float dampingFactor;      /* 1.0 (rigid write-back damping)               */
    int   numSubSteps;        /* 10                                           */
    int   threadsPerGroup;    /* 256 (only sizes the reference's bbox partials)*/
} lpe_fluid_config;

/* Rigid body as seen by the fluid coupling: byte-for-byte mirror of
 * Systems::GPURigidBody (fluid.hpp:94-125, 200 B).  Filled by the host
 * mirror's gatherRigidBodies (reference fluid.cpp:304-438). */
typedef struct lpe_gpu_rigid {
    int32_t shapeType;          /* 0 = Circle, 1 = Polygon                     */
    float posX, posY, angle, radius;
    int32_t vertCount;
    float vertsX[LPE_MAX_POLY_VERTS];
    float vertsY[LPE_MAX_POLY_VERTS];
    float vx, vy, omega, mass, inertia;
    float minX, maxX, minY, maxY;
    float accumFx, accumFy, accumTorque;
} lpe_gpu_rigid;

/* Per-tick statistics of the SPH step (for the parity harness / bench). */
typedef struct lpe_sph_stats {
    int32_t maxCellOccupancy;   /* max particles in one reference 2h cell     */
    int32_t notInserted;        /* particles outside the reference grid, last sub-step */
    int32_t capacityOverflow;   /* non-zero if a particle left the device grid */
    int32_t listOverflow;       /* non-zero if a per-particle rigid list overflowed */
    int32_t gridDimX, gridDimY; /* reference grid dims of the last sub-step   */
    int32_t gridMinX, gridMinY;
    float   cellSize;
    /* diagnostics, counted only while lpe_sph_diag(ctx, 1) is on (sums over
     * every sub-step since it was switched on): */
    int32_t nlistOverflow;      /* particles whose neighbour list exceeded 64  */
    int32_t rigidCandidates;    /* rigids tested by the coupling solvers       */
    int32_t neighbours;         /* neighbours with r < h found by the density pass */
    int32_t stageFallback;      /* blocks of the LDS-staged density pass (lpe_sph_probe_density)
                                   whose neighbourhood did not fit LDS (always counted) */
    /* reference cells holding more than LPE_REF_MAX_PER_CELL particles,
     * summed over the sub-steps of the last lpe_sph_step (any mode): where
     * this is non-zero the reference drops inserts and reads across cells */
    int32_t overCapCells;
    /* LPE_SPH_MODE_REF_CELL_CAP read past the last cell of the grid (the
     * reference reads stale or out-of-bounds memory there: undefined) */
    int32_t refUndefined;
    /* overCapCells summed, and maxCellOccupancy maximised, over every step
     * since the last lpe_sph_diag call (a bench window) */
    int32_t overCapCellsTotal;
    int32_t maxCellOccupancyTotal;
    /* slab decomposition: ghost records each exchange moves to the left /
     * right neighbour per sub-step (the wire capacity, wire_cap of
     * lpe_sph_set_slab; 0 without a neighbour or off a slab) */
    int32_t haloWire[2];
    /* slab decomposition: the particles this rank owns now, its slots in use
     * (owned + ghosts of the last sub-step), and the most ghost records the
     * left / right neighbour filed for it in a sub-step since the last
     * lpe_sph_diag; all 0 off a slab */
    int32_t slabOwned, slabSlots;
    int32_t ghostsIn[2];
    int32_t forcesGlobal;       /* forces-pass blocks whose neighbourhood exceeded the LDS image, summed
                                   since the upload (their neighbours are gathered from global memory:
                                   the same sums, slower) */
    /* the lagged checks of lpe_sph_step (ABI 2): times the device grid grew
     * (or recentred) to stay ahead of the fluid's bbox, times a slab rank's
     * slots grew, and the device grid in use (origin and size, cells) */
    int32_t gridRegrows, slotRegrows;
    int32_t deviceGrid[4];
} lpe_sph_stats;

/* ------------------------------------------------------------------------ */
/* Rigid path data: one solid body, its ECS components flattened.            */
/* Filled by the host mirror from entt views (reference components:           */
/* include/entities/entity_components.hpp:6-133, include/math/polygon.hpp:30-44). */
/* ------------------------------------------------------------------------ */
enum lpe_body_flags {
    LPE_BODY_HAS_PHASE   = 1u << 0,   /* Components::ParticlePhase present       */
    LPE_BODY_SOLID       = 1u << 1,   /* ... and phase == Solid                  */
    LPE_BODY_LIQUID      = 1u << 2,   /* ... and phase == Liquid                 */
    LPE_BODY_BOUNDARY    = 1u << 3,   /* Components::Boundary present            */
    LPE_BODY_HAS_SLEEP   = 1u << 4,   /* Components::Sleep present               */
    LPE_BODY_ASLEEP      = 1u << 5,   /* Sleep::asleep                           */
    LPE_BODY_HAS_ANGPOS  = 1u << 6,   /* Components::AngularPosition present     */
    LPE_BODY_HAS_ANGVEL  = 1u << 7,   /* Components::AngularVelocity present     */
    LPE_BODY_HAS_INERTIA = 1u << 8,   /* Components::Inertia present             */
    LPE_BODY_CIRCLE      = 1u << 9,   /* CircleShape present (narrowphase.cpp:38) */
    LPE_BODY_POLYGON     = 1u << 10,  /* PolygonShape present                    */
    LPE_BODY_HAS_MASS    = 1u << 11,  /* Components::Mass present                */
    LPE_BODY_HAS_VEL     = 1u << 12   /* Components::Velocity present            */
};

typedef struct lpe_body {
    uint32_t eid;        /* raw entt::entity value: orders pairs (broadphase.cpp:264) */
    uint32_t flags;      /* lpe_body_flags                                           */
    double x, y, angle;  /* Position, AngularPosition::angle                          */
    double vx, vy, omega;/* Velocity, AngularVelocity::omega                          */
    double mass, inertia;/* Mass::value, Inertia::I                                   */
    double radius;       /* CircleShape::radius                                       */
    int32_t vert_off;    /* PolygonShape vertices: [vert_off, vert_off+vert_cnt) of   */
    int32_t vert_cnt;    /*   the shared local-vertex array (x, y pairs, double)      */
    int32_t sleep_counter;
    int32_t pad;
} lpe_body;

/* A narrowphase contact (collision_data.hpp:22-28): a and b are body indices,
 * n points from A to B; pair is the index of its broadphase pair. */
typedef struct lpe_contact {
    int32_t a, b, pair, pad;
    double nx, ny, pen, px, py;
} lpe_contact;

/* Configuration of RigidBodyCollisionSystem::update and the integrator systems.
 * Reference defaults: BroadphaseConfig (broadphase.hpp:25-34),
 * ContactSolverConfig (contact_solver.hpp:21-27), PositionSolverConfig
 * (position_solver.hpp:21-34), GravityConfig (gravity.hpp:27-34),
 * RotationConfig (rotation.hpp:28-34), BoundaryConfig (boundary.hpp:30-39),
 * SleepConfig (sleep.hpp:31-40).  The reference hard-wires the rigid
 * sub-configs (rigid_body_collision.cpp:30, :44, :48); pgsIterations and
 * posIterations are exposed here with the reference defaults (10, 10). */
typedef struct lpe_rigid_config {
    double universeSize;          /* SharedSystemConfig::UniverseSizeMeters   */
    double metersPerPixel;        /* SharedSystemConfig::MetersPerPixel       */
    int32_t quadtreeCapacity;     /* 8 (tree shape only; pair SET unaffected) */
    int32_t pgsIterations;        /* 10                                        */
    double boundaryBuffer;        /* 500                                       */
    double smallParticleThreshold;/* 0.01                                      */
    float frictionCoeff;          /* 0.5f                                      */
    int32_t posIterations;        /* 10                                        */
    double baumgarte;             /* 0.02                                      */
    double slop;                  /* 0.001                                     */
    double gravity;               /* 9.8   (GravityConfig)                     */
    double planetaryMassThreshold;/* 1e10                                      */
    double angularDamping;        /* 0.98  (RotationConfig)                    */
    double maxAngularSpeed;       /* 20                                        */
    double marginPixels;          /* 15    (BoundaryConfig)                    */
    double bounceDamping;         /* 0.7                                       */
    double maxSpeed;              /* 1.0                                       */
    double linearSleepThreshold;  /* 0.5   (SleepConfig)                       */
    double angularSleepThreshold; /* 0.5                                       */
    int32_t sleepFramesThreshold; /* 60                                        */
    int32_t pgsMode;              /* LPE_PGS_GAUSS_SEIDEL (0, default): the
                                   * reference's sequential PGS in the canonical
                                   * striped order; LPE_PGS_JACOBI (1): opt-in
                                   * parallel Jacobi solve (mass-split contacts,
                                   * pgsIterations iterations) -- not the
                                   * reference's arithmetic, checked by the LCP
                                   * invariants and its own restatement */
} lpe_rigid_config;
#define LPE_PGS_GAUSS_SEIDEL 0
#define LPE_PGS_JACOBI 1

typedef struct lpe_ctx lpe_ctx;

/* ---- lifecycle -------------------------------------------------------- */
/* Replaces FluidSystem::FluidSystem (fluid.cpp:72-125): device, queue and
 * code-object set-up.  The code object is loaded once per process, so a
 * reference-style reset() that re-creates systems does not reload it. */
int  lpe_create(int device, lpe_ctx **out);
/* Replaces FluidSystem::~FluidSystem (fluid.cpp:127-147). */
int  lpe_destroy(lpe_ctx *ctx);
const char *lpe_last_error(const lpe_ctx *ctx);
int  lpe_abi_version(void);
int  lpe_device_count(int *count);
/* Blocks until all work queued on the context's stream is done. */
int  lpe_sync(lpe_ctx *ctx);
/* Hardware queues.  A context runs four streams (fluid step, prelaunch,
 * collision detection, position solver) and HIP maps streams round robin
 * onto GPU_MAX_HW_QUEUES queues, 4 by default: one per stream of a context.
 * Leave it at 4: more than 4 measured every kernel ~2x slower on MI355X /
 * ROCm 7.2 (round 6; round 4 advised 8).  Reports the value in effect
 * (*queues); *set_by_library is always 0 since round 6. */
int  lpe_hw_queues(int *queues, int *set_by_library);

/* ---- kernel timing (bench / profiling; no reference counterpart) ------- */
/* on = 1: every launch of a named kernel on the context's stream is
 * bracketed by a pair of HIP events; on = 2: only the dominant kernels
 * (k_density, k_forces_couple, k_pgs_solve, k_pos_solve, k_narrow,
 * k_bp_pairs), so the host stays ahead of the device; on = 0: off.  lpe_timing_read() waits for the stream,
 * accumulates the event durations and returns, for the i-th kernel name seen,
 * its name, total milliseconds and launch count (returns LPE_ERR_ARG when i is
 * past the last name).  lpe_timing_reset() clears the totals. */
int  lpe_timing_enable(lpe_ctx *ctx, int on);
int  lpe_timing_reset(lpe_ctx *ctx);
int  lpe_timing_read(lpe_ctx *ctx, int i, char *name, int name_cap,
                     double *total_ms, long *calls);

/* ---- SPH fluid (Systems::FluidSystem) ----------------------------------- */
int  lpe_fluid_config_default(lpe_fluid_config *cfg);
/* Replaces the FluidConfig → GPUFluidParams packing (fluid.cpp:614-666,
 * :759-818). */
int  lpe_sph_set_config(lpe_ctx *ctx, const lpe_fluid_config *cfg);
/* Replaces gatherFluidParticles' output copy into the particle buffer
 * (fluid.cpp:250-302, :996-1000).  n fluid particles in gather order; the
 * arrays are fp32 (the reference casts double→float at gather).  h is
 * config.gridConfig.smoothingLength for every particle (fluid.cpp:292), so it
 * is not an input.  ax = ay = 0 and vh = v at every gather (fluid.cpp:287-290);
 * lpe_sph_upload re-establishes that. */
int  lpe_sph_upload(lpe_ctx *ctx, int n,
                    const float *x, const float *y,
                    const float *vx, const float *vy,
                    const float *mass,
                    const float *density, const float *pressure);
/* Replaces the rigid part of FluidSystem::update (fluid.cpp:975-1007):
 * r bodies in gatherRigidBodies order.  accum* are ignored (reset to 0). */
int  lpe_sph_upload_rigids(lpe_ctx *ctx, int r, const lpe_gpu_rigid *rigids);
/* Replaces multiStepVelocityVerlet (fluid.cpp:582-956): numSubSteps
 * sub-steps of kick/drift → grid hash → density → forces → finish →
 * rigid–fluid impulse (if r > 0) → rigid–fluid push-out, followed by the
 * once-per-tick rigid velocity write-back arithmetic (fluid.cpp:545-562).
 * dt_tick = SharedSystemConfig.SecondsPerTick * TimeAcceleration
 * (fluid.cpp:592).  Asynchronous: results are read with lpe_sph_download*. */
int  lpe_sph_step(lpe_ctx *ctx, double dt_tick);
/* Replaces writeBackToECS's source data (fluid.cpp:496-524).  Any pointer
 * may be NULL to skip that field.  Blocks until the step is complete. */
int  lpe_sph_download(lpe_ctx *ctx, float *x, float *y, float *vx, float *vy,
                      float *density, float *pressure);
/* Extra fields for parity tests: half-step velocity and acceleration. */
int  lpe_sph_download_aux(lpe_ctx *ctx, float *vxHalf, float *vyHalf,
                          float *ax, float *ay);
/* Replaces writeBackRigidBodies' source data (fluid.cpp:526-580): the
 * rigid array after v += F/m, ω += τ/I, × dampingFactor (accum reset to 0).
 * The pre-write-back accumulators are returned in accumF{x,y},accumTorque
 * when accum is non-NULL (3 floats per body). */
int  lpe_sph_download_rigids(lpe_ctx *ctx, lpe_gpu_rigid *rigids, float *accum);
int  lpe_sph_get_stats(lpe_ctx *ctx, lpe_sph_stats *stats);
/* Diagnostics counters of lpe_sph_stats on (1, counters reset) or off (0);
 * either way the window totals (overCapCellsTotal, maxCellOccupancyTotal)
 * restart. */
int  lpe_sph_diag(lpe_ctx *ctx, int on);

/* SPH modes (flags, default 0).
 * LPE_SPH_MODE_REF_CELL_CAP: the reference's fixed-capacity grid semantics.
 *   Its GPUGridCell holds a count and 64 indices (GPU_MAX_PER_CELL,
 *   fluid.hpp:56); assignCells keeps incrementing count past 64 but stores no
 *   more indices (fluid_kernels.metal:237-240), and computeDensity /
 *   computeForces loop c < count unclamped (:281-283, :349-351), reading the
 *   next cells' count and indices as particle ids (values >= N skipped).  In
 *   this mode the device reproduces exactly that, with the canonical
 *   insertion order (cell quadrants row-major, ascending particle index) in
 *   place of the reference's atomic order; where no cell exceeds 64 it equals
 *   the default mode bit for bit.  Default (0): unbounded cell lists (the
 *   counting sort has no capacity), i.e. the reference's intent.  Not
 *   available on a slab rank (LPE_ERR_STATE). */
#define LPE_SPH_MODE_REF_CELL_CAP 1
/* LPE_SPH_MODE_PROBE_TICK_PASS: lpe_sph_probe_density runs the tick's density
 * pass (which also writes the forces pass's neighbour lists) instead of the
 * pure computeDensity pass; the same sums, bit for bit (the density
 * microbench times both). */
#define LPE_SPH_MODE_PROBE_TICK_PASS 2
int  lpe_sph_set_mode(lpe_ctx *ctx, int flags);

/* Parity probe: the reference's assignCells cell index for each particle
 * (fluid_kernels.metal:212-241: cellY*gridDimX + cellX, or -1 if "not
 * inserted") computed from the CURRENT device positions with the grid the
 * reference would derive from them (fluid.cpp:717-752).  Runs one kick-free
 * hash pass; does not advance the simulation. */
int  lpe_sph_probe_cells(lpe_ctx *ctx, int32_t *cell_index, lpe_sph_stats *stats);
/* Parity probe: density and pressure of the current positions (one hash +
 * density pass, no integration; fluid_kernels.metal:246-307). */
int  lpe_sph_probe_density(lpe_ctx *ctx, float *density, float *pressure);

/* ---- rigid bodies (Systems::RigidBodyCollisionSystem + integrators) ---- */
typedef struct lpe_rigid_stats {
    int32_t pairs;          /* broadphase pairs                                */
    int32_t contacts;       /* narrowphase contacts                            */
    int32_t pgsLevels;      /* dependency levels of one PGS sweep              */
    int32_t posLevels;      /* dependency levels of one position-solver sweep  */
    int32_t overflow;       /* non-zero if a fixed-capacity list overflowed    */
    int32_t colourRounds;   /* rounds of the parallel pair colouring           */
} lpe_rigid_stats;

int  lpe_rigid_config_default(lpe_rigid_config *cfg);
int  lpe_rigid_set_config(lpe_ctx *ctx, const lpe_rigid_config *cfg);
/* Bodies (ECS gather of every entity the rigid path or the integrators read)
 * and the shared local-vertex array (x, y pairs).  Body order is free; pair
 * order is by lpe_body::eid. */
int  lpe_rigid_upload(lpe_ctx *ctx, int nb, const lpe_body *bodies, int nverts,
                      const double *verts);
/* RigidBodyCollisionSystem::update (rigid_body_collision.cpp:24-50) on the
 * device: broadphase pair set (broadphase.cpp:233-295) in canonical order
 * (eid_a, eid_b); GJK/EPA/clipping narrowphase in fp64
 * (narrowphase.cpp:352-420); PGS (contact_solver.cpp:449-543) and Baumgarte
 * position solver (position_solver.cpp:299-325) as exact sequential
 * Gauss-Seidel sweeps in the graph-coloured order: pairs edge-coloured so
 * that one colour's pairs share no movable body, visited colour by colour,
 * each pair's contacts in narrowphase order (the reference visits its
 * unordered_map's order, contact_manager.cpp:169-245).  stats->pgsLevels and
 * posLevels report the colour count. */
int  lpe_rigid_step(lpe_ctx *ctx, lpe_rigid_stats *stats);
/* Pre-size the pair and contact buffers of lpe_rigid_step (re-allocated at
 * exactly these capacities; the defaults are 16 pairs and 64 contacts per
 * body).  A step whose pairs or contacts exceed them grows them and redoes
 * its detection (never a truncated list); lpe_rigid_buffer_info reports the
 * capacities and how often that happened.  Replaces the grow-only sizing of
 * the reference's per-pair std::vectors (narrowphase.cpp:352-420). */
int  lpe_rigid_reserve(lpe_ctx *ctx, int pairs, int contacts);
int  lpe_rigid_buffer_info(lpe_ctx *ctx, int *pairs, int *contacts, int *regrows);
/* Colour of each pair of the last lpe_rigid_step (-1: pair without contacts),
 * for the parity harness; cap entries at most, *ncolours the colour count. */
int  lpe_rigid_download_colours(lpe_ctx *ctx, int cap, int32_t *pair_colour, int32_t *ncolours);
/* Accumulated impulses of the last lpe_rigid_step's contact solve, per
 * contact in lpe_rigid_download_contacts order: lamN the normal row's
 * (>= 0), lamF the friction row's (|lamF| <= frictionCoeff * lamN) --
 * ContactRows::normal / ::friction .lambda (contact_solver.cpp:399-437),
 * which the reference keeps inside solveLcpPgs.  cap entries at most. */
int  lpe_rigid_download_impulses(lpe_ctx *ctx, int cap, float *lamN, float *lamF, int32_t *nc);
/* Same with caller-supplied orders (parity mode): `pairs` (np body-index
 * pairs) replaces the broadphase and fixes the narrowphase / position-solver
 * order; `pgs_order` (NULL = contact order) is the PGS contact visiting order,
 * e.g. the reference's unordered_map manifold order
 * (contact_manager.cpp:169-245). */
int  lpe_rigid_step_ordered(lpe_ctx *ctx, int np, const int32_t *pairs, int nc_order,
                            const int32_t *pgs_order, lpe_rigid_stats *stats);
/* Integrator systems on the device, in this order when their bit is set:
 * 1 Boundary (boundary.cpp:13-70), 2 Gravity (gravity.cpp:19-58),
 * 4 Rotation (rotation.cpp:18-60), 8 Movement (movement.cpp:13-39),
 * 16 Sleep (sleep.cpp:19-67).  dt_state = SecondsPerTick *
 * baseTimeAcceleration * timeScale (gravity, rotation); dt_move =
 * SecondsPerTick * TimeAcceleration (movement). */
int  lpe_rigid_integrate(lpe_ctx *ctx, int systems, double dt_state, double dt_move);
int  lpe_rigid_download(lpe_ctx *ctx, lpe_body *bodies);
/* Last step's pairs and contacts (parity probes). */
int  lpe_rigid_download_contacts(lpe_ctx *ctx, int pair_cap, int32_t *pairs, int contact_cap,
                                 lpe_contact *contacts, int32_t *np, int32_t *nc);

/* ---- resident world tick (ECSSimulator::tick, src/sim.cpp:156-163) ------ */
/* Time configuration of a tick: SharedSystemConfig::SecondsPerTick and
 * ::TimeAcceleration (FluidSystem, MovementSystem) and the SimulatorState
 * entity's baseTimeAcceleration * timeScale (Gravity, Rotation). */
typedef struct lpe_world_config {
    double secondsPerTick;
    double timeAcceleration;
    double baseTimeAcceleration;
    double timeScale;
} lpe_world_config;

/* Coupling rigids of FluidSystem::gatherRigidBodies (fluid.cpp:304-438): the
 * body indices (into the lpe_rigid_upload array) in the reference's view
 * order.  nr < 0 selects every uploaded body in descending index order
 * (reverse insertion, the EnTT view order for bodies uploaded in creation
 * order). */
int  lpe_world_set_coupling(lpe_ctx *ctx, int nr, const int32_t *body_index);
/* nticks device-resident ticks of the reference system order: FluidSystem
 * (rigid gather -> SPH sub-steps with coupling -> rigid velocity
 * write-back), Boundary, Gravity (bodies and fluid), RigidBodyCollision,
 * Rotation, Movement, Sleep (BarnesHut returns early: masses < 1e3,
 * barnes_hut.cpp:54-70; the call fails with LPE_ERR_ARG otherwise).  Fluid
 * state stays fp32 between ticks exactly as the ECS round trip of
 * fluid.cpp:496-524 leaves it. */
int  lpe_world_tick(lpe_ctx *ctx, const lpe_world_config *cfg, int nticks);

/* ---- x-slab decomposition of the SPH step -----------
 * The reference has one FluidSystem per process (fluid.cpp:958-1021); these
 * entry points split its particle set over ranks by x slab.  Rank r owns the
 * particles whose reference-cell column floor((x + eps) / 2h) lies in
 * [edges[r], edges[r+1]) / 2h (the first slab has no left edge, the last no
 * right edge), judged from the kicked position at every sub-step, and runs
 * lpe_sph_step / lpe_world_tick on them.  Per sub-step it exchanges with its
 * two neighbours the particles within two cell columns of (or past) an edge
 * -- ghosts, with their global ids and full state, so every density / force
 * sum is the single-domain one bit for bit and a particle that crossed an
 * edge is adopted by the rank it entered -- plus every rank's bbox record
 * (the reference grid is the global one).  Once per tick the rigid
 * accumulators are all-reduced (exact int64 limbs) before the write-back.
 * No host synchronisation: the exchanges are stream-ordered.
 * edges: nranks + 1 values in metres; the inner ones must be multiples of
 * the reference cell size 2h (0.1 m at the default h; the outer two are
 * ignored) and at least 8 cells apart.  wire_cap: ghost records per
 * direction and sub-step (both ends the same; more raise LPE_ERR_OVERFLOW at
 * the next download).  rebalance > 0: every that many fluid steps the inner
 * edges move one cell column towards equal owned counts (an all-reduced
 * histogram; identical on every rank), at most a quarter of the narrowest
 * slab from where they started.  Call after lpe_sph_set_config and before
 * lpe_sph_upload (the particle arrays get slots for the ghosts and growth).
 * A slab rank must not skip a tick or a step its neighbours take. */
int  lpe_sph_set_slab(lpe_ctx *ctx, int nranks, int rank, const float *edges, int wire_cap,
                      int rebalance);
/* A slab rank's current edges as reference-cell columns (nranks + 1 into
 * edges when cap allows; the outer two are -/+ 2^29), its rank count and
 * how many columns an edge may move from where it started (0: fixed). */
int  lpe_sph_slab_info(lpe_ctx *ctx, int cap, int32_t *edges, int *nranks, int *move);
/* Global particle ids of the n uploaded (owned) particles (default 0..n-1). */
int  lpe_sph_set_ids(lpe_ctx *ctx, int n, const int32_t *ids);
/* A slab rank: the particle count of the whole fluid (ids 0..n_global-1;
 * the reference's particleCount, fluid.cpp:981-984, bounds the values its
 * capped-cell loop takes for ids, fluid_kernels.metal:284-286).  Needed
 * before LPE_SPH_MODE_REF_CELL_CAP on a slab rank, which then files ghosts
 * in 3 columns each side instead of 2 (size wire_cap for them).  ABI 2. */
int  lpe_sph_set_global_count(lpe_ctx *ctx, int n_global);
/* The particles this context owns with their global ids (*n_out = count;
 * LPE_ERR_CAPACITY if it exceeds cap); in device order without a slab (ids
 * 0..n-1 permuted), in no particular order on a slab rank. */
int  lpe_sph_download_owned(lpe_ctx *ctx, int cap, float *x, float *y, float *vx, float *vy,
                            float *density, float *pressure, int32_t *ids, int *n_out);
/* Grow the device grid (fixed absolute cell grid, sized at upload from the
 * particles) to cover [x0, x1] x [y0, y1] (a slab rank: within its slab's
 * reach).  Call after lpe_sph_upload. */
int  lpe_sph_set_domain(lpe_ctx *ctx, double x0, double y0, double x1, double y1);
/* RCCL transport (one process per GPU, rank r of n, neighbours r-1 / r+1):
 * rank 0 creates the 128-byte id, every rank passes it to lpe_mg_init_rccl. */
int  lpe_mg_unique_id(char id[128]);
int  lpe_mg_init_rccl(lpe_ctx *ctx, int nranks, int rank, const char *id);
/* The context's transport: its rank count and rank, and the ranks its
 * communicator reports (ncclCommCount for RCCL -- the bench's check that the
 * N-GPU run really joined N ranks; the group size for the host-staged and
 * in-process transports; all 0 without a transport). */
int  lpe_mg_info(lpe_ctx *ctx, int *nranks, int *rank, int *comm_ranks);
/* Host-staged transport: the caller moves host copies of the exchange
 * buffers between the ranks' processes (e.g. torch.distributed over gloo).
 * halo: send sbL bytes of sendL to rank-1 and sbR of sendR to rank+1,
 * receive rbL bytes from rank-1 into recvL and rbR from rank+1 into recvR
 * (NULL / 0 where there is no neighbour); the sizes must equal the
 * neighbour's (the callback checks them and returns non-zero on a mismatch).
 * allreduce_f32 (op 0 sum, 1 min) and allreduce_i64 (sum, two's-complement
 * wrap) reduce n host values in place.  Every callback returns 0 on success;
 * a non-zero return fails the step with LPE_ERR_STATE.  Every call drains
 * the context's stream (validation transport, not the production path). */
typedef struct lpe_host_transport {
    void *user;
    int (*halo)(void *user, const void *sendL, size_t sbL, const void *sendR, size_t sbR, void *recvL,
                size_t rbL, void *recvR, size_t rbR);
    int (*allreduce_f32)(void *user, float *buf, int n, int op);
    int (*allreduce_i64)(void *user, long long *buf, int n);
} lpe_host_transport;
int  lpe_mg_init_host(lpe_ctx *ctx, int nranks, int rank, const lpe_host_transport *t);
/* In-process transport for tests: n contexts (ranks 0..n-1, any devices)
 * each advanced nticks by its own host thread — lpe_world_tick(cfg, 1) per
 * tick when cfg is non-NULL, else lpe_sph_step(dt_tick). */
int  lpe_mg_loopback_run(int n, lpe_ctx **ctxs, const lpe_world_config *cfg, double dt_tick,
                         int nticks);

/* ---- screen-space fluid density field -------- */
/* GPURenderParams (include/renderers/fluid_renderer_kernels.h:28-41): a
 * gridW x gridH grid of cellSize-metre cells from (originX, originY);
 * smoothingRadius is in cells (fluid_renderer.cpp:384-388 sets 10 and
 * cellSize = metres per pixel, origin (0, 0)). */
typedef struct lpe_render_params {
    int32_t gridW, gridH;
    float cellSize;
    float originX, originY;
    float smoothingRadius;
} lpe_render_params;
/* Replaces the compute passes of FluidRenderer::render (fluid_renderer.cpp:
 * 341-465, fluid_renderer_kernels.metal:36-124) on the context's current
 * fluid: unnormalised poly6 density per cell (h = smoothingRadius *
 * cellSize), two 5x5 box blurs, the maximum of the blurred grid, and the
 * normalised grid saturate(d / max) (0 where max <= 1e-12).  normalized
 * (gridW * gridH floats, row-major, may be NULL) and max_out (may be NULL)
 * are host pointers; blocks until done.  No fluid: a zero grid (the
 * reference skips the frame).  Not on a slab rank (LPE_ERR_STATE). */
int  lpe_render_density(lpe_ctx *ctx, const lpe_render_params *params, float *normalized,
                        float *max_out);

/* ---- Barnes-Hut gravity ----------------------- */
/* BarnesHutConfig (include/systems/barnes_hut.hpp:19-25) plus the
 * SharedSystemConfig fields BarnesHutSystem::update reads: UniverseSizeMeters
 * (root box, barnes_hut.cpp:110-112, :123-124), GravitationalSoftener (:261)
 * and SimulatorConstants::RealG (:277). */
typedef struct lpe_bh_config {
    double theta;                 /* 0.5 */
    double small_mass_threshold;  /* 1e3; <= 0 disables the early exit and the small-node skip */
    double universe_size;         /* root box [0, U) x [0, U) */
    double softener;              /* added as softener^2 to every distance^2 */
    double G;                     /* 6.674e-11 (src/core/constants.cpp:8) */
} lpe_bh_config;
typedef struct lpe_bh_stats {
    int32_t skipped;              /* 1: every mass below the threshold, nothing done (:55-71) */
    int32_t inserted;             /* bodies inside the universe, inserted into the tree */
    int32_t nodes;                /* quadtree nodes (the reference's nodePool_ use) */
    int32_t depth;                /* deepest level an insert reached (root = 0) */
} lpe_bh_stats;
/* Safety cap on the tree depth (LPE_ERR_OVERFLOW past it).  fp64 never gets
 * there: coincident bodies are dropped by the child's contains() test once the
 * box is below their ulp (depth ~55 for coordinates ~10 in a 64 m universe),
 * as in the reference. */
#define LPE_BH_MAX_DEPTH 128
int  lpe_bh_config_default(lpe_bh_config *cfg);
/* The bodies: the entities of view<Position, Mass>(exclude<Boundary>) in that
 * view's iteration order, which is buildTree's insertion order (:117-128);
 * has_vel[i] != 0 where the entity also has a Velocity (bodyView, :89; NULL:
 * all).  Host arrays, copied to the device. */
int  lpe_bh_upload(lpe_ctx *ctx, int n, const double *x, const double *y, const double *vx,
                   const double *vy, const double *mass, const uint8_t *has_vel);
/* One BarnesHutSystem::update (barnes_hut.cpp:50-99) on the uploaded bodies:
 * the small-mass early exit, the quadtree (same nodes, same centre-of-mass
 * fold order as the sequential insertion) and the force walk of every body
 * with a velocity, vel += a * dt in the reference's child order.
 * dt = SecondsPerTick * baseTimeAcceleration * timeScale (:284).  stats may
 * be NULL.  Blocks until done. */
int  lpe_bh_step(lpe_ctx *ctx, const lpe_bh_config *cfg, double dt, lpe_bh_stats *stats);
int  lpe_bh_download(lpe_ctx *ctx, double *vx, double *vy);
/* BarnesHutSystem inside lpe_world_tick (position 5 of sim.cpp:107-114, on
 * the rigid context's bodies, after the collision system and before
 * rotation).  Enabled by default with lpe_bh_config_default() and the rigid
 * config's universe size (the reference registers the system in every
 * scene, sim.cpp:111).  enable = 0 switches it off; cfg (may be NULL: the
 * defaults) replaces the config; order (n body indices, may be NULL / 0)
 * is the insertion order, i.e. the bodies of view<Position, Mass>
 * (exclude<Boundary>) in that view's iteration order - by default every
 * body with LPE_BODY_HAS_MASS and without LPE_BODY_BOUNDARY, last body
 * first (EnTT views iterate newest first).  The small-mass early exit is
 * decided once per upload / config change.  A world whose fluid particles
 * would make the system act fails with LPE_ERR_STATE (strict mode handles
 * it through lpe_bh_step).  Shares the buffers of lpe_bh_upload. */
int  lpe_world_set_barnes_hut(lpe_ctx *ctx, int enable, const lpe_bh_config *cfg, int n,
                              const int32_t *order);

#ifdef __cplusplus
}
#endif
#endif /* LPE_H */
