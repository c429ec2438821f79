/*
 * sph_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's SPH fluid step, used as the parity checker for the HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this code; the product library never links it.
 *
 * Parity status: UNPINNED BY EXECUTION.  The reference SPH path is Metal-only
 * (src/systems/fluid/fluid_kernels.metal) and cannot run in this container;
 * the reference holds no golden vectors, tests or fixtures for it (SURVEY.md
 * §4, §8c).  This file restates fluid_kernels.metal:19-924 and the
 * orchestration of src/systems/fluid/fluid.cpp:582-1021 line by line, with the
 * reference's non-deterministic orders replaced by canonical ones:
 *   - grid cell lists: ascending particle index (the reference inserts in
 *     atomic arrival order, fluid_kernels.metal:237);
 *   - rigid accumulators (reference: float atomics, fluid_kernels.metal:
 *     892-898, no defined order): the exact sum of the fp32 contributions,
 *     rounded once to nearest even (xacc_* below) -- the order-independent
 *     value that every sequence of float additions approximates.
 * Arithmetic is IEEE fp32 with no FMA contraction (build with
 * -ffp-contract=off); the reference compiles Metal with fast-math, which has
 * no single defined result.
 */
#include <math.h>
#include <float.h>
#include <stdlib.h>
#include <string.h>
#include "sph_oracle.h"

#define PI_F ((float)3.14159265358979323846)  /* MSL evaluates M_PI as float (fluid_kernels.metal:17) */

/* fluid_kernels.metal:19-24 */
static float poly6Coeff2D(float h) {
    float h2 = h * h;
    float h4 = h2 * h2;
    float h8 = h4 * h4;
    return 4.0f / (PI_F * h8);
}
/* fluid_kernels.metal:26-31 */
static float spikyCoeff2D(float h) {
    float h2 = h * h;
    float h4 = h2 * h2;
    float h5 = h4 * h;
    return -30.0f / (PI_F * h5);
}
/* fluid_kernels.metal:33-38 */
static float viscLaplacianCoeff2D(float h) {
    float h2 = h * h;
    float h4 = h2 * h2;
    float h5 = h4 * h;
    return 40.0f / (PI_F * h5);
}

/* fluid_kernels.metal:125-147 */
static int pointInPolygon(float px, float py, const lpe_gpu_rigid *b) {
    int vCount = b->vertCount;
    if (vCount < 3) return 0;
    int inside = 0;
    for (int i = 0, j = vCount - 1; i < vCount; j = i++) {
        float xi = b->vertsX[i], yi = b->vertsY[i];
        float xj = b->vertsX[j], yj = b->vertsY[j];
        int intersect = ((yi > py) != (yj > py)) &&
                        (px < (xj - xi) * (py - yi) / (yj - yi) + xi);
        if (intersect) inside = !inside;
    }
    return inside;
}

/* fluid_kernels.metal:149-194 */
static void closestPointOnPolygon(float px, float py, const lpe_gpu_rigid *b,
                                  float *ox, float *oy) {
    int vCount = b->vertCount;
    *ox = px; *oy = py;
    if (vCount < 2) return;
    float minDistSq = 1e12f;
    for (int i = 0; i < vCount; i++) {
        int j = (i + 1) % vCount;
        float x1 = b->vertsX[i], y1 = b->vertsY[i];
        float x2 = b->vertsX[j], y2 = b->vertsY[j];
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
        if (distSq < minDistSq) { minDistSq = distSq; *ox = cx; *oy = cy; }
    }
}

static float f2len(float x, float y) { return sqrtf(x * x + y * y); }

/* tanh and pow of the impulse solver (metal:810, :822).  Metal's fast-math
 * versions have no single defined result; the canonical value here (and in
 * the HIP path) is the fp64 function rounded once to fp32, i.e. the correctly
 * rounded fp32 result except in ~2^-29 of cases. */
static float lpe_tanhf(float x) { return (float)tanh((double)x); }
static float lpe_powf(float x, float e) { return (float)pow((double)x, (double)e); }

/* Exact accumulation of the rigid coupling forces.  A sum is 8 limbs of 32
 * bits (int64 containers, carries deferred) of the value * 2^160: every fp32
 * below 2^64 in magnitude, denormals included, is added exactly; the total is
 * rounded once to nearest even.  Independent restatement of the device's
 * xacc_add / xacc_round (little-physics-engine_amd/csrc/sph_coupling.h). */
#define XACC_LIMBS 8
#define XACC_BIAS 160
static int xacc_range_error = 0;

static void xacc_add(uint64_t *acc, float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    uint32_t e = (u >> 23) & 0xffu, m = u & 0x7fffffu;
    if (e == 0 && m == 0) return;
    if (e >= 127u + 64u) { __atomic_store_n(&xacc_range_error, 1, __ATOMIC_RELAXED); return; }
    uint32_t M = e ? (m | 0x800000u) : m;
    int pos = (e ? (int)e - 150 : -149) + XACC_BIAS;
    uint64_t v = (uint64_t)M << (pos & 31);
    uint64_t lo = v & 0xffffffffull, hi = v >> 32;
    if (u >> 31) { lo = 0ull - lo; hi = 0ull - hi; }
    /* atomic: the oracle's particle loops run on OpenMP threads; integer
     * adds commute, so the sum is the same in any order */
    __atomic_fetch_add(&acc[pos >> 5], lo, __ATOMIC_RELAXED);
    __atomic_fetch_add(&acc[(pos >> 5) + 1], hi, __ATOMIC_RELAXED);
}

static float xacc_round(const uint64_t *acc) {
    uint32_t d[XACC_LIMBS];
    int64_t carry = 0;
    for (int i = 0; i < XACC_LIMBS; i++) {
        int64_t t = (int64_t)acc[i] + carry;
        d[i] = (uint32_t)((uint64_t)t & 0xffffffffull);
        carry = (t - (int64_t)d[i]) / 4294967296LL;      /* exact: t - low is a multiple of 2^32 */
    }
    int neg = carry < 0;
    if (neg) {
        uint64_t c = 1;
        for (int i = 0; i < XACC_LIMBS; i++) {
            uint64_t t = (uint64_t)(uint32_t)~d[i] + c;
            d[i] = (uint32_t)t;
            c = t >> 32;
        }
    }
    int b = -1;
    for (int i = XACC_LIMBS - 1; i >= 0 && b < 0; i--)
        if (d[i]) for (int k = 31; k >= 0; k--) if ((d[i] >> k) & 1u) { b = i * 32 + k; break; }
    if (b < 0) return 0.0f;
    int p = b - 23 > 11 ? b - 23 : 11;
    uint32_t kept = 0;
    for (int k = b; k >= p; k--) kept = (kept << 1) | ((d[k >> 5] >> (k & 31)) & 1u);
    uint32_t guard = (d[(p - 1) >> 5] >> ((p - 1) & 31)) & 1u;
    int sticky = 0;
    for (int k = 0; k < p - 1; k++) sticky |= (int)((d[k >> 5] >> (k & 31)) & 1u);
    if (guard && (sticky || (kept & 1u))) kept++;
    float r = ldexpf((float)kept, p - XACC_BIAS);
    return neg ? -r : r;
}

#ifdef _OPENMP
#include <omp.h>
#endif
/* Threads of the per-particle loops (<= 0: OpenMP's default).  Every particle
 * is computed exactly as in the serial loop, so results do not depend on it. */
void lpeo_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n > 0 ? n : omp_get_num_procs());
#else
    (void)n;
#endif
}
int lpeo_get_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* Test hook: the exact, once-rounded sum of n floats (-1e30f on a range error). */
float lpeo_xacc_sum(const float *v, int n) {
    uint64_t acc[XACC_LIMBS] = {0};
    xacc_range_error = 0;
    for (int i = 0; i < n; i++) xacc_add(acc, v[i]);
    return xacc_range_error ? -1e30f : xacc_round(acc);
}

/* Grid of the reference: fluid.cpp:717-752 (host, fp32). */
void lpeo_grid_from_bbox(const lpeo_particle *p, int n, float smoothingLength,
                         lpeo_grid *g) {
    (void)smoothingLength;
    float minX = FLT_MAX, maxX = -FLT_MAX, minY = FLT_MAX, maxY = -FLT_MAX;
    /* computeBoundingBox + reduceBoundingBoxOnCPU (fluid_kernels.metal:446-514,
     * fluid.cpp:440-494): exact min/max over the n real particles. */
    for (int i = 0; i < n; i++) {
        if (p[i].x < minX) minX = p[i].x;
        if (p[i].x > maxX) maxX = p[i].x;
        if (p[i].y < minY) minY = p[i].y;
        if (p[i].y > maxY) maxY = p[i].y;
    }
    if (minX > maxX) { float t = minX; minX = maxX; maxX = t; }
    if (minY > maxY) { float t = minY; minY = maxY; maxY = t; }
    /* maxH scan over particle h (fluid.cpp:724-736) */
    float maxH = 0.05f;
    for (int i = 0; i < n; i++) if (p[i].h > maxH) maxH = p[i].h;
    float cellSize = 2.f * maxH;
    minX -= 1e-6f;
    minY -= 1e-6f;
    int gmx = (int)floorf(minX / cellSize);
    int gmy = (int)floorf(minY / cellSize);
    int gMx = (int)floorf(maxX / cellSize);
    int gMy = (int)floorf(maxY / cellSize);
    int dx = gMx - gmx + 1, dy = gMy - gmy + 1;
    if (dx < 1) dx = 1;
    if (dy < 1) dy = 1;
    g->cellSize = cellSize;
    g->gridMinX = gmx; g->gridMinY = gmy;
    g->gridDimX = dx;  g->gridDimY = dy;
    g->bbox[0] = minX + 1e-6f; g->bbox[1] = maxX; g->bbox[2] = minY + 1e-6f; g->bbox[3] = maxY;
}

/* assignCells cell index (fluid_kernels.metal:224-236); -1 = not inserted. */
static int cell_of(const lpeo_grid *g, float eps, float x, float y) {
    float px = x + eps, py = y + eps;
    int gx = (int)floorf(px / g->cellSize);
    int gy = (int)floorf(py / g->cellSize);
    int cx = gx - g->gridMinX, cy = gy - g->gridMinY;
    if (cx < 0 || cx >= g->gridDimX || cy < 0 || cy >= g->gridDimY) return -1;
    return cy * g->gridDimX + cx;
}

void lpeo_assign_cells(const lpeo_particle *p, int n, const lpeo_grid *g,
                       float eps, int32_t *cell) {
    for (int i = 0; i < n; i++) cell[i] = cell_of(g, eps, p[i].x, p[i].y);
}

/* Cell lists in canonical order.  The reference inserts in atomic arrival
 * order (fluid_kernels.metal:237), so any fixed order is a valid restatement;
 * this one is the HIP path's: inside each reference 2h cell, particles are
 * grouped by h-sized quadrant (qy, then qx, row-major) and ascending particle
 * index within a quadrant.  The stencil walk (ny, nx row-major over the 3x3
 * cells, metal:272-283) visits each cell's list in that order.  The quadrant
 * of a particle is floor(2t) - 2 floor(t) with t = (x + eps) / cellSize, so it
 * is consistent with the cell index bit for bit. start has C+1 entries. */
typedef struct {
    int32_t *start; int32_t *idx; int C; int maxOcc; int notIns;
    int overCap;          /* cells holding more than GPU_MAX_PER_CELL particles  */
    int32_t *F;           /* reference cell-capacity mode: the grid buffer      */
} cells_t;

/* Reference cell-capacity mode (lpeo_set_ref_cell_cap).  The reference's grid
 * is an array of GPUGridCell {int count; int indices[64];} (fluid.hpp:56-61,
 * 65 ints per cell), memset to 0 every sub-step (fluid.cpp:821-824).
 * assignCells increments count for every particle but stores only the first
 * 64 indices (fluid_kernels.metal:237-240); the readers loop c < count
 * UNCLAMPED over indices[c] (:281-283, :349-351), so past 64 they read the
 * next cell's count and indices (a flat 65-int stride), skipping values
 * >= particleCount.  Insertion order is the canonical cell order above (the
 * reference's is atomic arrival order).  F is that buffer, read exactly as
 * the kernels read it; a read past the last cell (undefined in the
 * reference: stale or out-of-bounds memory) sets lpeo_ref_undefined. */
#define REF_MAX_PER_CELL 64
#define REF_CELL_INTS (REF_MAX_PER_CELL + 1)
static int ref_cap_mode = 0;
static int ref_undefined = 0;
void lpeo_set_ref_cell_cap(int on) { ref_cap_mode = on ? 1 : 0; }
int lpeo_ref_undefined(void) { return ref_undefined; }

/* indices[k] of cell c as the reference kernels read it (k may exceed 63) */
static int ref_index(const cells_t *cl, int c, int k) {
    long pos = (long)REF_CELL_INTS * c + 1 + k;
    if (pos >= (long)REF_CELL_INTS * cl->C) { __atomic_store_n(&ref_undefined, 1, __ATOMIC_RELAXED); return 0; }
    return cl->F[pos];
}

static int quad_of(const lpeo_grid *g, float eps, float x, float y) {
    float tx = (x + eps) / g->cellSize, ty = (y + eps) / g->cellSize;
    int qx = (int)floorf(2.0f * tx) - 2 * (int)floorf(tx);
    int qy = (int)floorf(2.0f * ty) - 2 * (int)floorf(ty);
    return qy * 2 + qx;
}

static void build_cells(const lpeo_particle *p, int n, const lpeo_grid *g,
                        float eps, cells_t *cl) {
    int C = g->gridDimX * g->gridDimY;
    cl->C = C;
    cl->start = (int32_t *)calloc((size_t)C + 1, sizeof(int32_t));
    cl->idx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *bin = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int32_t *bstart = (int32_t *)calloc((size_t)4 * C + 1, sizeof(int32_t));
    cl->notIns = 0;
    for (int i = 0; i < n; i++) {
        int c = cell_of(g, eps, p[i].x, p[i].y);
        if (c < 0) { cl->notIns++; bin[i] = -1; continue; }
        bin[i] = 4 * c + quad_of(g, eps, p[i].x, p[i].y);
        bstart[bin[i] + 1]++;
    }
    for (int b = 0; b < 4 * C; b++) bstart[b + 1] += bstart[b];
    cl->maxOcc = 0;
    for (int c = 0; c < C; c++) {
        cl->start[c] = bstart[4 * c];
        int occ = bstart[4 * c + 4] - bstart[4 * c];
        if (occ > cl->maxOcc) cl->maxOcc = occ;
    }
    cl->start[C] = bstart[4 * C];
    int32_t *cur = (int32_t *)malloc(sizeof(int32_t) * (size_t)4 * C + 4);
    memcpy(cur, bstart, sizeof(int32_t) * (size_t)4 * C);
    for (int i = 0; i < n; i++)
        if (bin[i] >= 0) cl->idx[cur[bin[i]]++] = i;
    free(cur);
    free(bstart);
    free(bin);
    cl->overCap = 0;
    cl->F = NULL;
    for (int c = 0; c < C; c++)
        if (cl->start[c + 1] - cl->start[c] > REF_MAX_PER_CELL) cl->overCap++;
    if (ref_cap_mode) {                 /* assignCells into the memset grid buffer */
        cl->F = (int32_t *)calloc((size_t)REF_CELL_INTS * (C > 0 ? C : 1), sizeof(int32_t));
        for (int c = 0; c < C; c++) {
            int cnt = cl->start[c + 1] - cl->start[c];
            cl->F[(size_t)REF_CELL_INTS * c] = cnt;
            for (int k = 0; k < cnt && k < REF_MAX_PER_CELL; k++)
                cl->F[(size_t)REF_CELL_INTS * c + 1 + k] = cl->idx[cl->start[c] + k];
        }
    }
}
static void free_cells(cells_t *cl) { free(cl->start); free(cl->idx); free(cl->F); }

/* computeDensity (fluid_kernels.metal:246-307) for particle i. */
static void density_one(lpeo_particle *p, int n, int i, const lpeo_grid *g,
                        const cells_t *cl, const lpe_fluid_config *cfg,
                        float *rho_out, float *p_out) {
    const lpeo_particle self = p[i];
    float xi = self.x, yi = self.y;
    float hi = (self.h <= 0.f) ? cfg->gridConfig.smoothingLength : self.h;
    float h2 = hi * hi;
    float poly6 = poly6Coeff2D(hi);
    float acc = 0.0f;
    float px = xi + cfg->gridConfig.gridEpsilon, py = yi + cfg->gridConfig.gridEpsilon;
    int gx = (int)floorf(px / g->cellSize), gy = (int)floorf(py / g->cellSize);
    int cellX = gx - g->gridMinX, cellY = gy - g->gridMinY;
    for (int ny = -1; ny <= 1; ny++) {
        for (int nx = -1; nx <= 1; nx++) {
            int cx = cellX + nx, cy = cellY + ny;
            if (cx < 0 || cx >= g->gridDimX || cy < 0 || cy >= g->gridDimY) continue;
            int c = cy * g->gridDimX + cx;
            int kb = cl->start[c], ke = cl->start[c + 1];
            if (cl->F) { kb = 0; ke = cl->F[(size_t)REF_CELL_INTS * c]; }     /* count */
            for (int k = kb; k < ke; k++) {
                int j = cl->F ? ref_index(cl, c, k) : cl->idx[k];
                if (j >= n) continue;
                float dx = xi - p[j].x, dy = yi - p[j].y;
                float r2 = dx * dx + dy * dy;
                if (r2 < h2) {
                    float diff = h2 - r2;
                    float w = poly6 * diff * diff * diff;
                    acc += p[j].mass * w;
                }
            }
        }
    }
    float pres = cfg->stiffness * (acc - cfg->restDensity);
    if (pres < 0.f) pres = 0.f;
    *rho_out = acc;
    *p_out = pres;
}

/* computeForces (fluid_kernels.metal:312-403) for particle i. */
static void forces_one(const lpeo_particle *p, int n, int i, const lpeo_grid *g,
                       const cells_t *cl, const lpe_fluid_config *cfg,
                       float *ax_out, float *ay_out) {
    const lpeo_particle self = p[i];
    float xi = self.x, yi = self.y, pi = self.pressure, rhoi = self.density;
    float hi = (self.h <= 0.f) ? cfg->gridConfig.smoothingLength : self.h;
    float sumFx = 0.f, sumFy = 0.f;
    float px = xi + cfg->gridConfig.gridEpsilon, py = yi + cfg->gridConfig.gridEpsilon;
    int gx = (int)floorf(px / g->cellSize), gy = (int)floorf(py / g->cellSize);
    int cellX = gx - g->gridMinX, cellY = gy - g->gridMinY;
    for (int ny = -1; ny <= 1; ny++) {
        for (int nx = -1; nx <= 1; nx++) {
            int cx = cellX + nx, cy = cellY + ny;
            if (cx < 0 || cx >= g->gridDimX || cy < 0 || cy >= g->gridDimY) continue;
            int c = cy * g->gridDimX + cx;
            int kb = cl->start[c], ke = cl->start[c + 1];
            if (cl->F) { kb = 0; ke = cl->F[(size_t)REF_CELL_INTS * c]; }
            for (int k = kb; k < ke; k++) {
                int j = cl->F ? ref_index(cl, c, k) : cl->idx[k];
                if (j == i || j >= n) continue;
                const lpeo_particle nb = p[j];
                float dx = xi - nb.x, dy = yi - nb.y;
                float r2 = dx * dx + dy * dy;
                if (r2 < cfg->numericalConfig.minDistanceThreshold) continue;
                float hj = (nb.h <= 0.f) ? cfg->gridConfig.smoothingLength : nb.h;
                float h_ij = 0.5f * (hi + hj);
                float h_ij2 = h_ij * h_ij;
                if (r2 >= h_ij2) continue;
                float r = sqrtf(r2);
                float pj = nb.pressure, rhoj = nb.density;
                if (rhoj < cfg->numericalConfig.minDensityThreshold ||
                    rhoi < cfg->numericalConfig.minDensityThreshold) continue;
                float term = (pi / (rhoi * rhoi)) + (pj / (rhoj * rhoj));
                float spF = spikyCoeff2D(h_ij);
                float diff = (h_ij - r);
                float wSpiky = spF * (diff * diff);
                float rx = dx / r, ry = dy / r;
                float fxPress = -nb.mass * term * wSpiky;
                float fx = fxPress * rx;
                float fy = fxPress * ry;
                float vx_ij = self.vx - nb.vx, vy_ij = self.vy - nb.vy;
                float lapC = viscLaplacianCoeff2D(h_ij);
                float wVisc = lapC * diff;
                float fVisc = cfg->viscosity * nb.mass * (wVisc / rhoj);
                fx -= fVisc * vx_ij;
                fy -= fVisc * vy_ij;
                sumFx += fx;
                sumFy += fy;
            }
        }
    }
    *ax_out = sumFx;
    *ay_out = sumFy;
}

/* rigidFluidImpulseSolver (fluid_kernels.metal:679-924) for particle i;
 * the rigid accumulators are exact sums (xacc, 3 x XACC_LIMBS per rigid). */
static void impulse_one(lpeo_particle *fpp, const lpe_gpu_rigid *rigids, int rigidCount,
                        const lpe_fluid_config *cfg, float dt, uint64_t *acq) {
    const float GRAVITY = cfg->gravity;
    const float WATER_DENSITY = cfg->restDensity;
    const float MAX_FORCE = cfg->impulseSolver.maxForce;
    const float MAX_TORQUE = cfg->impulseSolver.maxTorque;
    const float VISCOSITY_SCALE = cfg->impulseSolver.viscosityScale;
    const float DEPTH_SCALE = cfg->impulseSolver.depthScale;
    const float DEPTH_TRANSITION_RATE = cfg->impulseSolver.depthTransitionRate;
    const float PRESSURE_FORCE_LIMIT_RATIO = cfg->impulseSolver.pressureForceRatio;
    const float VISCOUS_FORCE_LIMIT_RATIO = cfg->impulseSolver.viscousForceRatio;
    const float ANGULAR_DAMPING_THRESHOLD = cfg->impulseSolver.angularDampingThreshold;
    const float ANGULAR_DAMPING_FACTOR = cfg->impulseSolver.angularDampingFactor;
    const float DEPTH_ESTIMATE_SCALE = cfg->impulseSolver.depthEstimateScale;
    const float MAX_SAFE_VELOCITY_SQ = cfg->impulseSolver.maxSafeVelocitySq;
    const float MIN_PENETRATION = cfg->impulseSolver.minPenetration;
    const float MIN_REL_VELOCITY = cfg->impulseSolver.minRelVelocity;
    const float FLUID_FORCE_SCALE = cfg->impulseSolver.fluidForceScale;
    const float FLUID_FORCE_MAX = cfg->impulseSolver.fluidForceMax;
    const float BUOYANCY_STRENGTH = cfg->impulseSolver.buoyancyStrength;

    lpeo_particle fp = *fpp;
    float densityF = fp.density > 0.0f ? fp.density : WATER_DENSITY;
    float pressureF = fp.pressure;
    float tffx = 0.0f, tffy = 0.0f;
    int hadInteraction = 0;
    for (int r = 0; r < rigidCount; r++) {
        const lpe_gpu_rigid *rb = &rigids[r];
        float rbVelSq = rb->vx * rb->vx + rb->vy * rb->vy + rb->omega * rb->omega;
        if (rbVelSq > MAX_SAFE_VELOCITY_SQ) continue;
        if (fp.x < rb->minX || fp.x > rb->maxX || fp.y < rb->minY || fp.y > rb->maxY) continue;
        int inside = 0;
        float pen = 0.0f, relx = 0.f, rely = 0.f, nx = 0.f, ny = 0.f;
        if (rb->shapeType == 0) {
            float rx = fp.x - rb->posX, ry = fp.y - rb->posY;
            float dist2 = rx * rx + ry * ry;
            float radiusSq = rb->radius * rb->radius;
            if (dist2 < radiusSq) {
                inside = 1;
                float dist = sqrtf(dist2);
                if (dist < MIN_PENETRATION) dist = MIN_PENETRATION;
                pen = rb->radius - dist;
                if (pen < 0.0f) pen = 0.0f;
                relx = rx; rely = ry;
                nx = relx / dist; ny = rely / dist;
            }
        } else if (rb->shapeType == 1 && rb->vertCount >= 3) {
            inside = pointInPolygon(fp.x, fp.y, rb);
            if (inside) {
                float cx, cy;
                closestPointOnPolygon(fp.x, fp.y, rb, &cx, &cy);
                float dx = fp.x - cx, dy = fp.y - cy;
                float d2 = dx * dx + dy * dy;
                float d = sqrtf(d2);
                if (d < MIN_PENETRATION) d = MIN_PENETRATION;
                pen = d;
                if (pen < 0.0f) pen = 0.0f;
                relx = fp.x - rb->posX; rely = fp.y - rb->posY;
                nx = dx / d; ny = dy / d;
            }
        }
        if (!inside || pen < MIN_PENETRATION) continue;
        hadInteraction = 1;
        float rotx = -rb->omega * rely, roty = rb->omega * relx;
        float rvx = rb->vx + rotx, rvy = rb->vy + roty;
        float relVx = fp.vx - rvx, relVy = fp.vy - rvy;
        float depthFactor = lpe_tanhf(DEPTH_TRANSITION_RATE * pen / DEPTH_SCALE);
        float normalVel = relVx * nx + relVy * ny;
        float nvx = nx * normalVel, nvy = ny * normalVel;
        float tvx = relVx - nvx, tvy = relVy - nvy;
        float particleVolume = fp.mass / densityF;
        float effectiveArea = lpe_powf(particleVolume, 2.0f / 3.0f);
        float depth = fminf(fp.y / DEPTH_ESTIMATE_SCALE, 1.0f);
        float hydro = densityF * GRAVITY * depth;
        float totalPressure = pressureF + hydro;
        float pressureForce = totalPressure * effectiveArea * depthFactor;
        float pfm = fminf(pressureForce, MAX_FORCE * PRESSURE_FORCE_LIMIT_RATIO);
        float pfx = nx * pfm, pfy = ny * pfm;
        float tangentVelMag = f2len(tvx, tvy);
        if (tangentVelMag > MIN_REL_VELOCITY) {
            float tdx = tvx / tangentVelMag, tdy = tvy / tangentVelMag;
            float viscosityCoef = cfg->viscosity * VISCOSITY_SCALE;
            float viscousForce = viscosityCoef * tangentVelMag * densityF * depthFactor * dt;
            float vfm = fminf(viscousForce, MAX_FORCE * VISCOUS_FORCE_LIMIT_RATIO);
            pfx += -tdx * vfm;
            pfy += -tdy * vfm;
        }
        if (rb->mass > 0.1f) {
            float bx = 0.0f * BUOYANCY_STRENGTH * pen * effectiveArea * GRAVITY * densityF;
            float by = -1.0f * BUOYANCY_STRENGTH * pen * effectiveArea * GRAVITY * densityF;
            float cbx = pfx + bx, cby = pfy + by;
            if (f2len(cbx, cby) <= MAX_FORCE) { pfx = cbx; pfy = cby; }
        }
        float tfx = pfx, tfy = pfy;
        float forceMag = f2len(tfx, tfy);
        if (forceMag > MAX_FORCE) {
            float s = MAX_FORCE / forceMag;
            tfx = tfx * s; tfy = tfy * s;
        }
        float torque = relx * tfy - rely * tfx;
        torque = fminf(fmaxf(torque, -MAX_TORQUE), MAX_TORQUE);
        if (fabsf(rb->omega) > ANGULAR_DAMPING_THRESHOLD) {
            float sgn = (rb->omega > 0.f) ? 1.f : ((rb->omega < 0.f) ? -1.f : 0.f);
            torque -= ANGULAR_DAMPING_FACTOR * sgn * fabsf(rb->omega) * rb->inertia;
        }
        xacc_add(acq + (size_t)r * 3 * XACC_LIMBS, tfx);
        xacc_add(acq + (size_t)r * 3 * XACC_LIMBS + XACC_LIMBS, tfy);
        xacc_add(acq + (size_t)r * 3 * XACC_LIMBS + 2 * XACC_LIMBS, torque);
        tffx -= tfx * FLUID_FORCE_SCALE;
        tffy -= tfy * FLUID_FORCE_SCALE;
    }
    if (hadInteraction) {
        float fm = f2len(tffx, tffy);
        if (fm > FLUID_FORCE_MAX) {
            float s = FLUID_FORCE_MAX / fm;
            tffx = tffx * s; tffy = tffy * s;
        }
        float invMass = (fp.mass > 0.0001f) ? 1.0f / fp.mass : 1.0f;
        fp.ax += tffx * invMass;
        fp.ay += tffy * invMass;
        *fpp = fp;
    }
}

/* rigidFluidPositionSolver (fluid_kernels.metal:533-668) for particle i. */
static void position_one(lpeo_particle *pp, const lpe_gpu_rigid *rigids, int rigidCount,
                         const lpe_fluid_config *cfg) {
    const float SAFETY_MARGIN = cfg->positionSolver.safetyMargin;
    const float RELAX_FACTOR = cfg->positionSolver.relaxFactor;
    const float MIN_SAFE_DISTANCE = cfg->positionSolver.minSafeDistance;
    const float MIN_POSITION_CHANGE = cfg->positionSolver.minPositionChange;
    lpeo_particle p = *pp;
    float oldx = p.x, oldy = p.y;
    float acx = 0.0f, acy = 0.0f;
    float px = p.x, py = p.y;
    int hadCollision = 0;
    for (int r = 0; r < rigidCount; r++) {
        const lpe_gpu_rigid *b = &rigids[r];
        if (px < b->minX || px > b->maxX || py < b->minY || py > b->maxY) continue;
        if (b->shapeType == 0) {
            float dx = px - b->posX, dy = py - b->posY;
            float dist2 = dx * dx + dy * dy;
            float radius = b->radius;
            if (dist2 < radius * radius) {
                hadCollision = 1;
                float dist = sqrtf(dist2);
                if (dist < MIN_SAFE_DISTANCE) { dist = MIN_SAFE_DISTANCE; dx = 1.0f; dy = 0.0f; }
                float pen = (radius - dist) + SAFETY_MARGIN;
                float dirx = dx / dist, diry = dy / dist;
                acx -= dirx * pen * RELAX_FACTOR;
                acy -= diry * pen * RELAX_FACTOR;
            }
        } else if (b->shapeType == 1) {
            if (b->vertCount < 3) continue;
            if (pointInPolygon(px, py, b)) {
                hadCollision = 1;
                float cx, cy;
                closestPointOnPolygon(px, py, b, &cx, &cy);
                float cdx = px - cx, cdy = py - cy;
                float d2 = cdx * cdx + cdy * cdy;
                float d = sqrtf(d2);
                if (d < MIN_SAFE_DISTANCE) { d = MIN_SAFE_DISTANCE; cdx = 1.0f; cdy = 0.0f; }
                float pen = d + SAFETY_MARGIN;
                float dirx = cdx / d, diry = cdy / d;
                acx += dirx * pen * RELAX_FACTOR;
                acy += diry * pen * RELAX_FACTOR;
            }
        }
    }
    const float MAX_CORRECTION = cfg->positionSolver.maxCorrection;
    float cm = f2len(acx, acy);
    if (cm > MAX_CORRECTION) {
        acx = (acx / cm) * MAX_CORRECTION;
        acy = (acy / cm) * MAX_CORRECTION;
    }
    p.x -= acx;
    p.y -= acy;
    if (p.x < 0.f) p.x = cfg->gridConfig.boundaryOffset;
    if (p.y < 0.f) p.y = cfg->gridConfig.boundaryOffset;
    if (hadCollision) {
        float pdx = p.x - oldx, pdy = p.y - oldy;
        float pdm = f2len(pdx, pdy);
        if (pdm > MIN_POSITION_CHANGE) {
            float cdx = pdx / pdm, cdy = pdy / pdm;
            float cvx = p.vx, cvy = p.vy;
            float va = cvx * cdx + cvy * cdy;
            if (va < 0.0f) {
                float restitution = 0.0f;
                cvx -= (1.0f + restitution) * va * cdx;
                cvy -= (1.0f + restitution) * va * cdy;
                p.vx = cvx; p.vy = cvy;
                p.vxHalf = p.vx; p.vyHalf = p.vy;
            }
        }
    }
    *pp = p;
}

void lpeo_density(lpeo_particle *p, int n, const lpe_fluid_config *cfg, lpeo_grid *g_out,
                  lpeo_sub_stats *st) {
    lpeo_grid g;
    lpeo_grid_from_bbox(p, n, cfg->gridConfig.smoothingLength, &g);
    cells_t cl;
    build_cells(p, n, &g, cfg->gridConfig.gridEpsilon, &cl);
    float *rho = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    float *pr = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    #pragma omp parallel for schedule(dynamic, 1024)
    for (int i = 0; i < n; i++) density_one(p, n, i, &g, &cl, cfg, &rho[i], &pr[i]);
    for (int i = 0; i < n; i++) { p[i].density = rho[i]; p[i].pressure = pr[i]; }
    if (st) { st->maxOcc = cl.maxOcc; st->notInserted = cl.notIns; st->overCap = cl.overCap; }
    if (g_out) *g_out = g;
    free(rho); free(pr);
    free_cells(&cl);
}

int lpeo_fluid_tick(const lpe_fluid_config *cfg, double dt_tick,
                    lpeo_particle *p, int n, lpe_gpu_rigid *rigids, int nr,
                    float *accum_out, lpeo_tick_stats *st) {
    if (n <= 0) return 0;  /* FluidSystem::update returns early (fluid.cpp:969-972) */
    float dt = (float)dt_tick;                                  /* fluid.cpp:592 */
    float subDt = dt / (float)cfg->numSubSteps;                 /* fluid.cpp:593 */
    float halfDt = 0.5f * subDt;
    if (st) memset(st, 0, sizeof(*st));
    for (int r = 0; r < nr; r++) { rigids[r].accumFx = rigids[r].accumFy = rigids[r].accumTorque = 0.f; }
    /* gather re-establishes a = 0, vh = v, h = smoothingLength (fluid.cpp:287-292) */
    for (int i = 0; i < n; i++) {
        p[i].vxHalf = p[i].vx; p[i].vyHalf = p[i].vy;
        p[i].ax = 0.f; p[i].ay = 0.f;
        p[i].h = cfg->gridConfig.smoothingLength;
    }
    float *ax = (float *)malloc(sizeof(float) * (size_t)n);
    float *ay = (float *)malloc(sizeof(float) * (size_t)n);
    float *rho = (float *)malloc(sizeof(float) * (size_t)n);
    float *pr = (float *)malloc(sizeof(float) * (size_t)n);
    uint64_t *acq = (uint64_t *)calloc((size_t)(nr > 0 ? nr : 1) * 3 * XACC_LIMBS, sizeof(uint64_t));
    xacc_range_error = 0;
    ref_undefined = 0;
    for (int step = 0; step < cfg->numSubSteps; step++) {
        /* velocityVerletHalf (fluid_kernels.metal:408-423) */
        for (int i = 0; i < n; i++) {
            p[i].vxHalf = p[i].vx + halfDt * p[i].ax;
            p[i].vyHalf = p[i].vy + halfDt * p[i].ay;
            p[i].x += p[i].vxHalf * subDt;
            p[i].y += p[i].vyHalf * subDt;
        }
        lpeo_grid g;
        lpeo_grid_from_bbox(p, n, cfg->gridConfig.smoothingLength, &g);
        cells_t cl;
        build_cells(p, n, &g, cfg->gridConfig.gridEpsilon, &cl);
        if (st) {
            if (cl.maxOcc > st->maxOcc) st->maxOcc = cl.maxOcc;
            st->notInserted = cl.notIns;
            st->overCap += cl.overCap;
            st->grid = g;
        }
        #pragma omp parallel for schedule(dynamic, 1024)
        for (int i = 0; i < n; i++) density_one(p, n, i, &g, &cl, cfg, &rho[i], &pr[i]);
        for (int i = 0; i < n; i++) { p[i].density = rho[i]; p[i].pressure = pr[i]; }
        #pragma omp parallel for schedule(dynamic, 1024)
        for (int i = 0; i < n; i++) forces_one(p, n, i, &g, &cl, cfg, &ax[i], &ay[i]);
        for (int i = 0; i < n; i++) { p[i].ax = ax[i]; p[i].ay = ay[i]; }
        /* velocityVerletFinish (fluid_kernels.metal:428-441) */
        for (int i = 0; i < n; i++) {
            p[i].vx = p[i].vxHalf + halfDt * p[i].ax;
            p[i].vy = p[i].vyHalf + halfDt * p[i].ay;
        }
        if (nr > 0)
            #pragma omp parallel for schedule(dynamic, 1024)
            for (int i = 0; i < n; i++) impulse_one(&p[i], rigids, nr, cfg, subDt, acq);
        #pragma omp parallel for schedule(dynamic, 1024)
        for (int i = 0; i < n; i++) position_one(&p[i], rigids, nr, cfg);
        free_cells(&cl);
    }
    /* writeBackRigidBodies arithmetic (fluid.cpp:545-562) */
    for (int r = 0; r < nr; r++) {
        lpe_gpu_rigid *rb = &rigids[r];
        rb->accumFx = xacc_round(acq + (size_t)r * 3 * XACC_LIMBS);
        rb->accumFy = xacc_round(acq + (size_t)r * 3 * XACC_LIMBS + XACC_LIMBS);
        rb->accumTorque = xacc_round(acq + (size_t)r * 3 * XACC_LIMBS + 2 * XACC_LIMBS);
        if (accum_out) {
            accum_out[3 * r + 0] = rb->accumFx;
            accum_out[3 * r + 1] = rb->accumFy;
            accum_out[3 * r + 2] = rb->accumTorque;
        }
        float invMass = (rb->mass > 1e-12f) ? (1.f / rb->mass) : 0.f;
        float invInertia = (rb->inertia > 1e-12f) ? (1.f / rb->inertia) : 0.f;
        rb->vx += rb->accumFx * invMass;
        rb->vy += rb->accumFy * invMass;
        rb->vx *= cfg->dampingFactor;
        rb->vy *= cfg->dampingFactor;
        rb->omega += rb->accumTorque * invInertia;
        rb->omega *= cfg->dampingFactor;
        rb->accumFx = rb->accumFy = rb->accumTorque = 0.f;
    }
    free(ax); free(ay); free(rho); free(pr); free(acq);
    return xacc_range_error ? 2 : 0;
}

void lpeo_fluid_config_default(lpe_fluid_config *c) {
    memset(c, 0, sizeof(*c));
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
    c->numericalConfig.minDistanceThreshold = 1e-14f; c->numericalConfig.minDensityThreshold = 1e-12f;
    c->numericalConfig.minTimestep = 1e-10f; c->numericalConfig.fallbackTimestep = 1e-4f;
    c->dampingFactor = 1.0f; c->numSubSteps = 10; c->threadsPerGroup = 256;
}
