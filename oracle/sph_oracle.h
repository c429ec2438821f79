/* sph_oracle.h — TEST INFRASTRUCTURE ONLY (see sph_oracle.c header). */
#ifndef LPE_SPH_ORACLE_H
#define LPE_SPH_ORACLE_H
#include <stdint.h>
#include "../include/lpe.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Mirror of Systems::GPUFluidParticle (fluid.hpp:36-51), 52 B. */
typedef struct lpeo_particle {
    float x, y, vx, vy, vxHalf, vyHalf, ax, ay, mass, h, c, density, pressure;
} lpeo_particle;

/* The reference's per-sub-step grid (fluid.cpp:737-752). */
typedef struct lpeo_grid {
    float cellSize;
    int gridMinX, gridMinY, gridDimX, gridDimY;
    float bbox[4]; /* minX, maxX, minY, maxY of the particles */
} lpeo_grid;

typedef struct lpeo_sub_stats { int maxOcc; int notInserted; int overCap; } lpeo_sub_stats;
/* overCap: cells over GPU_MAX_PER_CELL, summed over the sub-steps */
typedef struct lpeo_tick_stats { int maxOcc; int notInserted; lpeo_grid grid; int overCap; } lpeo_tick_stats;

void lpeo_fluid_config_default(lpe_fluid_config *c);
void lpeo_grid_from_bbox(const lpeo_particle *p, int n, float smoothingLength, lpeo_grid *g);
void lpeo_assign_cells(const lpeo_particle *p, int n, const lpeo_grid *g, float eps, int32_t *cell);
/* One hash + density pass over the current positions (no integration). */
void lpeo_density(lpeo_particle *p, int n, const lpe_fluid_config *cfg, lpeo_grid *g_out,
                  lpeo_sub_stats *st);
/* FluidSystem::update minus the ECS gather/scatter: numSubSteps sub-steps and
 * the rigid write-back arithmetic.  accum_out (3 floats per rigid, optional)
 * receives the accumulators before write-back. */
int lpeo_fluid_tick(const lpe_fluid_config *cfg, double dt_tick,
                    lpeo_particle *p, int n, lpe_gpu_rigid *rigids, int nr,
                    float *accum_out, lpeo_tick_stats *st);

/* Exact sum of n floats rounded once to nearest even (the coupling
 * accumulators' arithmetic); -1e30f if a value is outside the range. */
float lpeo_xacc_sum(const float *v, int n);
/* Reference cell-capacity semantics on (1) / off (0, default: unbounded cell
 * lists); see sph_oracle.c.  lpeo_ref_undefined() reports a read past the
 * last cell since the last tick started (undefined in the reference). */
void lpeo_set_ref_cell_cap(int on);
/* OpenMP threads of the particle loops (results are independent of it). */
void lpeo_set_threads(int n);
int lpeo_get_threads(void);
int lpeo_ref_undefined(void);

#ifdef __cplusplus
}
#endif
#endif
