/* rigid_oracle.h — TEST INFRASTRUCTURE ONLY (see rigid_oracle.cpp header). */
#ifndef LPE_RIGID_ORACLE_H
#define LPE_RIGID_ORACLE_H
#include <stdint.h>
#include "../include/lpe.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lpeo_rigid_stats {
    int32_t pairs, contacts, manifolds, dynamicBodies;
} lpeo_rigid_stats;

void lpeo_rigid_config_default(lpe_rigid_config *c);

/* Broadphase::detectCollisions pair SET (broadphase.cpp:233-295), in the
 * canonical order (eid_a, eid_b) ascending, eid_a < eid_b.  pairs receives
 * body-index pairs.  Returns the pair count, or -(count) if cap is too small. */
int lpeo_broadphase(const lpe_rigid_config *cfg, int nb, const lpe_body *bodies,
                    const double *verts, int32_t *pairs, int cap);

/* narrowPhase (narrowphase.cpp:352-420) over the given pairs, in pair order.
 * Returns the contact count, or -(count) if cap is too small. */
int lpeo_narrowphase(int nb, const lpe_body *bodies, const double *verts, int np,
                     const int32_t *pairs, lpe_contact *out, int cap);

/* ContactSolver::solveContactConstraints (contact_solver.cpp:449-543): rows
 * are visited in `order` (contact indices; NULL = identity).  Updates vx, vy,
 * omega of dynamic bodies. */
int lpeo_pgs(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, int nc,
             const lpe_contact *contacts, const int32_t *order);

/* PositionSolver::positionalSolver (position_solver.cpp:299-325): contacts
 * visited in `order` (NULL = identity).  Updates x, y, angle. */
int lpeo_position_solver(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, int nc,
                         const lpe_contact *contacts, const int32_t *order);

/* Round-2 canonical order (k_pair_colour, kept for comparison): colour-major over the
 * edge-coloured contact pairs, pairs ascending inside a colour, contacts of a
 * pair in narrowphase order.  order receives nc contact indices; pair_colour
 * (optional, npairs entries) the colour of each pair (-1: no contact).
 * Returns the number of colours (-1: more than 64 needed). */
int lpeo_colour_order(int nb, const lpe_body *bodies, int nc, const lpe_contact *cs,
                      int32_t *order, int32_t *pair_colour, int npairs);

/* Canonical solver order since round 3: striped Gauss-Seidel (see
 * rigid_oracle.cpp): x-stripes of the movable bodies, per stripe an interior
 * and a boundary group, each coloured greedily; phase A (even stripes) then
 * phase B (odd stripes).  pair_step (optional) receives each pair's step,
 * nstripes (optional) the stripe count.  Returns the steps (-1: > 64 colours
 * in a group). */
int lpeo_stripe_order(int nb, const lpe_body *bodies, int nc, const lpe_contact *cs,
                      int32_t *order, int32_t *pair_step, int npairs, int32_t *nstripes);

/* RigidBodyCollisionSystem::update (rigid_body_collision.cpp:24-50) with the
 * canonical orders: pairs by (eid_a, eid_b); PGS and position solver in the
 * striped order of lpeo_stripe_order. */
int lpeo_rigid_update(const lpe_rigid_config *cfg, int nb, lpe_body *bodies,
                      const double *verts, lpeo_rigid_stats *stats);

/* Integrator / tick-parity systems (one pass each). */
void lpeo_boundary(const lpe_rigid_config *cfg, int nb, lpe_body *bodies);
void lpeo_gravity(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, double dt);
void lpeo_rotation(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, double dt);
void lpeo_movement(int nb, lpe_body *bodies, double dt);
void lpeo_sleep(const lpe_rigid_config *cfg, int nb, lpe_body *bodies);

/* ECSSimulator::tick for a scene without fluid (FluidSystem returns early,
 * fluid.cpp:969-972; Barnes-Hut returns early for masses < 1e3,
 * barnes_hut.cpp:54-70): Boundary, Gravity, RigidBodyCollision, Rotation,
 * Movement, Sleep.  dt_state = SecondsPerTick * baseTimeAcceleration *
 * timeScale (gravity, rotation); dt_move = SecondsPerTick * TimeAcceleration. */
int lpeo_rigid_tick(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, const double *verts,
                    double dt_state, double dt_move, lpeo_rigid_stats *stats);

/* One full tick with fluid: FluidSystem (gather of the `couple` bodies ->
 * SPH -> velocity write-back), Boundary, Gravity (bodies and fluid),
 * RigidBodyCollision, Rotation, Movement, Sleep.  parts: fluid in gather
 * order (sph_oracle.h).  The canonical orders of both oracles apply. */
struct lpeo_particle;
int lpeo_world_tick(const lpe_fluid_config *fcfg, const lpe_rigid_config *rcfg,
                    double spt, double time_accel, double bta, double ts,
                    struct lpeo_particle *parts, int n, lpe_body *bodies, int nb,
                    const double *verts, int nr, const int32_t *couple);

#ifdef __cplusplus
}
#endif
#endif
