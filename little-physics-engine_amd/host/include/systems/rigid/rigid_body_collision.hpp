/**
 * rigid_body_collision.hpp — MI355X drop-in for
 * include/systems/rigid/rigid_body_collision.hpp of the reference.
 *
 * Same class and config names (rigid_body_collision.hpp:23-59), so
 * src/sim.cpp:110 / :72-74 / :143-145 compile unchanged.  The reference
 * hard-wires its stage configs as default-constructed locals
 * (rigid_body_collision.cpp:30, :44, :48); the two iteration counts are
 * exposed here with the reference defaults.
 */
#pragma once

#include <entt/entt.hpp>
#include "systems/i_system.hpp"

namespace Systems {

struct RigidBodyCollisionConfig {
    double empty = 0.0;
    int pgsIterations = 10;        // ContactSolverConfig::iterations (contact_solver.hpp:21-27)
    float frictionCoeff = 0.5f;    // ContactSolverConfig::friction
    int positionIterations = 10;   // PositionSolverConfig::iterations (position_solver.hpp:21-34)
    double baumgarte = 0.02;       // PositionSolverConfig::baumgarte
    double slop = 0.001;           // PositionSolverConfig::slop
};

/**
 * Broadphase -> GJK/EPA/clip narrowphase -> PGS -> Baumgarte position solve,
 * on the device (lpe_rigid_step), behind the reference's update() surface.
 */
class RigidBodyCollisionSystem : public ConfigurableSystem<RigidBodyCollisionConfig> {
public:
    RigidBodyCollisionSystem();
    ~RigidBodyCollisionSystem() override = default;
    void update(entt::registry &registry) override;

    /** Pairs and contacts of the last update (parity harness). */
    int lastPairs() const { return lastPairs_; }
    int lastContacts() const { return lastContacts_; }

private:
    int lastPairs_ = 0;
    int lastContacts_ = 0;
};

} // namespace Systems
