/**
 * integrators.cpp — MI355X drop-ins for the tick-parity and integrator
 * systems of the reference: BoundarySystem (src/systems/boundary.cpp),
 * BasicGravitySystem (gravity.cpp), RotationSystem (rotation.cpp),
 * MovementSystem (movement.cpp) and SleepSystem (sleep.cpp).  Class names,
 * headers and configs are the reference's (include/systems/{boundary,gravity,...}.hpp); update()
 * runs the same per-entity arithmetic on the device (lpe_rigid_integrate,
 * fp64 like the reference).
 *
 * Strict mode gathers every Position entity (fluid included: Boundary and
 * Gravity act on the fluid too, boundary.cpp:23, gravity.cpp:36), integrates
 * and scatters.  Resident mode records each system's configuration and the
 * last system of the order (SleepSystem, sim.cpp:114) advances the whole
 * device tick (lpe_world_tick) once every system has run.
 */
#include "systems/boundary.hpp"
#include "systems/gravity.hpp"
#include "systems/movement.hpp"
#include "systems/rotation.hpp"
#include "systems/sleep.hpp"

#include "entities/entity_components.hpp"
#include "entities/sim_components.hpp"
#include "lpe_backend.hpp"

namespace Systems {

namespace {

enum Bits { BOUNDARY = 1, GRAVITY = 2, ROTATION = 4, MOVEMENT = 8, SLEEP = 16 };

// dt of Gravity and Rotation: SecondsPerTick * baseTimeAcceleration *
// timeScale from the SimulatorState entity (gravity.cpp:23-33, rotation.cpp:21-27)
double stateDt(entt::registry &reg, const SharedSystemConfig &sh) {
    auto v = reg.view<Components::SimulatorState>();
    if (v.empty()) return sh.SecondsPerTick;
    const auto &st = reg.get<Components::SimulatorState>(v.front());
    return sh.SecondsPerTick * st.baseTimeAcceleration * st.timeScale;
}

void integrate(entt::registry &reg, const lpe_rigid_config &cfg, int bits, double dtState,
               double dtMove) {
    lpe_ctx *ctx = lpe::host::context();
    if (!ctx) return;
    lpe::host::BodySet set;
    lpe::host::gatherBodies(reg, set, /*skipLiquid=*/false);
    if (set.bodies.empty()) return;
    if (!lpe::host::check(lpe_rigid_set_config(ctx, &cfg), "lpe_rigid_set_config")) return;
    if (!lpe::host::check(lpe_rigid_upload(ctx, (int)set.bodies.size(), set.bodies.data(),
                                           (int)(set.verts.size() / 2),
                                           set.verts.empty() ? nullptr : set.verts.data()),
                          "lpe_rigid_upload"))
        return;
    if (!lpe::host::check(lpe_rigid_integrate(ctx, bits, dtState, dtMove), "lpe_rigid_integrate")) return;
    std::vector<lpe_body> out(set.bodies.size());
    if (!lpe::host::check(lpe_rigid_download(ctx, out.data()), "lpe_rigid_download")) return;
    lpe::host::scatterBodies(reg, set, out.data());
}

bool resident() { return lpe::host::mode() == lpe::host::Mode::Resident; }

}  // namespace

// ---- BoundarySystem (boundary.cpp:13-70) ----------------------------------
BoundarySystem::BoundarySystem() = default;

void BoundarySystem::update(entt::registry &registry) {
    lpe_rigid_config &rc = lpe::host::residentConfigs().rigid;
    lpe_rigid_config c = resident() ? rc : lpe::host::rigidConfig(sysConfig);
    c.marginPixels = specificConfig.marginPixels;
    c.bounceDamping = specificConfig.bounceDamping;
    c.maxSpeed = specificConfig.maxSpeed;
    if (resident()) { rc = c; return; }
    integrate(registry, c, BOUNDARY, 0.0, 0.0);
}

// ---- BasicGravitySystem (gravity.cpp:19-58) --------------------------------
BasicGravitySystem::BasicGravitySystem() = default;

void BasicGravitySystem::update(entt::registry &registry) {
    lpe_rigid_config &rc = lpe::host::residentConfigs().rigid;
    lpe_rigid_config c = resident() ? rc : lpe::host::rigidConfig(sysConfig);
    c.gravity = specificConfig.gravitationalAcceleration;
    c.planetaryMassThreshold = specificConfig.planetaryMassThreshold;
    if (resident()) { rc = c; return; }
    integrate(registry, c, GRAVITY, stateDt(registry, sysConfig), 0.0);
}

// ---- RotationSystem (rotation.cpp:18-60) -----------------------------------
RotationSystem::RotationSystem() = default;

void RotationSystem::update(entt::registry &registry) {
    lpe_rigid_config &rc = lpe::host::residentConfigs().rigid;
    lpe_rigid_config c = resident() ? rc : lpe::host::rigidConfig(sysConfig);
    c.angularDamping = specificConfig.angularDamping;
    c.maxAngularSpeed = specificConfig.maxAngularSpeed;
    if (resident()) { rc = c; return; }
    integrate(registry, c, ROTATION, stateDt(registry, sysConfig), 0.0);
}

// ---- MovementSystem (movement.cpp:13-39) -----------------------------------
MovementSystem::MovementSystem() = default;

void MovementSystem::update(entt::registry &registry) {
    if (resident()) return;
    // dt = SecondsPerTick * TimeAcceleration (movement.cpp:17)
    integrate(registry, lpe::host::rigidConfig(sysConfig), MOVEMENT, 0.0,
              sysConfig.SecondsPerTick * sysConfig.TimeAcceleration);
}

// ---- SleepSystem (sleep.cpp:19-67) -------------------------------------------
SleepSystem::SleepSystem() = default;

void SleepSystem::update(entt::registry &registry) {
    lpe_rigid_config &rc = lpe::host::residentConfigs().rigid;
    lpe_rigid_config c = resident() ? rc : lpe::host::rigidConfig(sysConfig);
    c.linearSleepThreshold = specificConfig.linearSleepThreshold;
    c.angularSleepThreshold = specificConfig.angularSleepThreshold;
    c.sleepFramesThreshold = specificConfig.sleepFramesThreshold;
    if (resident()) {
        rc = c;
        lpe::host::residentTick(registry, sysConfig);   // the whole device tick
        return;
    }
    integrate(registry, c, SLEEP, 0.0, 0.0);
}

}  // namespace Systems
