// lpe_backend.hpp — the process-wide device context behind the drop-in
// systems (Systems::FluidSystem, RigidBodyCollisionSystem, BoundarySystem,
// BasicGravitySystem, RotationSystem, MovementSystem, SleepSystem) and the
// ECS <-> C-ABI gathers they share.
//
// Ownership follows SURVEY.md §8(b): the code object and the HIP context are
// process-lifetime (a reference-style reset() that re-creates the systems,
// src/sim.cpp:105, does not reload them); host arrays are only borrowed for
// the duration of a C-ABI call.  Error convention of the reference
// (fluid.cpp:97-100, :961-964): a failure is logged once to std::cerr and the
// backend disables itself, turning every update() into a no-op; lastStatus()
// keeps the lpe_status for callers that want to fail loudly.
#pragma once

#include <entt/entt.hpp>
#include <vector>

#include "lpe.h"
#include "systems/shared_system_config.hpp"

namespace lpe {
namespace host {

enum class Mode {
    Strict = 0,    // every system gathers and scatters the ECS each tick
    Resident = 1   // the device owns the state; ECS synced every syncEvery ticks
};

// Context on device LPE_DEVICE (env, default 0); nullptr once disabled.
lpe_ctx *context();
// false (and the backend disabled, message logged once) if st != LPE_OK
bool check(int st, const char *what);
int lastStatus();
void reset();            // drops the disabled flag and the resident world
void setMode(Mode m, int syncEvery = 1);
Mode mode();

// Wall time of the fluid system's phases (strict mode), accumulated since the
// last reset(): the ECS gather, the uploads, the device step, the downloads,
// the ECS write-back -- what the drop-in costs beyond the device's own work.
struct PhaseTimes {
    double gather = 0, upload = 0, device = 0, download = 0, scatter = 0;
    long calls = 0;
};
PhaseTimes &fluidTimes();

// ---- ECS gathers shared by the rigid and integrator systems ---------------
// Every entity with a Position (optionally skipping Liquid), in storage order,
// as lpe_body rows (components flattened into flags) plus the local polygon
// vertices.  eid is the raw entity value, which orders pairs like the
// reference's `f > e` test (broadphase.cpp:264).
struct BodySet {
    std::vector<entt::entity> ents;
    std::vector<lpe_body> bodies;
    std::vector<double> verts;
};
void gatherBodies(entt::registry &reg, BodySet &out, bool skipLiquid);
// Writes Position, Velocity, AngularPosition, AngularVelocity and Sleep back.
void scatterBodies(entt::registry &reg, const BodySet &set, const lpe_body *bodies);

// lpe_rigid_config with the reference defaults and the shared config's
// universe size and pixel scale.
lpe_rigid_config rigidConfig(const SharedSystemConfig &sh);

// ---- resident mode ---------------------------------------------------------
// Integrator configs recorded by the systems each tick (resident mode runs
// the whole tick in the last system of the order, SleepSystem).
struct ResidentConfigs {
    lpe_rigid_config rigid;
    lpe_fluid_config fluid;
    bool haveFluid = false;
    lpe_bh_config bh;            // BarnesHutSystem's (recorded by its update())
    bool haveBh = false;
};
ResidentConfigs &residentConfigs();
// Runs one device tick (lpe_world_tick) for the registry; uploads the world
// when it is not resident yet and syncs the ECS every syncEvery ticks.
void residentTick(entt::registry &reg, const SharedSystemConfig &sh);
// Download the device state into the ECS now.
void residentSync(entt::registry &reg);
void residentInvalidate();

}  // namespace host
}  // namespace lpe
