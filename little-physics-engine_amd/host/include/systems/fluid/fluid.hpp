/**
 * fluid.hpp — MI355X drop-in for include/systems/fluid/fluid.hpp of the
 * reference (little-physics-engine, snapshot 2025-05-23).
 *
 * Same namespace, class name, base class and FluidConfig fields/defaults as
 * the reference header (fluid.hpp:131-200), so src/sim.cpp (which constructs
 * Systems::FluidSystem by type, sim.cpp:107, and dynamic_casts to it,
 * sim.cpp:69-71 / :140-142) and every scenario (which fills FluidConfig
 * through i_scenario.hpp:35) compile unchanged.  The Metal members
 * (fluid.hpp:18, :328-355) are gone: the device work goes through the C ABI
 * of include/lpe.h, owned by the process-wide backend (lpe_backend.hpp).
 */
#pragma once

#include <entt/entt.hpp>
#include <vector>
#include <cstddef>
#include <limits>

#include "systems/i_system.hpp"

namespace Systems
{

/** Reference GPUFluidParticle (fluid.hpp:36-51), kept for source
 *  compatibility; the HIP backend stores particles as fp32 SoA. */
struct GPUFluidParticle
{
    float x, y, vx, vy, vxHalf, vyHalf, ax, ay, mass, h, c, density, pressure;
};

/** GPU_MAX_PER_CELL (fluid.hpp:56): the reference's per-cell capacity.  The
 *  HIP grid hash is a counting sort without a cap; occupancy is reported. */
static constexpr int GPU_MAX_PER_CELL = 64;

enum class GPURigidShapeType : int { Circle = 0, Polygon = 1 };

/** GPURigidBody (fluid.hpp:93-125), byte-identical to lpe_gpu_rigid. */
static constexpr int GPU_POLYGON_MAX_VERTS = 16;
struct GPURigidBody
{
    GPURigidShapeType shapeType;
    float posX, posY, angle, radius;
    int vertCount;
    float vertsX[GPU_POLYGON_MAX_VERTS];
    float vertsY[GPU_POLYGON_MAX_VERTS];
    float vx, vy, omega, mass, inertia;
    float minX, maxX, minY, maxY;
    float accumFx, accumFy, accumTorque;
};

/** FluidConfig: field-for-field and default-for-default the reference's
 *  (fluid.hpp:131-200). */
struct FluidConfig
{
    float gravity = 9.81f;
    float restDensity = 0.5f;
    float stiffness = 200.0f;
    float viscosity = 0.03f;

    struct {
        float safetyMargin = 0.001f;
        float relaxFactor = 0.9f;
        float maxCorrection = 0.1f;
        float maxVelocityUpdate = 1.0f;
        float minSafeDistance = 1e-10f;
        float velocityDamping = 0.3f;
        float minPositionChange = 1e-6f;
    } positionSolver;

    struct {
        float maxForce = 0.15f;
        float maxTorque = 0.03f;
        float fluidForceScale = 100.0f;
        float fluidForceMax = 50000.0f;
        float buoyancyStrength = 0.2f;
        float viscosityScale = 0.05f;
        float depthScale = 0.04f;
        float depthTransitionRate = 2.0f;
        float depthEstimateScale = 10.0f;
        float pressureForceRatio = 1.0f;
        float viscousForceRatio = 0.3f;
        float angularDampingThreshold = 0.5f;
        float angularDampingFactor = 0.005f;
        float maxSafeVelocitySq = 80.0f;
        float minPenetration = 1e-6f;
        float minRelVelocity = 1e-6f;
    } impulseSolver;

    struct {
        float gridEpsilon = 1e-6f;
        float smoothingLength = 0.05f;
        float boundaryOffset = 0.001f;
    } gridConfig;

    struct {
        float minDistanceThreshold = 1e-14f;
        float minDensityThreshold = 1e-12f;
        float minTimestep = 1e-10f;
        float fallbackTimestep = 1e-4f;
    } numericalConfig;

    float dampingFactor = 1.0f;
    int numSubSteps = 10;
    int threadsPerGroup = 256;
};

/**
 * FluidSystem: SPH fluid + rigid–fluid coupling on the MI355X.
 *
 * Strict mode (default) keeps the reference's contract of update()
 * (fluid.cpp:958-1021): gather the Liquid entities and the shaped non-Liquid
 * entities in EnTT view order, advance numSubSteps velocity-Verlet sub-steps
 * on the device, apply the fluid->rigid impulse once, and write x, v,
 * density, pressure and the rigid velocities back before returning.
 * Resident mode (lpe::host::setMode) hands the whole tick to the device.
 */
class FluidSystem : public ConfigurableSystem<FluidConfig>
{
public:
    FluidSystem();
    ~FluidSystem() override;
    void update(entt::registry &registry) override;

    /** Largest reference-cell occupancy of the last update (the reference
     *  drops inserts past GPU_MAX_PER_CELL); for the parity harness. */
    int lastMaxCellOccupancy() const { return lastMaxOcc_; }

private:
    std::vector<GPUFluidParticle> gatherFluidParticles(
        entt::registry &registry, std::vector<entt::entity> &entityList) const;
    std::vector<GPURigidBody> gatherRigidBodies(
        entt::registry &registry, std::vector<entt::entity> &rigidEntityList) const;

    int lastMaxOcc_ = 0;
};

} // namespace Systems
