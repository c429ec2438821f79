/**
 * fluid.cpp — MI355X drop-in for src/systems/fluid/fluid.cpp of the
 * reference.  The 9 Metal kernels and their 20 blocking command buffers per
 * tick (fluid.cpp:603-948) become one lpe_sph_step on the device
 * (little-physics-engine_amd/csrc/lpe_sph.hip); the gathers and write-backs
 * keep the reference's ECS contract.
 */
#include <chrono>
#include "systems/fluid/fluid.hpp"

#include <cstddef>
#include <cstring>
#include <limits>
#include <type_traits>

#include "entities/entity_components.hpp"
#include "lpe_backend.hpp"
#include "math/polygon.hpp"
#include "../csrc/lpe_trig.h"

namespace Systems
{

static_assert(sizeof(GPURigidBody) == sizeof(lpe_gpu_rigid), "GPURigidBody mirrors lpe_gpu_rigid");
static_assert(offsetof(GPURigidBody, accumTorque) == offsetof(lpe_gpu_rigid, accumTorque),
              "GPURigidBody mirrors lpe_gpu_rigid");
static_assert(sizeof(FluidConfig) == sizeof(lpe_fluid_config), "FluidConfig mirrors lpe_fluid_config");
static_assert(offsetof(FluidConfig, numSubSteps) == offsetof(lpe_fluid_config, numSubSteps),
              "FluidConfig mirrors lpe_fluid_config");
static_assert(offsetof(FluidConfig, gridConfig) == offsetof(lpe_fluid_config, gridConfig),
              "FluidConfig mirrors lpe_fluid_config");

static lpe_fluid_config toC(const FluidConfig &c)
{
    static_assert(std::is_trivially_copyable<FluidConfig>::value, "POD config");
    lpe_fluid_config out;
    std::memcpy(&out, &c, sizeof(out));
    return out;
}

FluidSystem::FluidSystem() = default;

// Systems are re-created on every reset() (sim.cpp:105): the device code
// object and context stay (process lifetime); only a resident world is
// dropped, because the registry it mirrors is about to be cleared.
FluidSystem::~FluidSystem()
{
    lpe::host::residentInvalidate();
}

// gatherFluidParticles (fluid.cpp:250-302): Liquid entities in view order;
// vh = v and a = 0 at every gather; h = smoothingLength.
std::vector<GPUFluidParticle> FluidSystem::gatherFluidParticles(
    entt::registry &registry, std::vector<entt::entity> &entityList) const
{
    std::vector<GPUFluidParticle> out;
    auto view = registry.view<Components::Position, Components::Velocity, Components::Mass,
                              Components::ParticlePhase, Components::SpeedOfSound,
                              Components::SPHTemp>();
    for (auto e : view)
    {
        if (view.get<Components::ParticlePhase>(e).phase != Components::Phase::Liquid)
        {
            continue;
        }
        const auto &pos = view.get<Components::Position>(e);
        const auto &vel = view.get<Components::Velocity>(e);
        const auto &spht = view.get<Components::SPHTemp>(e);
        GPUFluidParticle p{};
        p.x = (float)pos.x;
        p.y = (float)pos.y;
        p.vx = (float)vel.x;
        p.vy = (float)vel.y;
        p.vxHalf = p.vx;
        p.vyHalf = p.vy;
        p.mass = (float)view.get<Components::Mass>(e).value;
        p.h = getSpecificConfig().gridConfig.smoothingLength;
        p.c = (float)view.get<Components::SpeedOfSound>(e).value;
        p.density = (float)spht.density;
        p.pressure = (float)spht.pressure;
        out.push_back(p);
        entityList.push_back(e);
    }
    return out;
}

// gatherRigidBodies (fluid.cpp:304-438): every shaped non-Liquid entity in
// view order.  Polygon world vertices in double from float(angle), then
// float; at most GPU_POLYGON_MAX_VERTS; AABB of those vertices.
std::vector<GPURigidBody> FluidSystem::gatherRigidBodies(
    entt::registry &registry, std::vector<entt::entity> &rigidEntityList) const
{
    std::vector<GPURigidBody> out;
    auto view = registry.view<Components::Position, Components::Shape>();
    for (auto e : view)
    {
        if (const auto *ph = registry.try_get<Components::ParticlePhase>(e))
        {
            if (ph->phase == Components::Phase::Liquid)
            {
                continue;
            }
        }
        const auto &pos = view.get<Components::Position>(e);
        const auto &shape = view.get<Components::Shape>(e);
        GPURigidBody rb{};
        rb.posX = (float)pos.x;
        rb.posY = (float)pos.y;
        rb.angle = 0.0f;
        if (const auto *ap = registry.try_get<Components::AngularPosition>(e)) rb.angle = (float)ap->angle;
        if (const auto *v = registry.try_get<Components::Velocity>(e)) { rb.vx = (float)v->x; rb.vy = (float)v->y; }
        if (const auto *w = registry.try_get<Components::AngularVelocity>(e)) rb.omega = (float)w->omega;
        rb.mass = 1.f;
        rb.inertia = 1.f;
        if (const auto *m = registry.try_get<Components::Mass>(e)) rb.mass = (float)m->value;
        if (const auto *in = registry.try_get<Components::Inertia>(e)) rb.inertia = (float)in->I;
        rb.minX = rb.posX - 0.5f;
        rb.maxX = rb.posX + 0.5f;
        rb.minY = rb.posY - 0.5f;
        rb.maxY = rb.posY + 0.5f;
        if (shape.type == Components::ShapeType::Circle)
        {
            rb.shapeType = GPURigidShapeType::Circle;
            rb.radius = (float)shape.size;
            rb.vertCount = 0;
            rb.minX = rb.posX - rb.radius;
            rb.maxX = rb.posX + rb.radius;
            rb.minY = rb.posY - rb.radius;
            rb.maxY = rb.posY + rb.radius;
        }
        else if (shape.type == Components::ShapeType::Polygon)
        {
            rb.shapeType = GPURigidShapeType::Polygon;
            rb.radius = 0.f;
            const auto *poly = registry.try_get<PolygonShape>(e);
            if (!poly)
            {
                continue;
            }
            int cnt = (int)poly->vertices.size();
            if (cnt > GPU_POLYGON_MAX_VERTS) cnt = GPU_POLYGON_MAX_VERTS;
            rb.vertCount = cnt;
            // std::cos(float) as the reference (rb.angle is a float), evaluated by
            // the implementation the device and the oracle share (csrc/lpe_trig.h)
            double c = lpe_cosf(rb.angle), s = lpe_sinf(rb.angle);
            float mnx = std::numeric_limits<float>::max(), mxx = -std::numeric_limits<float>::max();
            float mny = std::numeric_limits<float>::max(), mxy = -std::numeric_limits<float>::max();
            for (int i = 0; i < cnt; i++)
            {
                double lx = poly->vertices[i].x, ly = poly->vertices[i].y;
                double wx = pos.x + (lx * c - ly * s);
                double wy = pos.y + (lx * s + ly * c);
                rb.vertsX[i] = (float)wx;
                rb.vertsY[i] = (float)wy;
                if (wx < mnx) mnx = (float)wx;
                if (wx > mxx) mxx = (float)wx;
                if (wy < mny) mny = (float)wy;
                if (wy > mxy) mxy = (float)wy;
            }
            rb.minX = mnx;
            rb.maxX = mxx;
            rb.minY = mny;
            rb.maxY = mxy;
        }
        else
        {
            continue;   // Square: skipped (fluid.cpp:427-431)
        }
        out.push_back(rb);
        rigidEntityList.push_back(e);
    }
    return out;
}

void FluidSystem::update(entt::registry &registry)
{
    if (lpe::host::mode() == lpe::host::Mode::Resident)
    {
        // the whole tick runs on the device in the last system of the
        // order (SleepSystem); record this system's configuration
        lpe::host::residentConfigs().fluid = toC(getSpecificConfig());
        lpe::host::residentConfigs().haveFluid = true;
        return;
    }
    lpe_ctx *ctx = lpe::host::context();
    if (!ctx)
    {
        return;   // fluid.cpp:961-964
    }
    using clock = std::chrono::steady_clock;
    lpe::host::PhaseTimes &pt = lpe::host::fluidTimes();
    auto since = [](clock::time_point t0) { return std::chrono::duration<double>(clock::now() - t0).count(); };
    clock::time_point t0 = clock::now();
    std::vector<entt::entity> fluidEntities;
    std::vector<GPUFluidParticle> parts = gatherFluidParticles(registry, fluidEntities);
    if (parts.empty())
    {
        return;   // fluid.cpp:969-972
    }
    std::vector<entt::entity> rigidEntities;
    std::vector<GPURigidBody> rigids = gatherRigidBodies(registry, rigidEntities);

    const int n = (int)parts.size();
    std::vector<float> x(n), y(n), vx(n), vy(n), m(n), rho(n), p(n);
    for (int i = 0; i < n; i++)
    {
        x[i] = parts[i].x; y[i] = parts[i].y;
        vx[i] = parts[i].vx; vy[i] = parts[i].vy;
        m[i] = parts[i].mass;
        rho[i] = parts[i].density; p[i] = parts[i].pressure;
    }
    pt.gather += since(t0);
    t0 = clock::now();
    const lpe_fluid_config cfg = toC(getSpecificConfig());
    if (!lpe::host::check(lpe_sph_set_config(ctx, &cfg), "lpe_sph_set_config")) return;
    if (!lpe::host::check(lpe_sph_upload(ctx, n, x.data(), y.data(), vx.data(), vy.data(), m.data(),
                                         rho.data(), p.data()), "lpe_sph_upload"))
        return;
    const int r = (int)rigids.size();
    if (!lpe::host::check(lpe_sph_upload_rigids(ctx, r, r ? (const lpe_gpu_rigid *)rigids.data() : nullptr),
                          "lpe_sph_upload_rigids"))
        return;
    // dt = float(SecondsPerTick * TimeAcceleration) (fluid.cpp:592)
    const double dt = getSharedSystemConfig().SecondsPerTick * getSharedSystemConfig().TimeAcceleration;
    pt.upload += since(t0);
    t0 = clock::now();
    if (!lpe::host::check(lpe_sph_step(ctx, dt), "lpe_sph_step")) return;
    if (!lpe::host::check(lpe_sync(ctx), "lpe_sync")) return;
    pt.device += since(t0);
    t0 = clock::now();
    if (!lpe::host::check(lpe_sph_download(ctx, x.data(), y.data(), vx.data(), vy.data(), rho.data(),
                                           p.data()), "lpe_sph_download"))
        return;
    pt.download += since(t0);
    t0 = clock::now();
    // writeBackToECS (fluid.cpp:496-524)
    for (int i = 0; i < n; i++)
    {
        entt::entity e = fluidEntities[(size_t)i];
        auto &pos = registry.get<Components::Position>(e);
        auto &vel = registry.get<Components::Velocity>(e);
        auto &spht = registry.get<Components::SPHTemp>(e);
        pos.x = x[i]; pos.y = y[i];
        vel.x = vx[i]; vel.y = vy[i];
        spht.density = rho[i];
        spht.pressure = p[i];
    }
    // writeBackRigidBodies (fluid.cpp:526-580): the device applied
    // v += F/m, w += tau/I and the damping; push v and w into the ECS
    if (r > 0)
    {
        if (!lpe::host::check(lpe_sph_download_rigids(ctx, (lpe_gpu_rigid *)rigids.data(), nullptr),
                              "lpe_sph_download_rigids"))
            return;
        for (int i = 0; i < r; i++)
        {
            entt::entity e = rigidEntities[(size_t)i];
            if (auto *v = registry.try_get<Components::Velocity>(e)) { v->x = rigids[i].vx; v->y = rigids[i].vy; }
            if (auto *w = registry.try_get<Components::AngularVelocity>(e)) w->omega = rigids[i].omega;
        }
    }
    lpe_sph_stats st;
    if (lpe_sph_get_stats(ctx, &st) == LPE_OK) lastMaxOcc_ = st.maxCellOccupancy;
    pt.scatter += since(t0);
    pt.calls++;
}

} // namespace Systems
