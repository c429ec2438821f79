/**
 * rigid_body_collision.cpp — MI355X drop-in for
 * src/systems/rigid/rigid_body_collision.cpp of the reference.
 *
 * The reference runs, on one CPU core, broadphase (quadtree) -> narrowphase
 * (GJK/EPA/clip) -> ContactManager -> PGS -> position solver
 * (rigid_body_collision.cpp:24-50).  Here the same stages run on the device
 * behind lpe_rigid_step (csrc/lpe_rigid.hip); update() gathers the non-Liquid
 * entities, steps, and writes poses and velocities back.
 */
#include "systems/rigid/rigid_body_collision.hpp"

#include "entities/entity_components.hpp"
#include "lpe_backend.hpp"

namespace Systems {

RigidBodyCollisionSystem::RigidBodyCollisionSystem() = default;

static void applyConfig(lpe_rigid_config &c, const RigidBodyCollisionConfig &s)
{
    c.pgsIterations = s.pgsIterations;
    c.frictionCoeff = s.frictionCoeff;
    c.posIterations = s.positionIterations;
    c.baumgarte = s.baumgarte;
    c.slop = s.slop;
}

void RigidBodyCollisionSystem::update(entt::registry &registry)
{
    if (lpe::host::mode() == lpe::host::Mode::Resident)
    {
        applyConfig(lpe::host::residentConfigs().rigid, getSpecificConfig());
        return;
    }
    lpe_ctx *ctx = lpe::host::context();
    if (!ctx) return;
    lpe::host::BodySet set;
    lpe::host::gatherBodies(registry, set, /*skipLiquid=*/true);
    if (set.bodies.empty()) return;
    lpe_rigid_config c = lpe::host::rigidConfig(getSharedSystemConfig());
    applyConfig(c, getSpecificConfig());
    if (!lpe::host::check(lpe_rigid_set_config(ctx, &c), "lpe_rigid_set_config")) return;
    if (!lpe::host::check(lpe_rigid_upload(ctx, (int)set.bodies.size(), set.bodies.data(),
                                           (int)(set.verts.size() / 2),
                                           set.verts.empty() ? nullptr : set.verts.data()),
                          "lpe_rigid_upload"))
        return;
    lpe_rigid_stats st;
    if (!lpe::host::check(lpe_rigid_step(ctx, &st), "lpe_rigid_step")) return;
    lastPairs_ = st.pairs;
    lastContacts_ = st.contacts;
    if (st.contacts == 0) return;   // rigid_body_collision.cpp:35-37
    std::vector<lpe_body> out(set.bodies.size());
    if (!lpe::host::check(lpe_rigid_download(ctx, out.data()), "lpe_rigid_download")) return;
    lpe::host::scatterBodies(registry, set, out.data());
}

} // namespace Systems
