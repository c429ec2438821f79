/*
 * ref_driver.cpp — TEST INFRASTRUCTURE ONLY.  Drives the REFERENCE's own
 * rigid-path and integrator sources (compiled from /root/reference by
 * oracle/Makefile.ref into oracle/_ref/) on scenes built from plain arrays,
 * to record golden fixtures.  This file is ours; it only includes the
 * reference headers and calls the reference functions.
 *
 * What runs here is reference code, except the PGS: contact_solver.cpp needs
 * <arm_neon.h> (absent on x86-64) and is unbuildable, so the driver calls the
 * restated lpeo_pgs (oracle/rigid_oracle.cpp) on the manifolds produced by the
 * reference's ContactManager, in their iteration order.  ECSSimulator::tick
 * (src/sim.cpp:156-163) is replaced by the same system order minus
 * FluidSystem (Metal; rigid-only scenes make it return early, fluid.cpp:
 * 969-972) and BarnesHutSystem (returns early for masses < 1e3,
 * barnes_hut.cpp:54-70).
 */
#include <entt/entt.hpp>

#include <cmath>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "entities/entity_components.hpp"
#include "entities/sim_components.hpp"
#include "math/polygon.hpp"
#include "systems/barnes_hut.hpp"
#include "systems/boundary.hpp"
#include "systems/gravity.hpp"
#include "systems/movement.hpp"
#include "systems/rotation.hpp"
#include "systems/shared_system_config.hpp"
#include "systems/sleep.hpp"
#include "systems/rigid/broadphase.hpp"
#include "systems/rigid/collision_data.hpp"
#include "systems/rigid/contact_manager.hpp"
#include "systems/rigid/narrowphase.hpp"
#include "systems/rigid/position_solver.hpp"

#include "rigid_oracle.h"

namespace {

struct Scene {
    entt::registry reg;
    std::vector<entt::entity> ents;
};

void build(Scene &s, int nb, const lpe_body *b, const double *verts, double bta, double ts) {
    auto st = s.reg.create();                    /* reset(): SimulatorState first (sim.cpp:95-96) */
    s.reg.emplace<Components::SimulatorState>(st, bta, ts);
    for (int i = 0; i < nb; i++) {
        const lpe_body &x = b[i];
        auto e = s.reg.create();
        s.ents.push_back(e);
        s.reg.emplace<Components::Position>(e, x.x, x.y);
        if (x.flags & LPE_BODY_HAS_VEL) s.reg.emplace<Components::Velocity>(e, x.vx, x.vy);
        if (x.flags & LPE_BODY_HAS_MASS) s.reg.emplace<Components::Mass>(e, x.mass);
        if (x.flags & LPE_BODY_BOUNDARY) s.reg.emplace<Components::Boundary>(e);
        if (x.flags & LPE_BODY_HAS_PHASE)
            s.reg.emplace<Components::ParticlePhase>(
                e, (x.flags & LPE_BODY_LIQUID) ? Components::Phase::Liquid : Components::Phase::Solid);
        if (x.flags & LPE_BODY_HAS_SLEEP) {
            auto &sl = s.reg.emplace<Components::Sleep>(e);
            sl.asleep = (x.flags & LPE_BODY_ASLEEP) != 0;
            sl.sleepCounter = x.sleep_counter;
        }
        if (x.flags & LPE_BODY_CIRCLE) s.reg.emplace<CircleShape>(e, CircleShape{x.radius});
        if (x.flags & LPE_BODY_POLYGON) {
            PolygonShape poly;
            poly.type = Components::ShapeType::Polygon;
            for (int k = 0; k < x.vert_cnt; k++)
                poly.vertices.emplace_back(verts[2 * (x.vert_off + k)], verts[2 * (x.vert_off + k) + 1]);
            s.reg.emplace<PolygonShape>(e, poly);
        }
        if (x.flags & LPE_BODY_HAS_INERTIA) s.reg.emplace<Components::Inertia>(e, x.inertia);
        if (x.flags & LPE_BODY_HAS_ANGPOS) s.reg.emplace<Components::AngularPosition>(e, x.angle);
        if (x.flags & LPE_BODY_HAS_ANGVEL) s.reg.emplace<Components::AngularVelocity>(e, x.omega);
    }
}

void extract(Scene &s, int nb, const lpe_body *tmpl, lpe_body *out) {
    for (int i = 0; i < nb; i++) {
        lpe_body x = tmpl[i];
        auto e = s.ents[i];
        const auto &p = s.reg.get<Components::Position>(e);
        x.x = p.x; x.y = p.y;
        if (x.flags & LPE_BODY_HAS_VEL) {
            const auto &v = s.reg.get<Components::Velocity>(e);
            x.vx = v.x; x.vy = v.y;
        }
        if (x.flags & LPE_BODY_HAS_ANGPOS) x.angle = s.reg.get<Components::AngularPosition>(e).angle;
        if (x.flags & LPE_BODY_HAS_ANGVEL) x.omega = s.reg.get<Components::AngularVelocity>(e).omega;
        if (x.flags & LPE_BODY_HAS_SLEEP) {
            const auto &sl = s.reg.get<Components::Sleep>(e);
            x.sleep_counter = sl.sleepCounter;
            if (sl.asleep) x.flags |= LPE_BODY_ASLEEP; else x.flags &= ~LPE_BODY_ASLEEP;
        }
        out[i] = x;
    }
}

void write_velocities(Scene &s, int nb, const lpe_body *b) {
    for (int i = 0; i < nb; i++) {
        auto e = s.ents[i];
        if (b[i].flags & LPE_BODY_HAS_VEL) {
            auto &v = s.reg.get<Components::Velocity>(e);
            v.x = b[i].vx; v.y = b[i].vy;
        }
        if (b[i].flags & LPE_BODY_HAS_ANGVEL) s.reg.get<Components::AngularVelocity>(e).omega = b[i].omega;
    }
}

}  // namespace

extern "C" int lpref_rigid_ticks(const lpe_rigid_config *cfg, double spt, double time_accel,
                                 double bta, double ts, int nb, lpe_body *bodies,
                                 const double *verts, int nticks, lpe_body *before_rigid,
                                 lpe_body *after_pgs, lpe_body *after_pos, int32_t *pairs_out,
                                 int pair_cap, int32_t *np_out, lpe_contact *contacts_out,
                                 int contact_cap, int32_t *nc_out, int32_t *pgs_order) {
    Scene s;
    build(s, nb, bodies, verts, bta, ts);
    std::vector<lpe_body> tmpl(bodies, bodies + nb);
    SharedSystemConfig sh{};                     /* no default initialisers (shared_system_config.hpp:10-20) */
    sh.UniverseSizeMeters = cfg->universeSize;
    sh.TimeAcceleration = time_accel;
    sh.MetersPerPixel = cfg->metersPerPixel;
    sh.SecondsPerTick = spt;
    sh.GravitationalSoftener = 0.0;
    sh.DragCoeff = 0.0;
    sh.ParticleDensity = 0.0;
    sh.GridSize = 50;
    sh.CellSizePixels = 12.0;
    Systems::BoundarySystem boundary;
    Systems::BasicGravitySystem gravity;
    Systems::RotationSystem rotation;
    Systems::MovementSystem movement;
    Systems::SleepSystem sleep;
    Systems::BoundaryConfig bc; bc.marginPixels = cfg->marginPixels; bc.bounceDamping = cfg->bounceDamping;
    bc.maxSpeed = cfg->maxSpeed;
    Systems::GravityConfig gc; gc.gravitationalAcceleration = cfg->gravity;
    gc.planetaryMassThreshold = cfg->planetaryMassThreshold;
    Systems::RotationConfig rc; rc.angularDamping = cfg->angularDamping; rc.maxAngularSpeed = cfg->maxAngularSpeed;
    Systems::SleepConfig sc; sc.linearSleepThreshold = cfg->linearSleepThreshold;
    sc.angularSleepThreshold = cfg->angularSleepThreshold; sc.sleepFramesThreshold = cfg->sleepFramesThreshold;
    boundary.setSpecificConfig(bc); gravity.setSpecificConfig(gc);
    rotation.setSpecificConfig(rc); sleep.setSpecificConfig(sc);
    for (Systems::ISystem *sys : {(Systems::ISystem *)&boundary, (Systems::ISystem *)&gravity,
                                  (Systems::ISystem *)&rotation, (Systems::ISystem *)&movement,
                                  (Systems::ISystem *)&sleep})
        sys->setSharedSystemConfig(sh);

    std::vector<lpe_body> work(nb);
    for (int t = 0; t < nticks; t++) {
        const bool last = (t == nticks - 1);
        boundary.update(s.reg);                                  /* sim.cpp:107-114 order */
        gravity.update(s.reg);
        if (last && before_rigid) extract(s, nb, tmpl.data(), before_rigid);
        /* RigidBodyCollisionSystem::update (rigid_body_collision.cpp:24-50) */
        using namespace RigidBodyCollision;
        BroadphaseConfig bp;
        bp.quadtreeCapacity = cfg->quadtreeCapacity;
        bp.boundaryBuffer = cfg->boundaryBuffer;
        bp.smallParticleThreshold = cfg->smallParticleThreshold;
        auto cand = Broadphase::detectCollisions(s.reg, sh, bp);
        auto manifold = narrowPhase(s.reg, cand);
        /* entity -> body index (a table: the piles have ~10k pairs, 30k contacts) */
        std::vector<int> idx_of;
        for (int i = 0; i < nb; i++) {
            size_t k = (size_t)entt::to_entity(s.ents[i]);
            if (idx_of.size() <= k) idx_of.resize(k + 1, -1);
            idx_of[k] = i;
        }
        auto body_index = [&](entt::entity e) {
            size_t k = (size_t)entt::to_entity(e);
            return k < idx_of.size() ? idx_of[k] : -1;
        };
        std::vector<lpe_contact> cs;
        for (size_t k = 0; k < manifold.collisions.size(); k++) {
            const auto &c = manifold.collisions[k];
            lpe_contact x{};
            x.a = body_index(c.a); x.b = body_index(c.b); x.pair = -1;
            x.nx = c.normal.x; x.ny = c.normal.y; x.pen = c.penetration;
            x.px = c.contactPoint.x; x.py = c.contactPoint.y;
            cs.push_back(x);
        }
        std::vector<int32_t> order;
        if (!manifold.collisions.empty()) {
            ContactManager mgr;
            mgr.updateContacts(manifold);
            auto &mans = mgr.getManifoldsForSolver();
            /* manifold iteration order -> contact indices (contacts keep
             * narrowphase order inside a manifold, contact_manager.cpp:206-240) */
            std::vector<char> used(cs.size(), 0);
            std::unordered_map<long long, std::vector<size_t>> by_pair;   /* (a, b) -> contacts, narrowphase order */
            for (size_t k = 0; k < cs.size(); k++) by_pair[(long long)cs[k].a * nb + cs[k].b].push_back(k);
            static const std::vector<size_t> none;
            for (const auto &m : mans) {
                int a = body_index(m.a), b = body_index(m.b);
                auto it = by_pair.find((long long)a * nb + b);
                for (size_t k : (it == by_pair.end() ? none : it->second)) {
                    if (used[k]) continue;
                    if (std::fabs(cs[k].nx - m.normal.x) >= 1e-7 || std::fabs(cs[k].ny - m.normal.y) >= 1e-7) continue;
                    used[k] = 1;
                    order.push_back((int32_t)k);
                }
            }
            extract(s, nb, tmpl.data(), work.data());
            lpeo_pgs(cfg, nb, work.data(), (int)cs.size(), cs.data(), order.data());
            write_velocities(s, nb, work.data());
            if (last && after_pgs) extract(s, nb, tmpl.data(), after_pgs);
            PositionSolverConfig pc;
            pc.iterations = cfg->posIterations;
            pc.baumgarte = cfg->baumgarte;
            pc.slop = cfg->slop;
            PositionSolver::positionalSolver(s.reg, manifold, pc);
        } else if (last && after_pgs) {
            extract(s, nb, tmpl.data(), after_pgs);
        }
        if (last && after_pos) extract(s, nb, tmpl.data(), after_pos);
        if (last) {
            *np_out = (int32_t)cand.size();
            for (size_t k = 0; k < cand.size() && (int)k < pair_cap; k++) {
                pairs_out[2 * k] = body_index(cand[k].eA);
                pairs_out[2 * k + 1] = body_index(cand[k].eB);
            }
            *nc_out = (int32_t)cs.size();
            for (size_t k = 0; k < cs.size() && (int)k < contact_cap; k++) {
                contacts_out[k] = cs[k];
                pgs_order[k] = k < order.size() ? order[k] : -1;
            }
        }
        rotation.update(s.reg);
        movement.update(s.reg);
        sleep.update(s.reg);
    }
    extract(s, nb, tmpl.data(), bodies);
    return 0;
}

/* BarnesHutSystem::update (src/systems/barnes_hut.cpp:50-99), the reference's
 * own code, on n bodies with Position + Mass (+ Velocity where has_vel[i]):
 * vx/vy updated in place (body index order); order_out[k] = the body index of
 * the k-th entity of view<Position, Mass>(exclude<Boundary>), buildTree's
 * insertion order (:117-128), which the oracle and the device take as their
 * input order.  Returns 0. */
extern "C" int lpref_barnes_hut(double theta, double small_mass, double universe, double softener,
                                double spt, double bta, double ts, int n, const double *x,
                                const double *y, double *vx, double *vy, const double *m,
                                const unsigned char *has_vel, int32_t *order_out) {
    entt::registry reg;
    auto st = reg.create();
    reg.emplace<Components::SimulatorState>(st, bta, ts);
    std::vector<entt::entity> ents(n);
    for (int i = 0; i < n; i++) {
        auto e = reg.create();
        ents[i] = e;
        reg.emplace<Components::Position>(e, x[i], y[i]);
        if (!has_vel || has_vel[i]) reg.emplace<Components::Velocity>(e, vx[i], vy[i]);
        reg.emplace<Components::Mass>(e, m[i]);
    }
    auto body_index = [&](entt::entity e) {
        for (int i = 0; i < n; i++) if (ents[i] == e) return i;
        return -1;
    };
    int k = 0;
    for (auto e : reg.view<Components::Position, Components::Mass>(entt::exclude<Components::Boundary>))
        order_out[k++] = body_index(e);
    SharedSystemConfig sh{};
    sh.UniverseSizeMeters = universe;
    sh.SecondsPerTick = spt;
    sh.GravitationalSoftener = softener;
    sh.TimeAcceleration = 1.0;
    sh.MetersPerPixel = 1.0;
    sh.DragCoeff = 0.0;
    sh.ParticleDensity = 0.0;
    sh.GridSize = 50;
    sh.CellSizePixels = 12.0;
    Systems::BarnesHutSystem bh;
    Systems::BarnesHutConfig bc;
    bc.theta = theta;
    bc.smallMassThreshold = small_mass;
    bh.setSpecificConfig(bc);
    bh.setSharedSystemConfig(sh);
    bh.update(reg);
    for (int i = 0; i < n; i++)
        if (!has_vel || has_vel[i]) {
            const auto &v = reg.get<Components::Velocity>(ents[i]);
            vx[i] = v.x;
            vy[i] = v.y;
        }
    return 0;
}
