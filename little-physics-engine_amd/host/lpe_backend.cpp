// lpe_backend.cpp — process-wide device context of the drop-in systems and
// the ECS <-> C-ABI gathers (see lpe_backend.hpp).
#include "lpe_backend.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <unordered_map>

#include "entities/entity_components.hpp"
#include "entities/sim_components.hpp"
#include "math/polygon.hpp"

namespace lpe {
namespace host {

namespace {

struct World {
    bool ready = false;
    long ticks = 0;
    size_t positions = 0;                  // Position storage size at upload
    BodySet bodies;                        // non-Liquid entities (rigid path)
    std::vector<entt::entity> fluid;       // Liquid entities in gather order
    bool bhSent = false;                   // Barnes-Hut config + order given to the device
    lpe_bh_config bhCfg{};
};

struct State {
    lpe_ctx *ctx = nullptr;
    bool disabled = false;
    int status = LPE_OK;
    Mode mode = Mode::Strict;
    int syncEvery = 1;
    ResidentConfigs cfgs;
    bool cfgsInit = false;
    World world;
};

State &state() {
    static State s;
    return s;
}

}  // namespace

lpe_ctx *context() {
    State &s = state();
    if (s.disabled) return nullptr;
    if (!s.ctx) {
        int dev = 0;
        if (const char *e = std::getenv("LPE_DEVICE")) dev = std::atoi(e);
        int st = lpe_create(dev, &s.ctx);
        if (st != LPE_OK) {
            // reference: no device => the fluid system silently disables
            // itself (fluid.cpp:97-100); here it is logged once
            std::cerr << "[lpe] no usable MI355X device (lpe_create status " << st
                      << "); device systems disabled\n";
            s.status = st;
            s.disabled = true;
            s.ctx = nullptr;
            return nullptr;
        }
    }
    return s.ctx;
}

bool check(int st, const char *what) {
    if (st == LPE_OK) return true;
    State &s = state();
    if (!s.disabled) {
        std::cerr << "[lpe] " << what << " failed (status " << st << "): "
                  << (s.ctx ? lpe_last_error(s.ctx) : "") << "; device systems disabled\n";
    }
    s.status = st;
    s.disabled = true;
    return false;
}

int lastStatus() { return state().status; }

PhaseTimes &fluidTimes() {
    static PhaseTimes t;
    return t;
}

void reset() {
    fluidTimes() = PhaseTimes();
    State &s = state();
    s.disabled = false;
    s.status = LPE_OK;
    s.world = World();
}

void setMode(Mode m, int syncEvery) {
    State &s = state();
    s.mode = m;
    s.syncEvery = syncEvery < 1 ? 1 : syncEvery;
    s.world = World();
}

Mode mode() { return state().mode; }

lpe_rigid_config rigidConfig(const SharedSystemConfig &sh) {
    lpe_rigid_config c;
    lpe_rigid_config_default(&c);
    c.universeSize = sh.UniverseSizeMeters;
    c.metersPerPixel = sh.MetersPerPixel;
    return c;
}

// ---------------------------------------------------------------------------
void gatherBodies(entt::registry &reg, BodySet &out, bool skipLiquid) {
    out.ents.clear();
    out.bodies.clear();
    out.verts.clear();
    auto view = reg.view<Components::Position>();
    out.ents.reserve(view.size());
    out.bodies.reserve(view.size());
    for (auto e : view) {
        const auto *ph = reg.try_get<Components::ParticlePhase>(e);
        if (skipLiquid && ph && ph->phase == Components::Phase::Liquid) continue;
        const auto &pos = view.get<Components::Position>(e);
        lpe_body b;
        std::memset(&b, 0, sizeof(b));
        b.eid = (uint32_t)entt::to_integral(e);
        b.x = pos.x;
        b.y = pos.y;
        uint32_t f = 0;
        if (ph) {
            f |= LPE_BODY_HAS_PHASE;
            if (ph->phase == Components::Phase::Solid) f |= LPE_BODY_SOLID;
            if (ph->phase == Components::Phase::Liquid) f |= LPE_BODY_LIQUID;
        }
        if (reg.any_of<Components::Boundary>(e)) f |= LPE_BODY_BOUNDARY;
        if (const auto *sl = reg.try_get<Components::Sleep>(e)) {
            f |= LPE_BODY_HAS_SLEEP;
            if (sl->asleep) f |= LPE_BODY_ASLEEP;
            b.sleep_counter = sl->sleepCounter;
        }
        if (const auto *ap = reg.try_get<Components::AngularPosition>(e)) {
            f |= LPE_BODY_HAS_ANGPOS;
            b.angle = ap->angle;
        }
        if (const auto *av = reg.try_get<Components::AngularVelocity>(e)) {
            f |= LPE_BODY_HAS_ANGVEL;
            b.omega = av->omega;
        }
        if (const auto *in = reg.try_get<Components::Inertia>(e)) {
            f |= LPE_BODY_HAS_INERTIA;
            b.inertia = in->I;
        }
        if (const auto *m = reg.try_get<Components::Mass>(e)) {
            f |= LPE_BODY_HAS_MASS;
            b.mass = m->value;
        }
        if (const auto *v = reg.try_get<Components::Velocity>(e)) {
            f |= LPE_BODY_HAS_VEL;
            b.vx = v->x;
            b.vy = v->y;
        }
        b.vert_off = (int32_t)(out.verts.size() / 2);
        if (const auto *c = reg.try_get<CircleShape>(e)) {
            f |= LPE_BODY_CIRCLE;
            b.radius = c->radius;
        } else if (const auto *p = reg.try_get<PolygonShape>(e)) {
            f |= LPE_BODY_POLYGON;
            b.vert_cnt = (int32_t)p->vertices.size();
            for (const auto &v : p->vertices) {
                out.verts.push_back(v.x);
                out.verts.push_back(v.y);
            }
        }
        b.flags = f;
        out.ents.push_back(e);
        out.bodies.push_back(b);
    }
}

void scatterBodies(entt::registry &reg, const BodySet &set, const lpe_body *bodies) {
    for (size_t i = 0; i < set.ents.size(); i++) {
        entt::entity e = set.ents[i];
        if (!reg.valid(e)) continue;
        const lpe_body &b = bodies[i];
        if (auto *p = reg.try_get<Components::Position>(e)) { p->x = b.x; p->y = b.y; }
        if (auto *v = reg.try_get<Components::Velocity>(e)) { v->x = b.vx; v->y = b.vy; }
        if (auto *a = reg.try_get<Components::AngularPosition>(e)) a->angle = b.angle;
        if (auto *w = reg.try_get<Components::AngularVelocity>(e)) w->omega = b.omega;
        if (auto *s = reg.try_get<Components::Sleep>(e)) {
            s->sleepCounter = b.sleep_counter;
            s->asleep = (b.flags & LPE_BODY_ASLEEP) != 0;
        }
    }
}

// ---------------------------------------------------------------------------
// resident mode
ResidentConfigs &residentConfigs() {
    State &s = state();
    if (!s.cfgsInit) {
        lpe_rigid_config_default(&s.cfgs.rigid);
        lpe_fluid_config_default(&s.cfgs.fluid);
        s.cfgsInit = true;
    }
    return s.cfgs;
}

void residentInvalidate() { state().world = World(); }

namespace {

// Liquid entities in FluidSystem::gatherFluidParticles view order
// (fluid.cpp:259-299)
void gatherFluidSoA(entt::registry &reg, std::vector<entt::entity> &ents, std::vector<float> &x,
                    std::vector<float> &y, std::vector<float> &vx, std::vector<float> &vy,
                    std::vector<float> &m, std::vector<float> &rho, std::vector<float> &p) {
    auto view = reg.view<Components::Position, Components::Velocity, Components::Mass,
                         Components::ParticlePhase, Components::SpeedOfSound, Components::SPHTemp>();
    for (auto e : view) {
        if (view.get<Components::ParticlePhase>(e).phase != Components::Phase::Liquid) continue;
        const auto &pos = view.get<Components::Position>(e);
        const auto &vel = view.get<Components::Velocity>(e);
        const auto &spht = view.get<Components::SPHTemp>(e);
        ents.push_back(e);
        x.push_back((float)pos.x);
        y.push_back((float)pos.y);
        vx.push_back((float)vel.x);
        vy.push_back((float)vel.y);
        m.push_back((float)view.get<Components::Mass>(e).value);
        rho.push_back((float)spht.density);
        p.push_back((float)spht.pressure);
    }
}

// Body indices of FluidSystem::gatherRigidBodies' rigids, in its view order
// (fluid.cpp:313-435): shaped non-Liquid entities; Square shapes and
// polygons without a PolygonShape are skipped.
std::vector<int32_t> couplingOrder(entt::registry &reg, const BodySet &set) {
    std::unordered_map<uint32_t, int32_t> index;
    for (size_t i = 0; i < set.ents.size(); i++) index[(uint32_t)entt::to_integral(set.ents[i])] = (int32_t)i;
    std::vector<int32_t> out;
    auto view = reg.view<Components::Position, Components::Shape>();
    for (auto e : view) {
        if (const auto *ph = reg.try_get<Components::ParticlePhase>(e))
            if (ph->phase == Components::Phase::Liquid) continue;
        const auto &shape = view.get<Components::Shape>(e);
        if (shape.type == Components::ShapeType::Polygon && !reg.all_of<PolygonShape>(e)) continue;
        if (shape.type != Components::ShapeType::Circle && shape.type != Components::ShapeType::Polygon)
            continue;
        auto it = index.find((uint32_t)entt::to_integral(e));
        if (it != index.end()) out.push_back(it->second);
    }
    return out;
}

bool residentUpload(entt::registry &reg, lpe_ctx *ctx) {
    State &s = state();
    World &w = s.world;
    w = World();
    gatherBodies(reg, w.bodies, /*skipLiquid=*/true);
    std::vector<float> x, y, vx, vy, m, rho, p;
    gatherFluidSoA(reg, w.fluid, x, y, vx, vy, m, rho, p);
    const double *vp = w.bodies.verts.empty() ? nullptr : w.bodies.verts.data();
    if (!check(lpe_rigid_upload(ctx, (int)w.bodies.bodies.size(), w.bodies.bodies.data(),
                                (int)(w.bodies.verts.size() / 2), vp), "lpe_rigid_upload"))
        return false;
    int n = (int)x.size();
    if (!check(lpe_sph_upload(ctx, n, n ? x.data() : nullptr, n ? y.data() : nullptr,
                              n ? vx.data() : nullptr, n ? vy.data() : nullptr,
                              n ? m.data() : nullptr, n ? rho.data() : nullptr,
                              n ? p.data() : nullptr), "lpe_sph_upload"))
        return false;
    std::vector<int32_t> couple = couplingOrder(reg, w.bodies);
    if (!check(lpe_world_set_coupling(ctx, (int)couple.size(), couple.empty() ? nullptr : couple.data()),
               "lpe_world_set_coupling"))
        return false;
    w.positions = reg.storage<Components::Position>().size();
    w.ready = true;
    return true;
}

}  // namespace

void residentSync(entt::registry &reg) {
    State &s = state();
    World &w = s.world;
    lpe_ctx *ctx = context();
    if (!ctx || !w.ready) return;
    size_t n = w.fluid.size();
    if (n) {
        std::vector<float> x(n), y(n), vx(n), vy(n), rho(n), p(n);
        if (!check(lpe_sph_download(ctx, x.data(), y.data(), vx.data(), vy.data(), rho.data(), p.data()),
                   "lpe_sph_download"))
            return;
        for (size_t i = 0; i < n; i++) {          // writeBackToECS (fluid.cpp:509-523)
            entt::entity e = w.fluid[i];
            if (!reg.valid(e)) continue;
            auto &pos = reg.get<Components::Position>(e);
            auto &vel = reg.get<Components::Velocity>(e);
            auto &spht = reg.get<Components::SPHTemp>(e);
            pos.x = x[i]; pos.y = y[i];
            vel.x = vx[i]; vel.y = vy[i];
            spht.density = rho[i];
            spht.pressure = p[i];
        }
    }
    if (!w.bodies.bodies.empty()) {
        std::vector<lpe_body> out(w.bodies.bodies.size());
        if (!check(lpe_rigid_download(ctx, out.data()), "lpe_rigid_download")) return;
        scatterBodies(reg, w.bodies, out.data());
    }
}

void residentTick(entt::registry &reg, const SharedSystemConfig &sh) {
    State &s = state();
    lpe_ctx *ctx = context();
    if (!ctx) return;
    ResidentConfigs &rc = residentConfigs();
    rc.rigid.universeSize = sh.UniverseSizeMeters;
    rc.rigid.metersPerPixel = sh.MetersPerPixel;
    World &w = s.world;
    if (w.ready && reg.storage<Components::Position>().size() != w.positions) {
        // entities were created or destroyed: hand the device state to the
        // ECS, then take the new world
        residentSync(reg);
        w.ready = false;
    }
    if (!check(lpe_sph_set_config(ctx, &rc.fluid), "lpe_sph_set_config")) return;
    if (!check(lpe_rigid_set_config(ctx, &rc.rigid), "lpe_rigid_set_config")) return;
    if (!w.ready && !residentUpload(reg, ctx)) return;
    lpe_world_config wc;
    wc.secondsPerTick = sh.SecondsPerTick;
    wc.timeAcceleration = sh.TimeAcceleration;
    wc.baseTimeAcceleration = 1.0;
    wc.timeScale = 1.0;
    auto sv = reg.view<Components::SimulatorState>();
    if (!sv.empty()) {
        const auto &st = reg.get<Components::SimulatorState>(sv.front());
        wc.baseTimeAcceleration = st.baseTimeAcceleration;
        wc.timeScale = st.timeScale;
    }
    if (rc.haveBh && (!w.bhSent || std::memcmp(&w.bhCfg, &rc.bh, sizeof(rc.bh)) != 0)) {
        // BarnesHutSystem's insertion order: view<Position, Mass>(exclude<Boundary>)
        // in its own iteration order (barnes_hut.cpp:117-128), as world body
        // indices (Liquid entities are not world bodies: a world whose fluid
        // would make the system act fails in lpe_world_tick)
        std::unordered_map<uint32_t, int32_t> idx;
        for (size_t i = 0; i < w.bodies.ents.size(); i++) idx[(uint32_t)w.bodies.ents[i]] = (int32_t)i;
        std::vector<int32_t> order;
        for (auto e : reg.view<Components::Position, Components::Mass>(entt::exclude<Components::Boundary>)) {
            auto it = idx.find((uint32_t)e);
            if (it != idx.end()) order.push_back(it->second);
        }
        if (!check(lpe_world_set_barnes_hut(ctx, 1, &rc.bh, (int)order.size(), order.empty() ? nullptr : order.data()),
                   "lpe_world_set_barnes_hut"))
            return;
        w.bhSent = true;
        w.bhCfg = rc.bh;
    }
    if (!check(lpe_world_tick(ctx, &wc, 1), "lpe_world_tick")) return;
    w.ticks++;
    if (w.ticks % s.syncEvery == 0) residentSync(reg);
}

}  // namespace host
}  // namespace lpe
