/**
 * barnes_hut.cpp — MI355X drop-in for Systems::BarnesHutSystem
 * (src/systems/barnes_hut.cpp, include/systems/barnes_hut.hpp).  Same class,
 * header and BarnesHutConfig; update() gathers the bodies of
 * view<Position, Mass>(exclude<Boundary>) in that view's order (buildTree's
 * insertion order, barnes_hut.cpp:117-128), builds the quadtree and walks it
 * on the device (lpe_bh_step: same nodes, same centre-of-mass fold order, same
 * child order as the recursion) and scatters the velocities back.
 *
 * Resident mode records the config; the device tick (lpe_world_tick, run by
 * the last system) applies Barnes-Hut at this system's place in the order,
 * on the world bodies in this view's order.  A resident world whose fluid
 * particles would make it act fails loudly there (LPE_ERR_STATE); strict
 * mode handles it.
 */
#include "systems/barnes_hut.hpp"

#include "entities/entity_components.hpp"
#include "entities/sim_components.hpp"
#include "lpe_backend.hpp"

namespace Systems {

BarnesHutSystem::BarnesHutSystem() = default;

void BarnesHutSystem::update(entt::registry &registry) {
    const double thr = specificConfig.smallMassThreshold;
    if (lpe::host::mode() == lpe::host::Mode::Resident) {
        // the device tick (SleepSystem, the last system) runs it - early exit
        // included - after the collision system as here (lpe_world_set_barnes_hut)
        lpe_bh_config &bc = lpe::host::residentConfigs().bh;
        lpe_bh_config_default(&bc);
        bc.theta = specificConfig.theta;
        bc.small_mass_threshold = thr;
        bc.universe_size = sysConfig.UniverseSizeMeters;
        bc.softener = sysConfig.GravitationalSoftener;
        lpe::host::residentConfigs().haveBh = true;
        return;
    }
    if (thr > 0.0) {                                                   // early exit (:55-71)
        bool skip = true;
        auto mv = registry.view<Components::Mass>(entt::exclude<Components::Boundary>);
        for (auto e : mv)
            if (mv.get<Components::Mass>(e).value >= thr) { skip = false; break; }
        if (skip) return;
    }
    auto sv = registry.view<Components::SimulatorState>();
    if (sv.empty()) return;                                            // (:75-79)
    const auto &state = registry.get<Components::SimulatorState>(sv.front());
    lpe_ctx *ctx = lpe::host::context();
    if (!ctx) return;

    std::vector<entt::entity> ents;
    std::vector<double> x, y, vx, vy, m;
    std::vector<uint8_t> hv;
    auto view = registry.view<Components::Position, Components::Mass>(entt::exclude<Components::Boundary>);
    for (auto e : view) {
        const auto &p = view.get<Components::Position>(e);
        ents.push_back(e);
        x.push_back(p.x);
        y.push_back(p.y);
        m.push_back(view.get<Components::Mass>(e).value);
        const auto *v = registry.try_get<Components::Velocity>(e);
        hv.push_back(v ? 1 : 0);
        vx.push_back(v ? v->x : 0.0);
        vy.push_back(v ? v->y : 0.0);
    }
    if (ents.empty()) return;
    lpe_bh_config cfg;
    lpe_bh_config_default(&cfg);
    cfg.theta = specificConfig.theta;
    cfg.small_mass_threshold = thr;
    cfg.universe_size = sysConfig.UniverseSizeMeters;
    cfg.softener = sysConfig.GravitationalSoftener;
    const double dt = sysConfig.SecondsPerTick * state.baseTimeAcceleration * state.timeScale;   // (:284)
    const int n = (int)ents.size();
    if (!lpe::host::check(lpe_bh_upload(ctx, n, x.data(), y.data(), vx.data(), vy.data(), m.data(), hv.data()),
                          "lpe_bh_upload"))
        return;
    if (!lpe::host::check(lpe_bh_step(ctx, &cfg, dt, nullptr), "lpe_bh_step")) return;
    if (!lpe::host::check(lpe_bh_download(ctx, vx.data(), vy.data()), "lpe_bh_download")) return;
    for (int i = 0; i < n; i++)
        if (hv[i]) {
            auto &v = registry.get<Components::Velocity>(ents[i]);
            v.x = vx[i];
            v.y = vy[i];
        }
}

}  // namespace Systems
