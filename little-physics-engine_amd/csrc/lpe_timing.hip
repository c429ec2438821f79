// lpe_timing.hip — HIP-event kernel timing on the context stream.
#include "lpe_internal.h"
#include <cstring>

namespace lpe {

// mode 2: the dominant kernels only, so the host keeps enough launches queued
// ahead of the device (per-kernel events on every launch make the host the
// bottleneck and the events then time the device idling between launches)
bool KernelTimer::wants(const char *name) const {
    // (a cross-stream wait, k_wait_flag, is no work of the tick: never timed)
    if (std::strcmp(name, "k_wait_flag") == 0) return false;
    if (on == 1) return true;
    static const char *hot[] = {"k_density", "k_density_plan", "k_forces_couple", "k_pgs_flow", "k_pos_flow", "k_pair_colour",
                                "k_narrow", "k_bg_pairs"};
    for (const char *h : hot)
        if (std::strcmp(h, name) == 0) return true;
    return false;
}

int KernelTimer::slot(const char *name) {
    for (size_t i = 0; i < names.size(); i++)
        if (names[i] == name) return (int)i;
    names.emplace_back(name);
    pending.emplace_back();
    total_ms.push_back(0.0);
    calls.push_back(0);
    return (int)names.size() - 1;
}

hipEvent_t KernelTimer::get() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    // device-scope release: the default system-scope release writes back L2
    // at every event, which slows the kernels being timed
    (void)hipEventCreateWithFlags(&e, hipEventReleaseToDevice);
    return e;
}

}  // namespace lpe

static void timer_resolve(lpe_ctx *ctx) {
    lpe::KernelTimer &t = ctx->timer;
    for (size_t i = 0; i < t.names.size(); i++) {
        for (auto &pr : t.pending[i]) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
                t.total_ms[i] += ms;
                t.calls[i] += 1;
            }
            t.pool.push_back(pr.first);
            t.pool.push_back(pr.second);
        }
        t.pending[i].clear();
    }
}

extern "C" int lpe_timing_enable(lpe_ctx *ctx, int on) {
    if (!ctx) return LPE_ERR_ARG;
    if (on < 0 || on > 2) return LPE_ERR_ARG;
    ctx->timer.on = on;
    return LPE_OK;
}

extern "C" int lpe_timing_reset(lpe_ctx *ctx) {
    if (!ctx) return LPE_ERR_ARG;
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    timer_resolve(ctx);
    for (auto &v : ctx->timer.total_ms) v = 0.0;
    for (auto &c : ctx->timer.calls) c = 0;
    return LPE_OK;
}

extern "C" int lpe_timing_read(lpe_ctx *ctx, int i, char *name, int name_cap, double *total_ms,
                               long *calls) {
    if (!ctx) return LPE_ERR_ARG;
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));
    timer_resolve(ctx);
    lpe::KernelTimer &t = ctx->timer;
    if (i < 0 || i >= (int)t.names.size()) return LPE_ERR_ARG;
    if (name && name_cap > 0) {
        std::strncpy(name, t.names[i].c_str(), (size_t)name_cap - 1);
        name[name_cap - 1] = 0;
    }
    if (total_ms) *total_ms = t.total_ms[i];
    if (calls) *calls = t.calls[i];
    return LPE_OK;
}

int lpe_timer_destroy_internal(lpe_ctx *ctx) {
    lpe::KernelTimer &t = ctx->timer;
    timer_resolve(ctx);
    for (hipEvent_t e : t.pool) (void)hipEventDestroy(e);
    t.pool.clear();
    return LPE_OK;
}
