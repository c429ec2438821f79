// lpe_world.hip — the device-resident tick: ECSSimulator::tick
// (src/sim.cpp:156-163) over the fluid (lpe_sph.hip) and the bodies
// (lpe_rigid.hip) without any ECS round trip.
//
// The fluid's ECS round trip is exact: FluidSystem writes fp32 state into the
// double ECS (fluid.cpp:496-524), Boundary and Gravity then update it in
// double (boundary.cpp:23-69, gravity.cpp:53-57) and the next gather casts it
// back to fp32 (fluid.cpp:283-286).  k_fluid_boundary_gravity performs exactly
// that: widen, update in double, narrow.
#include "lpe_internal.h"
#include <cstdlib>
#include "rigid_dev.h"
#include "sph_coupling.h"
#include "lpe_trig.h"
#include <algorithm>
#include <cmath>
#include <vector>

namespace lpe {

// gatherRigidBodies (fluid.cpp:304-438) for one coupling rigid
// (recs: also the fluid coupling's compact AABBs and records, k_rig_couple's work)
__global__ void k_gather_rigids(int nr, const int32_t *__restrict__ coupleBody,
                                const lpe_body *__restrict__ bodies, const double *__restrict__ verts,
                                lpe_gpu_rigid *__restrict__ rig, float maxSafeVelocitySq, float4 *__restrict__ recs) {
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr) return;
    const lpe_body b = bodies[coupleBody[r]];
    lpe_gpu_rigid rb;
    float *raw = (float *)&rb;
    for (int k = 0; k < (int)(sizeof(rb) / 4); k++) raw[k] = 0.f;   // GPURigidBody rb{}
    rb.posX = (float)b.x;
    rb.posY = (float)b.y;
    rb.angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? (float)b.angle : 0.0f;
    if (b.flags & LPE_BODY_HAS_VEL) { rb.vx = (float)b.vx; rb.vy = (float)b.vy; }
    if (b.flags & LPE_BODY_HAS_ANGVEL) rb.omega = (float)b.omega;
    rb.mass = (b.flags & LPE_BODY_HAS_MASS) ? (float)b.mass : 1.f;
    rb.inertia = (b.flags & LPE_BODY_HAS_INERTIA) ? (float)b.inertia : 1.f;
    rb.minX = rb.posX - 0.5f; rb.maxX = rb.posX + 0.5f;
    rb.minY = rb.posY - 0.5f; rb.maxY = rb.posY + 0.5f;
    if (b.flags & LPE_BODY_CIRCLE) {
        rb.shapeType = 0;
        rb.radius = (float)b.radius;
        rb.vertCount = 0;
        rb.minX = rb.posX - rb.radius; rb.maxX = rb.posX + rb.radius;
        rb.minY = rb.posY - rb.radius; rb.maxY = rb.posY + rb.radius;
    } else {
        rb.shapeType = 1;
        rb.radius = 0.f;
        int cnt = min(b.vert_cnt, LPE_MAX_POLY_VERTS);
        rb.vertCount = cnt;
        // std::cos(float) (fluid.cpp:399-400: rb.angle is a float)
        double c = (double)lpe_cosf(rb.angle), s = (double)lpe_sinf(rb.angle);
        float mnx = 3.402823466e38f, mxx = -3.402823466e38f, mny = 3.402823466e38f, mxy = -3.402823466e38f;
        const double *lv = verts + 2 * (size_t)b.vert_off;
        for (int i = 0; i < cnt; i++) {
            double lx = lv[2 * i], ly = lv[2 * i + 1];
            double wx = b.x + (lx * c - ly * s);
            double wy = b.y + (lx * s + ly * c);
            rb.vertsX[i] = (float)wx;
            rb.vertsY[i] = (float)wy;
            if (wx < mnx) mnx = (float)wx;
            if (wx > mxx) mxx = (float)wx;
            if (wy < mny) mny = (float)wy;
            if (wy > mxy) mxy = (float)wy;
        }
        rb.minX = mnx; rb.maxX = mxx; rb.minY = mny; rb.maxY = mxy;
    }
    rig[r] = rb;
    if (recs) rig_couple_one(rb, r, nr, maxSafeVelocitySq, recs);
}

// writeBackRigidBodies' ECS part (fluid.cpp:564-579: v and omega of every
// gathered rigid, fp32 -> double) is k_rigid_writeback's tail (lpe_sph.hip)

// Boundary (boundary.cpp:23-69) then Gravity (gravity.cpp:53-57) on fluid
// particles (no Sleep component, not Boundary): widen, update, narrow
__global__ void k_fluid_boundary_gravity(int n, PState P, double m, double U, double damp,
                                         double maxSpeed, double g, double dt,
                                         const int32_t *__restrict__ heavy_bodies, int heavy_fluid,
                                         const int32_t *__restrict__ nslot) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (nslot && (i >= *nslot || P.id[i] < 0)) return;     // (slab rank: slots in use, dropped ones skipped)
    double x = P.x[i], y = P.y[i], vx = P.vx[i], vy = P.vy[i];
    bool bounced = false;
    if (x < m) { x = m; vx = fabs(vx) * damp; bounced = true; }
    else if (x > U - m) { x = U - m; vx = -fabs(vx) * damp; bounced = true; }
    if (y < m) { y = m; vy = fabs(vy) * damp; bounced = true; }
    else if (y > U - m) { y = U - m; vy = -fabs(vy) * damp; bounced = true; }
    if (bounced) {
        double sp = sqrt(vx * vx + vy * vy);
        if (sp > maxSpeed) { vx = (vx / sp) * maxSpeed; vy = (vy / sp) * maxSpeed; }
    }
    if (!heavy_fluid && !(heavy_bodies && *heavy_bodies)) vy += g * dt;
    P.x[i] = (float)x; P.y[i] = (float)y; P.vx[i] = (float)vx; P.vy[i] = (float)vy;
}

}  // namespace lpe

using namespace lpe;

static inline int wblk(long n, int t = 256) { return (int)((n + t - 1) / t); }

extern "C" int lpe_world_set_coupling(lpe_ctx *ctx, int nr, const int32_t *body_index) {
    if (!ctx || (nr > 0 && !body_index)) return LPE_ERR_ARG;
    SphDev &d = ctx->sph;
    RigidDev *rd = rigid_dev(ctx);
    std::vector<int32_t> idx;
    if (nr < 0) {
        for (int i = rd->nb - 1; i >= 0; i--) idx.push_back(i);
    } else {
        for (int k = 0; k < nr; k++) {
            if (body_index[k] < 0 || body_index[k] >= rd->nb) return LPE_ERR_ARG;
            idx.push_back(body_index[k]);
        }
    }
    int n = (int)idx.size();
    if (n > d.cap_couple || !d.coupleBody) {
        if (d.coupleBody) (void)hipFree(d.coupleBody);
        LPE_HIP(ctx, hipMalloc((void **)&d.coupleBody, sizeof(int32_t) * std::max(n, 1)));
        d.cap_couple = n;
    }
    int st0 = sph_alloc_rigids(ctx, n);
    if (st0) return st0;
    if (n > 0) {
        LPE_HIP(ctx, hipMemcpyAsync(d.coupleBody, idx.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.accum, 0, sizeof(float) * 3 * n, ctx->stream));
        LPE_HIP(ctx, hipMemsetAsync(d.acq, 0, sizeof(unsigned long long) * 3 * XACC_LIMBS * n, ctx->stream));
    }
    d.couple_n = n;
    // bin-list capacity bound without a host sync per tick: bodies that cannot
    // rotate keep their AABB extent; the others are bounded by 2 x circumradius
    std::vector<lpe_body> hb(rd->nb);
    std::vector<double> hv(2 * (size_t)std::max(rd->nverts, 1));
    LPE_HIP(ctx, hipStreamSynchronize(ctx->stream));    // the bodies may still be in flight
    if (rd->nb) LPE_HIP(ctx, hipMemcpy(hb.data(), rd->bodies, sizeof(lpe_body) * rd->nb, hipMemcpyDeviceToHost));
    if (rd->nverts) LPE_HIP(ctx, hipMemcpy(hv.data(), rd->verts, sizeof(double) * 2 * rd->nverts, hipMemcpyDeviceToHost));
    float bcs = std::max(0.25f, d.cs);
    long bound = 0;
    for (int k = 0; k < n; k++) {
        const lpe_body &b = hb[idx[k]];
        double ex, ey;
        if (b.flags & LPE_BODY_CIRCLE) {
            ex = ey = 2 * b.radius;
        } else {
            double R = 0, mnx = 0, mxx = 0, mny = 0, mxy = 0;
            for (int v = 0; v < b.vert_cnt; v++) {
                double lx = hv[2 * (b.vert_off + v)], ly = hv[2 * (b.vert_off + v) + 1];
                R = std::max(R, std::sqrt(lx * lx + ly * ly));
                mnx = std::min(mnx, lx); mxx = std::max(mxx, lx);
                mny = std::min(mny, ly); mxy = std::max(mxy, ly);
            }
            bool rotates = (b.flags & LPE_BODY_HAS_ANGVEL) && !(b.flags & LPE_BODY_BOUNDARY);
            if (rotates) { ex = ey = 2 * R; }
            else { ex = mxx - mnx; ey = mxy - mny; }
        }
        long bx = (long)std::ceil(ex / bcs) + 2, by = (long)std::ceil(ey / bcs) + 2;
        bound += bx * by;
    }
    d.rlist_bound = (int)std::min<long>(bound + 1024, 1L << 30);
    d.fluid_heavy = false;
    return LPE_OK;
}

extern "C" int lpe_world_tick(lpe_ctx *ctx, const lpe_world_config *wc, int nticks) {
    if (!ctx || !wc || nticks < 0) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    SphDev &d = ctx->sph;
    RigidDev *rd = rigid_dev(ctx);
    const lpe_rigid_config &rc = rd->cfg;
    hipStream_t s = ctx->stream;
    const double dt_fluid = wc->secondsPerTick * wc->timeAcceleration;              // fluid.cpp:592
    const double dt_move = wc->secondsPerTick * wc->timeAcceleration;               // movement.cpp:17
    const double dt_state = wc->secondsPerTick * wc->baseTimeAcceleration * wc->timeScale;  // gravity.cpp:31-33
    // a slab rank (lpe_sph_set_slab) joins every fluid step, owned particles or not
    const bool fluid = d.n > 0 || d.shard;
    if (d.couple_n == 0 && rd->nb > 0 && fluid) {
        int st = lpe_world_set_coupling(ctx, -1, nullptr);
        if (st) return st;
    }
    {
        // the boundary system keeps the fluid inside the universe at the end
        // of every tick (boundary.cpp:13-70); the sub-steps of one tick move
        // a particle far less than a metre past it
        const double U = rc.universeSize;
        int st = lpe_sph_cover_box(ctx, -1.0, -1.0, U + 1.0, U + 1.0);
        if (st) return st;
    }
    {
        // BarnesHutSystem's guard (a fluid world it would act on) before any
        // work of the tick is queued
        int st = bh_world_prepare(ctx);
        if (st) return st;
    }
    // collision detection overlapped with the fluid step (LPE_SERIAL_TICK=1:
    // everything on the context stream, in the systems' order)
    const char *ser = std::getenv("LPE_SERIAL_TICK");
    const bool serial = ser && std::atoi(ser) != 0;
    const bool overlap = !serial && rd->nb > 0;
    for (int t = 0; t < nticks; t++) {
        // 1) FluidSystem::update (fluid.cpp:958-1021)
        int nr = fluid ? d.couple_n : 0;
        if (nr > 0) {
            float4 *recs = sph_rig_records(ctx, nr);
            if (!recs) return LPE_ERR_HIP;
            LPE_KERNEL(ctx, "k_gather_rigids", k_gather_rigids, dim3(wblk(nr, 128)), dim3(128), 0, s, nr,
                       d.coupleBody, rd->bodies, rd->verts, d.rig, d.cfg.impulseSolver.maxSafeVelocitySq, recs);
            d.nr = nr;
            d.rig_dirty = true;
            d.rig_coupled = true;
        }
        if (overlap) {          // after the gather: the fluid sees the unclamped poses
            int st = rigid_tick_begin(ctx, !fluid);
            if (st) return st;
        }
        if (fluid) {
            // the detection launches after the first sub-step, its host half
            // and the colouring after the third (rigid_tick_hook)
            // (the write-back of the coupled rigids' velocities scatters them
            // to their bodies in the same kernel: d.wb_bodies)
            d.wb_bodies = nr > 0 ? rd->bodies : nullptr;
            int st = sph_step_hooked(ctx, dt_fluid, overlap ? rigid_tick_hook : nullptr);
            d.wb_bodies = nullptr;
            if (st) return st;
        }
        // 2) BoundarySystem, 3) BasicGravitySystem: bodies and fluid
        // (the planetary-mass check spans bodies and fluid, gravity.cpp:43-51)
        // the bodies' boundary (velocity half) and gravity as one pass when
        // overlapped (the position half ran in rigid_tick_begin); the fluid's
        // boundary + gravity pass leads the prelaunch on its side stream
        // (it touches no body; the context stream joins it at the tick's end)
        int st;
        if (overlap) {
            st = lpe_rigid_integrate(ctx, 32, dt_state, dt_move);
            if (!st) st = rigid_tick_boundary(ctx, true, dt_state);
        } else {
            st = lpe_rigid_integrate(ctx, 1 | 32, dt_state, dt_move);
        }
        if (st) return st;
        // (LPE_NO_PRELAUNCH=1: the next tick's sub-step 0 runs in its own
        // tick, for A/B measurements of the overlap)
        static const bool nopre = std::getenv("LPE_NO_PRELAUNCH") != nullptr;
        const bool prelaunch = !serial && fluid && !nopre;
        const bool fbg_side = prelaunch && d.n > 0 && d.P.x;
        auto fbg = [&](hipStream_t fs) {
            LPE_KERNEL(ctx, "k_fluid_boundary_gravity", k_fluid_boundary_gravity, dim3(wblk(d.n)), dim3(256), 0, fs, d.n, d.P, rc.marginPixels * rc.metersPerPixel, rc.universeSize, rc.bounceDamping, rc.maxSpeed, rc.gravity, dt_state, rd->nb > 0 ? rd->counts + 5 : (const int32_t *)nullptr, d.fluid_heavy ? 1 : 0, sph_slab_slots(ctx));
            return LPE_OK;
        };
        if (d.n > 0 && !fbg_side) {
            st = fbg(s);
            if (st) return st;
        }
        if (!overlap) {
            st = lpe_rigid_integrate(ctx, 2, dt_state, dt_move);
            if (st) return st;
        }
        // the fluid state is final for this tick: the next tick's first
        // sub-step (up to its forces) runs beside the rigid solvers -- also
        // after the last tick of this call, for the next call (it writes only
        // scratch, so downloads and state changes in between are safe)
        if (prelaunch) {
            // (with the fluid's boundary/gravity on the side stream, the bodies'
            // pass is the context stream's last launch: its signal serves)
            st = fbg_side ? sph_prelaunch(ctx, dt_fluid, fbg, overlap ? rigid_boundary_event(ctx) : nullptr, overlap)
                          : sph_prelaunch(ctx, dt_fluid);
            if (st) return st;
        }
        // an error past this point still joins the side stream's fluid
        // boundary / gravity pass (it writes P), so later calls cannot race it
        auto fail = [&](int code) {
            if (fbg_side) (void)hipStreamWaitEvent(s, d.fbgDone, 0);
            return code;
        };
        // 4) RigidBodyCollisionSystem
        st = overlap ? rigid_tick_finish(ctx) : lpe_rigid_step(ctx, nullptr);
        if (st) return fail(st);
        // 5) BarnesHut (its small-mass early exit cached until an upload), 6) Rotation,
        // 7) Movement, 8) Sleep
        st = bh_world_tick(ctx, dt_state);
        if (st) return fail(st);
        st = lpe_rigid_integrate(ctx, 4 | 8 | 16, dt_state, dt_move);
        if (st) return fail(st);
        if (fbg_side) LPE_HIP(ctx, hipStreamWaitEvent(s, d.fbgDone, 0));
        LPE_CHECK_LAUNCH(ctx, "world tick");
    }
    return LPE_OK;
}
