// sph_coupling.h — per-particle rigid–fluid coupling (device functions).
//
// Restates rigidFluidImpulseSolver (fluid_kernels.metal:679-924) and
// rigidFluidPositionSolver (fluid_kernels.metal:533-668) for ONE particle,
// over a candidate list of rigids in ascending rigid index (the reference
// loops over all R rigids in ascending order; non-candidates fail its AABB
// test, so the candidate walk is equivalent).
#pragma once
#include "lpe_internal.h"

namespace lpe {

__device__ __forceinline__ bool pointInPolygon(float px, float py, const lpe_gpu_rigid &b) {
    int vCount = b.vertCount;
    if (vCount < 3) return false;
    bool inside = false;
    for (int i = 0, j = vCount - 1; i < vCount; j = i++) {
        float xi = b.vertsX[i], yi = b.vertsY[i];
        float xj = b.vertsX[j], yj = b.vertsY[j];
        bool intersect = ((yi > py) != (yj > py)) &&
                         (px < (xj - xi) * (py - yi) / (yj - yi) + xi);
        if (intersect) inside = !inside;
    }
    return inside;
}

__device__ __forceinline__ void closestPointOnPolygon(float px, float py, const lpe_gpu_rigid &b,
                                                      float &ox, float &oy) {
    int vCount = b.vertCount;
    ox = px; oy = py;
    if (vCount < 2) return;
    float minDistSq = 1e12f;
    for (int i = 0; i < vCount; i++) {
        int j = (i + 1) % vCount;
        float x1 = b.vertsX[i], y1 = b.vertsY[i];
        float x2 = b.vertsX[j], y2 = b.vertsY[j];
        float ex = x2 - x1, ey = y2 - y1;
        float eLenSq = ex * ex + ey * ey;
        if (eLenSq < 1e-16f) continue;
        float dx = px - x1, dy = py - y1;
        float t = (dx * ex + dy * ey) / eLenSq;
        if (t < 0.f) t = 0.f;
        if (t > 1.f) t = 1.f;
        float cx = x1 + t * ex, cy = y1 + t * ey;
        float cdx = px - cx, cdy = py - cy;
        float distSq = cdx * cdx + cdy * cdy;
        if (distSq < minDistSq) { minDistSq = distSq; ox = cx; oy = cy; }
    }
}

__device__ __forceinline__ float f2len(float x, float y) { return sqrtf(x * x + y * y); }

// tanh / pow of the impulse solver (metal:810, :822): fp64 rounded once to
// fp32, the same definition as oracle/sph_oracle.c.
__device__ __forceinline__ float lpe_tanhf(float x) { return (float)tanh((double)x); }
__device__ __forceinline__ float lpe_powf(float x, float e) { return (float)pow((double)x, (double)e); }

struct CoupleParams {
    float gravity, restDensity, viscosity;
    float maxForce, maxTorque, viscosityScale, depthScale, depthTransitionRate;
    float pressureForceRatio, viscousForceRatio, angDampThr, angDampFactor;
    float depthEstimateScale, maxSafeVelocitySq, minPenetration, minRelVelocity;
    float fluidForceScale, fluidForceMax, buoyancyStrength;
    float safetyMargin, relaxFactor, minSafeDistance, minPositionChange, maxCorrection;
    float boundaryOffset;
    int bx0, by0, bW, bH;
    float bcs;
    int nr;
};

// Particle state entering the coupling (after velocityVerletFinish).
struct CoupleState {
    float x, y, vx, vy, vhx, vhy, ax, ay, mass, rho, p;
};

// rigidFluidImpulseSolver for one particle; adds to the rigid accumulators.
__device__ __forceinline__ void couple_impulse(CoupleState &st, const CoupleParams &cp, float dt,
                                               const lpe_gpu_rigid *__restrict__ rig,
                                               const int32_t *__restrict__ list, int k0, int k1,
                                               float *__restrict__ accum) {
    float densityF = st.rho > 0.0f ? st.rho : cp.restDensity;
    float pressureF = st.p;
    float tffx = 0.0f, tffy = 0.0f;
    bool had = false;
    const float px = st.x, py = st.y;
    for (int k = k0; k < k1; k++) {
        const int r = list[k];
        const lpe_gpu_rigid &rb = rig[r];
        float rbVelSq = rb.vx * rb.vx + rb.vy * rb.vy + rb.omega * rb.omega;
        if (rbVelSq > cp.maxSafeVelocitySq) continue;
        if (px < rb.minX || px > rb.maxX || py < rb.minY || py > rb.maxY) continue;
        bool inside = false;
        float pen = 0.0f, relx = 0.f, rely = 0.f, nx = 0.f, ny = 0.f;
        if (rb.shapeType == 0) {
            float rx = px - rb.posX, ry = py - rb.posY;
            float dist2 = rx * rx + ry * ry;
            float radiusSq = rb.radius * rb.radius;
            if (dist2 < radiusSq) {
                inside = true;
                float dist = sqrtf(dist2);
                if (dist < cp.minPenetration) dist = cp.minPenetration;
                pen = rb.radius - dist;
                if (pen < 0.0f) pen = 0.0f;
                relx = rx; rely = ry;
                nx = relx / dist; ny = rely / dist;
            }
        } else if (rb.shapeType == 1 && rb.vertCount >= 3) {
            inside = pointInPolygon(px, py, rb);
            if (inside) {
                float cx, cy;
                closestPointOnPolygon(px, py, rb, cx, cy);
                float dx = px - cx, dy = py - cy;
                float d2 = dx * dx + dy * dy;
                float d = sqrtf(d2);
                if (d < cp.minPenetration) d = cp.minPenetration;
                pen = d;
                if (pen < 0.0f) pen = 0.0f;
                relx = px - rb.posX; rely = py - rb.posY;
                nx = dx / d; ny = dy / d;
            }
        }
        if (!inside || pen < cp.minPenetration) continue;
        had = true;
        float rotx = -rb.omega * rely, roty = rb.omega * relx;
        float rvx = rb.vx + rotx, rvy = rb.vy + roty;
        float relVx = st.vx - rvx, relVy = st.vy - rvy;
        float depthFactor = lpe_tanhf(cp.depthTransitionRate * pen / cp.depthScale);
        float normalVel = relVx * nx + relVy * ny;
        float nvx = nx * normalVel, nvy = ny * normalVel;
        float tvx = relVx - nvx, tvy = relVy - nvy;
        float particleVolume = st.mass / densityF;
        float effectiveArea = lpe_powf(particleVolume, 2.0f / 3.0f);
        float depth = fminf(py / cp.depthEstimateScale, 1.0f);
        float hydro = densityF * cp.gravity * depth;
        float totalPressure = pressureF + hydro;
        float pressureForce = totalPressure * effectiveArea * depthFactor;
        float pfm = fminf(pressureForce, cp.maxForce * cp.pressureForceRatio);
        float pfx = nx * pfm, pfy = ny * pfm;
        float tangentVelMag = f2len(tvx, tvy);
        if (tangentVelMag > cp.minRelVelocity) {
            float tdx = tvx / tangentVelMag, tdy = tvy / tangentVelMag;
            float viscosityCoef = cp.viscosity * cp.viscosityScale;
            float viscousForce = viscosityCoef * tangentVelMag * densityF * depthFactor * dt;
            float vfm = fminf(viscousForce, cp.maxForce * cp.viscousForceRatio);
            pfx += -tdx * vfm;
            pfy += -tdy * vfm;
        }
        if (rb.mass > 0.1f) {
            float bxf = 0.0f * cp.buoyancyStrength * pen * effectiveArea * cp.gravity * densityF;
            float byf = -1.0f * cp.buoyancyStrength * pen * effectiveArea * cp.gravity * densityF;
            float cbx = pfx + bxf, cby = pfy + byf;
            if (f2len(cbx, cby) <= cp.maxForce) { pfx = cbx; pfy = cby; }
        }
        float tfx = pfx, tfy = pfy;
        float forceMag = f2len(tfx, tfy);
        if (forceMag > cp.maxForce) {
            float sc = cp.maxForce / forceMag;
            tfx = tfx * sc; tfy = tfy * sc;
        }
        float torque = relx * tfy - rely * tfx;
        torque = fminf(fmaxf(torque, -cp.maxTorque), cp.maxTorque);
        if (fabsf(rb.omega) > cp.angDampThr) {
            float sgn = (rb.omega > 0.f) ? 1.f : ((rb.omega < 0.f) ? -1.f : 0.f);
            torque -= cp.angDampFactor * sgn * fabsf(rb.omega) * rb.inertia;
        }
        atomicAdd(&accum[3 * r + 0], tfx);
        atomicAdd(&accum[3 * r + 1], tfy);
        atomicAdd(&accum[3 * r + 2], torque);
        tffx -= tfx * cp.fluidForceScale;
        tffy -= tfy * cp.fluidForceScale;
    }
    if (had) {
        float fm = f2len(tffx, tffy);
        if (fm > cp.fluidForceMax) {
            float sc = cp.fluidForceMax / fm;
            tffx = tffx * sc; tffy = tffy * sc;
        }
        float invMass = (st.mass > 0.0001f) ? 1.0f / st.mass : 1.0f;
        st.ax += tffx * invMass;
        st.ay += tffy * invMass;
    }
}

// rigidFluidPositionSolver for one particle (always dispatched, fluid.cpp:929-942).
__device__ __forceinline__ void couple_position(CoupleState &st, const CoupleParams &cp,
                                                const lpe_gpu_rigid *__restrict__ rig,
                                                const int32_t *__restrict__ list, int k0, int k1) {
    float oldx = st.x, oldy = st.y;
    float acx = 0.0f, acy = 0.0f;
    const float px = st.x, py = st.y;
    bool hadCollision = false;
    for (int k = k0; k < k1; k++) {
        const lpe_gpu_rigid &b = rig[list[k]];
        if (px < b.minX || px > b.maxX || py < b.minY || py > b.maxY) continue;
        if (b.shapeType == 0) {
            float dx = px - b.posX, dy = py - b.posY;
            float dist2 = dx * dx + dy * dy;
            float radius = b.radius;
            if (dist2 < radius * radius) {
                hadCollision = true;
                float dist = sqrtf(dist2);
                if (dist < cp.minSafeDistance) { dist = cp.minSafeDistance; dx = 1.0f; dy = 0.0f; }
                float pen = (radius - dist) + cp.safetyMargin;
                float dirx = dx / dist, diry = dy / dist;
                acx -= dirx * pen * cp.relaxFactor;
                acy -= diry * pen * cp.relaxFactor;
            }
        } else if (b.shapeType == 1) {
            if (b.vertCount < 3) continue;
            if (pointInPolygon(px, py, b)) {
                hadCollision = true;
                float cx, cy;
                closestPointOnPolygon(px, py, b, cx, cy);
                float cdx = px - cx, cdy = py - cy;
                float d2 = cdx * cdx + cdy * cdy;
                float d = sqrtf(d2);
                if (d < cp.minSafeDistance) { d = cp.minSafeDistance; cdx = 1.0f; cdy = 0.0f; }
                float pen = d + cp.safetyMargin;
                float dirx = cdx / d, diry = cdy / d;
                acx += dirx * pen * cp.relaxFactor;
                acy += diry * pen * cp.relaxFactor;
            }
        }
    }
    float cm = f2len(acx, acy);
    if (cm > cp.maxCorrection) {
        acx = (acx / cm) * cp.maxCorrection;
        acy = (acy / cm) * cp.maxCorrection;
    }
    st.x -= acx;
    st.y -= acy;
    if (st.x < 0.f) st.x = cp.boundaryOffset;
    if (st.y < 0.f) st.y = cp.boundaryOffset;
    if (hadCollision) {
        float pdx = st.x - oldx, pdy = st.y - oldy;
        float pdm = f2len(pdx, pdy);
        if (pdm > cp.minPositionChange) {
            float cdx = pdx / pdm, cdy = pdy / pdm;
            float cvx = st.vx, cvy = st.vy;
            float va = cvx * cdx + cvy * cdy;
            if (va < 0.0f) {
                float restitution = 0.0f;
                cvx -= (1.0f + restitution) * va * cdx;
                cvy -= (1.0f + restitution) * va * cdy;
                st.vx = cvx; st.vy = cvy;
                st.vhx = st.vx; st.vhy = st.vy;
            }
        }
    }
}

}  // namespace lpe
