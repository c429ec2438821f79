// lpe_render.hip — the screen-space fluid density field.
//
// Replaces the compute half of FluidRenderer::render (fluid_renderer.cpp:341-465;
// fluid_renderer_kernels.metal:36-130): the density of the fluid particles at
// every cell of a W x H grid (calculateDensityGrid: unnormalised poly6,
// h = smoothingRadius * cellSize), two 5x5 box-blur passes (boxBlur), the
// maximum of the blurred grid (which the reference reads back to the CPU,
// fluid_renderer.cpp:426-447) and the normalisation to [0, 1]
// (normalizeDensity).  The reference's density kernel loops over every
// particle for every cell, O(cells x N); here the particles are sorted into
// the SPH grid hash first (lpe_sph_hash_current) and a cell walks only the
// reference cells within h of it.  The sum runs over those particles in bin
// order rather than particle order, so the density agrees with the reference
// order to fp32 summation rounding (tests/test_render_gpu.py: 1e-5 of the
// maximum); blur, maximum and normalisation are the reference's arithmetic in
// the reference's order.
#include "lpe_internal.h"
#include <algorithm>
#include <cstring>

namespace lpe {

static constexpr int RT = 16;                 // 16 x 16 cells per block

__global__ void __launch_bounds__(RT * RT)
k_render_density(int gw, int gh, float cellSize, float originX, float originY, float hrel, float eps,
                 float cs, int W, int H, int ox, int oy, const int32_t *__restrict__ start,
                 const float4 *__restrict__ nbA, float *__restrict__ out) {
    const int gx = blockIdx.x * RT + (int)(threadIdx.x % RT);
    const int gy = blockIdx.y * RT + (int)(threadIdx.x / RT);
    if (gx >= gw || gy >= gh) return;
    // cell centre (metal:50): gridOrigin + (float2(gid) + 0.5) * cellSize
    const float px = originX + ((float)gx + 0.5f) * cellSize;
    const float py = originY + ((float)gy + 0.5f) * cellSize;
    const float hSq = hrel * hrel;
    float density = 0.0f;
    if (!(hSq < 1e-12f)) {                    // kernelPoly6 returns 0 otherwise (metal:22)
        // the reference cells (key floor((x + eps) / cs)) that can hold a
        // particle within hrel, one cell of margin for rounding
        const int cx0 = max((int)floorf((px - hrel + eps) / cs) - 1, ox);
        const int cx1 = min((int)floorf((px + hrel + eps) / cs) + 1, ox + W - 1);
        const int cy0 = max((int)floorf((py - hrel + eps) / cs) - 1, oy);
        const int cy1 = min((int)floorf((py + hrel + eps) / cs) + 1, oy + H - 1);
        for (int cy = cy0; cy <= cy1; cy++) {
            // the cells of one row are contiguous bins: one slot range per row
            const int b = start[((cy - oy) * W + (cx0 - ox)) << 2];
            const int e = start[(((cy - oy) * W + (cx1 - ox)) << 2) + 4];
            for (int k = b; k < e; k++) {
                const float4 r = nbA[k];
                const float dx = px - r.x, dy = py - r.y;
                const float rSq = dx * dx + dy * dy;
                if (rSq < hSq) {
                    const float diff = hSq - rSq;
                    density += diff * diff * diff;
                }
            }
        }
    }
    out[(size_t)gy * gw + gx] = density;
}

// boxBlur (metal:72-100): mean over the in-bounds cells of the 5x5 window,
// summed row by row
__global__ void __launch_bounds__(RT * RT)
k_box_blur(int gw, int gh, const float *__restrict__ in, float *__restrict__ out) {
    const int gx = blockIdx.x * RT + (int)(threadIdx.x % RT);
    const int gy = blockIdx.y * RT + (int)(threadIdx.x / RT);
    if (gx >= gw || gy >= gh) return;
    float sum = 0.0f;
    int count = 0;
    for (int dy = -2; dy <= 2; ++dy)
        for (int dx = -2; dx <= 2; ++dx) {
            const int sx = gx + dx, sy = gy + dy;
            if (sx >= 0 && sx < gw && sy >= 0 && sy < gh) {
                sum += in[(size_t)sy * gw + sx];
                count++;
            }
        }
    out[(size_t)gy * gw + gx] = count > 0 ? sum / (float)count : 0.0f;
}

// the maximum of the blurred grid (fluid_renderer.cpp:436-441, on the CPU
// there); densities are >= 0, so the float bits order like the values
__global__ void __launch_bounds__(256)
k_grid_max(size_t n, const float *__restrict__ in, uint32_t *__restrict__ mx) {
    float m = 0.0f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        m = fmaxf(m, in[i]);
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    __shared__ float wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
        atomicMax(mx, __float_as_uint(m));
    }
}

// normalizeDensity (metal:106-124): saturate(density / max) if max > 1e-12
__global__ void __launch_bounds__(256)
k_normalize_density(size_t n, const float *__restrict__ in, const uint32_t *__restrict__ mx,
                    float *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float maxD = __uint_as_float(*mx);
    out[i] = (maxD > 1e-12f) ? fminf(fmaxf(in[i] / maxD, 0.0f), 1.0f) : 0.0f;
}

}  // namespace lpe

using namespace lpe;

extern "C" int lpe_render_density(lpe_ctx *ctx, const lpe_render_params *p, float *normalized, float *max_out) {
    if (!ctx || !p || p->gridW <= 0 || p->gridH <= 0 || !(p->cellSize > 0.f)) return LPE_ERR_ARG;
    const size_t n = (size_t)p->gridW * (size_t)p->gridH;
    if (n > (size_t)1 << 28) return LPE_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    SphDev &d = ctx->sph;
    if (d.shard) {
        ctx->err = "lpe_render_density: a slab rank holds part of the fluid; render from one context";
        return LPE_ERR_STATE;
    }
    hipStream_t s = ctx->stream;
    if (2 * n > d.cap_rgrid || !d.rgrid) {
        if (d.rgrid) (void)hipFree(d.rgrid);
        d.rgrid = nullptr;
        LPE_HIP(ctx, hipMalloc((void **)&d.rgrid, sizeof(float) * 2 * n));
        d.cap_rgrid = 2 * n;
    }
    if (!d.rmax) LPE_HIP(ctx, hipMalloc((void **)&d.rmax, sizeof(uint32_t)));
    float *A = d.rgrid, *B = d.rgrid + n;
    const dim3 grid((p->gridW + RT - 1) / RT, (p->gridH + RT - 1) / RT);
    if (d.n > 0) {
        int st = lpe_sph_hash_current(ctx);
        if (st) return st;
        LPE_KERNEL(ctx, "k_render_density", k_render_density, grid, dim3(RT * RT), 0, s, p->gridW, p->gridH,
                   p->cellSize, p->originX, p->originY, p->smoothingRadius * p->cellSize,
                   d.cfg.gridConfig.gridEpsilon, d.cs, d.W, d.H, d.ox, d.oy, d.start, d.nbA, A);
    } else {
        LPE_HIP(ctx, hipMemsetAsync(A, 0, sizeof(float) * n, s));
    }
    LPE_KERNEL(ctx, "k_box_blur", k_box_blur, grid, dim3(RT * RT), 0, s, p->gridW, p->gridH, A, B);
    LPE_KERNEL(ctx, "k_box_blur", k_box_blur, grid, dim3(RT * RT), 0, s, p->gridW, p->gridH, B, A);
    LPE_HIP(ctx, hipMemsetAsync(d.rmax, 0, sizeof(uint32_t), s));
    const unsigned mb = (unsigned)std::min<size_t>((n + 255) / 256, 2048);
    LPE_KERNEL(ctx, "k_grid_max", k_grid_max, dim3(mb), dim3(256), 0, s, n, A, d.rmax);
    LPE_KERNEL(ctx, "k_normalize_density", k_normalize_density, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
               s, n, A, d.rmax, B);
    LPE_CHECK_LAUNCH(ctx, "render density");
    if (normalized)
        LPE_HIP(ctx, hipMemcpyAsync(normalized, B, sizeof(float) * n, hipMemcpyDeviceToHost, s));
    uint32_t mbits = 0;
    LPE_HIP(ctx, hipMemcpyAsync(&mbits, d.rmax, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    LPE_HIP(ctx, hipStreamSynchronize(s));
    if (max_out) std::memcpy(max_out, &mbits, sizeof(float));
    return LPE_OK;
}
