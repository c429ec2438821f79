/*
 * render_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's screen-space fluid density field, the parity checker for
 * lpe_render_density (little-physics-engine_amd/csrc/lpe_render.hip).  Only
 * tests/ may load this code; the product library never links it.
 *
 * Parity status: UNPINNED BY EXECUTION.  The reference renderer is Metal-only
 * (src/renderers/fluid_renderer_kernels.metal) and ships no fixtures; this
 * file restates, in the reference's own loop orders:
 *   calculateDensityGrid  fluid_renderer_kernels.metal:36-66 (every particle,
 *                         in buffer order, for every grid cell)
 *   boxBlur               :72-100 (5x5, twice: fluid_renderer.cpp:407-419)
 *   maximum               fluid_renderer.cpp:426-441 (on the CPU there)
 *   normalizeDensity      :106-124
 * fp32, no FMA contraction (-ffp-contract=off).
 */
#include <math.h>
#include <stddef.h>

static float poly6_unnormalised(float rSq, float hSq) {         /* metal:20-28 */
    if (rSq >= hSq || hSq < 1e-12f) return 0.0f;
    float diff = hSq - rSq;
    return diff * diff * diff;
}

static void box_blur(int gw, int gh, const float *in, float *out) {   /* metal:72-100 */
    for (int gy = 0; gy < gh; gy++)
        for (int gx = 0; gx < gw; gx++) {
            float sum = 0.0f;
            int count = 0;
            for (int dy = -2; dy <= 2; ++dy)
                for (int dx = -2; dx <= 2; ++dx) {
                    int sx = gx + dx, sy = gy + dy;
                    if (sx >= 0 && sx < gw && sy >= 0 && sy < gh) {
                        sum += in[(size_t)sy * gw + sx];
                        count++;
                    }
                }
            out[(size_t)gy * gw + gx] = (count > 0) ? (sum / (float)count) : 0.0f;
        }
}

/* n particles (x, y: fp32 positions in gather order); grid gw x gh of
 * cellSize metres from (ox, oy); smoothingRadius in cells.  Writes the raw
 * density, the twice-blurred grid, its maximum and the normalised grid. */
void lpeo_render_density(int n, const float *x, const float *y, int gw, int gh, float cellSize,
                         float ox, float oy, float smoothingRadius, float *density, float *blurred,
                         float *scratch, float *maxd, float *normalized) {
    float hrel = smoothingRadius * cellSize;                        /* metal:55 */
    float hSq = hrel * hrel;
    for (int gy = 0; gy < gh; gy++)
        for (int gx = 0; gx < gw; gx++) {
            float cx = ox + ((float)gx + 0.5f) * cellSize;           /* metal:50 */
            float cy = oy + ((float)gy + 0.5f) * cellSize;
            float d = 0.0f;
            for (int i = 0; i < n; ++i) {                            /* metal:59-66 */
                float dx = cx - x[i], dy = cy - y[i];
                float distSq = dx * dx + dy * dy;
                d += poly6_unnormalised(distSq, hSq);
            }
            density[(size_t)gy * gw + gx] = d;
        }
    box_blur(gw, gh, density, scratch);                              /* fluid_renderer.cpp:407-413 */
    box_blur(gw, gh, scratch, blurred);                              /* :414-419 */
    float m = 0.0f;                                                  /* :426-441 */
    for (size_t i = 0; i < (size_t)gw * gh; i++) m = blurred[i] > m ? blurred[i] : m;
    *maxd = m;
    for (size_t i = 0; i < (size_t)gw * gh; i++) {                   /* metal:106-124 */
        float v = (m > 1e-12f) ? blurred[i] / m : 0.0f;
        normalized[i] = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v);
    }
}
