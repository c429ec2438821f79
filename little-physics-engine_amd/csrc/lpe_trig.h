/*
 * lpe_trig.h — portable sine and cosine, compiled identically for the device
 * (hipcc), the host mirror (g++) and the CPU oracle (gcc), so that every
 * angle-dependent value of the rigid path is bit-identical across them.
 *
 * Why: the reference transforms vertices with the platform's libm
 * (polygon.hpp:55-76 getSupport, narrowphase.cpp:56-81 getWorldVerts,
 * broadphase.cpp:178-189 computeAABB: std::cos/std::sin on double; and
 * fluid.cpp:399-400 gatherRigidBodies: std::cos(float) — the FLOAT overload,
 * rb.angle is a float).  The device's libm (ocml) and the host's (glibc)
 * round differently in a few percent of arguments (1 ulp), which used to
 * leave the device's rigid poses 1e-16 apart from the oracle's and made the
 * drop-in's strict (host-gathered) and resident (device-gathered) modes drift
 * apart.  One implementation, evaluated with IEEE operations only (no FMA
 * contraction: every build of this header uses -ffp-contract=off), removes
 * the platform from the result.
 *
 * Algorithm: the classic fdlibm/FreeBSD scheme — Cody–Waite reduction by
 * pi/2 in up to three 33-bit steps (exact for |x| < LPE_TRIG_MAX_ARG =
 * 2^20 * pi/2; angles here stay within a few multiples of 2 pi: rotation.cpp
 * wraps them every tick, and lpe_rigid_upload refuses larger ones; beyond
 * the range the functions return NaN instead of a silently wrong value),
 * then degree-13/14 minimax kernels on [-pi/4, pi/4].  Error < 1 ulp
 * (measured against glibc over 2^24 arguments: tests/test_oracle_rigid.py).
 * lpe_cosf / lpe_sinf, the reference's std::cos(float), are the double
 * results rounded once to float: the correctly rounded value except within
 * 1 double ulp of a float tie (glibc's cosf/sinf are within 0.56 ulp).
 */
#ifndef LPE_TRIG_H
#define LPE_TRIG_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define LPE_TRIG_FN static inline __host__ __device__
#else
#define LPE_TRIG_FN static inline
#endif

#define LPE_TRIG_MAX_ARG 1647099.0   /* just below 2^20 * pi / 2 (the high word 0x413921fb) */

LPE_TRIG_FN uint32_t lpe_trig_hi(double x) {
    uint64_t u;
    memcpy(&u, &x, sizeof u);
    return (uint32_t)(u >> 32);
}

/* sin on [-pi/4, pi/4]; y is the tail of the reduced argument (iy = 0: none) */
LPE_TRIG_FN double lpe_ksin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    double z = x * x, w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

/* cos on [-pi/4, pi/4] */
LPE_TRIG_FN double lpe_kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x, w = z * z;
    double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + (z * r - x * y));
}

/* x = n * pi/2 + (y0 + y1), |y0 + y1| <= pi/4 (Cody–Waite, 33-bit splits) */
LPE_TRIG_FN int lpe_rem_pio2(double x, double *y0, double *y1) {
    const double invpio2 = 6.36619772367581382433e-01,
                 pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11,
                 pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21,
                 pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    const double toint = 6755399441055744.0;   /* 1.5 * 2^52: round to nearest */
    double fn = x * invpio2 + toint;
    fn = fn - toint;
    int n = (int)fn;
    double r = x - fn * pio2_1;
    double w = fn * pio2_1t;
    int j = (int)((lpe_trig_hi(x) >> 20) & 0x7ff);
    *y0 = r - w;
    int i = j - (int)((lpe_trig_hi(*y0) >> 20) & 0x7ff);
    if (i > 16) {
        double t = r;
        w = fn * pio2_2;
        r = t - w;
        w = fn * pio2_2t - ((t - r) - w);
        *y0 = r - w;
        i = j - (int)((lpe_trig_hi(*y0) >> 20) & 0x7ff);
        if (i > 49) {
            t = r;
            w = fn * pio2_3;
            r = t - w;
            w = fn * pio2_3t - ((t - r) - w);
            *y0 = r - w;
        }
    }
    *y1 = (r - *y0) - w;
    return n;
}

LPE_TRIG_FN double lpe_sin(double x) {
    uint32_t ix = lpe_trig_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {                    /* |x| <~ pi/4 */
        if (ix < 0x3e500000u) return x;         /* |x| < 2^-26 */
        return lpe_ksin(x, 0.0, 0);
    }
    if (ix >= 0x7ff00000u) return x - x;        /* inf, nan */
    if (ix >= 0x413921fbu) return (x - x) / (x - x);   /* |x| >= 2^20 pi/2: outside the exact reduction */
    double y0, y1;
    int n = lpe_rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return lpe_ksin(y0, y1, 1);
    case 1: return lpe_kcos(y0, y1);
    case 2: return -lpe_ksin(y0, y1, 1);
    default: return -lpe_kcos(y0, y1);
    }
}

LPE_TRIG_FN double lpe_cos(double x) {
    uint32_t ix = lpe_trig_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        if (ix < 0x3e46a09eu) return 1.0;       /* |x| < 2^-27 * sqrt(2) */
        return lpe_kcos(x, 0.0);
    }
    if (ix >= 0x7ff00000u) return x - x;
    if (ix >= 0x413921fbu) return (x - x) / (x - x);
    double y0, y1;
    int n = lpe_rem_pio2(x, &y0, &y1);
    switch (n & 3) {
    case 0: return lpe_kcos(y0, y1);
    case 1: return -lpe_ksin(y0, y1, 1);
    case 2: return -lpe_kcos(y0, y1);
    default: return lpe_ksin(y0, y1, 1);
    }
}

/* std::cos(float) / std::sin(float) of the reference's fluid gather */
LPE_TRIG_FN float lpe_cosf(float x) { return (float)lpe_cos((double)x); }
LPE_TRIG_FN float lpe_sinf(float x) { return (float)lpe_sin((double)x); }

#endif /* LPE_TRIG_H */
