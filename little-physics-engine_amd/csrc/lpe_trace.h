// Profiling-only stamp machinery, kept out of the kernels' sources.
//
// profiles/trace_build.sh compiles ONE source with -DLPE_FTRACE (lpe_sph.hip)
// or -DLPE_PTRACE (lpe_rigid.hip) into a variant library under profiles/_var,
// read back by the profiles/*_trace.py scripts through the extern "C"
// accessors below.  Without those macros (the shipped build) every stamp is an
// empty statement and nothing here is compiled.
//
//   FTR(k), FTRMAX(k, v)   k_forces_couple phases, per trace block `ftb` (the bbox-partial slot: tiles, then filed blocks)
//   DTR(k), DTRMAX(k, v)   k_density<true> phases, per tile `dtb`
//   PTR(w, k), PTR_SET     k_pgs_colour / k_pos_colour colour steps
//   STR(w, j, k), STR_SET  k_pgs_stripes / k_pos_stripes phases per workgroup j
//   CTR(k, v), STP(k)      k_group_colour stages per group, k_stripe_setup stages
#pragma once
#include <hip/hip_runtime.h>

#ifdef LPE_FTRACE
__device__ unsigned long long g_ftrace[4096 * 8];
__device__ int g_ftrace_on;
__device__ unsigned long long g_ftrace2[4096 * 8];
// LPE_FTRACE_LITE: only the block's start / end stamps, its pair count and
// its HW_ID (the full set leaves a 432-byte stack frame in k_forces_couple
// since round 6 and triples its time; the lite set keeps the shipped frame)
#ifdef LPE_FTRACE_LITE
#define FTR(k) do { if (((k) == 0 || (k) == 3) && g_ftrace_on && threadIdx.x == 0) g_ftrace[ftb * 8 + (k)] = wall_clock64(); } while (0)
#else
#define FTR(k) do { if (g_ftrace_on && threadIdx.x == 0) g_ftrace[ftb * 8 + (k)] = wall_clock64(); } while (0)
#endif
#define FTRCLR() do { if (g_ftrace_on && threadIdx.x == 0) for (int k_ = 0; k_ < 8; k_++) { g_ftrace[ftb * 8 + k_] = 0; g_ftrace2[ftb * 8 + k_] = 0; } } while (0)
// the coupling pair's stages (sph_coupling.h CPT), per block
#ifdef LPE_FTRACE_LITE
#define FTR_PAIRS() ((unsigned long long *)nullptr)
#else
#define FTR_PAIRS() (g_ftrace_on ? g_ftrace2 + ftb * 8 : (unsigned long long *)nullptr)
#endif
#define FTR2SET(k, v) do { if (g_ftrace_on && threadIdx.x == 0) g_ftrace2[ftb * 8 + (k)] = (unsigned long long)(v); } while (0)
extern "C" int lpe_ftrace2(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ftrace2), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
#ifdef LPE_FTRACE_LITE
#define FTRMAX(k, v) do {} while (0)
#else
#define FTRMAX(k, v) do { if (g_ftrace_on && (threadIdx.x & 63) == 0) atomicMax(&g_ftrace[ftb * 8 + (k)], (unsigned long long)(v)); } while (0)
#endif
// where the block ran: ftrace2 slot 6 = HW_ID (cu, se, ...), slot 7 = XCC_ID
#define FTRHW() do { if (g_ftrace_on && threadIdx.x == 0) { unsigned hw_, xcc_; \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_)); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_)); \
    g_ftrace2[ftb * 8 + 6] = hw_; g_ftrace2[ftb * 8 + 7] = xcc_; } } while (0)
extern "C" int lpe_ftrace(int on, unsigned long long *host, int n) {
    if (host) (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ftrace), sizeof(unsigned long long) * n);
    unsigned long long z[4096 * 8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_ftrace), z, sizeof(z));
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ftrace_on), &on, sizeof(int)) == hipSuccess ? 0 : 1;
}
// k_density<true> per tile (dtb = the tile): 0 start, 1 staged, 2 walk done
// (max over waves), 3 filed, 4 end (max over waves), 5 longest list (max),
// 6 the staged record count
__device__ unsigned long long g_dtrace[4096 * 8];
#define DTR(k) do { if (g_ftrace_on && threadIdx.x == 0 && dtb < 4096) g_dtrace[dtb * 8 + (k)] = wall_clock64(); } while (0)
#define DTRSET(k, v) do { if (g_ftrace_on && threadIdx.x == 0 && dtb < 4096) g_dtrace[dtb * 8 + (k)] = (unsigned long long)(v); } while (0)
#define DTRMAX(k, v) do { if (g_ftrace_on && (threadIdx.x & 63) == 0 && dtb < 4096) atomicMax(&g_dtrace[dtb * 8 + (k)], (unsigned long long)(v)); } while (0)
#define DTRCLR() do { if (g_ftrace_on && threadIdx.x == 0 && dtb < 4096) for (int k_ = 0; k_ < 8; k_++) g_dtrace[dtb * 8 + k_] = 0; } while (0)
// slot 7: where the tile ran, XCC_ID << 24 | HW_ID's low 24 bits (cu, sh, se)
#define DTRHW() do { if (g_ftrace_on && threadIdx.x == 0 && dtb < 4096) { unsigned hw_, xcc_; \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_)); \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_)); \
    g_dtrace[dtb * 8 + 7] = ((unsigned long long)(xcc_ & 0xF) << 24) | (hw_ & 0xFFFFFF); } } while (0)
extern "C" int lpe_dtrace(unsigned long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dtrace), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 1;
}
#else
#define DTR(k) do {} while (0)
#define DTRSET(k, v) do {} while (0)
#define DTRMAX(k, v) do {} while (0)
#define DTRCLR() do {} while (0)
#define DTRHW() do {} while (0)
#define FTR(k) do {} while (0)
#define FTRCLR() do {} while (0)
#define FTR_PAIRS() ((unsigned long long *)nullptr)
#define FTR2SET(k, v) do {} while (0)
#define FTRMAX(k, v) do {} while (0)
#define FTRHW() do {} while (0)
#endif

#ifdef LPE_PTRACE
__device__ unsigned long long g_ptrace[2][2048];
extern "C" int lpe_ptrace(unsigned long long *host) {
    if (host) (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ptrace), sizeof(unsigned long long) * 2 * 2048);
    return 0;
}
#define PTR(w, k) do { if (threadIdx.x == 0 && (k) < 2048) g_ptrace[w][k] = wall_clock64(); } while (0)
#define PTR_SET(w, k, v) do { g_ptrace[w][k] = (v); } while (0)

__device__ unsigned long long g_strace[2][32][64];
extern "C" int lpe_strace(unsigned long long *host) {
    if (host) (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_strace), sizeof(unsigned long long) * 2 * 32 * 64);
    return 0;
}
#define STR(w, j, k) do { if (threadIdx.x == 0 && (k) < 64 && (j) < 32) g_strace[w][j][k] = wall_clock64(); } while (0)
#define STR_SET(w, j, k, v) do { if ((j) < 32) g_strace[w][j][k] = (v); } while (0)

// rows 0 .. LPE_CTRACE_GROUPS - 1: k_group_colour's groups; row LPE_CTRACE_GROUPS: k_stripe_setup
#define LPE_CTRACE_GROUPS 128
__device__ unsigned long long g_ctrace[LPE_CTRACE_GROUPS + 1][8];
extern "C" int lpe_ctrace(unsigned long long *host) {
    if (host)
        (void)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ctrace), sizeof(unsigned long long) * (LPE_CTRACE_GROUPS + 1) * 8);
    return 0;
}
#define CTR(k, v) do { if (threadIdx.x == 0) g_ctrace[blockIdx.x][k] = (v); } while (0)
#define STP(k) do { if (threadIdx.x == 0) g_ctrace[LPE_CTRACE_GROUPS][k] = wall_clock64(); } while (0)
#else
#define PTR(w, k) do {} while (0)
#define PTR_SET(w, k, v) do {} while (0)
#define STR(w, j, k) do {} while (0)
#define STR_SET(w, j, k, v) do {} while (0)
#define CTR(k, v) do {} while (0)
#define STP(k) do {} while (0)
#endif
