// gap_probe.hip — what a dependent kernel boundary costs on the box, measured
// with in-kernel wall-clock stamps (no profiler): each launch i records the
// earliest workgroup start and the latest workgroup end, so gap = start[i+1] -
// end[i].  Variants: grid / LDS / kernarg size, dirty bytes left behind, and
// other streams holding blocked barrier packets (the world tick's side and
// prelaunch streams wait on events of the context stream while it runs the
// sub-steps).  Measurement tooling only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct Stamp { unsigned long long s, e; };
struct Big { int v[256]; };

// one record per workgroup (plain vector stores, no contended atomics)
__device__ __forceinline__ void stamp_begin(Stamp *st) {
    if (threadIdx.x == 0) st[blockIdx.x].s = (unsigned long long)wall_clock64();
}
__device__ __forceinline__ void stamp_end(Stamp *st) {
    __syncthreads();
    if (threadIdx.x == 0) st[blockIdx.x].e = (unsigned long long)wall_clock64();
}

__global__ void k_triv(Stamp *st) {
    stamp_begin(st);
    stamp_end(st);
}

__global__ void k_lds(Stamp *st, int work) {
    extern __shared__ float sm[];
    stamp_begin(st);
    sm[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    float a = sm[(threadIdx.x + 1) & 255];
    for (int i = 0; i < work; i++) a = a * 1.0001f + 0.5f;
    if (a == -1.f) sm[0] = a;
    stamp_end(st);
}

__global__ void k_big(Stamp *st, Big b) {
    stamp_begin(st);
    if (b.v[threadIdx.x & 255] == -7) st[blockIdx.x].s = 0;
    stamp_end(st);
}

// writes `per` float4 a thread: dirty bytes = grid * 256 * per * 16
__global__ void k_dirty(Stamp *st, float4 *buf, int per) {
    stamp_begin(st);
    size_t base = ((size_t)blockIdx.x * per) * 256 + threadIdx.x;
    for (int i = 0; i < per; i++) buf[base + (size_t)i * 256] = make_float4(1.f, 2.f, 3.f, (float)i);
    stamp_end(st);
}

// the same bytes with non-temporal stores
__global__ void k_dirty_nt(Stamp *st, float4 *buf, int per) {
    stamp_begin(st);
    size_t base = ((size_t)blockIdx.x * per) * 256 + threadIdx.x;
    for (int i = 0; i < per; i++) {
        float *p = (float *)(buf + base + (size_t)i * 256);
        __builtin_nontemporal_store(1.f, p);
        __builtin_nontemporal_store(2.f, p + 1);
        __builtin_nontemporal_store(3.f, p + 2);
        __builtin_nontemporal_store((float)i, p + 3);
    }
    stamp_end(st);
}

__global__ void k_spin(long long ticks) {
    long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

static double tick_us() {
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    return 1000.0 / khz;
}

struct Res { double gap_med, gap_p90, ker_med, wall_per; };

static const int WGMAX = 2048;

// launch(i) must pass st + i * WGMAX and use at most WGMAX workgroups
template <class F>
static Res run(hipStream_t s, Stamp *d_st, int n, F launch) {
    const size_t nrec = (size_t)n * WGMAX;
    std::vector<Stamp> h(nrec);
    for (auto &x : h) { x.s = ~0ull; x.e = 0; }
    CK(hipMemcpy(d_st, h.data(), nrec * sizeof(Stamp), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; i++) launch(i % n);  // warm (stamps reset below)
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(d_st, h.data(), nrec * sizeof(Stamp), hipMemcpyHostToDevice));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < n; i++) launch(i);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(h.data(), d_st, nrec * sizeof(Stamp), hipMemcpyDeviceToHost));
    const double tu = tick_us();
    std::vector<Stamp> L(n);
    for (int i = 0; i < n; i++) {
        L[i].s = ~0ull;
        L[i].e = 0;
        for (int w = 0; w < WGMAX; w++) {
            const Stamp &x = h[(size_t)i * WGMAX + w];
            if (x.e == 0) continue;
            L[i].s = std::min(L[i].s, x.s);
            L[i].e = std::max(L[i].e, x.e);
        }
    }
    h.swap(L);
    std::vector<double> g, k;
    for (int i = 1; i < n; i++) g.push_back(((long long)h[i].s - (long long)h[i - 1].e) * tu);
    for (int i = 0; i < n; i++) k.push_back(((long long)h[i].e - (long long)h[i].s) * tu);
    std::sort(g.begin(), g.end());
    std::sort(k.begin(), k.end());
    Res r{g[g.size() / 2], g[g.size() * 9 / 10], k[k.size() / 2], ms * 1000.0 / n};
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return r;
}

static void show(const char *name, Res r) {
    std::printf("%-58s gap med %6.2f p90 %6.2f  kernel med %7.2f  wall/launch %7.2f us\n", name, r.gap_med,
                r.gap_p90, r.ker_med, r.wall_per);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 400;
    hipStream_t A, B, C, D;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&D, hipStreamNonBlocking));
    Stamp *st;
    CK(hipMalloc(&st, (size_t)n * WGMAX * sizeof(Stamp)));
    float4 *buf;
    const size_t dirtyMax = 80ull << 20;  // >= 1024 WG * 256 * per(<=16) * 16 B = 67 MB
    CK(hipMalloc(&buf, dirtyMax));
    Big big{};
    const double tu = tick_us();
    std::printf("wall clock tick %.4f us, n = %d launches per case\n", tu, n);

    show("trivial 256 WG", run(A, st, n, [&](int i) { k_triv<<<256, 256, 0, A>>>(st + (size_t)i * WGMAX); }));
    show("trivial 1024 WG", run(A, st, n, [&](int i) { k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX); }));
    show("trivial 2048 WG", run(A, st, n, [&](int i) { k_triv<<<2048, 256, 0, A>>>(st + (size_t)i * WGMAX); }));
    show("1024 WG, 38 KB LDS", run(A, st, n, [&](int i) { k_lds<<<1024, 256, 38 << 10, A>>>(st + (size_t)i * WGMAX, 0); }));
    show("1024 WG, 38 KB LDS, ~10 us work", run(A, st, n, [&](int i) { k_lds<<<1024, 256, 38 << 10, A>>>(st + (size_t)i * WGMAX, 3000); }));
    show("1024 WG, 1 KB kernarg", run(A, st, n, [&](int i) { k_big<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX, big); }));
    for (int per : {1, 4, 16}) {
        if ((size_t)1024 * 256 * per * 16 > dirtyMax) continue;
        char nm[96];
        std::snprintf(nm, sizeof nm, "1024 WG, %.1f MB dirty", 1024.0 * 256 * per * 16 / 1e6);
        show(nm, run(A, st, n, [&](int i) { k_dirty<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX, buf, per); }));
    }
    for (int per : {4, 16}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "1024 WG, %.1f MB dirty, non-temporal stores", 1024.0 * 256 * per * 16 / 1e6);
        show(nm, run(A, st, n, [&](int i) { k_dirty_nt<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX, buf, per); }));
    }
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipEvent_t evd;
    CK(hipEventCreateWithFlags(&evd, hipEventDisableTiming | hipEventReleaseToDevice));
    show("1024 WG + event record after each", run(A, st, n, [&](int i) {
        k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX);
        (void)hipEventRecord(ev, A);
    }));
    show("1024 WG + device-release event after each", run(A, st, n, [&](int i) {
        k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX);
        (void)hipEventRecord(evd, A);
    }));
    // the event carried by the launch itself (hipExtLaunchKernelGGL's stop
    // event: the dispatch packet's completion signal, no marker packet)
    show("1024 WG launched with a stop event", run(A, st, n, [&](int i) {
        hipExtLaunchKernelGGL(k_triv, dim3(1024), dim3(256), 0, A, nullptr, ev, 0, st + (size_t)i * WGMAX);
    }));
    show("1024 WG launched with a device-release stop event", run(A, st, n, [&](int i) {
        hipExtLaunchKernelGGL(k_triv, dim3(1024), dim3(256), 0, A, nullptr, evd, 0, st + (size_t)i * WGMAX);
    }));
    // a completed event of another stream waited on between launches (a join)
    k_triv<<<1, 64, 0, B>>>(st);
    CK(hipEventRecord(ev, B));
    CK(hipStreamSynchronize(B));
    show("1024 WG + wait on a completed foreign event each", run(A, st, n, [&](int i) {
        (void)hipStreamWaitEvent(A, ev, 0);
        k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX);
    }));
    // blocked barrier packets on other queues while A runs: B spins, C / D / E
    // wait on B's event (a barrier-AND packet at the head of their queues)
    hipStream_t E;
    CK(hipStreamCreateWithFlags(&E, hipStreamNonBlocking));
    const long long spin = (long long)(300000.0 / tu);  // 300 ms
    hipStream_t waiters[3] = {C, D, E};
    for (int rep = 0; rep < 2; rep++)
        for (int nb = 0; nb <= 3; nb++) {
            k_spin<<<1, 64, 0, B>>>(spin);
            hipEvent_t eb;
            CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
            CK(hipEventRecord(eb, B));
            for (int w = 0; w < nb; w++) {
                CK(hipStreamWaitEvent(waiters[w], eb, 0));
                k_triv<<<1, 64, 0, waiters[w]>>>(st);
            }
            char nm[96];
            std::snprintf(nm, sizeof nm, "1024 WG, spin on B, %d stream(s) blocked on it", nb);
            show(nm, run(A, st, n, [&](int i) { k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX); }));
            std::snprintf(nm, sizeof nm, "  ~10 us work kernels, %d blocked", nb);
            show(nm, run(A, st, n / 4, [&](int i) { k_lds<<<1024, 256, 38 << 10, A>>>(st + (size_t)i * WGMAX, 300); }));
            CK(hipDeviceSynchronize());
            CK(hipEventDestroy(eb));
        }
    {
        // the waits as spinning kernels instead (C and D each run a 1-wave poller)
        k_spin<<<1, 64, 0, B>>>(spin);
        k_spin<<<1, 64, 0, C>>>(spin);
        k_spin<<<1, 64, 0, D>>>(spin);
        show("1024 WG, three 1-wave spinners on B, C, D", run(A, st, n, [&](int i) { k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX); }));
        show("  ~10 us work kernels, three spinners", run(A, st, n / 4, [&](int i) { k_lds<<<1024, 256, 38 << 10, A>>>(st + (size_t)i * WGMAX, 300); }));
        CK(hipDeviceSynchronize());
    }
    show("trivial 1024 WG (again, end)", run(A, st, n, [&](int i) { k_triv<<<1024, 256, 0, A>>>(st + (size_t)i * WGMAX); }));
    CK(hipFree(st));
    CK(hipFree(buf));
    return 0;
}
