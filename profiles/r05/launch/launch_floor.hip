// Launch-floor probe (profiling only, not part of the library): back-to-back
// dependent launches on one stream, wall time per launch, for kernels that
// differ in what the library's short kernels have: an empty body, a large
// kernel-argument struct, a few global stores / atomics, 1 vs 256 blocks.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

struct Big { float f[100]; int i[20]; void *p[10]; };   // ~560 B of kernel arguments

__global__ void k_empty() {}
__global__ void k_bigarg(Big b) { if (b.i[0] == 12345 && threadIdx.x == 999) ((int *)b.p[0])[0] = 1; }
__global__ void k_store(int *p) { p[blockIdx.x * blockDim.x + threadIdx.x] = threadIdx.x; }
__global__ void k_atomic(int *p) { atomicAdd(&p[threadIdx.x & 15], 1); }
__global__ void k_load_store(const int *a, int *b) { int i = blockIdx.x * blockDim.x + threadIdx.x; b[i] = a[i] + 1; }

template <class F>
static double per_launch_us(hipStream_t s, int n, F launch) {
    for (int i = 0; i < 50; i++) launch();
    hipStreamSynchronize(s);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) launch();
    hipStreamSynchronize(s);
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int *buf, *buf2;
    hipMalloc(&buf, 1 << 24);
    hipMalloc(&buf2, 1 << 24);
    hipMemset(buf, 0, 1 << 24);
    Big big;
    memset(&big, 0, sizeof(big));
    big.p[0] = buf;
    const int n = 2000;
    for (int blocks : {1, 16, 256, 1024}) {
        printf("{\"blocks\": %d, \"empty\": %.2f, \"bigarg\": %.2f, \"store\": %.2f, \"atomic\": %.2f, \"load_store\": %.2f}\n",
               blocks,
               per_launch_us(s, n, [&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s); }),
               per_launch_us(s, n, [&] { hipLaunchKernelGGL(k_bigarg, dim3(blocks), dim3(256), 0, s, big); }),
               per_launch_us(s, n, [&] { hipLaunchKernelGGL(k_store, dim3(blocks), dim3(256), 0, s, buf); }),
               per_launch_us(s, n, [&] { hipLaunchKernelGGL(k_atomic, dim3(blocks), dim3(256), 0, s, buf); }),
               per_launch_us(s, n, [&] { hipLaunchKernelGGL(k_load_store, dim3(blocks), dim3(256), 0, s, buf, buf2); }));
        fflush(stdout);
    }
    // the same chain on two streams with an event join per launch (the tick's cross-stream pattern)
    hipStream_t s2;
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    double join = per_launch_us(s, n, [&] {
        hipLaunchKernelGGL(k_store, dim3(16), dim3(256), 0, s2, buf);
        hipEventRecord(ev, s2);
        hipStreamWaitEvent(s, ev, 0);
        hipLaunchKernelGGL(k_store, dim3(16), dim3(256), 0, s, buf2);
    });
    printf("{\"two_streams_join_pair_us\": %.2f}\n", join);
    return 0;
}
