// lpe_transport.hip — transports of the x-slab decomposition: RCCL over xGMI
// (one process per GPU) and an in-process loopback group (tests: several
// ranks on one GPU, one host thread per rank).
#include "lpe_transport.h"
#include <rccl/rccl.h>
#include <atomic>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace lpe {

// ---------------------------------------------------------------------------
// RCCL: one grouped launch per exchange -- the ghost buffers with the two
// slab neighbours and the 16-byte bbox record to / from every other rank
// (an all-gather as point-to-point pairs: over xGMI every peer is one hop);
// all-reduces in place; everything on the context's stream.
struct RcclTransport : Transport {
    ncclComm_t comm = nullptr;
    ~RcclTransport() override {
        if (comm) ncclCommDestroy(comm);
    }
    int exchange(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR, size_t bytes,
                 int, int, float4 *bbAll) override {
        if (ncclGroupStart() != ncclSuccess) return LPE_ERR_HIP;
        ncclResult_t r = ncclSuccess;
        auto keep = [&r](ncclResult_t x) { if (r == ncclSuccess) r = x; };
        if (sendL && recvL && rank > 0) {
            keep(ncclSend(sendL, bytes, ncclChar, rank - 1, comm, ctx->stream));
            keep(ncclRecv(recvL, bytes, ncclChar, rank - 1, comm, ctx->stream));
        }
        if (sendR && recvR && rank < nranks - 1) {
            keep(ncclSend(sendR, bytes, ncclChar, rank + 1, comm, ctx->stream));
            keep(ncclRecv(recvR, bytes, ncclChar, rank + 1, comm, ctx->stream));
        }
        for (int q = 0; q < nranks; q++) {
            if (q == rank) continue;
            keep(ncclSend(bbAll + rank, sizeof(float4), ncclChar, q, comm, ctx->stream));
            keep(ncclRecv(bbAll + q, sizeof(float4), ncclChar, q, comm, ctx->stream));
        }
        const ncclResult_t e = ncclGroupEnd();     // always closes the group
        if (r != ncclSuccess || e != ncclSuccess) {
            ctx->err = std::string("RCCL slab exchange failed: ") + ncclGetErrorString(r != ncclSuccess ? r : e);
            return LPE_ERR_HIP;
        }
        return LPE_OK;
    }
    int allreduce_i64(lpe_ctx *ctx, long long *buf, int n) override {
        if (nranks == 1 || n <= 0) return LPE_OK;
        if (ncclAllReduce(buf, buf, (size_t)n, ncclInt64, ncclSum, comm, ctx->stream) != ncclSuccess) {
            ctx->err = "RCCL all-reduce (int64) failed";
            return LPE_ERR_HIP;
        }
        return LPE_OK;
    }
    int comm_ranks() override {
        int c = 0;
        return (comm && ncclCommCount(comm, &c) == ncclSuccess) ? c : 0;
    }
    int allreduce(lpe_ctx *ctx, float *buf, int n, int op) override {
        if (nranks == 1 || n <= 0) return LPE_OK;
        if (ncclAllReduce(buf, buf, (size_t)n, ncclFloat, op ? ncclMin : ncclSum, comm, ctx->stream) !=
            ncclSuccess) {
            ctx->err = "RCCL all-reduce failed";
            return LPE_ERR_HIP;
        }
        return LPE_OK;
    }
};

int transport_unique_id(char *id) {
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return LPE_ERR_HIP;
    static_assert(sizeof(u) <= 128, "ncclUniqueId fits 128 bytes");
    std::memset(id, 0, 128);
    std::memcpy(id, &u, sizeof(u));
    return LPE_OK;
}

Transport *transport_rccl(lpe_ctx *ctx, int nranks, int rank, const char *id, std::string &err) {
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    auto *t = new RcclTransport();
    t->rank = rank;
    t->nranks = nranks;
    (void)hipSetDevice(ctx->device);
    ncclResult_t r = ncclCommInitRank(&t->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        t->comm = nullptr;
        delete t;
        return nullptr;
    }
    return t;
}

// ---------------------------------------------------------------------------
// Loopback: the ranks are contexts of one process on one device, each driven
// by its own host thread.  An operation is stream-ordered like RCCL's: each
// rank records an event after its inputs, a host barrier publishes the
// events and buffers, each rank's stream waits for the others' events and a
// kernel on it reads their buffers directly; a second event + barrier
// orders every rank's later writes to its buffers after the others' reads.
// The host threads never wait for the device, so the GPU queue of every
// rank stays full (the round-3 loopback drained each stream per exchange).
static constexpr int LOOP_MAX = 64;
struct LoopSrc { const void *p[LOOP_MAX]; };

__global__ void k_loop_gather(const float *__restrict__ srcL, const float *__restrict__ srcR, float *__restrict__ dstL,
                              float *__restrict__ dstR, int hdr, int rec, int maxrec, LoopSrc bb, int nranks,
                              float4 *__restrict__ bbAll) {
    const int side = (int)(blockIdx.x & 1), part = (int)(blockIdx.x >> 1), parts = (int)(gridDim.x >> 1);
    const float *src = side ? srcR : srcL;
    float *dst = side ? dstR : dstL;
    if (blockIdx.x == 0 && (int)threadIdx.x < nranks)
        bbAll[threadIdx.x] = ((const float4 *)bb.p[threadIdx.x])[threadIdx.x];
    if (!src || !dst) return;
    const int cnt = min(max(*(const int *)src, 0), maxrec);
    const int words = hdr + cnt * rec;
    for (int i = part * (int)blockDim.x + (int)threadIdx.x; i < words; i += parts * (int)blockDim.x) dst[i] = src[i];
}

template <typename T>
__global__ void k_loop_reduce(T *__restrict__ buf, LoopSrc c, int nranks, int n, int op) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        T acc = ((const T *)c.p[0])[i];
        for (int r = 1; r < nranks; r++) {          // rank order: deterministic
            const T v = ((const T *)c.p[r])[i];
            if (op) acc = v < acc ? v : acc;
            else acc = (T)((unsigned long long)acc + (unsigned long long)v);   // (int64: wrap-around)
        }
        buf[i] = acc;
    }
}
template <>
__global__ void k_loop_reduce<float>(float *__restrict__ buf, LoopSrc c, int nranks, int n, int op) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        float acc = ((const float *)c.p[0])[i];
        for (int r = 1; r < nranks; r++) {
            const float v = ((const float *)c.p[r])[i];
            acc = op ? fminf(acc, v) : acc + v;
        }
        buf[i] = acc;
    }
}

struct LoopGroup {
    int n = 0;
    std::atomic<int> arrived{0};
    std::atomic<long> gen{0};
    std::atomic<bool> abort{false};
    std::vector<const void *> pL, pR;
    std::vector<float4 *> bb;
    std::vector<size_t> sz;
    std::vector<hipEvent_t> evReady, evDone;
    std::vector<void *> contrib;                  // all-reduce staging, per rank (device)
    std::vector<size_t> ccap;
    bool barrier() {
        const long g = gen.load(std::memory_order_acquire);
        if (arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == n) {
            arrived.store(0, std::memory_order_relaxed);
            gen.fetch_add(1, std::memory_order_release);
        } else {
            int spins = 0;
            while (gen.load(std::memory_order_acquire) == g) {
                if (abort.load(std::memory_order_relaxed)) return false;
                if (++spins > 256) std::this_thread::yield();
            }
        }
        return !abort.load(std::memory_order_relaxed);
    }
    void fail() { abort.store(true, std::memory_order_relaxed); }
};

struct LoopTransport : Transport {
    LoopGroup *g = nullptr;
    // record this rank's event, meet the others, order this stream after theirs
    int meet(lpe_ctx *ctx, std::vector<hipEvent_t> &ev) {
        if (hipEventRecord(ev[rank], ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (!g->barrier()) return LPE_ERR_STATE;
        for (int r = 0; r < nranks; r++)
            if (r != rank && hipStreamWaitEvent(ctx->stream, ev[r], 0) != hipSuccess) return LPE_ERR_HIP;
        return LPE_OK;
    }
    int exchange(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR, size_t bytes,
                 int hdr, int rec, float4 *bbAll) override {
        g->pL[rank] = sendL;
        g->pR[rank] = sendR;
        g->bb[rank] = bbAll;
        g->sz[rank] = bytes;
        int st = meet(ctx, g->evReady);
        if (st) return st;
        const float *srcL = recvL && rank > 0 ? (const float *)g->pR[rank - 1] : nullptr;
        const float *srcR = recvR && rank < nranks - 1 ? (const float *)g->pL[rank + 1] : nullptr;
        // a size that differs from the neighbour's send is a protocol error
        // (RCCL would hang or truncate): fail loudly
        if ((srcL && g->sz[rank - 1] != bytes) || (srcR && g->sz[rank + 1] != bytes)) {
            ctx->err = "loopback exchange: the wire size differs from a neighbour's";
            g->fail();
            return LPE_ERR_STATE;
        }
        LoopSrc src{};
        for (int r = 0; r < nranks; r++) src.p[r] = g->bb[r];
        const int maxrec = (int)((bytes / sizeof(float) - (size_t)hdr) / (size_t)std::max(rec, 1));
        hipLaunchKernelGGL(k_loop_gather, dim3(2 * 32), dim3(256), 0, ctx->stream, srcL, srcR, (float *)recvL,
                           (float *)recvR, hdr, rec, maxrec, src, nranks, bbAll);
        if (hipGetLastError() != hipSuccess) return LPE_ERR_HIP;
        return meet(ctx, g->evDone);        // (my buffers are rewritten only after everyone read them)
    }
    template <typename T>
    int reduce(lpe_ctx *ctx, T *buf, int n, int op) {
        if (nranks == 1 || n <= 0) return LPE_OK;
        const size_t B = sizeof(T) * (size_t)n;
        if (g->ccap[rank] < B) {
            if (g->contrib[rank]) (void)hipFree(g->contrib[rank]);
            g->contrib[rank] = nullptr;
            g->ccap[rank] = 0;
            if (hipMalloc(&g->contrib[rank], B) != hipSuccess) { g->fail(); return LPE_ERR_HIP; }
            g->ccap[rank] = B;
        }
        if (hipMemcpyAsync(g->contrib[rank], buf, B, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        int st = meet(ctx, g->evReady);
        if (st) return st;
        LoopSrc c{};
        for (int r = 0; r < nranks; r++) c.p[r] = g->contrib[r];
        hipLaunchKernelGGL(k_loop_reduce<T>, dim3(std::min(1024, (n + 255) / 256)), dim3(256), 0, ctx->stream, buf,
                           c, nranks, n, op);
        if (hipGetLastError() != hipSuccess) return LPE_ERR_HIP;
        return meet(ctx, g->evDone);
    }
    int allreduce(lpe_ctx *ctx, float *buf, int n, int op) override { return reduce<float>(ctx, buf, n, op); }
    int allreduce_i64(lpe_ctx *ctx, long long *buf, int n) override { return reduce<long long>(ctx, buf, n, 0); }
};

// ---------------------------------------------------------------------------
// Host-staged: the caller's callbacks (lpe_host_transport) move host copies of
// the buffers between processes -- e.g. torch.distributed over gloo.  Each
// operation drains the context's stream, stages device -> pinned host, calls
// the callback, and copies the result back.  Slow by construction; it exists
// so the cross-process protocol (both ends' sizes, the order of the calls)
// runs on hardware that has one GPU (RCCL refuses two ranks on one device).
// The exchange's bbox records travel as one MIN all-reduce.
struct HostTransport : Transport {
    lpe_host_transport cb{};
    std::vector<char *> pinned;            // [sendL, sendR, recvL, recvR, reduce]
    std::vector<size_t> pcap;
    ~HostTransport() override {
        for (char *p : pinned)
            if (p) (void)hipHostFree(p);
    }
    char *stage(lpe_ctx *ctx, int k, size_t bytes) {
        if (pcap[k] < bytes) {
            if (pinned[k]) (void)hipHostFree(pinned[k]);
            pinned[k] = nullptr;
            pcap[k] = 0;
            if (hipHostMalloc((void **)&pinned[k], std::max<size_t>(bytes, 64), 0) != hipSuccess) {
                ctx->err = "host transport: hipHostMalloc failed";
                return nullptr;
            }
            pcap[k] = std::max<size_t>(bytes, 64);
        }
        return pinned[k];
    }
    int callback_failed(lpe_ctx *ctx, const char *what, int rc) {
        ctx->err = std::string("host transport: ") + what + " callback returned " + std::to_string(rc) +
                   " (a size that differs from the neighbour's, or a failed peer)";
        return LPE_ERR_STATE;
    }
    int exchange(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR, size_t bytes,
                 int, int, float4 *bbAll) override {
        const bool L = sendL && recvL && rank > 0, R = sendR && recvR && rank < nranks - 1;
        char *hs[2] = {L ? stage(ctx, 0, bytes) : nullptr, R ? stage(ctx, 1, bytes) : nullptr};
        char *hr[2] = {L ? stage(ctx, 2, bytes) : nullptr, R ? stage(ctx, 3, bytes) : nullptr};
        if ((L && (!hs[0] || !hr[0])) || (R && (!hs[1] || !hr[1]))) return LPE_ERR_HIP;
        if (L && hipMemcpyAsync(hs[0], sendL, bytes, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (R && hipMemcpyAsync(hs[1], sendR, bytes, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        const int rc = cb.halo(cb.user, hs[0], L ? bytes : 0, hs[1], R ? bytes : 0, hr[0], L ? bytes : 0, hr[1],
                               R ? bytes : 0);
        if (rc) return callback_failed(ctx, "halo", rc);
        if (L && hipMemcpyAsync(recvL, hr[0], bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (R && hipMemcpyAsync(recvR, hr[1], bytes, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        // the bbox records: MIN of (minX, minY, -maxX, -maxY) over the ranks,
        // given to every slot (the unpack reduces them all)
        int st = reduce(ctx, (float *)(bbAll + rank), 4, "allreduce_f32",
                        [&](float *h) { return cb.allreduce_f32(cb.user, h, 4, 1); });
        if (st) return st;
        for (int q = 0; q < nranks; q++)
            if (q != rank && hipMemcpyAsync(bbAll + q, bbAll + rank, sizeof(float4), hipMemcpyDeviceToDevice,
                                            ctx->stream) != hipSuccess)
                return LPE_ERR_HIP;
        // the pinned staging buffers are reused by the next call
        return hipStreamSynchronize(ctx->stream) == hipSuccess ? LPE_OK : LPE_ERR_HIP;
    }
    template <class T, class F>
    int reduce(lpe_ctx *ctx, T *buf, int n, const char *what, F call) {
        if (nranks == 1 || n <= 0) return LPE_OK;
        T *h = (T *)stage(ctx, 4, sizeof(T) * (size_t)n);
        if (!h) return LPE_ERR_HIP;
        if (hipMemcpyAsync(h, buf, sizeof(T) * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        const int rc = call(h);
        if (rc) return callback_failed(ctx, what, rc);
        if (hipMemcpyAsync(buf, h, sizeof(T) * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        return LPE_OK;
    }
    int allreduce(lpe_ctx *ctx, float *buf, int n, int op) override {
        return reduce(ctx, buf, n, "allreduce_f32", [&](float *h) { return cb.allreduce_f32(cb.user, h, n, op); });
    }
    int allreduce_i64(lpe_ctx *ctx, long long *buf, int n) override {
        return reduce(ctx, buf, n, "allreduce_i64", [&](long long *h) { return cb.allreduce_i64(cb.user, h, n); });
    }
};

}  // namespace lpe

using namespace lpe;

extern "C" int lpe_mg_init_host(lpe_ctx *ctx, int nranks, int rank, const lpe_host_transport *t) {
    if (!ctx || !t || !t->halo || !t->allreduce_f32 || !t->allreduce_i64 || nranks < 1 || rank < 0 ||
        rank >= nranks)
        return LPE_ERR_ARG;
    if (ctx->transport) { delete ctx->transport; ctx->transport = nullptr; }
    auto *h = new HostTransport();
    h->cb = *t;
    h->rank = rank;
    h->nranks = nranks;
    h->pinned.assign(5, nullptr);
    h->pcap.assign(5, 0);
    ctx->transport = h;
    return LPE_OK;
}

extern "C" int lpe_mg_info(lpe_ctx *ctx, int *nranks, int *rank, int *comm_ranks) {
    if (!ctx) return LPE_ERR_ARG;
    const Transport *t = ctx->transport;
    if (nranks) *nranks = t ? t->nranks : 0;
    if (rank) *rank = t ? t->rank : 0;
    if (comm_ranks) *comm_ranks = t ? ctx->transport->comm_ranks() : 0;
    return LPE_OK;
}

extern "C" int lpe_mg_unique_id(char *id) {
    if (!id) return LPE_ERR_ARG;
    return transport_unique_id(id);
}

extern "C" int lpe_mg_init_rccl(lpe_ctx *ctx, int nranks, int rank, const char *id) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) return LPE_ERR_ARG;
    if (ctx->transport) { delete ctx->transport; ctx->transport = nullptr; }
    Transport *t = transport_rccl(ctx, nranks, rank, id, ctx->err);
    if (!t) return LPE_ERR_HIP;
    ctx->transport = t;
    return LPE_OK;
}

extern "C" int lpe_mg_loopback_run(int n, lpe_ctx **ctxs, const lpe_world_config *wc, double dt_tick,
                                   int nticks) {
    if (n < 1 || n > LOOP_MAX || !ctxs || nticks < 0) return LPE_ERR_ARG;
    for (int r = 0; r < n; r++) if (!ctxs[r]) return LPE_ERR_ARG;
    for (int r = 1; r < n; r++)
        if (ctxs[r]->device != ctxs[0]->device) {
            ctxs[r]->err = "lpe_mg_loopback_run: every rank on one device (its kernels read the others' buffers)";
            return LPE_ERR_ARG;
        }
    LoopGroup g;
    g.n = n;
    g.pL.assign(n, nullptr);
    g.pR.assign(n, nullptr);
    g.bb.assign(n, nullptr);
    g.sz.assign(n, 0);
    g.contrib.assign(n, nullptr);
    g.ccap.assign(n, 0);
    g.evReady.assign(n, nullptr);
    g.evDone.assign(n, nullptr);
    (void)hipSetDevice(ctxs[0]->device);
    int st0 = LPE_OK;
    for (int r = 0; r < n && !st0; r++)
        if (hipEventCreateWithFlags(&g.evReady[r], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g.evDone[r], hipEventDisableTiming) != hipSuccess)
            st0 = LPE_ERR_HIP;
    std::vector<Transport *> saved(n);
    for (int r = 0; r < n; r++) {
        auto *t = new LoopTransport();
        t->g = &g;
        t->rank = r;
        t->nranks = n;
        saved[r] = ctxs[r]->transport;
        ctxs[r]->transport = t;
    }
    std::vector<int> st(n, st0);
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++)
        th.emplace_back([&, r] {
            (void)hipSetDevice(ctxs[r]->device);
            for (int t = 0; t < nticks && st[r] == LPE_OK; t++)
                st[r] = wc ? lpe_world_tick(ctxs[r], wc, 1) : lpe_sph_step(ctxs[r], dt_tick);
            if (st[r] != LPE_OK) g.fail();       // release the ranks waiting on this one
        });
    for (auto &t : th) t.join();
    // every rank's work (and its reads of the others' buffers) is done before
    // the group's events and staging go away
    for (int r = 0; r < n; r++)
        if (hipStreamSynchronize(ctxs[r]->stream) != hipSuccess && st[r] == LPE_OK) st[r] = LPE_ERR_HIP;
    for (int r = 0; r < n; r++) {
        if (ctxs[r]->sph.pside) (void)hipStreamSynchronize(ctxs[r]->sph.pside);
        delete ctxs[r]->transport;
        ctxs[r]->transport = saved[r];
    }
    for (int r = 0; r < n; r++) {
        if (g.contrib[r]) (void)hipFree(g.contrib[r]);
        if (g.evReady[r]) (void)hipEventDestroy(g.evReady[r]);
        if (g.evDone[r]) (void)hipEventDestroy(g.evDone[r]);
    }
    for (int r = 0; r < n; r++) if (st[r] != LPE_OK) return st[r];
    return LPE_OK;
}
