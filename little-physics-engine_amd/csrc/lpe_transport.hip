// lpe_transport.hip — transports of the x-slab decomposition: RCCL over xGMI
// (one process per GPU) and an in-process loopback group (tests: several
// ranks on one GPU, one host thread per rank).
#include "lpe_transport.h"
#include <rccl/rccl.h>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace lpe {

// ---------------------------------------------------------------------------
// RCCL: grouped send/recv with the two slab neighbours, all-reduce in place;
// everything is enqueued on the context's stream.
struct RcclTransport : Transport {
    ncclComm_t comm = nullptr;
    ~RcclTransport() override {
        if (comm) ncclCommDestroy(comm);
    }
    int halo(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR,
             size_t sbL, size_t sbR, size_t rbL, size_t rbR) override {
        if (ncclGroupStart() != ncclSuccess) return LPE_ERR_HIP;
        ncclResult_t r = ncclSuccess;
        auto keep = [&r](ncclResult_t x) { if (r == ncclSuccess) r = x; };
        if (sendL && recvL && rank > 0) {
            keep(ncclSend(sendL, sbL, ncclChar, rank - 1, comm, ctx->stream));
            keep(ncclRecv(recvL, rbL, ncclChar, rank - 1, comm, ctx->stream));
        }
        if (sendR && recvR && rank < nranks - 1) {
            keep(ncclSend(sendR, sbR, ncclChar, rank + 1, comm, ctx->stream));
            keep(ncclRecv(recvR, rbR, ncclChar, rank + 1, comm, ctx->stream));
        }
        const ncclResult_t e = ncclGroupEnd();     // always closes the group
        if (r != ncclSuccess || e != ncclSuccess) {
            ctx->err = std::string("RCCL halo exchange failed: ") +
                       ncclGetErrorString(r != ncclSuccess ? r : e);
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
// Loopback: the ranks are contexts of one process, each driven by its own
// host thread; an exchange is a barrier, device-to-device copies from the
// neighbours' send buffers, and a second barrier (so no send buffer is
// rewritten before every neighbour has copied it).
struct LoopGroup {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long gen = 0;
    bool abort = false;          // a rank failed: every barrier returns at once
    std::vector<const void *> pL, pR;
    std::vector<size_t> szL, szR;          // the send sizes of each rank (checked by the receivers)
    std::vector<std::vector<float>> red;
    std::vector<std::vector<long long>> redi;
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (abort) return false;
        long g = gen;
        if (++arrived == n) {
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || abort; });
        }
        return !abort;
    }
    void fail() {
        std::lock_guard<std::mutex> lk(mu);
        abort = true;
        cv.notify_all();
    }
};

struct LoopTransport : Transport {
    LoopGroup *g = nullptr;
    int halo(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR,
             size_t sbL, size_t sbR, size_t rbL, size_t rbR) override {
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        g->pL[rank] = sendL;
        g->pR[rank] = sendR;
        g->szL[rank] = sbL;
        g->szR[rank] = sbR;
        if (!g->barrier()) return LPE_ERR_STATE;
        // the copies run on this rank's stream and are complete before the
        // second barrier: the sender may then reuse its buffers, and this
        // rank's unpack (same stream) sees the data.  A size that differs
        // from the neighbour's send is a protocol error (RCCL would hang or
        // truncate): fail loudly.
        int st = LPE_OK;
        if (recvL && rank > 0 && g->pR[rank - 1]) {
            if (g->szR[rank - 1] != rbL) {
                ctx->err = "loopback halo: receive size differs from the left neighbour's send";
                st = LPE_ERR_STATE;
            } else if (hipMemcpyAsync(recvL, g->pR[rank - 1], rbL, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess)
                st = LPE_ERR_HIP;
        }
        if (recvR && rank < nranks - 1 && g->pL[rank + 1]) {
            if (g->szL[rank + 1] != rbR) {
                ctx->err = "loopback halo: receive size differs from the right neighbour's send";
                st = LPE_ERR_STATE;
            } else if (hipMemcpyAsync(recvR, g->pL[rank + 1], rbR, hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess)
                st = LPE_ERR_HIP;
        }
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) st = LPE_ERR_HIP;
        if (!g->barrier()) return LPE_ERR_STATE;
        return st;
    }
    int allreduce(lpe_ctx *ctx, float *buf, int n, int op) override {
        if (nranks == 1 || n <= 0) return LPE_OK;
        std::vector<float> &mine = g->red[rank];
        mine.resize(n);
        if (hipMemcpyAsync(mine.data(), buf, sizeof(float) * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        if (!g->barrier()) return LPE_ERR_STATE;
        std::vector<float> acc(g->red[0]);             // rank order: deterministic
        for (int r = 1; r < nranks; r++)
            for (int i = 0; i < n; i++)
                acc[i] = op ? (g->red[r][i] < acc[i] ? g->red[r][i] : acc[i]) : acc[i] + g->red[r][i];
        if (!g->barrier()) return LPE_ERR_STATE;
        if (hipMemcpyAsync(buf, acc.data(), sizeof(float) * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        return LPE_OK;
    }
    int allreduce_i64(lpe_ctx *ctx, long long *buf, int n) override {
        if (nranks == 1 || n <= 0) return LPE_OK;
        std::vector<long long> &mine = g->redi[rank];
        mine.resize(n);
        if (hipMemcpyAsync(mine.data(), buf, sizeof(long long) * n, hipMemcpyDeviceToHost, ctx->stream) !=
                hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        if (!g->barrier()) return LPE_ERR_STATE;
        std::vector<long long> acc(g->redi[0]);
        for (int r = 1; r < nranks; r++)
            for (int i = 0; i < n; i++)     // two's complement wrap-around, as the device limbs
                acc[i] = (long long)((unsigned long long)acc[i] + (unsigned long long)g->redi[r][i]);
        if (!g->barrier()) return LPE_ERR_STATE;
        if (hipMemcpyAsync(buf, acc.data(), sizeof(long long) * n, hipMemcpyHostToDevice, ctx->stream) !=
                hipSuccess ||
            hipStreamSynchronize(ctx->stream) != hipSuccess)
            return LPE_ERR_HIP;
        return LPE_OK;
    }
};

// ---------------------------------------------------------------------------
// Host-staged: the caller's callbacks (lpe_host_transport) move host copies of
// the buffers between processes -- e.g. torch.distributed over gloo.  Each
// operation drains the context's stream, stages device -> pinned host, calls
// the callback, and copies the result back.  Slow by construction; it exists
// so the cross-process protocol (both ends' sizes, the order of the calls)
// runs on hardware that has one GPU (RCCL refuses two ranks on one device).
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
    int halo(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR,
             size_t sbL, size_t sbR, size_t rbL, size_t rbR) override {
        const bool L = sendL && recvL && rank > 0, R = sendR && recvR && rank < nranks - 1;
        char *hs[2] = {L ? stage(ctx, 0, sbL) : nullptr, R ? stage(ctx, 1, sbR) : nullptr};
        char *hr[2] = {L ? stage(ctx, 2, rbL) : nullptr, R ? stage(ctx, 3, rbR) : nullptr};
        if ((L && (!hs[0] || !hr[0])) || (R && (!hs[1] || !hr[1]))) return LPE_ERR_HIP;
        if (L && hipMemcpyAsync(hs[0], sendL, sbL, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (R && hipMemcpyAsync(hs[1], sendR, sbR, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        const int rc = cb.halo(cb.user, hs[0], L ? sbL : 0, hs[1], R ? sbR : 0, hr[0], L ? rbL : 0, hr[1],
                               R ? rbR : 0);
        if (rc) return callback_failed(ctx, "halo", rc);
        if (L && hipMemcpyAsync(recvL, hr[0], rbL, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
        if (R && hipMemcpyAsync(recvR, hr[1], rbR, hipMemcpyHostToDevice, ctx->stream) != hipSuccess) return LPE_ERR_HIP;
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
    if (n < 1 || !ctxs || nticks < 0) return LPE_ERR_ARG;
    for (int r = 0; r < n; r++) if (!ctxs[r]) return LPE_ERR_ARG;
    LoopGroup g;
    g.n = n;
    g.pL.assign(n, nullptr);
    g.szL.assign(n, 0);
    g.szR.assign(n, 0);
    g.pR.assign(n, nullptr);
    g.red.resize(n);
    g.redi.resize(n);
    std::vector<Transport *> saved(n);
    for (int r = 0; r < n; r++) {
        auto *t = new LoopTransport();
        t->g = &g;
        t->rank = r;
        t->nranks = n;
        saved[r] = ctxs[r]->transport;
        ctxs[r]->transport = t;
    }
    std::vector<int> st(n, LPE_OK);
    std::vector<std::thread> th;
    for (int r = 0; r < n; r++)
        th.emplace_back([&, r] {
            (void)hipSetDevice(ctxs[r]->device);
            for (int t = 0; t < nticks && st[r] == LPE_OK; t++)
                st[r] = wc ? lpe_world_tick(ctxs[r], wc, 1) : lpe_sph_step(ctxs[r], dt_tick);
            if (st[r] == LPE_OK && hipStreamSynchronize(ctxs[r]->stream) != hipSuccess) st[r] = LPE_ERR_HIP;
            if (st[r] != LPE_OK) g.fail();       // release the ranks waiting on this one
        });
    for (auto &t : th) t.join();
    for (int r = 0; r < n; r++) {
        delete ctxs[r]->transport;
        ctxs[r]->transport = saved[r];
    }
    for (int r = 0; r < n; r++) if (st[r] != LPE_OK) return st[r];
    return LPE_OK;
}
