// lpe_transport.h — exchange / collective transport of the x-slab
// decomposition.  Not part of the ABI.
//
// Per sub-step a slab rank exchanges one fixed-size wire buffer with each of
// its two neighbours (the ghost records, lpe_sph.hip) and every rank's bbox
// record; per tick it joins an all-reduce of the rigid accumulators (int64)
// and, when re-balancing, one of a column histogram (float).  Everything is
// stream-ordered on the context's stream (no host synchronisation):
// production is RCCL over xGMI (one process per GPU, one grouped p2p launch
// per exchange); tests use an in-process group of contexts on one GPU (one
// host thread per rank, device copies ordered by events) or a host-staged
// transport whose callbacks move the buffers between processes.
#pragma once
#include "lpe_internal.h"

namespace lpe {

struct Transport {
    int rank = 0, nranks = 1;
    virtual ~Transport() = default;
    // One sub-step's exchange: `bytes` of sendL to rank - 1 and of sendR to
    // rank + 1, the neighbours' into recvL / recvR (null where there is no
    // neighbour; both ends use the same size).  A buffer's first int is its
    // record count; a transport may move only hdr + count * rec floats.
    // bbAll[rank] is this rank's bbox record; afterwards bbAll[r] holds rank
    // r's for every r.
    virtual int exchange(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR,
                         size_t bytes, int hdr, int rec, float4 *bbAll) = 0;
    // in-place all-reduce of n floats on the device; op 0 = sum, 1 = min
    virtual int allreduce(lpe_ctx *ctx, float *buf, int n, int op) = 0;
    // in-place SUM all-reduce of n int64 on the device (exact: the rigid
    // accumulators' fixed-point limbs; two's-complement wrap-around)
    virtual int allreduce_i64(lpe_ctx *ctx, long long *buf, int n) = 0;
    // ranks the underlying communicator reports (RCCL: ncclCommCount)
    virtual int comm_ranks() { return nranks; }
};

Transport *transport_rccl(lpe_ctx *ctx, int nranks, int rank, const char *id, std::string &err);
int transport_unique_id(char *id);

}  // namespace lpe
