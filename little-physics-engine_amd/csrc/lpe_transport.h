// lpe_transport.h — halo / collective transport of the x-slab decomposition
// (SURVEY.md §8(e)).  Not part of the ABI.
//
// A rank exchanges device buffers with its left (rank - 1) and right
// (rank + 1) slab neighbours, each direction sized by the receiver's request
// of the previous tick (lpe_sph.hip, sph_migrate) and joins small all-reduces (the 4-float
// global bbox every sub-step, the 3R rigid accumulators once per tick).
// Production: RCCL over xGMI, one process per GPU, ops enqueued on the
// context's stream (no host sync).  Tests: an in-process loopback group of
// contexts driven by one host thread each (several ranks on one GPU).
#pragma once
#include "lpe_internal.h"

namespace lpe {

struct Transport {
    int rank = 0, nranks = 1;
    virtual ~Transport() = default;
    // send sbL bytes of sendL to rank-1 / sbR of sendR to rank+1 and receive
    // rbL bytes from rank-1 into recvL / rbR from rank+1 into recvR (each
    // size equal to the matching send of the neighbour); absent neighbours
    // (nullptr buffers) are skipped
    virtual int halo(lpe_ctx *ctx, const void *sendL, const void *sendR, void *recvL, void *recvR,
                     size_t sbL, size_t sbR, size_t rbL, size_t rbR) = 0;
    // in-place all-reduce of n floats on the device; op 0 = sum, 1 = min
    virtual int allreduce(lpe_ctx *ctx, float *buf, int n, int op) = 0;
    // in-place SUM all-reduce of n int64 on the device (exact: the rigid
    // accumulators' fixed-point limbs)
    virtual int allreduce_i64(lpe_ctx *ctx, long long *buf, int n) = 0;
};

Transport *transport_rccl(lpe_ctx *ctx, int nranks, int rank, const char *id, std::string &err);
int transport_unique_id(char *id);

}  // namespace lpe
