// rccl_stub.cpp -- TEST INFRASTRUCTURE ONLY (tests/test_multi_cpu.py): the RCCL calls
// rsm_multi.cpp makes, over host memory, so the multi-GPU exchange of the C ABI
// runs at G > 1 on a machine without GPUs.  A clique of G communicators (one per
// host "device") from ncclCommInitAll; collectives are only accepted inside a
// group (as rsm_multi.cpp issues them: one group over all G ranks) and execute at
// ncclGroupEnd with RCCL's semantics:
//   ncclAllGather(send, recv, count): recv of rank g = concatenation over ranks h
//     of send_h (count bytes each, rank order); in place when send = recv + g*count;
//   ncclSend(buf, count, peer) / ncclRecv(buf, count, peer): matched pairwise
//     (g sends to h <-> h receives from g, equal counts).
// Any mismatch (a rank missing from an all-gather, unequal counts, an unmatched
// send or recv, a call outside a group) fails the group with ncclInvalidUsage.
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <vector>

struct ncclComm {
    int rank, n, clique;
};

namespace {
struct Op {
    int kind;  // 0 all-gather, 1 send, 2 recv
    ncclComm_t comm;
    const void* send;
    void* recv;
    size_t count;
    int peer;
};
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;
std::mutex g_mu;
int g_cliques = 0;

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        default: return 8;
    }
}

ncclResult_t run_group(std::vector<Op>& ops) {
    // all-gathers, per clique: every rank exactly once, equal counts
    std::vector<Op*> ag;
    for (auto& o : ops)
        if (o.kind == 0) ag.push_back(&o);
    if (!ag.empty()) {
        const int n = ag[0]->comm->n, cl = ag[0]->comm->clique;
        std::vector<Op*> by_rank(n, nullptr);
        for (Op* o : ag) {
            if (o->comm->clique != cl || o->count != ag[0]->count || by_rank[o->comm->rank]) return ncclInvalidUsage;
            by_rank[o->comm->rank] = o;
        }
        for (Op* o : by_rank)
            if (!o) return ncclInvalidUsage;
        // snapshot every rank's send block first (in place: send aliases recv)
        std::vector<std::vector<unsigned char>> blk(n);
        for (int h = 0; h < n; ++h) {
            const unsigned char* s = static_cast<const unsigned char*>(by_rank[h]->send);
            blk[h].assign(s, s + by_rank[h]->count);
        }
        for (int g = 0; g < n; ++g)
            for (int h = 0; h < n; ++h)
                memcpy(static_cast<unsigned char*>(by_rank[g]->recv) + (size_t)h * by_rank[g]->count, blk[h].data(),
                       by_rank[g]->count);
    }
    // point-to-point: each send (g -> h) matches exactly one recv (h <- g)
    std::vector<char> used(ops.size(), 0);
    for (size_t i = 0; i < ops.size(); ++i) {
        if (ops[i].kind != 1) continue;
        const Op& s = ops[i];
        size_t j = ops.size();
        for (size_t c = 0; c < ops.size(); ++c)
            if (!used[c] && ops[c].kind == 2 && ops[c].comm->clique == s.comm->clique &&
                ops[c].comm->rank == s.peer && ops[c].peer == s.comm->rank && ops[c].count == s.count) {
                j = c;
                break;
            }
        if (j == ops.size()) return ncclInvalidUsage;
        used[i] = used[j] = 1;
        memcpy(ops[j].recv, s.send, s.count);
    }
    for (size_t c = 0; c < ops.size(); ++c)
        if (ops[c].kind == 2 && !used[c]) return ncclInvalidUsage;
    return ncclSuccess;
}

ncclResult_t enqueue(const Op& o) {
    if (t_depth == 0) return ncclInvalidUsage;  // rsm_multi.cpp groups every collective
    t_ops.push_back(o);
    return ncclSuccess;
}
}  // namespace

extern "C" {
ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    if (!comms || ndev <= 0 || !devlist) return ncclInvalidArgument;
    int cl;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        cl = g_cliques++;
    }
    for (int g = 0; g < ndev; ++g) comms[g] = new ncclComm{g, ndev, cl};
    return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "success" : "stub: invalid usage"; }
ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
    if (t_depth == 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_group(ops);
}
ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t) {
    return enqueue(Op{0, comm, send, recv, count * type_bytes(t), -1});
}
ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t) {
    return enqueue(Op{1, comm, buf, nullptr, count * type_bytes(t), peer});
}
ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t) {
    return enqueue(Op{2, comm, nullptr, buf, count * type_bytes(t), peer});
}
}
