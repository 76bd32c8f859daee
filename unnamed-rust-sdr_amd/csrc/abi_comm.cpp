// abi_comm.cpp -- RCCL fan-out / gather for channel-sharded multi-GPU runs (configs[4]).
// The data path has no reduction: channels are independent, so scatter and
// gather of contiguous channel blocks from one root are the only collectives.
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

#include "abi_common.hpp"

using namespace sdrgpu::detail;

struct sdrgpu_comm {
    int device = 0;
    int nranks = 1, rank = 0;
    ncclComm_t comm = nullptr;
    float* d_one = nullptr;  // 1-float scratch for the barrier all-reduce
};

static int nccl_status(ncclResult_t r) {
    if (r == ncclSuccess) return SDRGPU_OK;
    if (r == ncclInvalidArgument || r == ncclInvalidUsage) return SDRGPU_ERR_INVALID;
    return SDRGPU_ERR_DEVICE;
}

extern "C" {

int sdrgpu_comm_unique_id(void* id_out) {
    if (!id_out) return SDRGPU_ERR_INVALID;
    static_assert(sizeof(ncclUniqueId) == SDRGPU_COMM_ID_BYTES, "id size");
    ncclUniqueId id;
    int st = nccl_status(ncclGetUniqueId(&id));
    if (st) return st;
    std::memcpy(id_out, &id, sizeof(id));
    return SDRGPU_OK;
}

int sdrgpu_comm_init(int device, int nranks, int rank, const void* id, sdrgpu_comm** out) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return SDRGPU_ERR_INVALID;
    *out = nullptr;
    int st = check_device(device);
    if (st) return st;
    DeviceGuard g(device);
    if (!g.ok()) return SDRGPU_ERR_DEVICE;
    auto* c = new (std::nothrow) sdrgpu_comm();
    if (!c) return SDRGPU_ERR_NOMEM;
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    st = nccl_status(ncclCommInitRank(&c->comm, nranks, uid, rank));
    if (!st && hipMalloc(&c->d_one, sizeof(float)) != hipSuccess) st = SDRGPU_ERR_NOMEM;
    if (st) {
        if (c->comm) ncclCommDestroy(c->comm);
        delete c;
        return st;
    }
    *out = c;
    return SDRGPU_OK;
}

int sdrgpu_comm_scatter(sdrgpu_comm* c, const void* d_send, void* d_recv, size_t bytes_per_rank,
                        int root, void* stream) {
    if (!c || !d_recv || root < 0 || root >= c->nranks || (c->rank == root && !d_send))
        return SDRGPU_ERR_INVALID;
    DeviceGuard g(c->device);
    return nccl_status(ncclScatter(d_send, d_recv, bytes_per_rank, ncclUint8, root, c->comm,
                                   static_cast<hipStream_t>(stream)));
}

int sdrgpu_comm_gather(sdrgpu_comm* c, const void* d_send, void* d_recv, size_t bytes_per_rank,
                       int root, void* stream) {
    if (!c || !d_send || root < 0 || root >= c->nranks || (c->rank == root && !d_recv))
        return SDRGPU_ERR_INVALID;
    DeviceGuard g(c->device);
    return nccl_status(ncclGather(d_send, d_recv, bytes_per_rank, ncclUint8, root, c->comm,
                                  static_cast<hipStream_t>(stream)));
}

// Uneven blocks (nch % nranks != 0): point-to-point sends from / to the root inside one
// RCCL group (every link of the root's xGMI fan-out is driven at once); the root's own
// block is a device-local copy.  bytes / displs: nranks host entries, identical on all ranks.
// sdrgpu_comm_plan_v is the whole decision (which ops, which peers, which offsets); the two
// collectives only execute its ops, so the CPU suite checks every split through the plan.
int sdrgpu_comm_plan_v(int nranks, int rank, int root, int gather, const size_t* bytes,
                       const size_t* displs, sdrgpu_comm_op* ops, int max_ops, int* n_ops) {
    if (!n_ops || !bytes || nranks < 1 || rank < 0 || rank >= nranks || root < 0 ||
        root >= nranks || (rank == root && !displs) || (ops && max_ops < 0))
        return SDRGPU_ERR_INVALID;
    int n = 0;
    auto add = [&](int kind, int peer, size_t off, size_t nb) {
        if (ops && n < max_ops) ops[n] = sdrgpu_comm_op{kind, peer, off, nb};
        ++n;
    };
    if (rank == root) {
        for (int r = 0; r < nranks; ++r)
            if (r != root && bytes[r])
                add(gather ? SDRGPU_COMM_RECV : SDRGPU_COMM_SEND, r, displs[r], bytes[r]);
        if (bytes[root]) add(SDRGPU_COMM_COPY, root, displs[root], bytes[root]);
    } else if (bytes[rank]) {
        add(gather ? SDRGPU_COMM_SEND : SDRGPU_COMM_RECV, root, 0, bytes[rank]);
    }
    *n_ops = n;
    return (ops && n > max_ops) ? SDRGPU_ERR_INVALID : SDRGPU_OK;
}

// Execute the plan: `root_buf` is the root's packed buffer (d_send of scatterv, d_recv of
// gatherv), `own` this rank's own block (d_recv of scatterv, d_send of gatherv).
static int comm_run_v(sdrgpu_comm* c, int gather, const void* root_buf_c, const void* own_c,
                      const size_t* bytes, const size_t* displs, int root, void* stream) {
    if (!c || !bytes || root < 0 || root >= c->nranks) return SDRGPU_ERR_INVALID;
    if (c->rank == root && (!root_buf_c || !displs)) return SDRGPU_ERR_INVALID;
    if (bytes[c->rank] && !own_c) return SDRGPU_ERR_INVALID;
    char* root_buf = const_cast<char*>(static_cast<const char*>(root_buf_c));
    char* own = const_cast<char*>(static_cast<const char*>(own_c));
    int n = 0;
    int st = sdrgpu_comm_plan_v(c->nranks, c->rank, root, gather, bytes, displs, nullptr, 0, &n);
    if (st) return st;
    std::vector<sdrgpu_comm_op> ops(n);
    if ((st = sdrgpu_comm_plan_v(c->nranks, c->rank, root, gather, bytes, displs, ops.data(), n, &n)))
        return st;
    DeviceGuard g(c->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if ((st = nccl_status(ncclGroupStart()))) return st;
    for (const auto& op : ops) {
        char* p = c->rank == root ? root_buf + op.offset : own;
        if (op.kind == SDRGPU_COMM_SEND)
            st = nccl_status(ncclSend(p, op.bytes, ncclUint8, op.peer, c->comm, s));
        else if (op.kind == SDRGPU_COMM_RECV)
            st = nccl_status(ncclRecv(p, op.bytes, ncclUint8, op.peer, c->comm, s));
        if (st) break;
    }
    const int end = nccl_status(ncclGroupEnd());
    if (st || end) return st ? st : end;
    for (const auto& op : ops)
        if (op.kind == SDRGPU_COMM_COPY)
            SDRGPU_HIP_TRY(hipMemcpyAsync(gather ? root_buf + op.offset : own,
                                          gather ? own : root_buf + op.offset, op.bytes,
                                          hipMemcpyDeviceToDevice, s));
    return SDRGPU_OK;
}

int sdrgpu_comm_scatterv(sdrgpu_comm* c, const void* d_send, const size_t* bytes,
                         const size_t* displs, void* d_recv, int root, void* stream) {
    return comm_run_v(c, 0, d_send, d_recv, bytes, displs, root, stream);
}

int sdrgpu_comm_gatherv(sdrgpu_comm* c, const void* d_send, void* d_recv, const size_t* bytes,
                        const size_t* displs, int root, void* stream) {
    return comm_run_v(c, 1, d_recv, d_send, bytes, displs, root, stream);
}

int sdrgpu_comm_barrier(sdrgpu_comm* c, void* stream) {
    if (!c) return SDRGPU_ERR_INVALID;
    DeviceGuard g(c->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    int st = nccl_status(ncclAllReduce(c->d_one, c->d_one, 1, ncclFloat32, ncclSum, c->comm, s));
    if (st) return st;
    SDRGPU_HIP_TRY(hipStreamSynchronize(s));
    return SDRGPU_OK;
}

void sdrgpu_comm_destroy(sdrgpu_comm* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->d_one) (void)hipFree(c->d_one);
    delete c;
}

}  // extern "C"
