// abi_comm.cpp -- RCCL fan-out / gather for channel-sharded multi-GPU runs (configs[4]).
// The data path has no reduction: channels are independent, so scatter and
// gather of contiguous channel blocks from one root are the only collectives.
#include <rccl/rccl.h>

#include <cstring>

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
int sdrgpu_comm_scatterv(sdrgpu_comm* c, const void* d_send, const size_t* bytes,
                         const size_t* displs, void* d_recv, int root, void* stream) {
    if (!c || !bytes || root < 0 || root >= c->nranks) return SDRGPU_ERR_INVALID;
    if (c->rank == root && (!d_send || !displs)) return SDRGPU_ERR_INVALID;
    if (bytes[c->rank] && !d_recv) return SDRGPU_ERR_INVALID;
    DeviceGuard g(c->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const char* src = static_cast<const char*>(d_send);
    int st = nccl_status(ncclGroupStart());
    if (st) return st;
    if (c->rank == root) {
        for (int r = 0; r < c->nranks; ++r)
            if (r != root && bytes[r])
                if ((st = nccl_status(ncclSend(src + displs[r], bytes[r], ncclUint8, r, c->comm, s))))
                    break;
    } else if (bytes[c->rank]) {
        st = nccl_status(ncclRecv(d_recv, bytes[c->rank], ncclUint8, root, c->comm, s));
    }
    const int end = nccl_status(ncclGroupEnd());
    if (st || end) return st ? st : end;
    if (c->rank == root && bytes[root])
        SDRGPU_HIP_TRY(hipMemcpyAsync(d_recv, src + displs[root], bytes[root],
                                      hipMemcpyDeviceToDevice, s));
    return SDRGPU_OK;
}

int sdrgpu_comm_gatherv(sdrgpu_comm* c, const void* d_send, void* d_recv, const size_t* bytes,
                        const size_t* displs, int root, void* stream) {
    if (!c || !bytes || root < 0 || root >= c->nranks) return SDRGPU_ERR_INVALID;
    if (c->rank == root && (!d_recv || !displs)) return SDRGPU_ERR_INVALID;
    if (bytes[c->rank] && !d_send) return SDRGPU_ERR_INVALID;
    DeviceGuard g(c->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    char* dst = static_cast<char*>(d_recv);
    int st = nccl_status(ncclGroupStart());
    if (st) return st;
    if (c->rank == root) {
        for (int r = 0; r < c->nranks; ++r)
            if (r != root && bytes[r])
                if ((st = nccl_status(ncclRecv(dst + displs[r], bytes[r], ncclUint8, r, c->comm, s))))
                    break;
    } else if (bytes[c->rank]) {
        st = nccl_status(ncclSend(d_send, bytes[c->rank], ncclUint8, root, c->comm, s));
    }
    const int end = nccl_status(ncclGroupEnd());
    if (st || end) return st ? st : end;
    if (c->rank == root && bytes[root])
        SDRGPU_HIP_TRY(hipMemcpyAsync(dst + displs[root], d_send, bytes[root],
                                      hipMemcpyDeviceToDevice, s));
    return SDRGPU_OK;
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
