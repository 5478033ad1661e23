// mgmc_comm.hip -- the RCCL communicator of a handle: the end-of-run all-gather of every chain's
// (n, mean, M2), the bench's barrier and max-over-ranks time.
#include "mgmc_internal.hpp"

extern "C" {

#define NCCLCHK(h, call)                                                                     \
    do {                                                                                     \
        ncclResult_t r_ = (call);                                                            \
        if (r_ != ncclSuccess)                                                               \
            return fail(h, MGMC_E_HIP, std::string("RCCL error ") + ncclGetErrorString(r_) + " at " #call); \
    } while (0)

int mgmc_comm_unique_id(unsigned char out[MGMC_UNIQUE_ID_BYTES]) {
    if (!out) return fail(nullptr, MGMC_E_INVALID, "null argument");
    ncclUniqueId id;
    NCCLCHK(nullptr, ncclGetUniqueId(&id));
    memcpy(out, id.internal, MGMC_UNIQUE_ID_BYTES);
    return MGMC_OK;
}

int mgmc_comm_init(mgmc_handle* h, int nranks, int rank, const unsigned char id_bytes[MGMC_UNIQUE_ID_BYTES]) {
    if (!h || !id_bytes || nranks < 1 || rank < 0 || rank >= nranks) return fail(h, MGMC_E_INVALID, "invalid argument");
    HIPCHK(h, hipSetDevice(h->device));
    if (h->comm) {
        ncclCommDestroy(h->comm);
        h->comm = nullptr;
    }
    ncclUniqueId id;
    memcpy(id.internal, id_bytes, MGMC_UNIQUE_ID_BYTES);
    NCCLCHK(h, ncclCommInitRank(&h->comm, nranks, id, rank));
    h->nranks = nranks;
    h->rank = rank;
    if (h->comm_buf) HIPCHK(h, hipFree(h->comm_buf));
    HIPCHK(h, hipMalloc(&h->comm_buf, (size_t)(4 * nranks + 4) * h->nchains * sizeof(double)));
    return MGMC_OK;
}

int mgmc_comm_allgather_moments(mgmc_handle* h, double* out) {
    if (!h || !out) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    const int nch = h->nchains;
    if (!h->comm) {  // one rank: this handle's chains
        for (int c = 0; c < nch; ++c) {
            int rc = mgmc_qoi_moments_chain(h, c, out + 3 * c);
            if (rc) return rc;
        }
        return MGMC_OK;
    }
    // (count, mean, M2) of every chain packed to 3 doubles (the device moments are 4 apart), one
    // all-gather of 3 * nchains doubles per rank
    double* send = h->comm_buf + (size_t)4 * h->nranks * nch;
    HIPCHK(h, hipMemcpy2DAsync(send, 3 * sizeof(double), h->mom, 4 * sizeof(double), 3 * sizeof(double), nch,
                               hipMemcpyDeviceToDevice, h->stream));
    NCCLCHK(h, ncclAllGather(send, h->comm_buf, 3 * nch, ncclDouble, h->comm, h->stream));
    HIPCHK(h, hipMemcpyAsync(out, h->comm_buf, (size_t)3 * h->nranks * nch * sizeof(double), hipMemcpyDeviceToHost,
                             h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_comm_allreduce_max(mgmc_handle* h, double* value) {
    if (!h || !value) return fail(h, MGMC_E_INVALID, "null argument");
    if (!h->comm) return MGMC_OK;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemcpyAsync(h->comm_buf, value, sizeof(double), hipMemcpyHostToDevice, h->stream));
    NCCLCHK(h, ncclAllReduce(h->comm_buf, h->comm_buf, 1, ncclDouble, ncclMax, h->comm, h->stream));
    HIPCHK(h, hipMemcpyAsync(value, h->comm_buf, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_comm_barrier(mgmc_handle* h) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    HIPCHK(h, hipSetDevice(h->device));
    if (h->comm) NCCLCHK(h, ncclAllReduce(h->comm_buf, h->comm_buf, 1, ncclDouble, ncclSum, h->comm, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipDeviceSynchronize());
    return MGMC_OK;
}

int mgmc_comm_info(const mgmc_handle* h, int* rccl_ranks, int* rccl_rank, int* pci_bus_id) {
    if (!h || !rccl_ranks || !rccl_rank || !pci_bus_id) return fail(nullptr, MGMC_E_INVALID, "null argument");
    *rccl_ranks = 0;
    *rccl_rank = -1;
    if (h->comm) {
        NCCLCHK(const_cast<mgmc_handle*>(h), ncclCommCount(h->comm, rccl_ranks));
        NCCLCHK(const_cast<mgmc_handle*>(h), ncclCommUserRank(h->comm, rccl_rank));
    }
    if (hipDeviceGetAttribute(pci_bus_id, hipDeviceAttributePciBusId, h->device) != hipSuccess)
        return fail(const_cast<mgmc_handle*>(h), MGMC_E_HIP, "hipDeviceGetAttribute(PciBusId) failed");
    return MGMC_OK;
}

int mgmc_comm_destroy(mgmc_handle* h) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    if (h->comm) ncclCommDestroy(h->comm);
    h->comm = nullptr;
    h->nranks = 1;
    h->rank = 0;
    return MGMC_OK;
}

}  // extern "C"
