// comm.cpp — RCCL communicator for the normal-equation all-reduce (see comm.h).
#include "comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "bf_runtime.h"

namespace bf {

#define BF_NCCL(call)                                                                                       \
    do {                                                                                                    \
        ncclResult_t r_ = (call);                                                                           \
        if (r_ != ncclSuccess)                                                                              \
            throw ::bf::Error(::bf::BF_ERR_INTERNAL, std::string(#call) + " failed: " + ncclGetErrorString(r_)); \
    } while (0)

static_assert(sizeof(ncclUniqueId) == Comm::kIdBytes, "RCCL unique id size");

void Comm::uniqueId(uint8_t* out) {
    ncclUniqueId id;
    BF_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, id.internal, kIdBytes);
}

Comm::Comm(const uint8_t* id, int nranks, int rank) : nranks_(nranks), rank_(rank) {
    BF_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, BF_ERR_ARG, "rank / nranks");
    ncclUniqueId u;
    std::memcpy(u.internal, id, kIdBytes);
    ncclComm_t c = nullptr;
    BF_NCCL(ncclCommInitRank(&c, nranks, u, rank));  // collective: every rank calls it with the same id
    comm_ = c;
}

Comm::~Comm() {
    if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void Comm::allreduceSum(double* buf, size_t n, hipStream_t stream) {
    if (n == 0) return;
    if (lb_) return loopbackCollective(buf, n, sizeof(double), 0, 0, stream);
    BF_NCCL(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, static_cast<ncclComm_t>(comm_), stream));
}

void Comm::checkError() const {
    if (lb_) return loopbackCheck();
    if (!comm_) return;
    ncclResult_t async = ncclSuccess;
    BF_NCCL(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &async));
    BF_REQUIRE(async == ncclSuccess, BF_ERR_INTERNAL, std::string("RCCL communicator error: ") + ncclGetErrorString(async));
}

void Comm::orderedLaunchBegin() {
    if (lb_) loopbackTurn(true);
}
void Comm::orderedLaunchEnd() {
    if (lb_) loopbackTurn(false);
}

void Comm::broadcast(float* buf, size_t n, int root, hipStream_t stream) {
    if (n == 0) return;
    if (lb_) {
        BF_REQUIRE(root >= 0 && root < nranks_, BF_ERR_ARG, "broadcast root");
        return loopbackCollective(buf, n, sizeof(float), 1, root, stream);
    }
    BF_NCCL(ncclBroadcast(buf, buf, n, ncclFloat, root, static_cast<ncclComm_t>(comm_), stream));
}

}  // namespace bf
