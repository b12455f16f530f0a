// comm.cpp — RCCL communicator for the normal-equation all-reduce (see comm.h).
#include "comm.h"

#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
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

struct Loopback {
    int nranks = 1, timeoutMs = 60000;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<std::vector<unsigned char>> slot;  // per rank: its contribution of the current collective
    // every rank of the group waits here; a rank that never arrives fails the others after timeoutMs
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        if (++arrived == nranks) {
            arrived = 0;
            generation++;
            cv.notify_all();
            return;
        }
        if (!cv.wait_for(lk, std::chrono::milliseconds(timeoutMs), [&] { return generation != gen; }))
            throw Error(BF_ERR_INTERNAL, "loopback communicator: a rank did not reach the collective "
                                         "(ranks issued different collective sequences)");
    }
};

std::shared_ptr<Loopback> Comm::loopbackGroup(int nranks, int timeoutMs) {
    BF_REQUIRE(nranks >= 1, BF_ERR_ARG, "nranks");
    auto g = std::make_shared<Loopback>();
    g->nranks = nranks;
    g->timeoutMs = timeoutMs > 0 ? timeoutMs : 60000;
    g->slot.resize((size_t)nranks);
    return g;
}

Comm::Comm(std::shared_ptr<Loopback> group, int rank) : lb_(std::move(group)), nranks_(lb_ ? lb_->nranks : 1), rank_(rank) {
    BF_REQUIRE(lb_ && rank >= 0 && rank < nranks_, BF_ERR_ARG, "loopback rank");
}

void Comm::allreduceSum(double* buf, size_t n, hipStream_t stream) {
    if (n == 0) return;
    if (lb_) {
        BF_HIP(hipStreamSynchronize(stream));  // this rank's contribution is complete
        std::vector<unsigned char>& mine = lb_->slot[(size_t)rank_];
        mine.resize(n * sizeof(double));
        BF_HIP(hipMemcpy(mine.data(), buf, n * sizeof(double), hipMemcpyDeviceToHost));
        lb_->barrier();
        std::vector<double> sum(n, 0.0);
        for (int r = 0; r < nranks_; r++) {  // rank order
            BF_REQUIRE(lb_->slot[(size_t)r].size() == n * sizeof(double), BF_ERR_INTERNAL,
                       "loopback all-reduce: ranks passed different counts");
            const double* v = reinterpret_cast<const double*>(lb_->slot[(size_t)r].data());
            for (size_t i = 0; i < n; i++) sum[i] += v[i];
        }
        lb_->barrier();  // every rank has read every slot before the next collective refills them
        BF_HIP(hipMemcpy(buf, sum.data(), n * sizeof(double), hipMemcpyHostToDevice));
        return;
    }
    BF_NCCL(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, static_cast<ncclComm_t>(comm_), stream));
}

void Comm::broadcast(float* buf, size_t n, int root, hipStream_t stream) {
    if (n == 0) return;
    if (lb_) {
        BF_REQUIRE(root >= 0 && root < nranks_, BF_ERR_ARG, "broadcast root");
        BF_HIP(hipStreamSynchronize(stream));
        std::vector<unsigned char>& rs = lb_->slot[(size_t)root];
        if (rank_ == root) {
            rs.resize(n * sizeof(float));
            BF_HIP(hipMemcpy(rs.data(), buf, n * sizeof(float), hipMemcpyDeviceToHost));
        }
        lb_->barrier();
        if (rank_ != root) {
            BF_REQUIRE(rs.size() == n * sizeof(float), BF_ERR_INTERNAL, "loopback broadcast: ranks passed different counts");
            BF_HIP(hipMemcpy(buf, rs.data(), n * sizeof(float), hipMemcpyHostToDevice));
        }
        lb_->barrier();
        return;
    }
    BF_NCCL(ncclBroadcast(buf, buf, n, ncclFloat, root, static_cast<ncclComm_t>(comm_), stream));
}

}  // namespace bf
