// comm.h — the one data-path collective of the multi-GPU build: the sum all-reduce of the global
// bundle adjuster's normal equations over RCCL (xGMI), once per Gauss-Newton iteration
// (SURVEY.md §8(e)3). One process per GPU; rank 0 draws the RCCL unique id, the host side hands it
// to the other ranks over its own channel (torch.distributed / gloo in bench.py), every rank then
// creates its communicator with bf_comm_create.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>

namespace bf {

struct Loopback;

class Comm {
public:
    static constexpr size_t kIdBytes = 128;  // NCCL_UNIQUE_ID_BYTES
    static void uniqueId(uint8_t* out);
    Comm(const uint8_t* id, int nranks, int rank);
    // In-process loopback group (tests): nranks communicators in one process, each rank driven from its
    // own host thread (ranks may share a GPU). A collective synchronizes the calling rank's stream,
    // exchanges through host memory behind a barrier (a rank that never arrives fails it after
    // timeoutMs instead of hanging) and sums in rank order, so the call sites of the multi-rank path
    // run without one GPU per rank; RCCL itself is not exercised.
    static std::shared_ptr<Loopback> loopbackGroup(int nranks, int timeoutMs);
    Comm(std::shared_ptr<Loopback> group, int rank);
    ~Comm();
    int size() const { return nranks_; }
    int rank() const { return rank_; }
    // in-place sum over ranks of n doubles, enqueued on stream (no host synchronisation)
    void allreduceSum(double* buf, size_t n, hipStream_t stream);
    // root's n floats to every rank, in place, enqueued on stream
    void broadcast(float* buf, size_t n, int root, hipStream_t stream);

private:
    void* comm_ = nullptr;  // ncclComm_t
    std::shared_ptr<Loopback> lb_;
    int nranks_ = 1, rank_ = 0;
};

}  // namespace bf
