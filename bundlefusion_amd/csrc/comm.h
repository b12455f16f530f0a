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
    // own host thread (ranks share a GPU). A collective is a one-workgroup kernel on the caller's stream,
    // as RCCL's are: it publishes the rank's contribution in a device slot, waits on the device for every
    // rank's arrival (bounded by timeoutMs: a rank that never arrives makes the next call throw) and sums
    // in rank order (comm_loopback.hip). Nothing waits on the host, so the call sites see RCCL's
    // asynchronous, stream-ordered semantics; RCCL itself is not exercised. As with RCCL, a rank's streams
    // must not share a hardware queue with another rank's (one process per GPU has its own queues; ranks in
    // one process need GPU_MAX_HW_QUEUES above their stream count, tests/conftest.py). capacityBytes: the
    // largest collective (0: 16 MiB).
    static std::shared_ptr<Loopback> loopbackGroup(int nranks, int timeoutMs, size_t capacityBytes = 0);
    Comm(std::shared_ptr<Loopback> group, int rank);
    ~Comm();
    int size() const { return nranks_; }
    int rank() const { return rank_; }
    // in-place sum over ranks of n doubles, enqueued on stream (no host synchronisation)
    void allreduceSum(double* buf, size_t n, hipStream_t stream);
    // root's n floats to every rank, in place, enqueued on stream
    void broadcast(float* buf, size_t n, int root, hipStream_t stream);
    // after synchronising the streams that carried this communicator's collectives: throws BF_ERR_INTERNAL when
    // one of them failed (loopback: a wait for a rank timed out, so its sums are not valid; RCCL: the
    // communicator's asynchronous error)
    void checkError() const;
    // Loopback groups share one GPU: a persistent launch (k_pcg_persist, which needs nearly every CU and is
    // serialized per device) of one rank must not be queued ahead of another rank's earlier one, or each waits
    // on a collective the other can only reach after its own launch. The ranks' persistent launches are
    // therefore issued in rank order per round: begin waits (host) for this rank's turn, end passes it on.
    // No-ops for RCCL (one process per GPU).
    void orderedLaunchBegin();
    void orderedLaunchEnd();

private:
    void loopbackCollective(void* buf, size_t n, size_t elemBytes, int kind, int root, hipStream_t stream);
    void loopbackCheck() const;
    void loopbackTurn(bool begin);
    void* comm_ = nullptr;  // ncclComm_t
    std::shared_ptr<Loopback> lb_;
    int nranks_ = 1, rank_ = 0;
};

}  // namespace bf
