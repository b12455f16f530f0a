// comm_loopback.hip — the loopback communicator's collectives (comm.h) as stream-ordered kernels, the way
// RCCL runs its own: the collective is one workgroup enqueued on the caller's stream that publishes its
// contribution, waits on the device for every rank's arrival and then reduces, so nothing on the host
// waits and every dependency a caller forgets between its own kernels and the collective's buffer shows
// as it would with ncclAllReduce / ncclBroadcast (an unsynchronised host read, a kernel on another
// stream that does not wait for the collective). The ranks share one GPU; arrivals are device-scope
// counters, one per slot parity, so slots are reused every other collective without a departure barrier
// (a rank refills parity p only after every rank arrived at the collective in between, hence finished
// reading p). Every wait is bounded: a rank that never arrives sets the group's error word (host memory)
// and the collective ends with whatever the slots hold. Nothing may consume those: the next collective
// call throws, and so does Comm::checkError, which the callers run after synchronising the streams that
// carry collectives (bf_comm_allreduce_sum_f64, Recon::apply before a submap's poses are used,
// Recon::synchronize); a group destroyed with the word set reports it on stderr.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "bf_runtime.h"
#include "comm.h"

namespace bf {

namespace {

__device__ __forceinline__ unsigned long long lb_rtc() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// kind 0: in-place sum of n doubles over the ranks, in rank order; kind 1: broadcast of root's n floats
__global__ __launch_bounds__(256) void k_loopback_collective(double* dbuf, float* fbuf, size_t n, int kind, int root,
                                                             int rank, int nranks, uint32_t seq, unsigned char* slots,
                                                             size_t slotBytes, uint32_t* arrive, uint32_t* err,
                                                             unsigned long long ticks) {
    const uint32_t p = seq & 1u;
    unsigned char* base = slots + (size_t)p * (size_t)nranks * slotBytes;
    if (kind == 0) {
        double* mine = reinterpret_cast<double*>(base + (size_t)rank * slotBytes);
        for (size_t i = threadIdx.x; i < n; i += blockDim.x) mine[i] = dbuf[i];
    } else if (rank == root) {
        float* mine = reinterpret_cast<float*>(base + (size_t)rank * slotBytes);
        for (size_t i = threadIdx.x; i < n; i += blockDim.x) mine[i] = fbuf[i];
    }
    // every wave's slot stores reach device scope before the arrival is counted
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(&arrive[p], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t target = (uint32_t)nranks * (seq / 2u + 1u);  // arrivals ever at parity p after this one
        const unsigned long long t0 = lb_rtc();
        while (__hip_atomic_load(&arrive[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (lb_rtc() - t0 > ticks) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (kind == 0) {
        for (size_t i = threadIdx.x; i < n; i += blockDim.x) {
            double s = 0.0;
            for (int r = 0; r < nranks; r++) s += reinterpret_cast<const double*>(base + (size_t)r * slotBytes)[i];
            dbuf[i] = s;
        }
    } else if (rank != root) {
        const float* rs = reinterpret_cast<const float*>(base + (size_t)root * slotBytes);
        for (size_t i = threadIdx.x; i < n; i += blockDim.x) fbuf[i] = rs[i];
    }
}

}  // namespace

struct Loopback {
    int nranks = 1;
    unsigned long long ticks = 0;
    size_t slotBytes = 0;
    DevBuf<unsigned char> slots;  // [2 parities][nranks][slotBytes]
    DevBuf<uint32_t> arrive;      // arrivals ever, per parity
    uint32_t* err = nullptr;      // pinned host word: a wait ran out
    std::mutex mu;
    std::condition_variable turnCv;            // ordered persistent launches (Comm::orderedLaunchBegin)
    uint64_t turn = 0;                         // launches issued by the group so far
    std::vector<uint64_t> launches;            // per rank
    std::vector<uint32_t> seq;                 // next collective of each rank
    std::vector<std::pair<uint32_t, size_t>> sizes;  // (collective, bytes) of recent collectives, by seq % 64
    ~Loopback() {
        (void)hipDeviceSynchronize();  // no collective kernel may still use the slots
        if (err && __atomic_load_n(err, __ATOMIC_ACQUIRE) != 0)
            fprintf(stderr, "bf loopback communicator: a collective timed out waiting for a rank (results after it are invalid)\n");
        if (err) (void)hipHostFree(err);
    }
};

std::shared_ptr<Loopback> Comm::loopbackGroup(int nranks, int timeoutMs, size_t capacityBytes) {
    BF_REQUIRE(nranks >= 1, BF_ERR_ARG, "nranks");
    auto g = std::make_shared<Loopback>();
    g->nranks = nranks;
    g->ticks = 100000ull * (unsigned long long)(timeoutMs > 0 ? timeoutMs : 60000);
    g->slotBytes = (capacityBytes ? capacityBytes : (size_t)16 << 20) & ~(size_t)255;
    g->slots.alloc(2 * (size_t)nranks * g->slotBytes);
    g->arrive.alloc(2);
    BF_HIP(hipMemset(g->arrive.p, 0, 2 * sizeof(uint32_t)));
    BF_HIP(hipHostMalloc((void**)&g->err, sizeof(uint32_t), hipHostMallocCoherent));
    *g->err = 0;
    g->seq.assign((size_t)nranks, 0u);
    g->launches.assign((size_t)nranks, 0u);
    g->sizes.assign(64, {0xFFFFFFFFu, 0});
    BF_HIP(hipDeviceSynchronize());
    return g;
}

Comm::Comm(std::shared_ptr<Loopback> group, int rank) : lb_(std::move(group)), nranks_(lb_ ? lb_->nranks : 1), rank_(rank) {
    BF_REQUIRE(lb_ && rank >= 0 && rank < nranks_, BF_ERR_ARG, "loopback rank");
}

void Comm::loopbackCheck() const {
    BF_REQUIRE(__atomic_load_n(lb_->err, __ATOMIC_ACQUIRE) == 0, BF_ERR_INTERNAL,
               "loopback communicator: a rank did not reach a collective in time "
               "(ranks issued different collective sequences)");
}

void Comm::loopbackTurn(bool begin) {
    Loopback& g = *lb_;
    std::unique_lock<std::mutex> lk(g.mu);
    const uint64_t mine = g.launches[(size_t)rank_] * (uint64_t)nranks_ + (uint64_t)rank_;
    if (begin) {
        // bounded like the device-side waits: a rank that stopped issuing launches fails the others
        const bool ok = g.turnCv.wait_for(lk, std::chrono::microseconds(g.ticks / 100ull), [&] { return g.turn == mine; });
        BF_REQUIRE(ok, BF_ERR_INTERNAL, "loopback communicator: a rank did not reach its persistent launch in time");
    } else {
        g.launches[(size_t)rank_]++;
        g.turn = mine + 1;
        lk.unlock();
        g.turnCv.notify_all();
    }
}

void Comm::loopbackCollective(void* buf, size_t n, size_t elemBytes, int kind, int root, hipStream_t stream) {
    Loopback& g = *lb_;
    loopbackCheck();
    const size_t bytes = n * elemBytes;
    BF_REQUIRE(bytes <= g.slotBytes, BF_ERR_CAPACITY, "loopback collective larger than the group's slot capacity");
    uint32_t s;
    {
        std::lock_guard<std::mutex> lk(g.mu);
        s = g.seq[(size_t)rank_]++;
        auto& e = g.sizes[s % 64];
        if (e.first == s) {
            BF_REQUIRE(e.second == bytes, BF_ERR_INTERNAL, "loopback collective: ranks passed different counts");
        } else {
            e = {s, bytes};
        }
    }
    k_loopback_collective<<<1, 256, 0, stream>>>(kind == 0 ? static_cast<double*>(buf) : nullptr,
                                                 kind == 1 ? static_cast<float*>(buf) : nullptr, n, kind, root, rank_,
                                                 nranks_, s, g.slots.p, g.slotBytes, g.arrive.p, g.err, g.ticks);
    BF_LAUNCH_CHECK();
}

}  // namespace bf
