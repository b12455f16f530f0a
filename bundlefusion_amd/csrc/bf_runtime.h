// bf_runtime.h — error handling and small host utilities shared by the HIP library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <vector>

namespace bf {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

enum Status {
    BF_OK = 0,
    BF_ERR_HIP = -1,
    BF_ERR_ARG = -2,
    BF_ERR_CAPACITY = -3,
    BF_ERR_STATE = -4,
    BF_ERR_IO = -5,
    BF_ERR_INTERNAL = -6,
};

void set_last_error(const std::string& msg);

#define BF_HIP(call)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            throw ::bf::Error(::bf::BF_ERR_HIP, std::string(#call) + " failed: " + hipGetErrorString(e_) + \
                                                    " (" __FILE__ ":" + std::to_string(__LINE__) + ")");  \
    } while (0)

#define BF_REQUIRE(cond, code, msg)                                                 \
    do {                                                                            \
        if (!(cond)) throw ::bf::Error((code), std::string(msg) + " [" #cond "]"); \
    } while (0)

// Launch-error check after a kernel launch (does not synchronize).
#define BF_LAUNCH_CHECK() BF_HIP(hipGetLastError())

inline unsigned div_up(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// Owns a device allocation.
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) BF_HIP(hipMalloc((void**)&p, count * sizeof(T)));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    size_t bytes() const { return n * sizeof(T); }
};

// Live per-launch timing of one kernel with HIP events on the stream it is launched on, for
// the roofline figure bench.py reports. A ring of event pairs; a slot is harvested (event
// synchronize + elapsed time) only when the ring wraps, i.e. ~RING launches later, so the
// host never waits on work it just queued.
class KernelClock {
public:
    static constexpr size_t RING = 512;
    ~KernelClock() { destroy(); }
    void enable(bool on) {
        if (on && a_.empty()) {
            a_.resize(RING);
            b_.resize(RING);
            for (size_t i = 0; i < RING; i++) {
                BF_HIP(hipEventCreate(&a_[i]));
                BF_HIP(hipEventCreate(&b_[i]));
            }
        }
        on_ = on;
    }
    bool enabled() const { return on_; }
    void start(hipStream_t s) {
        if (pending_ == RING) harvest(head_);
        BF_HIP(hipEventRecord(a_[head_], s));
    }
    void stop(hipStream_t s) {
        BF_HIP(hipEventRecord(b_[head_], s));
        head_ = (head_ + 1) % RING;
        pending_++;
    }
    // event pair for hipExtLaunchKernelGGL, which stamps them at the dispatch's own start and
    // end (no queue gap between a separately recorded start event and the kernel): slot(), launch
    // with the pair, then commit()
    void slot(hipEvent_t& a, hipEvent_t& b) {
        if (pending_ == RING) harvest(head_);
        a = a_[head_];
        b = b_[head_];
    }
    void commit() {
        head_ = (head_ + 1) % RING;
        pending_++;
    }
    // sampled timing (period p): slotSampled() hands out the event pair for one launch in p (the events stamp
    // the dispatch, which costs the stream a little time per launch) and counts every launch; totalMs() then
    // scales the sampled time to all launches (their mean is the sampled mean) and launches() counts them all
    void setPeriod(uint32_t p) { period_ = p ? p : 1u; }
    bool slotSampled(hipEvent_t& a, hipEvent_t& b) {
        const bool s = (calls_++ % period_) == 0;
        if (s) slot(a, b);
        return s;
    }
    // drains every pending slot (synchronizes on the newest event)
    double totalMs() {
        while (pending_) harvest((head_ + RING - pending_) % RING);
        return (calls_ && n_) ? total_ * (double)calls_ / (double)n_ : total_;
    }
    uint64_t launches() {
        totalMs();
        return calls_ ? calls_ : n_;
    }
    void reset() {
        totalMs();
        total_ = 0.0;
        n_ = 0;
        calls_ = 0;
    }

private:
    void harvest(size_t slot) {
        BF_HIP(hipEventSynchronize(b_[slot]));
        float ms = 0.0f;
        BF_HIP(hipEventElapsedTime(&ms, a_[slot], b_[slot]));
        total_ += ms;
        n_++;
        pending_--;
    }
    void destroy() {
        for (auto e : a_) (void)hipEventDestroy(e);
        for (auto e : b_) (void)hipEventDestroy(e);
        a_.clear();
        b_.clear();
    }
    std::vector<hipEvent_t> a_, b_;
    size_t head_ = 0, pending_ = 0;
    double total_ = 0.0;
    uint64_t n_ = 0, calls_ = 0;
    uint32_t period_ = 1;
    bool on_ = false;
};

}  // namespace bf
