// bf_runtime.h — error handling and small host utilities shared by the HIP library.
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>

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

}  // namespace bf
