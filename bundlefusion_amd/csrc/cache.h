// cache.h — the dense-term frame cache (replaces CUDACache, /root/reference/FriedLiver/Source/
// CUDACache.h/.cpp/.cu): per frame, at s_downsampledWidth x s_downsampledHeight (80x60), the
// depth, camera-space positions, normals (float4 + uchar4), intensity and its Sobel derivatives the
// bundle adjuster's dense term reads (BFCachedFrame). See cache.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/bf/types.h"
#include "bf_runtime.h"
#include "frames.h"

namespace bf {

struct CacheConfig {
    uint32_t inputWidth, inputHeight;   // depth input (the SIFT depth size, Bundler.cpp:33-37)
    uint32_t width, height;             // downsampled cache size
    uint32_t maxFrames;
    float inputIntrinsics[16];          // row-major mat4f of the input depth camera
    float colorSigma;                   // s_colorDownSigma [2.5]
    float depthSigmaD, depthSigmaR;     // s_depthDownSigmaD [1.0], s_depthDownSigmaR [0.05]
};

class Cache {
public:
    Cache(const CacheConfig& cfg, hipStream_t stream);
    // storeFrame (CUDACache.cpp:45-94): device depth (inputWidth x inputHeight, metres, -inf
    // invalid) and colour (uchar4, colorW x colorH) -> the next cache frame; returns its index
    uint32_t storeFrame(const float* depth, const uint8_t* color, uint32_t colorW, uint32_t colorH);
    // copyCacheFrameFrom (CUDACache.h:24-39) / incrementCache (:41-43)
    uint32_t copyFrameFrom(const Cache& other, uint32_t frame);
    void increment();
    BFCachedFrame frame(uint32_t i) const;
    uint32_t numFrames() const { return cur_; }
    const CacheConfig& config() const { return cfg_; }
    const float* intrinsics() const { return K_; }     // m_intrinsics (scaled to the cache size)
    const float* intrinsicsInv() const { return Kinv_; }
    hipStream_t stream() const { return stream_; }

private:
    CacheConfig cfg_;
    hipStream_t stream_;
    uint32_t cur_ = 0;
    size_t hw_;
    float K_[16], Kinv_[16], inKinv_[16];
    GaussTable depthGauss_{}, colorGauss_{};
    DevBuf<float> depth_, intensity_;
    DevBuf<float4> campos_, normals_;
    DevBuf<uchar4> normalsU8_;
    DevBuf<float2> deriv_;
};

}  // namespace bf
