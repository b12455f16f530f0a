// frames.h — input preprocessing (CUDAImageManager::process, CUDAImageManager.cpp:22-158): see
// frames.hip. The CPU oracle restates the same steps in oracle/frames.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/bf/types.h"
#include "bf_runtime.h"

namespace bf {

struct GaussTable {  // gaussD weights per integer offset, radius (int)ceil(2 sigmaD) <= 7
    int radius;
    float w[15 * 15];
};
GaussTable gauss_table(float sigmaD);

class Preproc {
public:
    Preproc(uint32_t depthW, uint32_t depthH, uint32_t colorW, uint32_t colorH, uint32_t integrationW, uint32_t integrationH,
            const BFPreprocessOptions& opt, hipStream_t stream);
    // device pointers; queued on the stream. slot (0 / 1): which of two sensor-size raw buffers this run
    // ends in (rawDepth()), so a reader of one frame's raw image (the loop's cache) need not finish
    // before the next frame's preprocessing starts
    void run(const uint16_t* depthU16, const uint8_t* rgbx, float* depthOut, uint8_t* colorOut, int slot = 0);
    hipStream_t stream() const { return stream_; }
    uint32_t integrationWidth() const { return iw_; }
    uint32_t integrationHeight() const { return ih_; }
    uint32_t depthWidth() const { return dw_; }
    uint32_t depthHeight() const { return dh_; }
    uint32_t colorWidth() const { return cw_; }
    uint32_t colorHeight() const { return ch_; }
    // the sensor-size images of the last run that CUDAImageManager::copyToBundling hands the bundler
    // (CUDAImageManager.h:223-227): d_depthInputRaw (the two erosion passes end in it) and
    // d_depthInputFiltered (the bilateral filter's output; the raw image when the filter is off)
    const float* rawDepth() const { return a_[slot_].p; }
    const float* filteredDepth() const { return filteredOut_ ? filteredOut_ : (opt_.depthFilter ? b_.p : a_[slot_].p); }

private:
    uint32_t dw_, dh_, cw_, ch_, iw_, ih_;
    BFPreprocessOptions opt_;
    hipStream_t stream_;
    GaussTable gauss_{};
    DevBuf<float> a_[2], b_;
    int slot_ = 0;  // the last run's raw buffer
    const float* filteredOut_ = nullptr;  // the last run's filtered image (depthOut when no resampling)
};

}  // namespace bf
