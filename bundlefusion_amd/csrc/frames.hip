// frames.hip — input preprocessing of CUDAImageManager::process (CUDAImageManager.cpp:22-158) for
// gfx950: ushort depth -> metres (SensorDataReader.cpp:104-107), erodeDepthMap x2
// (CUDAImageUtil.cu:701-748), gaussFilterDepthMap (:759-806), nearest resampling of depth and colour
// to the integration size (resampleFloat / resampleUCHAR4, :93-186).
//
// The images are small (0.3 - 1.2 Mpixel) and every kernel is a stencil over them, so the layout is
// the plain row-major image; each workgroup stages its tile plus halo in LDS once, so a pixel's
// (2r+1)^2 neighbourhood is read from LDS instead of 25-81 global loads. Arithmetic follows the
// reference expression by expression (-ffp-contract=off); the Gaussian weights depend only on the
// integer offset, so they are a host-computed table shared with the CPU oracle.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <limits>

#include "../../include/bf/bf.h"
#include "bf_runtime.h"
#include "frames.h"

namespace bf {

namespace {

constexpr int TX = 32, TY = 8;   // workgroup tile: 32 x 8 pixels, 256 threads
constexpr int MAXR = 7;          // stencil radius cap (erode structure size / ceil(2 sigmaD))

__global__ __launch_bounds__(256) void k_depth_u16(const uint16_t* __restrict__ in, float* __restrict__ out, uint32_t n,
                                                   float shift) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint16_t d = in[i];
    out[i] = d == 0 ? -INFINITY : (float)d / shift;
}

// stage a (TX + 2R) x (TY + 2R) tile with halo; out-of-image cells are filled but never read: the
// callers keep the reference's `x + j >= 0 && ...` bounds tests
template <int R>
__device__ __forceinline__ void stage_tile(float (*t)[TX + 2 * MAXR], const float* __restrict__ in, int W, int H) {
    const int x0 = blockIdx.x * TX - R, y0 = blockIdx.y * TY - R;
    for (int k = threadIdx.x; k < (TX + 2 * R) * (TY + 2 * R); k += blockDim.x) {
        const int ty = k / (TX + 2 * R), tx = k % (TX + 2 * R);
        const int x = x0 + tx, y = y0 + ty;
        t[ty][tx] = (x >= 0 && x < W && y >= 0 && y < H) ? in[y * W + x] : 0.0f;
    }
    __syncthreads();
}
// the same from the sensor's ushort depth, converted as k_depth_u16 does (the first erosion's input)
template <int R>
__device__ __forceinline__ void stage_tile_u16(float (*t)[TX + 2 * MAXR], const uint16_t* __restrict__ in, int W, int H,
                                               float shift) {
    const int x0 = blockIdx.x * TX - R, y0 = blockIdx.y * TY - R;
    for (int k = threadIdx.x; k < (TX + 2 * R) * (TY + 2 * R); k += blockDim.x) {
        const int ty = k / (TX + 2 * R), tx = k % (TX + 2 * R);
        const int x = x0 + tx, y = y0 + ty;
        float v = 0.0f;
        if (x >= 0 && x < W && y >= 0 && y < H) {
            const uint16_t d = in[y * W + x];
            v = d == 0 ? -INFINITY : (float)d / shift;
        }
        t[ty][tx] = v;
    }
    __syncthreads();
}

// erodeDepthMapDevice (CUDAImageUtil.cu:701-739)
// BOUNDS false: the workgroup's tile and halo lie inside the image, so the reference's per-tap
// `x + j >= 0 && ...` tests are all true and are left out (the same taps, the same result)
template <int R, bool BOUNDS>
__device__ __forceinline__ unsigned int erode_count(const float (*t)[TX + 2 * MAXR], int lx, int ly, int x, int y, int W, int H,
                                                    float oldDepth, float dThresh) {
    unsigned int count = 0;
#pragma unroll
    for (int i = -R; i <= R; i++)
#pragma unroll
        for (int j = -R; j <= R; j++)
            if (!BOUNDS || (x + j >= 0 && x + j < W && y + i >= 0 && y + i < H)) {
                const float depth = t[ly + R + i][lx + R + j];
                if (depth == -INFINITY || depth == 0.0f || fabsf(depth - oldDepth) > dThresh) count++;
            }
    return count;
}
template <int R>
__device__ __forceinline__ bool tile_interior(int W, int H) {
    const int x0 = blockIdx.x * TX - R, y0 = blockIdx.y * TY - R;
    return x0 >= 0 && y0 >= 0 && x0 + TX + 2 * R <= W && y0 + TY + 2 * R <= H;
}
// inU16 != nullptr: the input is the sensor's ushort depth (k_depth_u16 folded into the staging)
template <int R>
__global__ __launch_bounds__(256) void k_erode(float* __restrict__ out, const float* __restrict__ in, int W, int H, float dThresh,
                                               float fracReq, const uint16_t* __restrict__ inU16, float shift) {
    __shared__ float t[TY + 2 * MAXR][TX + 2 * MAXR];
    if (inU16) stage_tile_u16<R>(t, inU16, W, H, shift);
    else stage_tile<R>(t, in, W, H);
    const int lx = threadIdx.x % TX, ly = threadIdx.x / TX;
    const int x = blockIdx.x * TX + lx, y = blockIdx.y * TY + ly;
    if (x >= W || y >= H) return;
    const float oldDepth = t[ly + R][lx + R];
    const unsigned int count = tile_interior<R>(W, H) ? erode_count<R, false>(t, lx, ly, x, y, W, H, oldDepth, dThresh)
                                                      : erode_count<R, true>(t, lx, ly, x, y, W, H, oldDepth, dThresh);
    const unsigned int sum = (2 * R + 1) * (2 * R + 1);
    out[y * W + x] = ((float)count / (float)sum >= fracReq) ? -INFINITY : oldDepth;
}

// gaussFilterDepthMapDevice (CUDAImageUtil.cu:759-797): m (x) outer, n (y) inner, as the reference
template <int R, bool BOUNDS>
__device__ __forceinline__ float gauss_at(const float (*t)[TX + 2 * MAXR], int lx, int ly, int x, int y, int W, int H,
                                          float depthCenter, float sigmaR, const GaussTable& g) {
    float sum = 0.0f, sumWeight = 0.0f;
#pragma unroll
    for (int dm = -R; dm <= R; dm++)
#pragma unroll
        for (int dn = -R; dn <= R; dn++)
            if (!BOUNDS || (x + dm >= 0 && y + dn >= 0 && x + dm < W && y + dn < H)) {
                const float currentDepth = t[ly + R + dn][lx + R + dm];
                if (currentDepth != -INFINITY && fabsf(depthCenter - currentDepth) < sigmaR) {
                    const float weight = g.w[(dn + R) * (2 * R + 1) + (dm + R)];
                    sumWeight += weight;
                    sum += weight * currentDepth;
                }
            }
    return sumWeight > 0.0f ? sum / sumWeight : -INFINITY;
}
template <int R>
__global__ __launch_bounds__(256) void k_gauss(float* __restrict__ out, const float* __restrict__ in, int W, int H, float sigmaR,
                                               GaussTable g) {
    __shared__ float t[TY + 2 * MAXR][TX + 2 * MAXR];
    stage_tile<R>(t, in, W, H);
    const int lx = threadIdx.x % TX, ly = threadIdx.x / TX;
    const int x = blockIdx.x * TX + lx, y = blockIdx.y * TY + ly;
    if (x >= W || y >= H) return;
    const float depthCenter = t[ly + R][lx + R];
    float r = -INFINITY;
    if (depthCenter != -INFINITY)
        r = tile_interior<R>(W, H) ? gauss_at<R, false>(t, lx, ly, x, y, W, H, depthCenter, sigmaR, g)
                                   : gauss_at<R, true>(t, lx, ly, x, y, W, H, depthCenter, sigmaR, g);
    out[y * W + x] = r;
}

// resampleFloat_Kernel / resampleUCHAR4_Kernel (CUDAImageUtil.cu:93-111, 160-177): nearest sample
template <class T>
__global__ __launch_bounds__(256) void k_resample(T* __restrict__ out, uint32_t oW, uint32_t oH, const T* __restrict__ in,
                                                  uint32_t iW, uint32_t iH) {
    const uint32_t x = blockIdx.x * TX + threadIdx.x % TX, y = blockIdx.y * TY + threadIdx.x / TX;
    if (x >= oW || y >= oH) return;
    const float scaleWidth = (float)(iW - 1) / (float)(oW - 1);
    const float scaleHeight = (float)(iH - 1) / (float)(oH - 1);
    const uint32_t xi = (uint32_t)((float)x * scaleWidth + 0.5f), yi = (uint32_t)((float)y * scaleHeight + 0.5f);
    if (xi < iW && yi < iH) out[y * oW + x] = in[yi * iW + xi];
}

template <int R>
void launch_erode(float* out, const float* in, int W, int H, float dT, float fr, hipStream_t s, const uint16_t* inU16 = nullptr,
                  float shift = 1.0f) {
    k_erode<R><<<dim3(div_up(W, TX), div_up(H, TY)), 256, 0, s>>>(out, in, W, H, dT, fr, inU16, shift);
}
template <int R>
void launch_gauss(float* out, const float* in, int W, int H, float sR, const GaussTable& g, hipStream_t s) {
    k_gauss<R><<<dim3(div_up(W, TX), div_up(H, TY)), 256, 0, s>>>(out, in, W, H, sR, g);
}

}  // namespace

// gaussD (CUDAImageUtil.cu:531-534) per integer offset, kernel radius (int)ceil(2.0 * sigmaD)
GaussTable gauss_table(float sigmaD) {
    GaussTable g{};
    g.radius = (int)std::ceil(2.0 * (double)sigmaD);
    BF_REQUIRE(g.radius >= 0 && g.radius <= MAXR, BF_ERR_ARG, "sigmaD out of range (radius <= 7)");
    for (int dy = -g.radius; dy <= g.radius; dy++)
        for (int dx = -g.radius; dx <= g.radius; dx++) {
            const int xx = dx * dx + dy * dy;
            g.w[(dy + g.radius) * (2 * g.radius + 1) + (dx + g.radius)] = expf(-((float)xx / (2.0f * sigmaD * sigmaD)));
        }
    return g;
}

Preproc::Preproc(uint32_t dw, uint32_t dh, uint32_t cw, uint32_t ch, uint32_t iw, uint32_t ih, const BFPreprocessOptions& o,
                 hipStream_t stream)
    : dw_(dw), dh_(dh), cw_(cw), ch_(ch), iw_(iw), ih_(ih), opt_(o), stream_(stream) {
    BF_REQUIRE(dw && dh && iw && ih, BF_ERR_ARG, "empty image size");
    BF_REQUIRE(o.erodeStructureSize >= 0 && o.erodeStructureSize <= MAXR, BF_ERR_ARG, "erode structure size 0..7");
    BF_REQUIRE(o.depthShift > 0.0f, BF_ERR_ARG, "depthShift");
    if (o.depthFilter) gauss_ = gauss_table(o.sigmaD);
    a_[0].alloc((size_t)dw * dh);
    a_[1].alloc((size_t)dw * dh);
    b_.alloc((size_t)dw * dh);
}

// CUDAImageManager::process: raw -> [erode x2 (raw <-> filtered)] -> [gauss | copy] -> resample
void Preproc::run(const uint16_t* depthU16, const uint8_t* rgbx, float* depthOut, uint8_t* colorOut, int slot) {
    BF_REQUIRE(slot == 0 || slot == 1, BF_ERR_ARG, "preprocessing buffer slot 0 / 1");
    const uint32_t n = dw_ * dh_;
    slot_ = slot;
    float* raw = a_[slot].p;
    float* filtered = b_.p;
    const int W = (int)dw_, H = (int)dh_;
    if (opt_.erode) {  // the first erosion converts the ushort depth as it stages its tile
        for (int i = 0; i < 2; i++) {
            float* out = (i % 2 == 0) ? filtered : raw;
            const float* in = (i % 2 == 0) ? raw : filtered;
            const uint16_t* u = i == 0 ? depthU16 : nullptr;
            const float sh = opt_.depthShift;
            switch (opt_.erodeStructureSize) {
                case 0: launch_erode<0>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                case 1: launch_erode<1>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                case 2: launch_erode<2>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                case 3: launch_erode<3>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                case 4: launch_erode<4>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                case 5: launch_erode<5>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                case 6: launch_erode<6>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
                default: launch_erode<7>(out, in, W, H, opt_.erodeDepthThresh, opt_.erodeFraction, stream_, u, sh); break;
            }
            BF_LAUNCH_CHECK();
        }
    } else {
        k_depth_u16<<<div_up(n, 256), 256, 0, stream_>>>(depthU16, raw, n, opt_.depthShift);
        BF_LAUNCH_CHECK();
    }
    const float* result = raw;
    // no resampling: the filter writes straight into the output (it is then the filtered image too)
    const bool direct = dw_ == iw_ && dh_ == ih_ && depthOut != nullptr;
    if (direct && opt_.depthFilter) filtered = depthOut;
    filteredOut_ = opt_.depthFilter ? filtered : raw;
    if (opt_.depthFilter) {
        switch (gauss_.radius) {
            case 0: launch_gauss<0>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            case 1: launch_gauss<1>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            case 2: launch_gauss<2>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            case 3: launch_gauss<3>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            case 4: launch_gauss<4>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            case 5: launch_gauss<5>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            case 6: launch_gauss<6>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
            default: launch_gauss<7>(filtered, raw, W, H, opt_.sigmaR, gauss_, stream_); break;
        }
        BF_LAUNCH_CHECK();
        result = filtered;
    }
    if (direct) {
        if (result != depthOut) BF_HIP(hipMemcpyAsync(depthOut, result, sizeof(float) * n, hipMemcpyDeviceToDevice, stream_));
    } else {
        k_resample<float><<<dim3(div_up(iw_, TX), div_up(ih_, TY)), 256, 0, stream_>>>(depthOut, iw_, ih_, result, dw_, dh_);
        BF_LAUNCH_CHECK();
    }
    if (rgbx && colorOut) {
        if (cw_ == iw_ && ch_ == ih_) {
            BF_HIP(hipMemcpyAsync(colorOut, rgbx, 4ull * cw_ * ch_, hipMemcpyDeviceToDevice, stream_));
        } else {
            k_resample<uchar4><<<dim3(div_up(iw_, TX), div_up(ih_, TY)), 256, 0, stream_>>>(
                reinterpret_cast<uchar4*>(colorOut), iw_, ih_, reinterpret_cast<const uchar4*>(rgbx), cw_, ch_);
            BF_LAUNCH_CHECK();
        }
    }
}

}  // namespace bf
