// cache.hip — gfx950 CUDACache::storeFrame (/root/reference/FriedLiver/Source/CUDACache.cpp:45-94,
// both CUDACACHE_FLOAT_NORMALS and CUDACACHE_UCHAR_NORMALS, CUDACacheUtil.h:7-8).
//
// The reference runs ten full-image passes per frame: gaussFilterDepthMap, convertDepthFloatTo-
// CameraSpaceFloat4 and computeNormals at the INPUT size (640x480), then nearest resampling of
// three of those images to 80x60, the uchar4 normal packing, resampleToIntensity, gaussFilter-
// Intensity and computeIntensityDerivatives. Every output pixel of the resampled images depends
// only on the input pixel it samples and that pixel's 4-neighbourhood, so here:
//
//  * k_cache_geometry: per CACHE pixel, five threads evaluate the bilateral depth filter at just the
//    5 input pixels it needs (sample + 4 neighbours), their camera-space positions, the normal, and
//    writes depth / campos / normals / uchar4 normals: 5 x 4 800 filter windows (one per thread)
//    instead of 307 200 full-resolution ones, with the same float expressions in the same order,
//    so the results are bit-identical to the staged pipeline (checked against the oracle, which stages).
//  * k_cache_intensity: per 8x8 tile, the resampled intensity (tile + radius + 1 halo) and its
//    Gaussian (tile + 1 halo) are staged in LDS: resample + convertToIntensity, the Gaussian and
//    the Sobel derivatives in one launch instead of three.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/bf/bf.h"
#include "bf_math.h"
#include "bf_runtime.h"
#include "cache.h"

namespace bf {

namespace {

constexpr int GEOM_WG = 320;  // 5 waves: one per stencil point of 64 cache pixels
constexpr uint32_t MAX_CACHE_PIXELS = 1u << 20;

struct GeomArgs {
    const float* depth;
    uint32_t iW, iH, oW, oH;
    float kinv[16];  // m_inputIntrinsicsInv (row-major float4x4)
    float sigmaR;
    int useGauss;
    GaussTable g;
    float* outDepth;
    float4* outCampos;
    float4* outNormals;
    uchar4* outNU8;
};

// gaussFilterDepthMapDevice (CUDAImageUtil.cu:759-797) evaluated at one pixel: m (x) outer, n (y) inner.
// R = the kernel radius as a template argument (R < 0: no filter), so the taps unroll: their loads
// issue together and the weights are compile-time offsets into the argument table
template <int R>
__device__ __forceinline__ float filtered_at(const GeomArgs& A, int x, int y) {
    const int W = (int)A.iW, H = (int)A.iH;
    const float depthCenter = A.depth[y * W + x];
    if constexpr (R < 0) {
        return depthCenter;
    } else {
        float sum = 0.0f, sumWeight = 0.0f;
        if (depthCenter != -INFINITY) {
#pragma unroll
            for (int dm = -R; dm <= R; dm++)
#pragma unroll
                for (int dn = -R; dn <= R; dn++) {
                    const int m = x + dm, n = y + dn;
                    if (m >= 0 && n >= 0 && m < W && n < H) {
                        const float currentDepth = A.depth[n * W + m];
                        if (currentDepth != -INFINITY && fabsf(depthCenter - currentDepth) < A.sigmaR) {
                            const float weight = A.g.w[(dn + R) * (2 * R + 1) + (dm + R)];
                            sumWeight += weight;
                            sum += weight * currentDepth;
                        }
                    }
                }
        }
        return sumWeight > 0.0f ? sum / sumWeight : -INFINITY;
    }
}

// convertDepthFloatToCameraSpaceFloat4_Kernel (CUDAImageUtil.cu:367-384) at one pixel
__device__ float4 campos_at(const GeomArgs& A, int x, int y, float depth) {
    if (depth == -INFINITY) return make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    const float* m = A.kinv;
    const float vx = (float)x * depth, vy = (float)y * depth, vz = depth, vw = depth;
    const float cx = m[0] * vx + m[1] * vy + m[2] * vz + m[3] * vw;
    const float cy = m[4] * vx + m[5] * vy + m[6] * vz + m[7] * vw;
    const float cw = m[12] * vx + m[13] * vy + m[14] * vz + m[15] * vw;
    return make_float4(cx, cy, cw, 1.0f);
}

// 64 cache pixels per workgroup; wave w evaluates the filtered depth at point w of each pixel's
// stencil (the sample, then +y, +x, -y, -x), so each thread runs one 5x5 bilateral window; wave 0
// then forms camera positions, the normal and the outputs from LDS.
template <int R>
__global__ __launch_bounds__(GEOM_WG) void k_cache_geometry(GeomArgs A) {
    __shared__ float sd[5][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t p = blockIdx.x * 64 + lane;
    const bool on = p < A.oW * A.oH;
    const uint32_t x = on ? p % A.oW : 0, y = on ? p / A.oW : 0;
    // resampleFloat4 / resampleFloat nearest sample (CUDAImageUtil.cu:113-150)
    const float scaleWidth = (float)(A.iW - 1) / (float)(A.oW - 1);
    const float scaleHeight = (float)(A.iH - 1) / (float)(A.oH - 1);
    const int xi = (int)(uint32_t)((float)x * scaleWidth + 0.5f), yi = (int)(uint32_t)((float)y * scaleHeight + 0.5f);
    const int dx[5] = {0, 0, 1, 0, -1}, dy[5] = {0, 1, 0, -1, 0};
    const bool interior = xi > 0 && xi < (int)A.iW - 1 && yi > 0 && yi < (int)A.iH - 1;
    float f = -INFINITY;
    if (on && (w == 0 || interior)) f = filtered_at<R>(A, xi + dx[w], yi + dy[w]);
    sd[w][lane] = f;
    __syncthreads();
    if (w != 0 || !on) return;
    const float d = sd[0][lane];
    const float4 CC = campos_at(A, xi, yi, d);
    A.outDepth[p] = d;
    A.outCampos[p] = CC;
    // computeNormals_Kernel (CUDAImageUtil.cu:404-432) at the sampled pixel
    float4 nrm = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (interior && CC.x != -INFINITY) {
        const float4 PC = campos_at(A, xi, yi + 1, sd[1][lane]);
        const float4 CP = campos_at(A, xi + 1, yi, sd[2][lane]);
        const float4 MC = campos_at(A, xi, yi - 1, sd[3][lane]);
        const float4 CM = campos_at(A, xi - 1, yi, sd[4][lane]);
        if (PC.x != -INFINITY && CP.x != -INFINITY && MC.x != -INFINITY && CM.x != -INFINITY) {
            const f3 n = cross3(mk3(PC.x, PC.y, PC.z) - mk3(MC.x, MC.y, MC.z), mk3(CP.x, CP.y, CP.z) - mk3(CM.x, CM.y, CM.z));
            const float l = length3(n);
            if (l > 0.0f) nrm = make_float4(n.x / -l, n.y / -l, n.z / -l, 0.0f);
        }
    }
    A.outNormals[p] = nrm;
    // convertNormalsFloat4ToUCHAR4_Kernel (CUDAImageUtil.cu:497-513)
    uchar4 u = make_uchar4(0, 0, 0, 0);
    if (nrm.x != -INFINITY) {
        const float px = (nrm.x + 1.0f) / 2.0f, py = (nrm.y + 1.0f) / 2.0f, pz = (nrm.z + 1.0f) / 2.0f;
        u = make_uchar4((unsigned char)roundf(px * 255), (unsigned char)roundf(py * 255), (unsigned char)roundf(pz * 255), 0);
    }
    A.outNU8[p] = u;
}

struct IntArgs {
    const uchar4* color;
    uint32_t cW, cH, oW, oH;
    int useGauss;
    GaussTable g;
    float* outIntensity;
    float2* outDeriv;
};

// IT x IT cache pixels per workgroup: the resampled intensity of the tile + (R + 1) halo and the
// Gaussian of the tile + 1 halo are staged in LDS, then the Sobel derivatives of the tile.
constexpr int IT = 8;  // 8x8 tiles: 80 workgroups at 80x60 (16x16: 20, each with twice the serial work)
// R: the Gaussian's radius, R < 0: unfiltered (template argument: the taps unroll, see filtered_at)
template <int R>
__global__ __launch_bounds__(256) void k_cache_intensity(IntArgs A) {
    constexpr int h = (R < 0 ? 0 : R) + 1, E = IT + 2 * h;  // staged edge for this radius
    __shared__ float I[E * E];
    __shared__ float G[(IT + 2) * (IT + 2)];
    const int W = (int)A.oW, H = (int)A.oH;
    const int x0 = blockIdx.x * IT - h, y0 = blockIdx.y * IT - h;
    // resampleToIntensity_Kernel (CUDAImageUtil.cu:224-241) + convertToIntensity (:197-199)
    const float scaleWidth = (float)(A.cW - 1) / (float)(W - 1);
    const float scaleHeight = (float)(A.cH - 1) / (float)(H - 1);
    for (int k = threadIdx.x; k < E * E; k += 256) {
        const int x = x0 + k % E, y = y0 + k / E;
        float v = 0.0f;
        if (x >= 0 && y >= 0 && x < W && y < H) {
            const uint32_t xi = (uint32_t)((float)(uint32_t)x * scaleWidth + 0.5f), yi = (uint32_t)((float)(uint32_t)y * scaleHeight + 0.5f);
            if (xi < A.cW && yi < A.cH) {
                const uchar4 c = A.color[yi * A.cW + xi];
                v = (0.299f * (float)c.x + 0.587f * (float)c.y + 0.114f * (float)c.z) / 255.0f;
            }
        }
        I[k] = v;
    }
    __syncthreads();
    // gaussFilterIntensityDevice (CUDAImageUtil.cu:811-847) over the tile + 1 halo; sigma <= 0: unfiltered
    for (int k = threadIdx.x; k < (IT + 2) * (IT + 2); k += 256) {
        const int gx = blockIdx.x * IT - 1 + k % (IT + 2), gy = blockIdx.y * IT - 1 + k / (IT + 2);
        float out = 0.0f;
        if (gx >= 0 && gy >= 0 && gx < W && gy < H) {
            out = I[(gy - y0) * E + (gx - x0)];
            if constexpr (R >= 0) {
                float sum = 0.0f, sumWeight = 0.0f;
#pragma unroll
                for (int dm = -R; dm <= R; dm++)  // offsets: wave-uniform weight index (scalar loads)
#pragma unroll
                    for (int dq = -R; dq <= R; dq++) {
                        const int m = gx + dm, q = gy + dq;
                        if (m >= 0 && q >= 0 && m < W && q < H) {
                            const float weight = A.g.w[(dq + R) * (2 * R + 1) + (dm + R)];
                            sumWeight += weight;
                            sum += weight * I[(q - y0) * E + (m - x0)];
                        }
                    }
                if (sumWeight > 0.0f) out = sum / sumWeight;
            }
            const int lx = gx - blockIdx.x * IT, ly = gy - blockIdx.y * IT;
            if (lx >= 0 && ly >= 0 && lx < IT && ly < IT) A.outIntensity[gy * W + gx] = out;
        }
        G[k] = out;
    }
    __syncthreads();
    // computeIntensityDerivatives_Kernel (CUDAImageUtil.cu:260-296)
    if (threadIdx.x >= IT * IT) return;
    const int lx = threadIdx.x % IT, ly = threadIdx.x / IT;
    const int x = blockIdx.x * IT + lx, y = blockIdx.y * IT + ly;
    if (x >= W || y >= H) return;
    auto g = [&](int xx, int yy) { return G[(yy - (int)blockIdx.y * IT + 1) * (IT + 2) + (xx - (int)blockIdx.x * IT + 1)]; };
    float2 r = make_float2(-INFINITY, -INFINITY);
    if (x > 0 && x < W - 1 && y > 0 && y < H - 1) {
        const float pos00 = g(x - 1, y - 1), pos01 = g(x - 1, y), pos02 = g(x - 1, y + 1);
        const float pos10 = g(x, y - 1), pos12 = g(x, y + 1);
        const float pos20 = g(x + 1, y - 1), pos21 = g(x + 1, y), pos22 = g(x + 1, y + 1);
        if (pos00 != -INFINITY && pos01 != -INFINITY && pos02 != -INFINITY && pos10 != -INFINITY && pos12 != -INFINITY &&
            pos20 != -INFINITY && pos21 != -INFINITY && pos22 != -INFINITY) {
            float resU = (-1.0f) * pos00 + (1.0f) * pos20 + (-2.0f) * pos01 + (2.0f) * pos21 + (-1.0f) * pos02 + (1.0f) * pos22;
            resU /= 8.0f;
            float resV = (-1.0f) * pos00 + (-2.0f) * pos10 + (-1.0f) * pos20 + (1.0f) * pos02 + (2.0f) * pos12 + (1.0f) * pos22;
            resV /= 8.0f;
            r = make_float2(resU, resV);
        }
    }
    A.outDeriv[y * W + x] = r;
}

}  // namespace

BFMat4 mat4_inverse(const BFMat4& m);  // api.cpp

Cache::Cache(const CacheConfig& cfg, hipStream_t stream) : cfg_(cfg), stream_(stream) {
    BF_REQUIRE(cfg.inputWidth >= 2 && cfg.inputHeight >= 2 && cfg.width >= 2 && cfg.height >= 2, BF_ERR_ARG,
               "cache and input sizes must be >= 2");
    BF_REQUIRE((size_t)cfg.width * cfg.height <= MAX_CACHE_PIXELS, BF_ERR_ARG, "cache size above 2^20 pixels");
    BF_REQUIRE(cfg.maxFrames > 0, BF_ERR_ARG, "maxFrames");
    hw_ = (size_t)cfg.width * cfg.height;
    // CUDACache::CUDACache (CUDACache.cpp:15-42): intrinsics scaled to the cache size
    std::memcpy(K_, cfg.inputIntrinsics, 64);
    K_[0] *= (float)cfg.width / (float)cfg.inputWidth;
    K_[5] *= (float)cfg.height / (float)cfg.inputHeight;
    K_[2] *= (float)(cfg.width - 1) / (float)(cfg.inputWidth - 1);
    K_[6] *= (float)(cfg.height - 1) / (float)(cfg.inputHeight - 1);
    BFMat4 k, ik;
    std::memcpy(k.m, K_, 64);
    ik = mat4_inverse(k);
    std::memcpy(Kinv_, ik.m, 64);
    std::memcpy(k.m, cfg.inputIntrinsics, 64);
    ik = mat4_inverse(k);
    std::memcpy(inKinv_, ik.m, 64);
    if (cfg.depthSigmaD > 0.0f) depthGauss_ = gauss_table(cfg.depthSigmaD);
    if (cfg.colorSigma > 0.0f) colorGauss_ = gauss_table(cfg.colorSigma);
    const size_t n = hw_ * cfg.maxFrames;
    depth_.alloc(n);
    intensity_.alloc(n);
    campos_.alloc(n);
    normals_.alloc(n);
    normalsU8_.alloc(n);
    deriv_.alloc(n);
}

uint32_t Cache::storeFrame(const float* depth, const uint8_t* color, uint32_t colorW, uint32_t colorH) {
    BF_REQUIRE(cur_ < cfg_.maxFrames, BF_ERR_CAPACITY, "cache full (maxFrames)");
    BF_REQUIRE(depth && color, BF_ERR_ARG, "null frame");
    BF_REQUIRE(colorW >= 2 && colorH >= 2, BF_ERR_ARG, "colour size");
    const uint32_t f = cur_;
    const size_t o = hw_ * f;
    GeomArgs g{};
    g.depth = depth;
    g.iW = cfg_.inputWidth; g.iH = cfg_.inputHeight; g.oW = cfg_.width; g.oH = cfg_.height;
    std::memcpy(g.kinv, inKinv_, 64);
    g.sigmaR = cfg_.depthSigmaR;
    g.useGauss = cfg_.depthSigmaD > 0.0f;
    g.g = depthGauss_;
    g.outDepth = depth_.p + o; g.outCampos = campos_.p + o; g.outNormals = normals_.p + o; g.outNU8 = normalsU8_.p + o;
    const int rg = g.useGauss ? depthGauss_.radius : -1;
    switch (rg) {
#define BF_GEOM(r) case r: k_cache_geometry<r><<<div_up((uint32_t)hw_, 64u), GEOM_WG, 0, stream_>>>(g); break;
        BF_GEOM(-1) BF_GEOM(0) BF_GEOM(1) BF_GEOM(2) BF_GEOM(3) BF_GEOM(4) BF_GEOM(5) BF_GEOM(6) BF_GEOM(7)
#undef BF_GEOM
        default: BF_REQUIRE(false, BF_ERR_ARG, "depth filter radius above 7");
    }
    BF_LAUNCH_CHECK();
    IntArgs ia{};
    ia.color = reinterpret_cast<const uchar4*>(color);
    ia.cW = colorW; ia.cH = colorH; ia.oW = cfg_.width; ia.oH = cfg_.height;
    ia.useGauss = cfg_.colorSigma > 0.0f;
    ia.g = colorGauss_;
    ia.outIntensity = intensity_.p + o;
    ia.outDeriv = deriv_.p + o;
    const dim3 ig(div_up(cfg_.width, (uint32_t)IT), div_up(cfg_.height, (uint32_t)IT));
    switch (ia.useGauss ? colorGauss_.radius : -1) {
#define BF_INT(r) case r: k_cache_intensity<r><<<ig, 256, 0, stream_>>>(ia); break;
        BF_INT(-1) BF_INT(0) BF_INT(1) BF_INT(2) BF_INT(3) BF_INT(4) BF_INT(5) BF_INT(6) BF_INT(7)
#undef BF_INT
        default: BF_REQUIRE(false, BF_ERR_ARG, "colour filter radius above 7");
    }
    BF_LAUNCH_CHECK();
    cur_++;
    return f;
}

uint32_t Cache::copyFrameFrom(const Cache& other, uint32_t frame) {
    BF_REQUIRE(cur_ < cfg_.maxFrames, BF_ERR_CAPACITY, "cache full (maxFrames)");
    BF_REQUIRE(frame < other.cur_, BF_ERR_ARG, "source frame not stored");
    BF_REQUIRE(other.hw_ == hw_, BF_ERR_ARG, "cache sizes differ");
    const size_t d = hw_ * cur_, s = hw_ * frame;
    BF_HIP(hipMemcpyAsync(depth_.p + d, other.depth_.p + s, hw_ * sizeof(float), hipMemcpyDeviceToDevice, stream_));
    BF_HIP(hipMemcpyAsync(campos_.p + d, other.campos_.p + s, hw_ * sizeof(float4), hipMemcpyDeviceToDevice, stream_));
    BF_HIP(hipMemcpyAsync(intensity_.p + d, other.intensity_.p + s, hw_ * sizeof(float), hipMemcpyDeviceToDevice, stream_));
    BF_HIP(hipMemcpyAsync(deriv_.p + d, other.deriv_.p + s, hw_ * sizeof(float2), hipMemcpyDeviceToDevice, stream_));
    BF_HIP(hipMemcpyAsync(normalsU8_.p + d, other.normalsU8_.p + s, hw_ * sizeof(uchar4), hipMemcpyDeviceToDevice, stream_));
    BF_HIP(hipMemcpyAsync(normals_.p + d, other.normals_.p + s, hw_ * sizeof(float4), hipMemcpyDeviceToDevice, stream_));
    return cur_++;
}

void Cache::increment() {
    BF_REQUIRE(cur_ < cfg_.maxFrames, BF_ERR_CAPACITY, "cache full (maxFrames)");
    cur_++;
}

BFCachedFrame Cache::frame(uint32_t i) const {
    BF_REQUIRE(i < cfg_.maxFrames, BF_ERR_ARG, "cache frame index");
    const size_t o = hw_ * i;
    BFCachedFrame f;
    f.depth = depth_.p + o;
    f.campos = reinterpret_cast<const float*>(campos_.p + o);
    f.normals = reinterpret_cast<const float*>(normals_.p + o);
    f.normalsU8 = reinterpret_cast<const uint8_t*>(normalsU8_.p + o);
    f.intensity = intensity_.p + o;
    f.intensityDeriv = reinterpret_cast<const float*>(deriv_.p + o);
    return f;
}

}  // namespace bf
