// oracle/frames.cpp — TEST INFRASTRUCTURE: serial restatement of the input preprocessing of
// CUDAImageManager::process (Source/CUDAImageManager.cpp:22-158) and the .sens depth conversion
// (Source/SensorDataReader.cpp:104-107): ushort -> metres, erodeDepthMap x2
// (Source/CUDAImageUtil.cu:701-739), gaussFilterDepthMap (:759-797), resampleFloat /
// resampleUCHAR4 (:93-111, :160-177). The Gaussian weights are gaussD (:531-534) tabulated per
// integer offset with the host expf, the same table the HIP build uses.
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

const float MINF = -INFINITY;

void erode(float* out, const float* in, int s, int W, int H, float dThresh, float fracReq) {
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            unsigned int count = 0;
            const float oldDepth = in[y * W + x];
            for (int i = -s; i <= s; i++)
                for (int j = -s; j <= s; j++)
                    if (x + j >= 0 && x + j < W && y + i >= 0 && y + i < H) {
                        const float depth = in[(y + i) * W + (x + j)];
                        if (depth == MINF || depth == 0.0f || std::fabs(depth - oldDepth) > dThresh) count++;
                    }
            const unsigned int sum = (2 * s + 1) * (2 * s + 1);
            out[y * W + x] = ((float)count / (float)sum >= fracReq) ? MINF : in[y * W + x];
        }
}

void gauss(float* out, const float* in, float sigmaD, float sigmaR, int W, int H) {
    const int R = (int)std::ceil(2.0 * (double)sigmaD);
    std::vector<float> w((2 * R + 1) * (2 * R + 1));
    for (int dy = -R; dy <= R; dy++)
        for (int dx = -R; dx <= R; dx++)
            w[(dy + R) * (2 * R + 1) + (dx + R)] = expf(-((float)(dx * dx + dy * dy) / (2.0f * sigmaD * sigmaD)));
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            out[y * W + x] = MINF;
            float sum = 0.0f, sumWeight = 0.0f;
            const float depthCenter = in[y * W + x];
            if (depthCenter != MINF) {
                for (int m = x - R; m <= x + R; m++)
                    for (int n = y - R; n <= y + R; n++)
                        if (m >= 0 && n >= 0 && m < W && n < H) {
                            const float currentDepth = in[n * W + m];
                            if (currentDepth != MINF && std::fabs(depthCenter - currentDepth) < sigmaR) {
                                const float weight = w[(n - y + R) * (2 * R + 1) + (m - x + R)];
                                sumWeight += weight;
                                sum += weight * currentDepth;
                            }
                        }
            }
            if (sumWeight > 0.0f) out[y * W + x] = sum / sumWeight;
        }
}

template <class T>
void resample(T* out, unsigned oW, unsigned oH, const T* in, unsigned iW, unsigned iH) {
    for (unsigned y = 0; y < oH; y++)
        for (unsigned x = 0; x < oW; x++) {
            const float scaleWidth = (float)(iW - 1) / (float)(oW - 1);
            const float scaleHeight = (float)(iH - 1) / (float)(oH - 1);
            const unsigned xi = (unsigned)((float)x * scaleWidth + 0.5f), yi = (unsigned)((float)y * scaleHeight + 0.5f);
            if (xi < iW && yi < iH) out[y * oW + x] = in[yi * iW + xi];
        }
}

struct RGBX { uint8_t v[4]; };

}  // namespace

extern "C" void or_preprocess(const BFPreprocessOptions* o, const uint16_t* depthU16, uint32_t dw, uint32_t dh,
                              const uint8_t* rgbx, uint32_t cw, uint32_t ch, uint32_t iw, uint32_t ih, float* depthOut,
                              uint8_t* colorOut) {
    const size_t n = (size_t)dw * dh;
    std::vector<float> raw(n), filtered(n);
    for (size_t i = 0; i < n; i++) raw[i] = depthU16[i] == 0 ? MINF : (float)depthU16[i] / o->depthShift;
    if (o->erode) {
        for (int i = 0; i < 2; i++) {
            if (i % 2 == 0) erode(filtered.data(), raw.data(), o->erodeStructureSize, (int)dw, (int)dh, o->erodeDepthThresh, o->erodeFraction);
            else erode(raw.data(), filtered.data(), o->erodeStructureSize, (int)dw, (int)dh, o->erodeDepthThresh, o->erodeFraction);
        }
    }
    const float* result = raw.data();
    if (o->depthFilter) {
        gauss(filtered.data(), raw.data(), o->sigmaD, o->sigmaR, (int)dw, (int)dh);
        result = filtered.data();
    }
    if (dw == iw && dh == ih) std::memcpy(depthOut, result, sizeof(float) * n);
    else resample(depthOut, iw, ih, result, dw, dh);
    if (rgbx && colorOut) {
        if (cw == iw && ch == ih) std::memcpy(colorOut, rgbx, 4ull * cw * ch);
        else resample(reinterpret_cast<RGBX*>(colorOut), iw, ih, reinterpret_cast<const RGBX*>(rgbx), cw, ch);
    }
}
