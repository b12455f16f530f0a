// synth_ba.cpp — host-side generators for bundle-adjustment inputs from the synthetic scene:
// EntryJ correspondences (stand-in for the out-of-scope SIFT front end, with the EntryJ
// convention of AddCurrToResidualsCU, SiftGPU/SIFTImageManager.cu:610-686) and dense-term
// cache frames (CUDACache::storeFrame, CUDACache.cpp:45-86, built with the reference's cache
// kernels from a noiseless render; the reference's bilateral/Gaussian pre-filters are skipped).
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "synth.h"

namespace bf {

static inline void inv_rigid(const float* T, float* Ti) {  // rigid inverse [R^T | -R^T t]
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) Ti[r * 4 + c] = T[c * 4 + r];
    for (int r = 0; r < 3; r++) Ti[r * 4 + 3] = -(Ti[r * 4 + 0] * T[3] + Ti[r * 4 + 1] * T[7] + Ti[r * 4 + 2] * T[11]);
    Ti[12] = Ti[13] = Ti[14] = 0.0f;
    Ti[15] = 1.0f;
}
static inline f3 apply(const float* T, f3 p) {
    return mk3(T[0] * p.x + T[1] * p.y + T[2] * p.z + T[3], T[4] * p.x + T[5] * p.y + T[6] * p.z + T[7],
               T[8] * p.x + T[9] * p.y + T[10] * p.z + T[11]);
}

static inline float gauss(uint32_t& st) {
    st = pcg_hash(st);
    float u1 = u01(st);
    st = pcg_hash(st);
    float u2 = u01(st);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
}

uint32_t synth_correspondences(const BFSynthScene& sc, const float* poses, uint32_t K, const BFDepthCameraParams& cam,
                               uint32_t maxPerPair, float minCovis, float noise, float outlierFrac, uint32_t seed,
                               BFEntryJ* out, uint32_t cap) {
    std::vector<float> inv((size_t)K * 16);
    for (uint32_t k = 0; k < K; k++) inv_rigid(poses + 16 * k, inv.data() + 16 * k);
    const uint32_t S = 40;
    uint32_t n = 0;
    for (uint32_t i = 0; i < K && n < cap; i++) {
        const float* Ti = poses + 16 * i;
        const f3 ci = mk3(Ti[3], Ti[7], Ti[11]);
        const f3 zi = mk3(Ti[2], Ti[6], Ti[10]);
        for (uint32_t j = i + 1; j < K && n < cap; j++) {
            const float* Tj = poses + 16 * j;
            const f3 cj = mk3(Tj[3], Tj[7], Tj[11]);
            const f3 zj = mk3(Tj[2], Tj[6], Tj[10]);
            if (length3(ci - cj) > 3.0f || dot3(zi, zj) < 0.26f) continue;  // > 3 m apart or > 75 deg
            uint32_t st = pcg_hash(seed * 0x9E3779B9u ^ pcg_hash(i * 7919u + j * 104729u + 17u));
            f3 ptsI[256], ptsJ[256];
            uint32_t acc = 0, tries = 0;
            const uint32_t maxTries = std::max(S, 4 * maxPerPair);
            uint32_t accInFirstS = 0;
            while (tries < maxTries && acc < maxPerPair && acc < 256) {
                tries++;
                st = pcg_hash(st);
                const uint32_t px = st % cam.imageWidth;
                st = pcg_hash(st);
                const uint32_t py = st % cam.imageHeight;
                // ray of pixel (px, py) in frame i
                BFMat4 Tm;
                std::memcpy(Tm.m, Ti, 64);
                const f3 dcam = mk3(((float)px - cam.mx) / cam.fx, ((float)py - cam.my) / cam.fy, 1.0f);
                const f3 d = xform4(Tm, dcam, 0.0f);
                float t;
                f3 X, nrm;
                int obj;
                if (!synth_trace(sc, ci, d, t, X, nrm, obj) || t < 0.1f || t > 4.0f) continue;
                const f3 Xj = apply(inv.data() + 16 * j, X);
                if (Xj.z < 0.1f || Xj.z > 4.0f) continue;
                const float u = Xj.x * cam.fx / Xj.z + cam.mx, v = Xj.y * cam.fy / Xj.z + cam.my;
                if (u < 0.0f || v < 0.0f || u > (float)cam.imageWidth - 1.0f || v > (float)cam.imageHeight - 1.0f) continue;
                float t2;
                f3 X2, n2;
                int o2;
                if (!synth_trace(sc, cj, X - cj, t2, X2, n2, o2) || length3(X2 - X) > 0.01f) continue;  // occluded in j
                ptsI[acc] = apply(inv.data() + 16 * i, X);
                ptsJ[acc] = Xj;
                acc++;
                if (tries <= S) accInFirstS++;
            }
            const float covis = (float)accInFirstS / (float)std::min(tries, S);
            if (covis < minCovis || acc == 0) continue;
            for (uint32_t q = 0; q < acc && n < cap; q++) {
                BFEntryJ e;
                e.imgIdx_i = i;
                e.imgIdx_j = j;
                f3 a = ptsI[q] + mk3(gauss(st), gauss(st), gauss(st)) * noise;
                f3 b = ptsJ[q] + mk3(gauss(st), gauss(st), gauss(st)) * noise;
                st = pcg_hash(st);
                if (u01(st) < outlierFrac) {
                    f3 dir = normalize3(mk3(gauss(st), gauss(st), gauss(st)));
                    st = pcg_hash(st);
                    b = b + dir * (0.1f + 0.2f * u01(st));
                }
                e.pos_i = {a.x, a.y, a.z};
                e.pos_j = {b.x, b.y, b.z};
                out[n++] = e;
            }
        }
    }
    return n;
}

// CUDACache::storeFrame restated for one noiseless render (see header comment).
void synth_cache_frame(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, float* depth, float* campos,
                       float* normals, uint8_t* normalsU8, float* intensity, float* intensityDeriv) {
    const uint32_t W = cam.imageWidth, H = cam.imageHeight;
    const float MINF = -std::numeric_limits<float>::infinity();
    std::vector<uint32_t> color(W * H);
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) synth_pixel(sc, T, cam, 0, 0, x, y, depth[y * W + x], color[y * W + x]);
    // convertDepthFloatToCameraSpaceFloat4 (CUDAImageUtil.cu:367-384)
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) {
            float* o = campos + 4 * (y * W + x);
            const float d = depth[y * W + x];
            if (d == MINF) { o[0] = o[1] = o[2] = o[3] = MINF; continue; }
            o[0] = ((float)x - cam.mx) / cam.fx * d;
            o[1] = ((float)y - cam.my) / cam.fy * d;
            o[2] = d;
            o[3] = 1.0f;
        }
    // computeNormals_Kernel (CUDAImageUtil.cu:404-431), w = 0
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) {
            float* o = normals + 4 * (y * W + x);
            o[0] = o[1] = o[2] = o[3] = MINF;
            if (x > 0 && x < W - 1 && y > 0 && y < H - 1) {
                const float* CC = campos + 4 * (y * W + x);
                const float* PC = campos + 4 * ((y + 1) * W + x);
                const float* CP = campos + 4 * (y * W + x + 1);
                const float* MC = campos + 4 * ((y - 1) * W + x);
                const float* CM = campos + 4 * (y * W + x - 1);
                if (CC[0] != MINF && PC[0] != MINF && CP[0] != MINF && MC[0] != MINF && CM[0] != MINF) {
                    const f3 n = cross3(mk3(PC[0], PC[1], PC[2]) - mk3(MC[0], MC[1], MC[2]), mk3(CP[0], CP[1], CP[2]) - mk3(CM[0], CM[1], CM[2]));
                    const float l = length3(n);
                    if (l > 0.0f) { o[0] = n.x / -l; o[1] = n.y / -l; o[2] = n.z / -l; o[3] = 0.0f; }
                }
            }
        }
    // convertNormalsFloat4ToUCHAR4 (CUDAImageUtil.cu:497-513)
    for (uint32_t k = 0; k < W * H; k++) {
        const float* n = normals + 4 * k;
        uint8_t* o = normalsU8 + 4 * k;
        o[0] = o[1] = o[2] = o[3] = 0;
        if (n[0] != MINF) {
            o[0] = (uint8_t)roundf((n[0] + 1.0f) / 2.0f * 255);
            o[1] = (uint8_t)roundf((n[1] + 1.0f) / 2.0f * 255);
            o[2] = (uint8_t)roundf((n[2] + 1.0f) / 2.0f * 255);
        }
    }
    // convertToIntensity (CUDAImageUtil.cu:197-199)
    for (uint32_t k = 0; k < W * H; k++) {
        const uint32_t c = color[k];
        intensity[k] = (0.299f * (float)(c & 0xFF) + 0.587f * (float)((c >> 8) & 0xFF) + 0.114f * (float)((c >> 16) & 0xFF)) / 255.0f;
    }
    // computeIntensityDerivatives_Kernel (CUDAImageUtil.cu:260-296)
    for (uint32_t y = 0; y < H; y++)
        for (uint32_t x = 0; x < W; x++) {
            float* o = intensityDeriv + 2 * (y * W + x);
            o[0] = o[1] = MINF;
            if (x > 0 && x < W - 1 && y > 0 && y < H - 1) {
                auto I = [&](int dx, int dy) { return intensity[(y + dy) * W + (x + dx)]; };
                const float p00 = I(-1, -1), p01 = I(-1, 0), p02 = I(-1, 1), p10 = I(0, -1), p12 = I(0, 1), p20 = I(1, -1), p21 = I(1, 0), p22 = I(1, 1);
                float u = (-1.0f) * p00 + (1.0f) * p20 + (-2.0f) * p01 + (2.0f) * p21 + (-1.0f) * p02 + (1.0f) * p22;
                float v = (-1.0f) * p00 + (-2.0f) * p10 + (-1.0f) * p20 + (1.0f) * p02 + (2.0f) * p12 + (1.0f) * p22;
                o[0] = u / 8.0f;
                o[1] = v / 8.0f;
            }
        }
}

}  // namespace bf
