// synth.hip — GPU renderer for the seeded synthetic RGB-D stream (see synth.h).
#include "synth.h"
#include "bf_runtime.h"

#include <cmath>
#include <cstring>

namespace bf {

__global__ __launch_bounds__(256) void k_synth_render(BFSynthScene sc, BFMat4 T, BFDepthCameraParams cam, uint32_t noiseSeed,
                                                      uint32_t frame, float* depth, uint32_t* color) {
    const uint32_t x = blockIdx.x * 16 + threadIdx.x % 16, y = blockIdx.y * 16 + threadIdx.x / 16;
    if (x >= cam.imageWidth || y >= cam.imageHeight) return;
    float d;
    uint32_t c;
    synth_pixel(sc, T, cam, noiseSeed, frame, x, y, d, c);
    depth[y * cam.imageWidth + x] = d;
    if (color) color[y * cam.imageWidth + x] = c;
}

void synth_render_device(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, uint32_t noiseSeed,
                         uint32_t frame, float* depth, uint8_t* color, hipStream_t stream) {
    dim3 g(div_up(cam.imageWidth, 16), div_up(cam.imageHeight, 16));
    k_synth_render<<<g, 256, 0, stream>>>(sc, T, cam, noiseSeed, frame, depth, reinterpret_cast<uint32_t*>(color));
    BF_LAUNCH_CHECK();
}

__global__ void k_synth_to_raw(const float* d, const uint32_t* c, uint32_t n, float shift, uint16_t* du, uint32_t* rgbx) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float v = d[i];
        du[i] = (v > 0.0f && v < INFINITY) ? (uint16_t)fminf(rintf(v * shift), 65535.0f) : (uint16_t)0;
        rgbx[i] = c[i];
    }
}
void synth_to_raw(const float* depth, const uint8_t* color, uint32_t n, float shift, uint16_t* du, uint8_t* rgbx,
                  hipStream_t stream) {
    if (!n) return;
    k_synth_to_raw<<<std::min(div_up(n, 256u), 4096u), 256, 0, stream>>>(depth, reinterpret_cast<const uint32_t*>(color), n, shift, du,
                                                                      reinterpret_cast<uint32_t*>(rgbx));
    BF_LAUNCH_CHECK();
}

void synth_render_host(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, uint32_t noiseSeed,
                       uint32_t frame, float* depth, uint8_t* color) {
    for (uint32_t y = 0; y < cam.imageHeight; y++)
        for (uint32_t x = 0; x < cam.imageWidth; x++) {
            float d;
            uint32_t c;
            synth_pixel(sc, T, cam, noiseSeed, frame, x, y, d, c);
            depth[y * cam.imageWidth + x] = d;
            if (color) std::memcpy(color + 4 * (y * cam.imageWidth + x), &c, 4);
        }
}

// 6x5x3 m room, 12 boxes on the floor + 12 spheres, placed in the ring the camera loop
// does not enter (|x| > ~1.9 or |z| > ~1.6).
void synth_scene_default(uint32_t seed, BFSynthScene* out) {
    std::memset(out, 0, sizeof(*out));
    out->seed = seed;
    out->roomMin[0] = -3.0f; out->roomMin[1] = -3.0f; out->roomMin[2] = -2.5f;
    out->roomMax[0] = 3.0f;  out->roomMax[1] = 0.0f;  out->roomMax[2] = 2.5f;
    uint32_t st = pcg_hash(seed + 12345u);
    auto rnd = [&]() { st = pcg_hash(st); return u01(st); };
    out->numPrimitives = 24;
    for (int k = 0; k < 24; k++) {
        float* P = out->prims[k];
        const bool box = k < 12;
        const float phi = 6.2831853f * ((float)k + rnd()) / 12.0f;
        const float size = 0.2f + 0.8f * rnd();
        const float half = 0.5f * size;
        float cx = 2.55f * cosf(phi), cz = 2.1f * sinf(phi);
        cx = fmaxf(-3.0f + half + 0.05f, fminf(3.0f - half - 0.05f, cx));
        cz = fmaxf(-2.5f + half + 0.05f, fminf(2.5f - half - 0.05f, cz));
        P[0] = box ? 0.0f : 1.0f;
        P[1] = cx;
        P[3] = cz;
        if (box) {
            const float h = 0.2f + 0.8f * rnd();
            P[4] = half;
            P[5] = 0.5f * h;
            P[6] = 0.5f * (0.2f + 0.8f * rnd());
            P[2] = -0.5f * h;  // resting on the floor (y = 0)
        } else {
            P[4] = half;  // radius 0.1 .. 0.5
            P[2] = -0.6f - 1.6f * rnd();
        }
        P[7] = rnd();
    }
}

}  // namespace bf
