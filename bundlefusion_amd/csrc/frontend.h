// frontend.h — the stand-in for the SiftGPU tracking front end's frame-to-frame estimate.
//
// In the reference, the pose the reconstruction integrates a new frame with is the SIFT-matched
// Kabsch transform to the previous frame chained onto the last optimized pose
// (computeSiftTransformCU, Source/OnlineBundler.cu:6-71; computeCurrentSiftTransform,
// Source/OnlineBundler.cpp:117-134). SIFT is out of scope; a `.sens` file
// carries a camera trajectory, so the estimate here is that trajectory's relative motion with a
// seeded error step, which gives the local and global solves a drift to remove:
//
//   Tinc(f) = inv(T[f-1]) * T[f] * [R(w) | t],  w ~ N(0, driftRad^2 I3), t ~ N(0, driftM^2 I3)
//
// computed in double and rounded to float once. The normals come from a counter-based generator
// (splitmix64 of seed, frame and component -> uniform in (0, 1) -> Box-Muller), so the estimate of
// frame f does not depend on the order frames are read in. An invalid pose on either side (any
// non-finite entry, the .sens convention for a lost frame) gives the identity: "no motion".
// oracle/frames.cpp (or_front_end_tinc) restates the same arithmetic for the parity tests.
#pragma once
#include <cmath>
#include <cstdint>

#include "../../include/bf/types.h"

namespace bf {

inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// uniform in (0, 1) from the 53 high bits
inline double front_end_uniform(uint32_t seed, uint32_t frame, uint32_t k) {
    const uint64_t key = ((uint64_t)seed << 32) ^ ((uint64_t)frame << 3) ^ (uint64_t)k;
    return ((double)(splitmix64(key) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

inline BFMat4 front_end_tinc(const float* prev, const float* cur, uint32_t frame, uint32_t seed, float driftRad,
                             float driftM) {
    BFMat4 out{};
    out.m[0] = out.m[5] = out.m[10] = out.m[15] = 1.0f;
    for (int k = 0; k < 16; k++)
        if (!std::isfinite(prev[k]) || !std::isfinite(cur[k])) return out;
    // rigid inverse of prev (R^T, -R^T t), then inv(prev) * cur
    double A[16] = {0}, B[16], rel[16];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) A[4 * i + j] = (double)prev[4 * j + i];
        A[4 * i + 3] = -((double)prev[4 * 0 + i] * prev[3] + (double)prev[4 * 1 + i] * prev[7] + (double)prev[4 * 2 + i] * prev[11]);
    }
    A[15] = 1.0;
    for (int k = 0; k < 16; k++) B[k] = cur[k];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += A[4 * i + k] * B[4 * k + j];
            rel[4 * i + j] = s;
        }
    // six normals: Box-Muller over three uniform pairs
    double g[6];
    for (int p = 0; p < 3; p++) {
        const double u1 = front_end_uniform(seed, frame, 2 * p), u2 = front_end_uniform(seed, frame, 2 * p + 1);
        const double r = std::sqrt(-2.0 * std::log(u1)), a = 6.283185307179586 * u2;
        g[2 * p] = r * std::cos(a);
        g[2 * p + 1] = r * std::sin(a);
    }
    const double w[3] = {g[0] * driftRad, g[1] * driftRad, g[2] * driftRad};
    double step[16] = {0};
    const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (th > 1e-12) {  // Rodrigues
        const double kx = w[0] / th, ky = w[1] / th, kz = w[2] / th;
        const double K[9] = {0, -kz, ky, kz, 0, -kx, -ky, kx, 0};
        double K2[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) K2[3 * i + j] = K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j] + K[3 * i + 2] * K[6 + j];
        const double s = std::sin(th), c = 1.0 - std::cos(th);
        for (int i = 0; i < 9; i++) R[i] += s * K[i] + c * K2[i];
    }
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) step[4 * i + j] = R[3 * i + j];
        step[4 * i + 3] = g[3 + i] * driftM;
    }
    step[15] = 1.0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += rel[4 * i + k] * step[4 * k + j];
            out.m[4 * i + j] = (float)s;
        }
    return out;
}

}  // namespace bf
