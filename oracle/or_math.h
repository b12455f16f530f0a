// oracle/or_math.h — TEST INFRASTRUCTURE (CPU oracle). Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may use anything under oracle/.
//
// Scalar float3/int3/float4x4 helpers restating the reference's cutil_math.h and
// cuda_SimpleMatrixUtil.h arithmetic in plain IEEE float32 (compiled with
// -ffp-contract=off so every a*b+c is two rounded operations, as in the HIP build).
#pragma once
#include <cmath>
#include <cstdint>
#include <climits>

namespace orc {

struct f3 { float x, y, z; };
struct i3 { int x, y, z; };

inline f3 mk(float x, float y, float z) { return {x, y, z}; }
inline f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline f3 operator/(f3 a, f3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
inline f3 mul(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline f3 cross(f3 a, f3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline float length(f3 a) { return std::sqrt(dot(a, a)); }
// cutil_math.h:81-84 host rsqrtf = 1/sqrtf; normalize = v * rsqrtf(dot(v,v)) (cutil_math.h:1207-1210)
inline f3 normalize(f3 v) { float inv = 1.0f / std::sqrt(dot(v, v)); return v * inv; }

// cutil_math.h:31-33: sign() returns 0 at 0
inline int sgn(float v) { return (0.0f < v) - (v < 0.0f); }

// float -> int conversion with CUDA cvt.rzi.s32.f32 semantics (truncate toward zero,
// saturate, NaN -> 0): what make_int3(float3) (cutil_math.h:179) computes on the GPU.
inline int f2i(float v) {
    if (std::isnan(v)) return 0;
    if (v >= 2147483648.0f) return INT_MAX;
    if (v <= -2147483648.0f) return INT_MIN;
    return (int)v;
}

struct m4 { float e[16]; };  // row-major (cuda_SimpleMatrixUtil.h:855-875)

// float4x4 * float3, w = 1 (cuda_SimpleMatrixUtil.h:937-945)
inline f3 xform(const m4& m, f3 v) {
    const float* e = m.e;
    return {e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * 1.0f,
            e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * 1.0f,
            e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * 1.0f};
}
// float4x4 * float4 (cuda_SimpleMatrixUtil.h:925-933), returning xyz of (v, w)
inline f3 xform4(const m4& m, f3 v, float w) {
    const float* e = m.e;
    return {e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * w,
            e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * w,
            e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * w};
}

inline m4 matmul(const m4& a, const m4& b) {
    m4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = 0.0f;
            for (int k = 0; k < 4; k++) s += a.e[i * 4 + k] * b.e[k * 4 + j];
            r.e[i * 4 + j] = s;
        }
    return r;
}

// General cofactor inverse, cuda_SimpleMatrixUtil.h:980-1090 (same term order).
m4 inverse(const m4& m);

}  // namespace orc
