// bf_math.h — float3/int3/float4x4 helpers for the gfx950 kernels and the host
// runtime. Arithmetic is written as explicit IEEE float32 operations (the library
// is compiled with -ffp-contract=off) in the operand order of the reference's
// cutil_math.h / cuda_SimpleMatrixUtil.h, so integer outcomes that hinge on float
// comparisons (which block a DDA visits, which pixel a voxel projects to) are
// reproducible between this build and the CPU oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits.h>
#include "../../include/bf/types.h"

#define BF_HD __host__ __device__ __forceinline__

namespace bf {

struct f3 { float x, y, z; };
struct i3 { int x, y, z; };

BF_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
BF_HD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
BF_HD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
BF_HD f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
BF_HD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
BF_HD f3 operator*(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
BF_HD f3 operator/(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
BF_HD f3 operator/(f3 a, f3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
BF_HD f3& operator+=(f3& a, f3 b) { a.x += b.x; a.y += b.y; a.z += b.z; return a; }
BF_HD f3& operator-=(f3& a, f3 b) { a.x -= b.x; a.y -= b.y; a.z -= b.z; return a; }
BF_HD f3 mul3(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
BF_HD float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
BF_HD f3 cross3(f3 a, f3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
BF_HD float length3(f3 a) { return sqrtf(dot3(a, a)); }
// normalize = v * rsqrtf(dot(v,v)) with the host definition rsqrtf = 1/sqrtf (cutil_math.h:81-84,1207-1210)
BF_HD f3 normalize3(f3 v) { float inv = 1.0f / sqrtf(dot3(v, v)); return v * inv; }

// cutil_math.h:31-33
BF_HD int sgn(float v) { return (0.0f < v) - (v < 0.0f); }

// float -> int with CUDA cvt.rzi.s32.f32 semantics (truncate, saturate, NaN -> 0): the
// conversion make_int3(float3) (cutil_math.h:179) performs in the reference kernels.
BF_HD int f2i(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
    // v_cvt_i32_f32 truncates, saturates out-of-range values and maps NaN to 0: exactly the
    // semantics above, in one instruction (inline asm: the C++ cast would be UB out of range)
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return r;
#else
    if (v != v) return 0;
    if (v >= 2147483648.0f) return INT_MAX;
    if (v <= -2147483648.0f) return INT_MIN;
    return (int)v;
#endif
}

struct m4 { float e[16]; };  // row-major, cuda_SimpleMatrixUtil.h:855-875

BF_HD m4 toM4(const BFMat4& a) { m4 r; for (int i = 0; i < 16; i++) r.e[i] = a.m[i]; return r; }

// float4x4 * float3 with implicit w = 1 (cuda_SimpleMatrixUtil.h:937-945)
BF_HD f3 xform(const m4& m, f3 v) {
    const float* e = m.e;
    return mk3(e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * 1.0f,
               e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * 1.0f,
               e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * 1.0f);
}
BF_HD f3 xform(const BFMat4& m, f3 v) {
    const float* e = m.m;
    return mk3(e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * 1.0f,
               e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * 1.0f,
               e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * 1.0f);
}
// float4x4 * float4 (cuda_SimpleMatrixUtil.h:925-933), xyz of the result
BF_HD f3 xform4(const BFMat4& m, f3 v, float w) {
    const float* e = m.m;
    return mk3(e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * w,
               e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * w,
               e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * w);
}

// Host-side general cofactor inverse (same term order as cuda_SimpleMatrixUtil.h:980-1090);
// defined in runtime.cpp.
BFMat4 mat4_inverse(const BFMat4& m);
BFMat4 mat4_mul(const BFMat4& a, const BFMat4& b);

// ---- voxel-hash coordinate maps (VoxelUtilHashSDF.h) --------------------------------
// computeHashPos :225-234 — wrapping int32 products
BF_HD uint32_t hash_bucket(int x, int y, int z, uint32_t numBuckets) {
    int32_t a = (int32_t)((uint32_t)x * 73856093u);
    int32_t b = (int32_t)((uint32_t)y * 19349669u);
    int32_t c = (int32_t)((uint32_t)z * 83492791u);
    int res = (a ^ b ^ c) % (int)numBuckets;
    if (res < 0) res += (int)numBuckets;
    return (uint32_t)res;
}

// worldToVirtualVoxelPos :283-287
BF_HD i3 world_to_vvox(f3 pos, float voxelSize) {
    f3 p = pos / voxelSize;
    f3 q = p + mk3((float)sgn(p.x), (float)sgn(p.y), (float)sgn(p.z)) * 0.5f;
    i3 r; r.x = f2i(q.x); r.y = f2i(q.y); r.z = f2i(q.z); return r;
}
// virtualVoxelPosToSDFBlock :290-299
BF_HD i3 vvox_to_block(i3 v) {
    if (v.x < 0) v.x -= BF_SDF_BLOCK_SIZE - 1;
    if (v.y < 0) v.y -= BF_SDF_BLOCK_SIZE - 1;
    if (v.z < 0) v.z -= BF_SDF_BLOCK_SIZE - 1;
    i3 r; r.x = v.x / BF_SDF_BLOCK_SIZE; r.y = v.y / BF_SDF_BLOCK_SIZE; r.z = v.z / BF_SDF_BLOCK_SIZE; return r;
}
BF_HD f3 vvox_to_world(int x, int y, int z, float voxelSize) {  // :308-310
    return mk3((float)x, (float)y, (float)z) * voxelSize;
}
BF_HD f3 block_to_world(int bx, int by, int bz, float voxelSize) {  // :313-315
    return vvox_to_world(bx * BF_SDF_BLOCK_SIZE, by * BF_SDF_BLOCK_SIZE, bz * BF_SDF_BLOCK_SIZE, voxelSize);
}
BF_HD i3 world_to_block(f3 w, float voxelSize) { return vvox_to_block(world_to_vvox(w, voxelSize)); }

// isInCameraFrustumApprox, DepthCameraUtil.h:95-107,137-144
BF_HD bool in_frustum(const BFDepthCameraParams& c, const BFMat4& viewInv, f3 pos) {
    f3 pc = xform(viewInv, pos);
    float px = pc.x * c.fx / pc.z + c.mx;
    float py = pc.y * c.fy / pc.z + c.my;
    float wm1 = (float)c.imageWidth - 1.0f, hm1 = (float)c.imageHeight - 1.0f;
    float x = (2.0f * px - wm1) / wm1;
    float y = (hm1 - 2.0f * py) / hm1;
    float z = (pc.z - c.sensorDepthWorldMin) / (c.sensorDepthWorldMax - c.sensorDepthWorldMin);
    x = x * 0.95f; y = y * 0.95f; z = z * 0.95f;  // pProj *= 0.95 (float operator*=, cutil_math.h:761)
    return !(x < -1.0f || x > 1.0f || y < -1.0f || y > 1.0f || z < 0.0f || z > 1.0f);
}
// isSDFBlockInCameraFrustumApprox, VoxelUtilHashSDF.h:322-326
BF_HD bool block_in_frustum(const BFDepthCameraParams& c, const BFMat4& viewInv, int bx, int by, int bz, float voxelSize) {
    f3 w = block_to_world(bx, by, bz, voxelSize) + mk3(1.0f, 1.0f, 1.0f) * (voxelSize * 0.5f * (BF_SDF_BLOCK_SIZE - 1.0f));
    return in_frustum(c, viewInv, w);
}

// kinectDepthToSkeleton, DepthCameraUtil.h:114-119
BF_HD f3 depth_to_camera(const BFDepthCameraParams& c, uint32_t ux, uint32_t uy, float depth) {
    const float x = ((float)ux - c.mx) / c.fx;
    const float y = ((float)uy - c.my) / c.fy;
    return mk3(depth * x, depth * y, depth);
}

// packed 63-bit key of a block coordinate (21 bits per axis, biased)
BF_HD uint64_t block_key(int x, int y, int z) {
    return ((uint64_t)(uint32_t)(x + (1 << 20)) << 42) | ((uint64_t)(uint32_t)(y + (1 << 20)) << 21) |
           (uint64_t)(uint32_t)(z + (1 << 20));
}
BF_HD i3 key_block(uint64_t k) {
    i3 r;
    r.x = (int)((k >> 42) & 0x1FFFFF) - (1 << 20);
    r.y = (int)((k >> 21) & 0x1FFFFF) - (1 << 20);
    r.z = (int)(k & 0x1FFFFF) - (1 << 20);
    return r;
}

}  // namespace bf
