// raycast.hip — gfx950 raycaster of the voxel-hash TSDF (replaces CUDARayCastSDF,
// /root/reference/FriedLiver/Source/DepthSensing/CUDARayCastSDF.cu/.cpp, RayCastSDFUtil.h, and the
// D3D11 ray-interval splatting of DX11RayIntervalSplatting.cpp + Shaders/RayIntervalSplatting.hlsl).
//
//  * Ray-interval splat without a rasteriser: one wave per visible block projects the block's 8
//    corners (cameraToDepthProj), takes the NDC bounding rectangle and depth range, and updates the
//    covered pixels with atomicMin / atomicMax on order-preserving integer encodings of the world
//    depth. Coverage follows the D3D11 pixel-centre rule (left/top edges inclusive); the depth
//    tests are those of the two passes with depth clipping disabled (min pass: LESS against a
//    depth buffer cleared to 1, so quads with NDC z >= 1 never write; max pass: GREATER against 0).
//  * renderKernel / traverseCoarseGridSimpleSampleAll: one thread per pixel marches the splatted
//    interval in rayIncrement steps with trilinear SDF samples (8 voxel fetches, any zero weight
//    invalidates the sample), 3 linear-bisection refinements at a + -> - crossing. A per-thread
//    one-entry block cache skips the hash probe when consecutive fetches hit the same block
//    (results are unchanged: it caches the lookup, not the voxel).
//  * computeNormals from the camera-space points (or the SDF gradient when useGradients).
#include "hash_dev.h"
#include "tsdf.h"
#include <cstdlib>

#include <cstring>

namespace bf {

BFMat4 mat4_inverse(const BFMat4& M);  // api.cpp

namespace {

const float MINF_F = -__builtin_inff();
enum RenderStat { RS_SAMPLES = 0, RS_LOADS, RS_PROBES, RS_RAYS, RS_QUADS, RS_ATOMICS, RS_RENDERS, RS_PIXELS, RS_WAVESAMPLES, RS_COUNT };

__device__ __forceinline__ uint32_t enc_f(float f) {  // monotone float -> uint32
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}
__device__ __forceinline__ float dec_f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }

struct RayArgs {
    const BFHashEntry* hash;
    const BFVoxel* voxels;
    uint32_t numBuckets, numEntries, maxList;
    float voxelSize;
    uint32_t ldsTable;  // 1: the workgroup's LDS block table may hold heap indices (numBlocks < 2^24 - 1)
};

// The workgroup's block table in LDS: the rays of a 16x16 tile cross the same blocks, so a block one ray
// located is found by its neighbours without a hash probe (a probe is a dependent load from a table of
// 2^23 buckets in HBM; this is one LDS read). Direct-mapped, one 64-bit word per slot: 39 key bits (block
// coordinates + 4096, 13 bits each, in [0, 8190]) and 24 bits of heap index (0xFFFFFF: a free block). A
// 64-bit LDS store is single-copy atomic, so a reader sees an empty slot or a whole entry; the hash does
// not change during a render, so every entry stays valid. Blocks outside the key range take the probe.
constexpr int RC_SLOTS = 1024;
constexpr unsigned long long RC_EMPTY = ~0ull;
__device__ __forceinline__ bool rc_key(i3 b, unsigned long long& key) {
    const uint32_t x = (uint32_t)(b.x + 4096), y = (uint32_t)(b.y + 4096), z = (uint32_t)(b.z + 4096);
    key = ((unsigned long long)x << 26) | ((unsigned long long)y << 13) | (unsigned long long)z;
    return x <= 8190u && y <= 8190u && z <= 8190u;
}
__device__ __forceinline__ uint32_t rc_slot(i3 b) {
    return ((uint32_t)b.x * 73856093u ^ (uint32_t)b.y * 19349669u ^ (uint32_t)b.z * 83492791u) & (RC_SLOTS - 1);
}

// cameraToDepthProj (RayCastSDFUtil.h:208-222)
__device__ __forceinline__ f3 camera_to_depth_proj(const BFRayCastParams& p, f3 pos) {
    const float px = pos.x * p.fx / pos.z + p.mx;
    const float py = pos.y * p.fy / pos.z + p.my;
    f3 r;
    r.x = (2.0f * px - ((float)p.width - 1.0f)) / ((float)p.width - 1.0f);
    r.y = (((float)p.height - 1.0f) - 2.0f * py) / ((float)p.height - 1.0f);
    r.z = (pos.z - p.minDepth) / (p.maxDepth - p.minDepth);
    return r;
}
// depthToCamera with the ray-cast intrinsics (RayCastSDFUtil.h:201-206)
__device__ __forceinline__ f3 rc_depth_to_camera(const BFRayCastParams& p, uint32_t ux, uint32_t uy, float depth) {
    const float x = ((float)ux - p.mx) / p.fx;
    const float y = ((float)uy - p.my) / p.fy;
    return mk3(depth * x, depth * y, depth);
}

__device__ __forceinline__ f3 fmin3(f3 a, f3 b) { return mk3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
__device__ __forceinline__ f3 fmax3(f3 a, f3 b) { return mk3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }

__global__ void k_splat_clear(uint32_t* smin, uint32_t* smax, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        smin[i] = enc_f(__builtin_inff());
        smax[i] = enc_f(-__builtin_inff());
    }
}

// rayIntervalSplatKernel (CUDARayCastSDF.cu:101-190) for both passes + the raster of its quads
__global__ __launch_bounds__(256) void k_splat(const int4* __restrict__ visible, const uint32_t* ctrl, float voxelSize,
                                               BFDepthCameraParams cam, BFRayCastParams rp, uint32_t* smin, uint32_t* smax,
                                               unsigned long long* stats) {
    const uint32_t n = ctrl[C_VISIBLE];
    uint32_t quads = 0, atoms = 0;  // per wave (uniform): rasterised blocks, atomic depth updates
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const BFMat4 V = rp.viewMatrix;
    for (uint32_t b = wave; b < n; b += nwaves) {
        const int4 e = visible[b];
        if (!block_in_frustum(cam, V, e.x, e.y, e.z, voxelSize)) continue;  // :107 (isSDFBlockInCameraFrustumApprox)
        const f3 wv = block_to_world(e.x, e.y, e.z, voxelSize);
        const float hv = voxelSize / 2.0f;
        const f3 MINV = mk3(wv.x - hv, wv.y - hv, wv.z - hv);
        const float ext = (float)BF_SDF_BLOCK_SIZE * voxelSize;
        const f3 maxv = mk3(MINV.x + ext, MINV.y + ext, MINV.z + ext);
        const f3 p000 = camera_to_depth_proj(rp, xform(V, mk3(MINV.x, MINV.y, MINV.z)));
        const f3 p100 = camera_to_depth_proj(rp, xform(V, mk3(maxv.x, MINV.y, MINV.z)));
        const f3 p010 = camera_to_depth_proj(rp, xform(V, mk3(MINV.x, maxv.y, MINV.z)));
        const f3 p001 = camera_to_depth_proj(rp, xform(V, mk3(MINV.x, MINV.y, maxv.z)));
        const f3 p110 = camera_to_depth_proj(rp, xform(V, mk3(maxv.x, maxv.y, MINV.z)));
        const f3 p011 = camera_to_depth_proj(rp, xform(V, mk3(MINV.x, maxv.y, maxv.z)));
        const f3 p101 = camera_to_depth_proj(rp, xform(V, mk3(maxv.x, MINV.y, maxv.z)));
        const f3 p111 = camera_to_depth_proj(rp, xform(V, mk3(maxv.x, maxv.y, maxv.z)));
        const f3 mn = fmin3(fmin3(fmin3(p000, p100), fmin3(p010, p001)), fmin3(fmin3(p110, p011), fmin3(p101, p111)));
        const f3 mx = fmax3(fmax3(fmax3(p000, p100), fmax3(p010, p001)), fmax3(fmax3(p110, p011), fmax3(p101, p111)));
        // depthProjToCameraZ (RayCastSDFUtil.h:196-199)
        const float dwMin = mn.z * (rp.maxDepth - rp.minDepth) + rp.minDepth;
        const float dwMax = mx.z * (rp.maxDepth - rp.minDepth) + rp.minDepth;
        const bool minOk = mn.z < 1.0f;  // LESS vs depth cleared to 1 (NDC z clamped to [0,1])
        const bool maxOk = mx.z > 0.0f;  // GREATER vs depth cleared to 0
        if (!minOk && !maxOk) continue;
        const float W = (float)rp.width, H = (float)rp.height;
        const float left = (mn.x + 1.0f) * 0.5f * W, right = (mx.x + 1.0f) * 0.5f * W;
        const float top = (1.0f - mx.y) * 0.5f * H, bottom = (1.0f - mn.y) * 0.5f * H;
        if (!(left < right) || !(top < bottom)) continue;  // empty or NaN
        const float fx0 = ceilf(left - 0.5f), fx1 = ceilf(right - 0.5f) - 1.0f;
        const float fy0 = ceilf(top - 0.5f), fy1 = ceilf(bottom - 0.5f) - 1.0f;
        if (fx1 < 0.0f || fy1 < 0.0f || fx0 > W - 1.0f || fy0 > H - 1.0f) continue;
        const int x0 = (int)fmaxf(fx0, 0.0f), x1 = (int)fminf(fx1, W - 1.0f);
        const int y0 = (int)fmaxf(fy0, 0.0f), y1 = (int)fminf(fy1, H - 1.0f);
        if (x1 < x0 || y1 < y0) continue;
        const uint32_t w = (uint32_t)(x1 - x0 + 1), npx = w * (uint32_t)(y1 - y0 + 1);
        const uint32_t emin = enc_f(dwMin), emax = enc_f(dwMax);
        quads++;
        // every covered pixel takes an atomic min / max (no return value: the wave does not wait on
        // them). Reading the target first to skip the atomics that cannot change it cut them 3x
        // (8.9 -> 2.9 M per render) but put a dependent load in front of each: 143 -> 178 us
        atoms += npx * ((minOk ? 1u : 0u) + (maxOk ? 1u : 0u));
        for (uint32_t k = lane; k < npx; k += 64) {
            const uint32_t idx = (uint32_t)(y0 + (int)(k / w)) * rp.width + (uint32_t)(x0 + (int)(k % w));
            if (minOk) atomicMin(&smin[idx], emin);
            if (maxOk) atomicMax(&smax[idx], emax);
        }
    }
    if (lane == 0 && quads) {
        atomicAdd(&stats[RS_QUADS], (unsigned long long)quads);
        atomicAdd(&stats[RS_ATOMICS], (unsigned long long)atoms);
    }
}

// getVoxel(worldPos) (VoxelUtilHashSDF.h:406-417) with a two-entry per-thread block cache: a trilinear
// sample's corners straddle a block face about a third of the time, and a one-entry cache re-probed the hash
// as the corners alternated between the two blocks (up to six probes per sample instead of two)
struct BlockCache {
    int ax = INT_MIN, ay = 0, az = 0, ap = BF_FREE_ENTRY;  // entry A
    int bx = INT_MIN, by = 0, bz = 0, bp = BF_FREE_ENTRY;  // entry B
    bool replaceB = false;  // the entry a miss replaces (the one not used last)
    uint32_t samples = 0, loads = 0, probes = 0;  // render statistics (trilinear samples, voxel loads, hash probes)
    unsigned long long* table = nullptr;  // the workgroup's LDS block table (nullptr: probe every miss)
    __device__ __forceinline__ int lookup(const RayArgs& R, i3 b) {
        // hits and updates as register selects: written as branches on the two entries, the compiler kept the
        // pair {ap, bp} in scratch and read it back on every hit (a memory round trip per corner lookup)
        const bool hitA = b.x == ax && b.y == ay && b.z == az;
        const bool hitB = b.x == bx && b.y == by && b.z == bz;
        if (hitA || hitB) {
            replaceB = hitA;
            return hitA ? ap : bp;
        }
        int p;
        unsigned long long key;
        const bool keyed = table && rc_key(b, key);
        const uint32_t slot = rc_slot(b);
        const unsigned long long e = keyed ? table[slot] : RC_EMPTY;
        if (keyed && e != RC_EMPTY && (e >> 24) == key) {
            const uint32_t q = (uint32_t)e & 0xFFFFFFu;
            p = q == 0xFFFFFFu ? BF_FREE_ENTRY : (int)q;
        } else {
            p = hash_lookup(R.hash, R.numBuckets, R.numEntries, R.maxList, b.x, b.y, b.z);
            probes++;
            if (keyed) table[slot] = (key << 24) | (p < 0 ? 0xFFFFFFull : (unsigned long long)(uint32_t)p);
        }
        const bool toB = replaceB;
        bx = toB ? b.x : bx; by = toB ? b.y : by; bz = toB ? b.z : bz; bp = toB ? p : bp;
        ax = toB ? ax : b.x; ay = toB ? ay : b.y; az = toB ? az : b.z; ap = toB ? ap : p;
        replaceB = !replaceB;
        return p;
    }
};
__device__ __forceinline__ void get_voxel(const RayArgs& R, BlockCache& c, f3 pos, float& sdf, float& weight, uint32_t& color) {
    const i3 v = world_to_vvox(pos, R.voxelSize);
    const i3 b = vvox_to_block(v);
    const int ptr = c.lookup(R, b);
    if (ptr == BF_FREE_ENTRY) {  // deleteVoxel
        sdf = 0.0f; weight = 0.0f; color = 0u;
        return;
    }
    int lx = v.x % BF_SDF_BLOCK_SIZE, ly = v.y % BF_SDF_BLOCK_SIZE, lz = v.z % BF_SDF_BLOCK_SIZE;
    if (lx < 0) lx += BF_SDF_BLOCK_SIZE;
    if (ly < 0) ly += BF_SDF_BLOCK_SIZE;
    if (lz < 0) lz += BF_SDF_BLOCK_SIZE;
    const BFVoxel* vp = R.voxels + (size_t)ptr * BF_VOXELS_PER_BLOCK + (lz * BF_SDF_BLOCK_SIZE * BF_SDF_BLOCK_SIZE + ly * BF_SDF_BLOCK_SIZE + lx);
    c.loads++;
    sdf = vp->sdf;
    weight = vp->weight;
    color = *reinterpret_cast<const uint32_t*>(vp->color);
}

// the voxel of worldPos without loading it: nullptr for a free block (deleteVoxel: sdf 0, weight 0)
__device__ __forceinline__ const BFVoxel* voxel_ptr(const RayArgs& R, BlockCache& c, f3 pos) {
    const i3 v = world_to_vvox(pos, R.voxelSize);
    const i3 b = vvox_to_block(v);
    const int ptr = c.lookup(R, b);
    if (ptr == BF_FREE_ENTRY) return nullptr;
    int lx = v.x % BF_SDF_BLOCK_SIZE, ly = v.y % BF_SDF_BLOCK_SIZE, lz = v.z % BF_SDF_BLOCK_SIZE;
    if (lx < 0) lx += BF_SDF_BLOCK_SIZE;
    if (ly < 0) ly += BF_SDF_BLOCK_SIZE;
    if (lz < 0) lz += BF_SDF_BLOCK_SIZE;
    return R.voxels + (size_t)ptr * BF_VOXELS_PER_BLOCK + (lz * BF_SDF_BLOCK_SIZE * BF_SDF_BLOCK_SIZE + ly * BF_SDF_BLOCK_SIZE + lx);
}

__device__ __forceinline__ float frac1(float v) { return v - floorf(v); }

// trilinearInterpolationSimpleFastFast (RayCastSDFUtil.h:96-116). On a zero-weight corner it returns
// false with dist holding the partial sum, which gradientForPoint then uses as the reference does.
__device__ __forceinline__ bool trilinear(const RayArgs& R, BlockCache& c, f3 pos, float& dist, uint32_t& rgb) {
    const float oSet = R.voxelSize;
    const f3 posDual = pos - mk3(oSet / 2.0f, oSet / 2.0f, oSet / 2.0f);
    const f3 vv = pos / R.voxelSize;
    c.samples++;
    const f3 weight = mk3(frac1(vv.x), frac1(vv.y), frac1(vv.z));
    dist = 0.0f;
    f3 colorFloat = mk3(0.0f, 0.0f, 0.0f);
    // corner k's offset (the reference's order: 000, 100, 010, 001, 110, 011, 101, 111), selected per
    // component rather than read from a table (an offset table was kept in scratch)
    auto offs = [&](int k) {
        return mk3((k == 1 || k == 4 || k == 6 || k == 7) ? oSet : 0.0f, (k == 2 || k == 4 || k == 5 || k == 7) ? oSet : 0.0f,
                   (k == 3 || k == 5 || k == 6 || k == 7) ? oSet : 0.0f);
    };
    // the 8 corners' voxels located first (hash probes only where the block changes), then loaded
    // together: the reference reads them one after another and stops at the first zero weight, which
    // made each load wait for the previous one; the sums below keep its order and its stop
    float vs[8], vw[8];
    uint32_t vc[8];
    // corner 000 in a free block: the reference's first corner read has weight 0 and the sample ends
    // there, so the other corners are not located (no probes in free space)
    const BFVoxel* v0 = voxel_ptr(R, c, posDual + offs(0));
    if (!v0) return false;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const BFVoxel* vp = k == 0 ? v0 : voxel_ptr(R, c, posDual + offs(k));
        vs[k] = 0.0f; vw[k] = 0.0f; vc[k] = 0u;
        if (vp) {
            vs[k] = vp->sdf;
            vw[k] = vp->weight;
            vc[k] = *reinterpret_cast<const uint32_t*>(vp->color);
            c.loads++;
        }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const float sdf = vs[k], w = vw[k];
        const uint32_t col = vc[k];
        if (w == 0.0f) return false;
        const f3 vColor = mk3((float)(col & 0xFF), (float)((col >> 8) & 0xFF), (float)((col >> 16) & 0xFF));
        const float a = (k == 1 || k == 4 || k == 6 || k == 7) ? weight.x : 1.0f - weight.x;
        const float bq = (k == 2 || k == 4 || k == 5 || k == 7) ? weight.y : 1.0f - weight.y;
        const float cq = (k == 3 || k == 5 || k == 6 || k == 7) ? weight.z : 1.0f - weight.z;
        const float wt = a * bq * cq;
        dist += wt * sdf;
        colorFloat += wt * vColor;
    }
    // make_uchar3(float, float, float): float -> unsigned char conversion
    rgb = (uint32_t)(uint8_t)colorFloat.x | ((uint32_t)(uint8_t)colorFloat.y << 8) | ((uint32_t)(uint8_t)colorFloat.z << 16);
    return true;
}

// gradientForPoint (RayCastSDFUtil.h:172-194)
__device__ __forceinline__ f3 gradient_for_point(const RayArgs& R, BlockCache& c, f3 pos) {
    const float vs = R.voxelSize;
    const f3 offset = mk3(vs, vs, vs);
    float dp00, d0p0, d00p, d100, d010, d001;
    uint32_t col;
    trilinear(R, c, pos - mk3(0.5f * offset.x, 0.0f, 0.0f), dp00, col);
    trilinear(R, c, pos - mk3(0.0f, 0.5f * offset.y, 0.0f), d0p0, col);
    trilinear(R, c, pos - mk3(0.0f, 0.0f, 0.5f * offset.z), d00p, col);
    trilinear(R, c, pos + mk3(0.5f * offset.x, 0.0f, 0.0f), d100, col);
    trilinear(R, c, pos + mk3(0.0f, 0.5f * offset.y, 0.0f), d010, col);
    trilinear(R, c, pos + mk3(0.0f, 0.0f, 0.5f * offset.z), d001, col);
    const f3 grad = mk3((dp00 - d100) / offset.x, (d0p0 - d010) / offset.y, (d00p - d001) / offset.z);
    const float l = length3(grad);
    if (l == 0.0f) return mk3(0.0f, 0.0f, 0.0f);
    return (-grad) / l;
}

// renderKernel (CUDARayCastSDF.cu:17-57) + traverseCoarseGridSimpleSampleAll (RayCastSDFUtil.h:224-290)
__device__ __forceinline__ void render_pixel(const RayArgs& R, const BFRayCastParams& rp, BlockCache& cache, uint32_t x, uint32_t y,
                             const uint32_t* __restrict__ smin, const uint32_t* __restrict__ smax, float* d_depth,
                             float4* d_depth4, float4* d_normals, float4* d_colors, float* outMin, float* outMax, bool& rayed) {
    const uint32_t pix = y * rp.width + x;
    const float MINF = -__builtin_inff();
    d_depth[pix] = MINF;
    d_depth4[pix] = make_float4(MINF, MINF, MINF, MINF);
    d_normals[pix] = make_float4(MINF, MINF, MINF, MINF);
    d_colors[pix] = make_float4(MINF, MINF, MINF, MINF);
    const uint32_t emn = smin[pix], emx = smax[pix];
    // min target cleared to -inf, max target to 0 (DX11RayIntervalSplatting.cpp:174,203)
    float minInterval = (emn == enc_f(__builtin_inff())) ? MINF : dec_f(emn);
    float maxInterval = (emx == enc_f(-__builtin_inff())) ? 0.0f : dec_f(emx);
    if (outMin) outMin[pix] = minInterval;
    if (outMax) outMax[pix] = maxInterval;

    const f3 camDir = normalize3(rc_depth_to_camera(rp, x, y, 1.0f));
    const f3 worldCamPos = xform(rp.viewMatrixInverse, mk3(0.0f, 0.0f, 0.0f));
    const f3 w4 = xform4(rp.viewMatrixInverse, camDir, 0.0f);
    const f3 worldDir = normalize3(w4);
    if (minInterval == 0.0f || minInterval == MINF) return;
    if (maxInterval == 0.0f || maxInterval == MINF) return;
    minInterval = fmaxf(minInterval, rp.minDepth);
    maxInterval = fminf(maxInterval, rp.maxDepth);
    rayed = true;

    float lastSdf = 0.0f, lastAlpha = 0.0f;
    int lastWeight = 0;
    const float depthToRayLength = 1.0f / camDir.z;
    float rayCurrent = depthToRayLength * fmaxf(rp.minDepth, minInterval);
    const float rayEnd = depthToRayLength * fminf(rp.maxDepth, maxInterval);
    while (rayCurrent < rayEnd) {
        const f3 cur = worldCamPos + rayCurrent * worldDir;
        float dist;
        uint32_t rgb;
        if (trilinear(R, cache, cur, dist, rgb)) {
            if (lastWeight > 0 && lastSdf > 0.0f && dist < 0.0f) {
                // findIntersectionBisection (RayCastSDFUtil.h:130-156), 3 iterations
                float a = lastAlpha, aDist = lastSdf, b = rayCurrent, bDist = dist, c = 0.0f;
                uint32_t rgb2 = 0;
                bool ok = true;
                for (int it = 0; it < 3; it++) {
                    c = a + (aDist / (aDist - bDist)) * (b - a);
                    float cDist;
                    if (!trilinear(R, cache, worldCamPos + c * worldDir, cDist, rgb2)) { ok = false; break; }
                    if (aDist * cDist > 0.0f) { a = c; aDist = cDist; }
                    else { b = c; bDist = cDist; }
                }
                const float alpha = c;
                if (ok && fabsf(lastSdf - dist) < rp.thresSampleDist) {
                    if (fabsf(dist) < rp.thresDist) {
                        const float depth = alpha / depthToRayLength;
                        d_depth[pix] = depth;
                        const f3 cp = rc_depth_to_camera(rp, x, y, depth);
                        d_depth4[pix] = make_float4(cp.x, cp.y, cp.z, 1.0f);
                        d_colors[pix] = make_float4((float)(rgb2 & 0xFF) / 255.f, (float)((rgb2 >> 8) & 0xFF) / 255.f,
                                                    (float)((rgb2 >> 16) & 0xFF) / 255.f, 1.0f);
                        if (rp.useGradients) {
                            const f3 iso = worldCamPos + alpha * worldDir;
                            const f3 nrm = -gradient_for_point(R, cache, iso);
                            const f3 n = xform4(rp.viewMatrix, nrm, 0.0f);
                            d_normals[pix] = make_float4(n.x, n.y, n.z, 1.0f);
                        }
                        return;
                    }
                }
            }
            lastSdf = dist;
            lastAlpha = rayCurrent;
            lastWeight = 1;
            rayCurrent += rp.rayIncrement;
        } else {
            lastWeight = 0;
            rayCurrent += rp.rayIncrement;
        }
    }
}
// stats: [RS_SAMPLES] trilinear samples, [RS_LOADS] voxel loads, [RS_PROBES] hash probes, [RS_RAYS] marched rays
// Pixel shape: each wave marches an 8x8 pixel square (neighbouring rays cross the same blocks and end at
// similar depths); TPB 256: a workgroup is a 16x16 tile of four such squares, TPB 64: one square per
// workgroup, so a slot frees as soon as its one wave ends (A/B, BF_RENDER_TPB)
#ifndef BF_RENDER_WPE  // A/B builds: waves per SIMD asked of the compiler (0: its own choice, 101 VGPRs -> 4)
#define BF_RENDER_WPE 0
#endif
#if BF_RENDER_WPE
#define BF_RENDER_ATTR __attribute__((amdgpu_waves_per_eu(BF_RENDER_WPE)))
#else
#define BF_RENDER_ATTR
#endif
template <int TPB>
__global__ __launch_bounds__(TPB) BF_RENDER_ATTR void k_render(RayArgs R, BFRayCastParams rp, const uint32_t* __restrict__ smin,
                                                const uint32_t* __restrict__ smax, float* d_depth, float4* d_depth4,
                                                float4* d_normals, float4* d_colors, float* outMin, float* outMax,
                                                unsigned long long* stats) {
    constexpr uint32_t TILE = TPB == 256 ? 16u : 8u;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t x = blockIdx.x * TILE + (wv & 1u) * 8u + (lane & 7u), y = blockIdx.y * TILE + (wv >> 1) * 8u + (lane >> 3);
    __shared__ unsigned long long s_table[RC_SLOTS];
    for (uint32_t i = threadIdx.x; i < (uint32_t)RC_SLOTS; i += TPB) s_table[i] = RC_EMPTY;
    __syncthreads();
    BlockCache cache;
    if (R.ldsTable) cache.table = s_table;
    bool rayed = false;
    if (x < rp.width && y < rp.height)
        render_pixel(R, rp, cache, x, y, smin, smax, d_depth, d_depth4, d_normals, d_colors, outMin, outMax, rayed);
    const uint32_t s = wave_sum_u32(cache.samples), l = wave_sum_u32(cache.loads), p = wave_sum_u32(cache.probes);
    const uint32_t r = wave_sum_u32(rayed ? 1u : 0u);
    uint32_t wmax = cache.samples;  // the wave's longest march
    for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off));
    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
        atomicAdd(&stats[RS_RENDERS], 1ull);
        atomicAdd(&stats[RS_PIXELS], (unsigned long long)rp.width * rp.height);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&stats[RS_SAMPLES], (unsigned long long)s);
        atomicAdd(&stats[RS_LOADS], (unsigned long long)l);
        atomicAdd(&stats[RS_PROBES], (unsigned long long)p);
        atomicAdd(&stats[RS_RAYS], (unsigned long long)r);
        atomicAdd(&stats[RS_WAVESAMPLES], 64ull * wmax);
    }
}

// computeNormalsDevice (CameraUtil.cu:665-692)
__global__ void k_normals(float4* out, const float4* in, uint32_t W, uint32_t H) {
    const uint32_t x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= W || y >= H) return;
    const float MINF = -__builtin_inff();
    float4 o = make_float4(MINF, MINF, MINF, MINF);
    if (x > 0 && x < W - 1 && y > 0 && y < H - 1) {
        const float4 CC = in[y * W + x], PC = in[(y + 1) * W + x], CP = in[y * W + x + 1];
        const float4 MC = in[(y - 1) * W + x], CM = in[y * W + x - 1];
        if (CC.x != MINF && PC.x != MINF && CP.x != MINF && MC.x != MINF && CM.x != MINF) {
            const f3 n = cross3(mk3(PC.x, PC.y, PC.z) - mk3(MC.x, MC.y, MC.z), mk3(CP.x, CP.y, CP.z) - mk3(CM.x, CM.y, CM.z));
            const float l = length3(n);
            if (l > 0.0f) o = make_float4(n.x / -l, n.y / -l, n.z / -l, 1.0f);
        }
    }
    out[y * W + x] = o;
}

}  // namespace

void Scene::renderStats(BFRenderStats& out) {
    uint64_t c[RS_COUNT];
    BF_HIP(hipMemcpyAsync(c, renderStats_.p, sizeof(c), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    out.samples = c[RS_SAMPLES]; out.voxelLoads = c[RS_LOADS]; out.hashProbes = c[RS_PROBES]; out.rays = c[RS_RAYS];
    out.splatBlocks = c[RS_QUADS]; out.splatAtomics = c[RS_ATOMICS]; out.renders = c[RS_RENDERS]; out.pixels = c[RS_PIXELS];
    out.waveSamples = c[RS_WAVESAMPLES];
    out.timedRenders = renderClock_.enabled() ? renderClock_.launches() : 0;
    out.renderMs = renderClock_.enabled() ? renderClock_.totalMs() : 0.0;
    out.splatMs = splatClock_.enabled() ? splatClock_.totalMs() : 0.0;
}

void Scene::raycast(const BFMat4& T, const BFDepthCameraParams& cam, const BFRayCastParams& rpIn, float* depth, float4* depth4,
                    float4* normals, float4* colors, float* rayMin, float* rayMax) {
    BF_REQUIRE(depth && depth4 && normals && colors, BF_ERR_ARG, "raycast outputs");
    BF_REQUIRE(rpIn.width > 0 && rpIn.height > 0, BF_ERR_ARG, "raycast size");
    compactify(T, cam);  // setLastRigidTransformAndCompactify (CUDASceneRepHashSDF.h:128-139)
    BFRayCastParams rp = rpIn;
    rp.viewMatrixInverse = T;  // CUDARayCastSDF::rayIntervalSplatting sets both from the transform
    rp.viewMatrix = Tinv_;
    const size_t P = (size_t)rp.width * rp.height;
    if (P > splatCap_) {
        splatMin_.alloc(P);
        splatMax_.alloc(P);
        splatCap_ = P;
    }
    k_splat_clear<<<std::max(1u, std::min(div_up(P, 256), 2048u)), 256, 0, stream_>>>(splatMin_.p, splatMax_.p, (uint32_t)P);
    BF_LAUNCH_CHECK();
    const bool timed = renderClock_.enabled();
    if (timed) {
        if (!splatClock_.enabled()) splatClock_.enable(true);
        splatClock_.start(stream_);
    }
    k_splat<<<(unsigned)numCUs_ * 4, 256, 0, stream_>>>(visible_.p, ctrl_.p, cfg_.hp.virtualVoxelSize, cam, rp, splatMin_.p,
                                                          splatMax_.p, renderStats_.p);
    BF_LAUNCH_CHECK();
    if (timed) splatClock_.stop(stream_);
    RayArgs R;
    R.hash = hash_.p;
    R.voxels = voxels_.p;
    R.numBuckets = cfg_.hp.hashNumBuckets;
    R.numEntries = E_;
    R.maxList = cfg_.hp.hashMaxCollisionLinkedListSize;
    R.voxelSize = cfg_.hp.virtualVoxelSize;
    static const bool ldsTable = [] {
        const char* e = std::getenv("BF_RENDER_LDS_TABLE");  // A/B: 0 = probe every block-cache miss
        return !(e && std::atoi(e) == 0);
    }();
    R.ldsTable = ldsTable && cfg_.hp.numSDFBlocks < 0xFFFFFFu ? 1u : 0u;
    const dim3 g(div_up(rp.width, 16), div_up(rp.height, 16));
    static const int tpb = [] {
        const char* e = std::getenv("BF_RENDER_TPB");
        return e && std::atoi(e) == 64 ? 64 : 256;
    }();
    if (timed) renderClock_.start(stream_);
    if (tpb == 64)
        k_render<64><<<dim3(div_up(rp.width, 8), div_up(rp.height, 8)), 64, 0, stream_>>>(
            R, rp, splatMin_.p, splatMax_.p, depth, depth4, normals, colors, rayMin, rayMax, renderStats_.p);
    else
        k_render<256><<<g, 256, 0, stream_>>>(R, rp, splatMin_.p, splatMax_.p, depth, depth4, normals, colors, rayMin, rayMax,
                                              renderStats_.p);
    BF_LAUNCH_CHECK();
    if (timed) renderClock_.stop(stream_);
    if (!rp.useGradients) {
        k_normals<<<g, 256, 0, stream_>>>(normals, depth4, rp.width, rp.height);
        BF_LAUNCH_CHECK();
    }
}

}  // namespace bf
