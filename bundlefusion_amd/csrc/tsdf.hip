// tsdf.hip — gfx950 kernels + host class for the voxel-hash TSDF scene.
//
// Replaces the reference's CUDASceneRepHashSDF.cu kernels (citations are to
// /root/reference/FriedLiver/Source/DepthSensing/). Design points:
//  * alloc is two-phase and lock-free: a per-pixel DDA emits absent, in-frustum blocks,
//    de-duplicated per 16x16 tile in an LDS hash set and appended with wave-aggregated
//    atomics; a per-candidate insert dedups globally (64-bit CAS set) and claims a bucket
//    slot with a CAS on HashEntry.ptr. One pass replaces the reference's repeat-until-
//    stable try-lock loop and its host round trips (CUDASceneRepHashSDF.h:335-348).
//  * compactify streams the allocated prefix of a 16-B per-block position array instead of
//    the whole 32-B-per-entry hash table, with wave ballot + popcount compaction.
//  * integrate runs one wave per 8^3 block (8 z-slices of 64 voxels), touching a voxel's
//    12 B only when it lies inside the truncation band.
//  * GC reads a per-block count of voxels with (uint)weight != 0, maintained by the
//    integrate kernel, instead of re-reading 512 voxels per block.
#include "tsdf.h"
#include "../../include/bf/bf.h"
#include "hash_dev.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace bf {

namespace {

constexpr unsigned long long EMPTY_KEY = ~0ull;
constexpr int ALLOC_TILE = 16;          // 16x16 pixels per workgroup
constexpr int LDS_SET = 1024;           // per-tile candidate dedup set (8 KiB); slot = 10 low coordinate bits
constexpr uint32_t OVF_CAP = 1u << 16;  // collision-list inserts per op (serial path)
constexpr uint32_t GC_LIST_CAP = 4096;  // collision-list deletes per GC pass (serial path)

struct HashArgs {
    BFHashEntry* hash;
    uint32_t* heap;
    BFVoxel* voxels;
    int4* blockPos;
    uint32_t* blockCount;
    int4* visible;
    int4* band;
    const float2* tiles;
    uint32_t tilesW, tilesH;
    const float2* tiles2;  // 32x32-pixel depth bounds (footprints wider than 2x2 fine tiles)
    uint32_t tiles2W;
    uint32_t* ctrl;
    unsigned long long* stats;  // [STAT_SLOTS][16] counters, field order of BFTsdfStats
    uint32_t numBuckets, numEntries, numBlocks, maxList;
    float voxelSize, truncation, truncScale, maxIntegrationDistance, weightMax;
    // RN(1 / x) of the launch-uniform divisors the alloc walk's setup divides by (div_by_uniform), or 0
    // when x is outside [2^-20, 2^20] (the IEEE division runs); rFx / rFy are set per batch (camera)
    float rVoxelSize, rFx, rFy;
    uint32_t shardCount, shardIndex;
    uint32_t allocForceDirect;
    float shardChunk;
    // reference streaming bitmask (isSDFBlockStreamedOut, CUDASceneRepHashSDF.cu:152-163)
    const uint32_t* bitMask;
    BFFloat3 streamExtents;
    BFInt3 streamGridDims;
    BFInt3 streamMinGridPos;
};

// Sequence of voxel ops (integrate / de-integrate one depth map at one pose) applied as one pass
// (Scene::applyOps). Passed by value as a kernel argument: 3x4 matrices, image pointers, op kinds.
struct OpTable {
    float tinv[Scene::kMaxOps][12];  // world -> camera, rows 0-2
    float t[Scene::kMaxOps][12];     // camera -> world (alloc DDA)
    const float* depth[Scene::kMaxOps];
    const uint32_t* color[Scene::kMaxOps];
    uint8_t intIdx[Scene::kMaxOps];  // op index of the i-th integrate op
    float2* tiles[Scene::kMaxOps];   // per op: 8x8-pixel depth bounds of its depth map ...
    float2* tiles2[Scene::kMaxOps];  // ... and the 16x16 level
    uint2* dc[Scene::kMaxOps];       // per op: {depth bits, colour} per pixel, one 8-B gather per voxel
    uint8_t tileIdx[Scene::kMaxOps];  // op index of the i-th op whose frame caches this batch fills
    uint32_t n, deintMask, nInt, tileMask, nTile;  // tileMask: ops whose tiles and dc image this batch computes
};
__host__ __device__ __forceinline__ BFMat4 op_mat(const float* m) {
    BFMat4 r;
    for (int i = 0; i < 12; i++) r.m[i] = m[i];
    r.m[12] = 0.0f; r.m[13] = 0.0f; r.m[14] = 0.0f; r.m[15] = 1.0f;
    return r;
}

__device__ __forceinline__ unsigned lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ unsigned long long lanemask_lt() {
    unsigned l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// 12-B voxel as one 4-byte-aligned unit, so loads/stores become single dwordx3 accesses
struct __attribute__((packed, aligned(4))) Vox3 {
    uint32_t a, b, c;
};

enum StatField { S_PIXELS = 0, S_CAND, S_ALLOC, S_SCANNED, S_VISIBLE, S_VOXELS, S_GCBLOCKS, S_GCFREED, S_OVERFLOW, S_OPS,
                 S_BAND, S_RMW, S_BOPS, S_BBLOCKS, S_BRMW, S_BUPD, S_BEVAL, S_BHALF };
constexpr int DEPTH_TILE = 8;    // 8x8-pixel depth-bound tiles for the band cull
constexpr int DEPTH_TILE2 = 16;  // coarse level: 16x16 pixels
constexpr int STAT_SLOTS = 64;
constexpr int STAT_FIELDS = 32;  // counters per slot (BFTsdfStats uses the first sizeof/8)

// The lane index, re-read where it is used: an asm statement the compiler cannot hoist, so a long
// kernel does not keep lane-derived values live (or spilled) across its loops.
__device__ __forceinline__ unsigned lane_id_here() {
    unsigned l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
// Sum over the 64 lanes of a fully active wave through DPP row permutes (no LDS addresses to keep
// live): pairs, quads, half rows, rows, then the four row sums read into scalars.
__device__ __forceinline__ uint32_t dpp_row_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true);  // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true);  // row_mirror
    return v;
}
__device__ __forceinline__ int wave_sum(int v) {
    const uint32_t r = dpp_row_sum((uint32_t)v);
    return (int)(__builtin_amdgcn_readlane(r, 0) + __builtin_amdgcn_readlane(r, 16) + __builtin_amdgcn_readlane(r, 32) +
                 __builtin_amdgcn_readlane(r, 48));
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
    // 16-bit limbs: every partial sum of 64 lanes stays below 2^22, so no carries are lost
    unsigned long long s = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t r = dpp_row_sum((uint32_t)(v >> (16 * k)) & 0xFFFFu);
        s += (unsigned long long)(__builtin_amdgcn_readlane(r, 0) + __builtin_amdgcn_readlane(r, 16) +
                                  __builtin_amdgcn_readlane(r, 32) + __builtin_amdgcn_readlane(r, 48)) << (16 * k);
    }
    return s;
}

// Workgroup-level counter flush: wave sum, LDS add, then one global atomic per workgroup into one
// of 64 slots (no single hot word; summed on the host at query time). Every thread of the workgroup
// must call it (it contains a barrier).
__device__ void flush_stats2(unsigned long long* stats, int f0, unsigned long long v0, int f1, unsigned long long v1) {
    __shared__ unsigned long long s_st[2];
    if (threadIdx.x < 2) s_st[threadIdx.x] = 0;
    __syncthreads();
    v0 = wave_sum_u64(v0);
    v1 = wave_sum_u64(v1);
    if ((threadIdx.x & 63) == 0) {
        if (v0) atomicAdd(&s_st[0], v0);
        if (v1) atomicAdd(&s_st[1], v1);
    }
    __syncthreads();
    const unsigned slot = ((blockIdx.y * gridDim.x + blockIdx.x) % STAT_SLOTS) * STAT_FIELDS;
    if (threadIdx.x == 0) {
        if (s_st[0]) atomicAdd(&stats[slot + f0], s_st[0]);
        if (s_st[1] && f1 >= 0) atomicAdd(&stats[slot + f1], s_st[1]);
    }
}

__device__ __forceinline__ void load_entry(const BFHashEntry* h, uint32_t i, int4& a, int4& b) { hash_load_entry(h, i, a, b); }

// getHashEntryForSDFBlockPos, VoxelUtilHashSDF.h:440-485 -> ptr or FREE
__device__ __forceinline__ int lookup_ptr(const HashArgs& A, int x, int y, int z) {
    return hash_lookup(A.hash, A.numBuckets, A.numEntries, A.maxList, x, y, z);
}

// Spatial ownership for multi-GPU sharding: the chunk of the block's corner (worldToChunks
// rounding, CUDASceneRepHashSDF.cu:136-150) hashed onto the shard count.
__device__ __forceinline__ bool owned(const HashArgs& A, int bx, int by, int bz) {
    if (A.shardCount <= 1) return true;
    f3 w = block_to_world(bx, by, bz, A.voxelSize) / A.shardChunk;
    int cx = f2i(w.x + (float)sgn(w.x) * 0.5f), cy = f2i(w.y + (float)sgn(w.y) * 0.5f), cz = f2i(w.z + (float)sgn(w.z) * 0.5f);
    return hash_bucket(cx, cy, cz, A.shardCount) == A.shardIndex;
}

// Does this rank own a chunk of any block in the box spanned by blocks b0 and b1? Same float
// arithmetic as owned() at the box's corners; at most 4 chunks per axis are tested (a truncation
// band is far shorter than a chunk), beyond that the walk runs.
__device__ __forceinline__ bool segment_may_own(const HashArgs& A, i3 b0, i3 b1) {
    const f3 wl = block_to_world(min(b0.x, b1.x), min(b0.y, b1.y), min(b0.z, b1.z), A.voxelSize) / A.shardChunk;
    const f3 wh = block_to_world(max(b0.x, b1.x), max(b0.y, b1.y), max(b0.z, b1.z), A.voxelSize) / A.shardChunk;
    const int x0 = f2i(wl.x + (float)sgn(wl.x) * 0.5f), y0 = f2i(wl.y + (float)sgn(wl.y) * 0.5f), z0 = f2i(wl.z + (float)sgn(wl.z) * 0.5f);
    const int x1 = f2i(wh.x + (float)sgn(wh.x) * 0.5f), y1 = f2i(wh.y + (float)sgn(wh.y) * 0.5f), z1 = f2i(wh.z + (float)sgn(wh.z) * 0.5f);
    if (x1 - x0 > 3 || y1 - y0 > 3 || z1 - z0 > 3) return true;
    for (int cz = z0; cz <= z1; cz++)
        for (int cy = y0; cy <= y1; cy++)
            for (int cx = x0; cx <= x1; cx++)
                if (hash_bucket(cx, cy, cz, A.shardCount) == A.shardIndex) return true;
    return false;
}

// isSDFBlockStreamedOut, CUDASceneRepHashSDF.cu:152-163
__device__ __forceinline__ bool streamed_out(const HashArgs& A, int bx, int by, int bz) {
    if (!A.bitMask) return false;
    f3 w = block_to_world(bx, by, bz, A.voxelSize);
    f3 p = mk3(w.x / A.streamExtents.x, w.y / A.streamExtents.y, w.z / A.streamExtents.z);
    int cx = f2i(p.x + (float)sgn(p.x) * 0.5f) - A.streamMinGridPos.x;
    int cy = f2i(p.y + (float)sgn(p.y) * 0.5f) - A.streamMinGridPos.y;
    int cz = f2i(p.z + (float)sgn(p.z) * 0.5f) - A.streamMinGridPos.z;
    uint32_t index = (uint32_t)(cz * A.streamGridDims.x * A.streamGridDims.y + cy * A.streamGridDims.x + cx);
    return (A.bitMask[index / 32] & (1u << (index % 32))) != 0;
}

__device__ __forceinline__ uint32_t mix_hash(unsigned long long k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (uint32_t)k;
}

// ------------------------------------------------------------------------------------
__global__ void k_reset_hash(BFHashEntry* hash, uint32_t E) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < E; i += gridDim.x * blockDim.x) {
        int4* p = reinterpret_cast<int4*>(hash + i);
        p[0] = make_int4(0, 0, 0, BF_FREE_ENTRY);
        p[1] = make_int4(0, 0, 0, 0);
    }
}

// resetHeapKernel, CUDASceneRepHashSDF.cu:27-45 (voxels are cleared by a memset)
__global__ void k_reset_heap(uint32_t* heap, int4* blockPos, uint32_t* blockCount, uint32_t B, uint32_t* ctrl) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < B; i += gridDim.x * blockDim.x) {
        heap[i] = B - i - 1;
        blockPos[i] = make_int4(0, 0, 0, 0);
        blockCount[i] = 0;
    }
    if (blockIdx.x == 0 && threadIdx.x < C_COUNT) ctrl[threadIdx.x] = (threadIdx.x == C_HEAP) ? B - 1 : 0;
}

// Per-op counter reset (replaces the reference's memset + D2H of d_hashCompactifiedCounter).
__global__ void k_begin_op(uint32_t* ctrl, unsigned long long* stats) {
    if (threadIdx.x == 0) {
        ctrl[C_VISIBLE] = 0;
        ctrl[C_BAND] = 0;
        ctrl[C_CAND] = 0;
        ctrl[C_OVF] = 0;
        stats[S_OPS]++;
    }
}

// Depth-bound tiles of the band cull: min / max over the depths integrate would accept (not -inf,
// below maxIntegrationDistance, CUDASceneRepHashSDF.cu:450-457); empty tiles get (+inf, -inf).
// Wave t < nFine reduces one 8x8 tile, the next nCoarse waves one 32x32 tile each.
__device__ __forceinline__ void depth_tile_wave(uint32_t t, const float* __restrict__ depthImg, uint32_t W, uint32_t H,
                                                uint32_t tilesW, uint32_t tilesH, uint32_t tiles2W, uint32_t tiles2H,
                                                float maxDist, float2* tiles, float2* tiles2) {
    const uint32_t lane = lane_id();
    const uint32_t nFine = tilesW * tilesH;
    float lo = INFINITY, hi = -INFINITY;
    if (t < nFine) {
        const uint32_t x = (t % tilesW) * DEPTH_TILE + (lane & 7), y = (t / tilesW) * DEPTH_TILE + (lane >> 3);
        if (x < W && y < H) {
            const float d = depthImg[y * W + x];
            if (d != -INFINITY && d < maxDist) { lo = d; hi = d; }
        }
    } else {
        const uint32_t c = t - nFine;
        if (c >= tiles2W * tiles2H) return;
        constexpr int ROWS = 64 / DEPTH_TILE2;  // pixel rows per pass of the wave
        const uint32_t x = (c % tiles2W) * DEPTH_TILE2 + (lane % DEPTH_TILE2), y0 = (c / tiles2W) * DEPTH_TILE2 + (lane / DEPTH_TILE2);
#pragma unroll
        for (int i = 0; i < DEPTH_TILE2 / ROWS; i++) {
            const uint32_t y = y0 + ROWS * i;
            if (x < W && y < H) {
                const float d = depthImg[y * W + x];
                if (d != -INFINITY && d < maxDist) { lo = fminf(lo, d); hi = fmaxf(hi, d); }
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, off));
        hi = fmaxf(hi, __shfl_xor(hi, off));
    }
    if (lane == 0) {
        if (t < nFine) tiles[t] = make_float2(lo, hi);
        else tiles2[t - nFine] = make_float2(lo, hi);
    }
}

// Per-op counter reset fused with the depth-bound tiles of the op.
__global__ __launch_bounds__(256) void k_begin_op_tiles(uint32_t* ctrl, unsigned long long* stats,
                                                        const float* __restrict__ depthImg, uint32_t W, uint32_t H,
                                                        uint32_t tilesW, uint32_t tilesH, uint32_t tiles2W, uint32_t tiles2H,
                                                        float maxDist, float2* tiles, float2* tiles2, uint32_t nops) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctrl[C_VISIBLE] = 0;
        ctrl[C_BAND] = 0;
        ctrl[C_CAND] = 0;
        ctrl[C_OVF] = 0;
        stats[S_OPS] += nops;
    }
    depth_tile_wave((blockIdx.x * blockDim.x + threadIdx.x) >> 6, depthImg, W, H, tilesW, tilesH, tiles2W, tiles2H, maxDist,
                    tiles, tiles2);
}

// The screen rectangle of a block's corner projections, grown for the voxel pass's pixel rule: a voxel at
// screen x takes column (int)(x + 0.5), truncated toward zero, so x in (-1.5, -0.5] lands in column 0. The
// rectangle [floor(lo - 0.5), floor(hi + RECT_HI)] holds every column a voxel can take; at the left / top edge
// the bound is that truncation itself (hi just above -1.5 keeps column 0), so it carries 1/64 px for the
// corner projections' rounding (~1e-4 px): without it a corner computed 7.5e-5 px past -1.5 dropped a half
// whose corner voxel lands in row 0 (test_app_gpu's end phase, one weight off).
constexpr float RECT_HI = 1.5f + 0x1p-6f;
// Conservative test that a block may contain a voxel integrate will update: project the 8 voxel-
// centre corners (convex hull -> bounding pixel rectangle, grown by one pixel), take the depth
// bounds of the covered tiles and reject when every depth is too far behind or in front of the
// block for |d - z| < truncation + truncScale * d to hold (1 mm slack for rounding, ~1000x the
// float error). Exactness: a rejected block has no voxel with an in-band sample, so skipping it
// changes no voxel. The corner projections use rcp (1 ulp, far inside the one-pixel growth);
// footprints within 3x3 fine (8-pixel) tiles read those tiles, wider ones up to 3x3 coarse
// (16-pixel) tiles, all loads independent.
// z0 / z1: the voxel z-range (offsets in the block) the test covers; a half-block test covers 0..3
// or 4..7, the block test 0..7
__device__ bool block_may_update(const HashArgs& A, const BFDepthCameraParams& cam, const BFMat4& Tinv, int bx, int by,
                                 int bz, const float2* __restrict__ tiles, const float2* __restrict__ tiles2, int z0 = 0,
                                 int z1 = BF_SDF_BLOCK_SIZE - 1) {
    const f3 c0 = block_to_world(bx, by, bz, A.voxelSize) + mk3(0.0f, 0.0f, A.voxelSize * (float)z0);
    const float ext = A.voxelSize * (float)(BF_SDF_BLOCK_SIZE - 1), extz = A.voxelSize * (float)(z1 - z0);
    float zlo = INFINITY, zhi = -INFINITY, xlo = INFINITY, xhi = -INFINITY, ylo = INFINITY, yhi = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const f3 w = c0 + mk3((k & 1) ? ext : 0.0f, (k & 2) ? ext : 0.0f, (k & 4) ? extz : 0.0f);
        const f3 p = xform(Tinv, w);
        if (!(p.z > 1e-3f)) return true;  // straddles the camera plane: keep
        const float rz = __builtin_amdgcn_rcpf(p.z);
        const float sx = p.x * cam.fx * rz + cam.mx, sy = p.y * cam.fy * rz + cam.my;
        zlo = fminf(zlo, p.z); zhi = fmaxf(zhi, p.z);
        xlo = fminf(xlo, sx); xhi = fmaxf(xhi, sx);
        ylo = fminf(ylo, sy); yhi = fmaxf(yhi, sy);
    }
    const float W = (float)cam.imageWidth, H = (float)cam.imageHeight;
    const float fx0 = floorf(xlo - 0.5f), fx1 = floorf(xhi + RECT_HI), fy0 = floorf(ylo - 0.5f), fy1 = floorf(yhi + RECT_HI);
    if (fx1 < 0.0f || fy1 < 0.0f || fx0 > W - 1.0f || fy0 > H - 1.0f) return false;  // every voxel off-screen
    const int x0 = (int)fmaxf(fx0, 0.0f), x1 = (int)fminf(fx1, W - 1.0f);
    const int y0 = (int)fmaxf(fy0, 0.0f), y1 = (int)fminf(fy1, H - 1.0f);
    const int tx0 = x0 / DEPTH_TILE, tx1 = x1 / DEPTH_TILE, ty0 = y0 / DEPTH_TILE, ty1 = y1 / DEPTH_TILE;
    float dlo = INFINITY, dhi = -INFINITY;
    if (tx1 - tx0 <= 2 && ty1 - ty0 <= 2) {  // footprint within 3x3 fine tiles (<= 17 px)
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const float2 t = tiles[min(ty0 + j, ty1) * A.tilesW + min(tx0 + i, tx1)];
                dlo = fminf(dlo, t.x);
                dhi = fmaxf(dhi, t.y);
            }
    } else {
        const int cx0 = x0 / DEPTH_TILE2, cx1 = x1 / DEPTH_TILE2, cy0 = y0 / DEPTH_TILE2, cy1 = y1 / DEPTH_TILE2;
        if (cx1 - cx0 > 2 || cy1 - cy0 > 2) return true;  // very close block: keep
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const float2 t = tiles2[min(cy0 + j, cy1) * A.tiles2W + min(cx0 + i, cx1)];
                dlo = fminf(dlo, t.x);
                dhi = fmaxf(dhi, t.y);
            }
    }
    if (!(dlo <= dhi)) return false;  // no integrable depth under the block
    const float slack = 0.001f;  // >> the float error of zlo / zhi and of the kernel's band test
    if (dlo * (1.0f - A.truncScale) >= zhi + A.truncation + slack) return false;  // surface far behind
    if (dhi * (1.0f + A.truncScale) <= zlo - A.truncation - slack) return false;  // surface far in front
    return true;
}

// block_may_update for the two z-halves of the block at once (bit h: half h, voxel z 4h..4h+3, may
// hold an in-band voxel), from per-op constants (cull_op_consts, 28 floats). The screen footprint and
// its depth bounds are the whole block's (a superset of each half's pixels: still conservative); the
// depth range is each half's own. The camera-space corner positions are affine in the corner
// offsets, so the block's corner voxel is transformed once (fma, the focal lengths folded into the
// x / y rows) and the other corners are that point plus sums of the three scaled columns; each
// half's depth range is the corner point's depth plus per-op minima / maxima of the column terms.
// Float differences against the per-corner transforms are ~1e-6 relative, far inside the one-pixel
// growth and the 1 mm slack. Against eight full corner transforms plus eight depth rows per (block,
// op) pair: k_compactify_ops 57.3 -> 48.8 us per batch (profiles/r11_scan_ab.txt).
constexpr int CULL_CONSTS = 28;
// q: [0..11] rows fx r0, fy r1, r2 of Tinv; [12..20] columns 0, 1, 2 of those rows times 7 voxels;
// [21..24] half 0 depth offset min / max, half 1 min / max (over the xy corners and its z levels)
__host__ __device__ __forceinline__ void cull_op_consts(const float* t, const BFDepthCameraParams& cam, float voxelSize, float* q) {
    const float ext = voxelSize * (float)(BF_SDF_BLOCK_SIZE - 1);
    for (int c = 0; c < 4; c++) {
        q[c] = cam.fx * t[c];
        q[4 + c] = cam.fy * t[4 + c];
        q[8 + c] = t[8 + c];
    }
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) q[12 + 3 * c + r] = ext * q[4 * r + c];
    const float ab0 = fminf(0.0f, q[14]) + fminf(0.0f, q[17]), ab1 = fmaxf(0.0f, q[14]) + fmaxf(0.0f, q[17]);
    const float z3 = voxelSize * 3.0f * t[10], z4 = voxelSize * 4.0f * t[10], z7 = voxelSize * 7.0f * t[10];
    q[21] = ab0 + fminf(0.0f, z3);
    q[22] = ab1 + fmaxf(0.0f, z3);
    q[23] = ab0 + fminf(z4, z7);
    q[24] = ab1 + fmaxf(z4, z7);
    q[25] = q[26] = q[27] = 0.0f;
}
__device__ __forceinline__ uint32_t block_may_update_halves_q(const HashArgs& A, const BFDepthCameraParams& cam, const float* __restrict__ q,
                                                              int bx, int by, int bz, const float2* __restrict__ tiles,
                                                              const float2* __restrict__ tiles2) {
    const f3 c0 = block_to_world(bx, by, bz, A.voxelSize);
    const float p0x = __builtin_fmaf(q[0], c0.x, __builtin_fmaf(q[1], c0.y, __builtin_fmaf(q[2], c0.z, q[3])));
    const float p0y = __builtin_fmaf(q[4], c0.x, __builtin_fmaf(q[5], c0.y, __builtin_fmaf(q[6], c0.z, q[7])));
    const float p0z = __builtin_fmaf(q[8], c0.x, __builtin_fmaf(q[9], c0.y, __builtin_fmaf(q[10], c0.z, q[11])));
    const float zlo[2] = {p0z + q[21], p0z + q[23]}, zhi[2] = {p0z + q[22], p0z + q[24]};
    if (!(fminf(zlo[0], zlo[1]) > 1e-3f)) return 3u;  // reaches the camera plane: keep
    float xlo = INFINITY, xhi = -INFINITY, ylo = INFINITY, yhi = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float px = p0x, py = p0y, pz = p0z;
#pragma unroll
        for (int c = 0; c < 3; c++)
            if ((k >> c) & 1) { px += q[12 + 3 * c]; py += q[13 + 3 * c]; pz += q[14 + 3 * c]; }
        const float rz = __builtin_amdgcn_rcpf(pz);
        const float sx = __builtin_fmaf(px, rz, cam.mx), sy = __builtin_fmaf(py, rz, cam.my);
        xlo = fminf(xlo, sx); xhi = fmaxf(xhi, sx);
        ylo = fminf(ylo, sy); yhi = fmaxf(yhi, sy);
    }
    const float W = (float)cam.imageWidth, H = (float)cam.imageHeight;
    const float fx0 = floorf(xlo - 0.5f), fx1 = floorf(xhi + RECT_HI), fy0 = floorf(ylo - 0.5f), fy1 = floorf(yhi + RECT_HI);
    if (fx1 < 0.0f || fy1 < 0.0f || fx0 > W - 1.0f || fy0 > H - 1.0f) return 0u;  // every voxel off-screen
    const int x0 = (int)fmaxf(fx0, 0.0f), x1 = (int)fminf(fx1, W - 1.0f);
    const int y0 = (int)fmaxf(fy0, 0.0f), y1 = (int)fminf(fy1, H - 1.0f);
    const int tx0 = x0 / DEPTH_TILE, tx1 = x1 / DEPTH_TILE, ty0 = y0 / DEPTH_TILE, ty1 = y1 / DEPTH_TILE;
    float dlo = INFINITY, dhi = -INFINITY;
    if (tx1 - tx0 <= 2 && ty1 - ty0 <= 2) {
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const float2 t = tiles[min(ty0 + j, ty1) * A.tilesW + min(tx0 + i, tx1)];
                dlo = fminf(dlo, t.x);
                dhi = fmaxf(dhi, t.y);
            }
    } else {
        const int cx0 = x0 / DEPTH_TILE2, cx1 = x1 / DEPTH_TILE2, cy0 = y0 / DEPTH_TILE2, cy1 = y1 / DEPTH_TILE2;
        if (cx1 - cx0 > 2 || cy1 - cy0 > 2) return 3u;  // very close block: keep
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const float2 t = tiles2[min(cy0 + j, cy1) * A.tiles2W + min(cx0 + i, cx1)];
                dlo = fminf(dlo, t.x);
                dhi = fmaxf(dhi, t.y);
            }
    }
    if (!(dlo <= dhi)) return 0u;  // no integrable depth under the block
    const float slack = 0.001f;
    uint32_t bits = 0;
#pragma unroll
    for (int hh = 0; hh < 2; hh++)
        if (!(dlo * (1.0f - A.truncScale) >= zhi[hh] + A.truncation + slack) &&
            !(dhi * (1.0f + A.truncScale) <= zlo[hh] - A.truncation - slack))
            bits |= 1u << hh;
    return bits;
}

// isSDFBlockInCameraFrustumApprox (VoxelUtilHashSDF.h:322-326, DepthCameraUtil.h:95-107) with the
// five IEEE divisions replaced by rcp products. The test is a set of comparisons of monotone
// quotients against +-1 / 0 / 1, so the fast result is taken when every compared value is farther
// from its bound than the rcp error (<= 2^-20 relative, taken with a 4x margin); otherwise the exact
// test decides. Identical outcome to block_in_frustum.
__device__ __forceinline__ bool block_in_frustum_fast(const BFDepthCameraParams& c, const BFMat4& viewInv, int bx, int by,
                                                      int bz, float voxelSize) {
    const f3 w = block_to_world(bx, by, bz, voxelSize) + mk3(1.0f, 1.0f, 1.0f) * (voxelSize * 0.5f * (BF_SDF_BLOCK_SIZE - 1.0f));
    const f3 pc = xform(viewInv, w);
    const float rz = __builtin_amdgcn_rcpf(pc.z);
    const float wm1 = (float)c.imageWidth - 1.0f, hm1 = (float)c.imageHeight - 1.0f;
    const float px = pc.x * c.fx * rz + c.mx, py = pc.y * c.fy * rz + c.my;
    const float x = (2.0f * px - wm1) * __builtin_amdgcn_rcpf(wm1) * 0.95f;
    const float y = (hm1 - 2.0f * py) * __builtin_amdgcn_rcpf(hm1) * 0.95f;
    const float z = (pc.z - c.sensorDepthWorldMin) * __builtin_amdgcn_rcpf(c.sensorDepthWorldMax - c.sensorDepthWorldMin) * 0.95f;
    const float ex = (fabsf(x) + 4.0f) * 0x1p-18f, ey = (fabsf(y) + 4.0f) * 0x1p-18f, ez = (fabsf(z) + 1.0f) * 0x1p-18f;
    const bool sure = fabsf(fabsf(x) - 1.0f) > ex && fabsf(fabsf(y) - 1.0f) > ey && fabsf(z - 1.0f) > ez && fabsf(z) > ez;
    if (!sure) return block_in_frustum(c, viewInv, bx, by, bz, voxelSize);
    return !(x < -1.0f || x > 1.0f || y < -1.0f || y > 1.0f || z < 0.0f || z > 1.0f);
}

// allocKernel, CUDASceneRepHashSDF.cu:165-251: per-pixel DDA over 8^3-block cells. Emits the
// absent, in-frustum, owned blocks (deduplicated per tile in LDS) into `cand`.
// a / b for a launch-uniform divisor b in [2^-20, 2^20] with rb = RN(1 / b) from the host: a * rb, then
// two residual corrections. The first leaves a faithful quotient; the second, from a faithful quotient with
// the correctly rounded reciprocal, rounds to nearest (Markstein's theorem) while the residuals are normal,
// i.e. for 2^-100 <= |a| <= 2^100 or a = 0 — bit-identical to the IEEE division there (tools/check_uniform_div.c:
// 8.6e9 cases). 5 VALU against ~11 for the division's scale / fmas / fixup sequence.
__device__ __forceinline__ float div_by_uniform(float a, float b, float rb) {
    const float q0 = a * rb;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), rb, q0);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), rb, q1);
}
// world_to_block (VoxelUtilHashSDF.h:283-299) of a point with the division by the voxel size through
// div_by_uniform. Below 2^-100 a coordinate's quotient is off by ulps but stays below 2^-60 with the
// point's sign, so f2i(p + sgn(p) 0.5) is 0 for it as for the IEEE quotient: only |w| > 2^100 (or no
// usable reciprocal) needs the IEEE path, which the caller runs under a ballot.
__device__ __forceinline__ i3 world_to_block_rcp(f3 w, float vs, float rvs) {
    const f3 p = mk3(div_by_uniform(w.x, vs, rvs), div_by_uniform(w.y, vs, rvs), div_by_uniform(w.z, vs, rvs));
    const f3 q = p + mk3((float)sgn(p.x), (float)sgn(p.y), (float)sgn(p.z)) * 0.5f;
    i3 v;
    v.x = f2i(q.x); v.y = f2i(q.y); v.z = f2i(q.z);
    return vvox_to_block(v);
}
struct RayWalk {  // one pixel's DDA state (CUDASceneRepHashSDF.cu:196-230)
    i3 id, idBound;
    f3 tMax, tDelta, step;
    bool active;
};
__device__ __forceinline__ RayWalk ray_walk_setup(const HashArgs& A, const float* __restrict__ depthImg,
                                                  const BFDepthCameraParams& cam, const BFMat4& T, uint32_t x, uint32_t y) {
    RayWalk r;
    r.active = x < cam.imageWidth && y < cam.imageHeight;
    const float d = r.active ? depthImg[y * cam.imageWidth + x] : 0.0f;
    if (d == -INFINITY || d == 0.0f) r.active = false;
    if (d >= A.maxIntegrationDistance) r.active = false;
    const float t = A.truncation + A.truncScale * d;
    const float minDepth = fminf(A.maxIntegrationDistance, d - t);
    const float maxDepth = fminf(A.maxIntegrationDistance, d + t);
    if (minDepth >= maxDepth) r.active = false;
    r.id = {0, 0, 0};
    r.idBound = {0, 0, 0};
    r.tMax = mk3(0, 0, 0);
    r.tDelta = mk3(0, 0, 0);
    r.step = mk3(0, 0, 0);
    if (r.active) {
        // depth_to_camera's two divisions by fx / fy and world_to_block's six by the voxel size go through
        // div_by_uniform (bit-identical in the ranges checked below; otherwise the IEEE form, per wave)
        f3 rayMin, rayMax;
        i3 idEnd;
        if (A.rFx != 0.0f) {  // launch-uniform
            const float cx = div_by_uniform((float)x - cam.mx, cam.fx, A.rFx), cy = div_by_uniform((float)y - cam.my, cam.fy, A.rFy);
            rayMin = xform(T, mk3(minDepth * cx, minDepth * cy, minDepth));
            rayMax = xform(T, mk3(maxDepth * cx, maxDepth * cy, maxDepth));
        } else {
            rayMin = xform(T, depth_to_camera(cam, x, y, minDepth));
            rayMax = xform(T, depth_to_camera(cam, x, y, maxDepth));
        }
        r.id = world_to_block_rcp(rayMin, A.voxelSize, A.rVoxelSize);
        idEnd = world_to_block_rcp(rayMax, A.voxelSize, A.rVoxelSize);
        const float big = fmaxf(fmaxf(fmaxf(fabsf(rayMin.x), fabsf(rayMin.y)), fmaxf(fabsf(rayMin.z), fabsf(rayMax.x))),
                                fmaxf(fabsf(rayMax.y), fabsf(rayMax.z)));
        const bool exactNeeded = A.rVoxelSize == 0.0f || big > 0x1p100f;
        if (__builtin_amdgcn_ballot_w64(exactNeeded)) {
            asm volatile("" ::: "memory");
            if (exactNeeded) {
                r.id = world_to_block(rayMin, A.voxelSize);
                idEnd = world_to_block(rayMax, A.voxelSize);
            }
        }
        const f3 rayDir = normalize3(rayMax - rayMin);
        r.step = mk3((float)sgn(rayDir.x), (float)sgn(rayDir.y), (float)sgn(rayDir.z));
        const f3 bp = block_to_world(r.id.x + f2i(fmaxf(0.0f, fminf(r.step.x, 1.0f))), r.id.y + f2i(fmaxf(0.0f, fminf(r.step.y, 1.0f))),
                                     r.id.z + f2i(fmaxf(0.0f, fminf(r.step.z, 1.0f))), A.voxelSize) -
                      mk3(1.0f, 1.0f, 1.0f) * (0.5f * A.voxelSize);
        r.tMax = (bp - rayMin) / rayDir;
        r.tDelta = (r.step * (float)BF_SDF_BLOCK_SIZE * A.voxelSize) / rayDir;
        r.idBound.x = f2i((float)idEnd.x + r.step.x);
        r.idBound.y = f2i((float)idEnd.y + r.step.y);
        r.idBound.z = f2i((float)idEnd.z + r.step.z);
        if (rayDir.x == 0.0f) { r.tMax.x = INFINITY; r.tDelta.x = INFINITY; }
        if (bp.x - rayMin.x == 0.0f) { r.tMax.x = INFINITY; r.tDelta.x = INFINITY; }
        if (rayDir.y == 0.0f) { r.tMax.y = INFINITY; r.tDelta.y = INFINITY; }
        if (bp.y - rayMin.y == 0.0f) { r.tMax.y = INFINITY; r.tDelta.y = INFINITY; }
        if (rayDir.z == 0.0f) { r.tMax.z = INFINITY; r.tDelta.z = INFINITY; }
        if (bp.z - rayMin.z == 0.0f) { r.tMax.z = INFINITY; r.tDelta.z = INFINITY; }
        // multi-GPU: the walk visits only blocks inside the box of its first and last block; when no
        // chunk of that box belongs to this rank, none of its blocks can be emitted, so skip the walk
        // (chunk indices are monotone in the block coordinate: the box's corners bound them)
        if (A.shardCount > 1) r.active = segment_may_own(A, r.id, idEnd);
    }
    return r;
}
__device__ __forceinline__ void ray_walk_advance(RayWalk& r) {  // traverse (CUDASceneRepHashSDF.cu:231-246)
    if (r.tMax.x < r.tMax.y && r.tMax.x < r.tMax.z) {
        r.id.x = f2i((float)r.id.x + r.step.x);
        if (r.id.x == r.idBound.x) r.active = false;
        r.tMax.x += r.tDelta.x;
    } else if (r.tMax.z < r.tMax.y) {
        r.id.z = f2i((float)r.id.z + r.step.z);
        if (r.id.z == r.idBound.z) r.active = false;
        r.tMax.z += r.tDelta.z;
    } else {
        r.id.y = f2i((float)r.id.y + r.step.y);
        if (r.id.y == r.idBound.y) r.active = false;
        r.tMax.y += r.tDelta.y;
    }
}
// the absent, in-frustum, owned, not streamed-out blocks are emitted (allocKernel's per-block tests)
__device__ __forceinline__ bool alloc_wants(const HashArgs& A, const BFDepthCameraParams& cam, const BFMat4& Tinv, i3 b) {
    return block_in_frustum_fast(cam, Tinv, b.x, b.y, b.z, A.voxelSize) && owned(A, b.x, b.y, b.z) &&
           !streamed_out(A, b.x, b.y, b.z) && lookup_ptr(A, b.x, b.y, b.z) == BF_FREE_ENTRY;
}
// A tile whose keys overflowed both the LDS set and its overflow list (never seen at the bench workloads):
// the tile's walk again, every visited block tested and emitted directly. Blocks phase 2 already emitted
// come out twice; the global dedup of k_alloc_insert removes them. It runs after phase 2, outside the hot
// walk loop (the first form tested and emitted an unplaced key inside the loop: 141 SGPR spills there).
__device__ __forceinline__ unsigned long long alloc_walk_direct(const HashArgs& A, const float* __restrict__ depthImg,
                                                             const BFDepthCameraParams& cam, const BFMat4& T, const BFMat4& Tinv,
                                                             unsigned long long* __restrict__ cand, uint32_t candCap,
                                                             uint8_t* __restrict__ candOp, uint8_t opIdx, uint32_t x, uint32_t y) {
    RayWalk r = ray_walk_setup(A, depthImg, cam, T, x, y);
    unsigned long long emitted = 0;
    for (uint32_t iter = 0; iter < 1024 && r.active; iter++) {
        const i3 b = r.id;
        ray_walk_advance(r);
        if (alloc_wants(A, cam, Tinv, b)) {
            const uint32_t k = atomicAdd(&A.ctrl[C_CAND], 1u);
            if (k < candCap) {
                cand[k] = block_key(b.x, b.y, b.z);
                if (candOp) candOp[k] = opIdx;
            } else {
                atomicOr(&A.ctrl[C_ERR], 1u);
            }
            emitted++;
        }
    }
    return emitted;
}
constexpr int ALLOC_OVF = 256;  // per tile: keys the congested LDS set could not place, tested in phase 2
__device__ __forceinline__ void alloc_collect(const HashArgs& A, const float* __restrict__ depthImg,
                                              const BFDepthCameraParams& cam, const BFMat4& T, const BFMat4& Tinv,
                                              unsigned long long* __restrict__ cand, uint32_t candCap,
                                              uint8_t* __restrict__ candOp = nullptr, uint8_t opIdx = 0) {
    __shared__ unsigned long long set[LDS_SET + ALLOC_OVF];  // the set, then the overflow keys
    __shared__ uint32_t s_novf;
    const uint32_t x = blockIdx.x * ALLOC_TILE + (threadIdx.x % ALLOC_TILE);
    const uint32_t y = blockIdx.y * ALLOC_TILE + (threadIdx.x / ALLOC_TILE);
    RayWalk r = ray_walk_setup(A, depthImg, cam, T, x, y);
    // a tile none of whose rays walks (no valid depth, or, sharded, no ray near an owned chunk) ends here
    if (!__syncthreads_or(r.active ? 1 : 0)) return;
    for (int k = threadIdx.x; k < LDS_SET; k += blockDim.x) set[k] = EMPTY_KEY;
    if (threadIdx.x == 0) s_novf = 0;
    __syncthreads();

    // phase 1: walk the ray's blocks and collect the tile's distinct blocks in the LDS set (compute
    // only, no global memory on the DDA's critical path). The per-block tests (frustum, ownership,
    // streaming mask) depend only on the block, so they run once per distinct block in phase 2
    // instead of once per DDA step: same emitted set, far fewer projections.
    const uint32_t lane = lane_id();
    // The loop runs while any lane of the wave walks (wave-uniform trip) so that lanes can compare
    // keys: a lane whose left (same pixel row) or upper neighbour pixel reaches the same block in
    // the same step leaves the insert to it (the chain ends at a lane that inserts or emits it), so
    // the LDS set sees far fewer same-address CAS. The emitted set is unchanged.
    // Two DDA steps per trip: both steps' first-probe CAS are issued back to back, so a walk pays one
    // LDS round trip per two blocks (probing past a taken slot, rare, follows per step). Which lane
    // inserts a key and in what order changes nothing: the set ends up holding the same keys, and a
    // key that finds no slot goes to the tile's overflow list (phase 2 tests it like the set's keys).
    auto is_dup = [&](unsigned long long myKey) {
        const unsigned long long left = __shfl_up(myKey, 1, ALLOC_TILE), up = __shfl_up(myKey, ALLOC_TILE);
        return ((lane % ALLOC_TILE) != 0 && left == myKey) || (lane >= ALLOC_TILE && up == myKey);
    };
    // slot from the low coordinate bits (3 + 4 + 3 = 10 bits = LDS_SET): the blocks one 16x16-pixel
    // tile reaches span a few blocks per axis, so they land in distinct slots without a mixing hash
    auto slot_of = [](i3 b) { return ((uint32_t)b.x & 7u) | (((uint32_t)b.y & 15u) << 3) | (((uint32_t)b.z & 7u) << 7); };
    auto finish_insert = [&](unsigned long long key, uint32_t h) {  // probes 2..16, then the overflow list
        for (int p = 1; p < 16; p++) {
            h = (h + 1) & (LDS_SET - 1);
            const unsigned long long old = atomicCAS(&set[h], EMPTY_KEY, key);
            if (old == EMPTY_KEY || old == key) return;
        }
        const uint32_t j = atomicAdd(&s_novf, 1u);
        if (j < (uint32_t)ALLOC_OVF) set[LDS_SET + j] = key;
    };
    for (uint32_t iter = 0; iter < 512; iter++) {
        if (!__any(r.active)) break;
        const bool actA = r.active;
        const i3 idA = r.id;
        if (r.active) ray_walk_advance(r);
        const bool actB = r.active;
        const i3 idB = r.id;
        if (r.active) ray_walk_advance(r);
        const unsigned long long keyA = actA ? block_key(idA.x, idA.y, idA.z) : EMPTY_KEY;
        const unsigned long long keyB = actB ? block_key(idB.x, idB.y, idB.z) : EMPTY_KEY;
        const bool doA = actA && !is_dup(keyA), doB = actB && !is_dup(keyB);
        const uint32_t hA = slot_of(idA), hB = slot_of(idB);
        const unsigned long long oldA = doA ? atomicCAS(&set[hA], EMPTY_KEY, keyA) : EMPTY_KEY;
        const unsigned long long oldB = doB ? atomicCAS(&set[hB], EMPTY_KEY, keyB) : EMPTY_KEY;
        if (doA && oldA != EMPTY_KEY && oldA != keyA) finish_insert(keyA, hA);
        if (doB && oldB != EMPTY_KEY && oldB != keyB) finish_insert(keyB, hB);
    }
    // phase 2: compact the distinct blocks to the front of the set, append the overflow keys, then every
    // thread checks one of them against the hash (one round of parallel lookups per 256 distinct blocks —
    // a tile reaches far fewer — instead of a round per 256 slots, each waiting on its hash loads) and
    // emits the absent ones
    __shared__ uint32_t s_nkeys;
    constexpr int SLOTS_PER_THREAD = LDS_SET / 256;
    unsigned long long mine[SLOTS_PER_THREAD];
    __syncthreads();
    const uint32_t novf = s_novf;
    const uint32_t nOvfKept = min(novf, (uint32_t)ALLOC_OVF);
    unsigned long long ovfKey = threadIdx.x < nOvfKept ? set[LDS_SET + threadIdx.x] : EMPTY_KEY;
#pragma unroll
    for (int j = 0; j < SLOTS_PER_THREAD; j++) mine[j] = set[j * 256 + threadIdx.x];
    if (threadIdx.x == 0) s_nkeys = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SLOTS_PER_THREAD + 1; j++) {
        const unsigned long long key = j < SLOTS_PER_THREAD ? mine[j] : ovfKey;
        const bool full = key != EMPTY_KEY;
        const unsigned long long m = __ballot(full);
        if (m == 0) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&s_nkeys, (uint32_t)__popcll(m));
        base = __shfl(base, 0);
        if (full) set[base + __popcll(m & lanemask_lt())] = key;
    }
    __syncthreads();
    const uint32_t nkeys = s_nkeys;
    unsigned long long emitted = 0;
    for (uint32_t k0 = 0; k0 < nkeys; k0 += 256) {
        const unsigned long long key = k0 + threadIdx.x < nkeys ? set[k0 + threadIdx.x] : EMPTY_KEY;
        const bool want = key != EMPTY_KEY && alloc_wants(A, cam, Tinv, key_block(key));
        const unsigned long long m = __ballot(want);
        if (want) {
            const int leader = __ffsll((long long)m) - 1;
            const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
            uint32_t base = 0;
            if ((int)lane_id() == leader) base = atomicAdd(&A.ctrl[C_CAND], (uint32_t)__popcll(m));
            base = __shfl(base, leader);
            if (base + rank < candCap) {
                cand[base + rank] = key;
                if (candOp) candOp[base + rank] = opIdx;
            }
            else atomicOr(&A.ctrl[C_ERR], 1u);
            emitted++;
        }
    }
    // the overflow list itself overflowed: the tile's walk again with direct emission (workgroup-uniform)
    // (A.allocForceDirect, a test switch: every walking tile also takes the direct path; same candidate set)
    if (novf > (uint32_t)ALLOC_OVF || A.allocForceDirect) emitted += alloc_walk_direct(A, depthImg, cam, T, Tinv, cand, candCap, candOp, opIdx, x, y);
    // pixels are counted on the host (W x H per walk); candidates are rare in steady state, so the
    // workgroup adds its count only when it emitted some (every workgroup adding to a few counters
    // serialised ~10^5 atomics per frame on them)
    if (__syncthreads_or(emitted != 0 ? 1 : 0)) flush_stats2(A.stats, S_CAND, emitted, -1, 0);
}
__global__ __launch_bounds__(256) void k_alloc_collect(HashArgs A, const float* __restrict__ depthImg,
                                                       BFDepthCameraParams cam, BFMat4 T, BFMat4 Tinv,
                                                       unsigned long long* __restrict__ cand, uint32_t candCap) {
    alloc_collect(A, depthImg, cam, T, Tinv, cand, candCap);
}
// batched: blockIdx.z selects the integrate op of the table (all ops' candidates land in one list;
// the global dedup of k_alloc_insert removes blocks several ops want)
// waves per SIMD asked of the compiler for the batched walk: 8 (63 VGPRs, 78 SGPRs with 65 spilled to VGPR lanes)
// against its own choice of 7 (SGPR-limited): k_alloc_collect_ops 90 -> 86.5 us per frame (gpurun_out/s21)
#ifndef BF_ALLOC_WPE
#define BF_ALLOC_WPE 8
#endif
#if BF_ALLOC_WPE
#define BF_ALLOC_ATTR __attribute__((amdgpu_waves_per_eu(BF_ALLOC_WPE)))
#else
#define BF_ALLOC_ATTR
#endif
__global__ __launch_bounds__(256) BF_ALLOC_ATTR void k_alloc_collect_ops(HashArgs A, BFDepthCameraParams cam, OpTable ops,
                                                           unsigned long long* __restrict__ cand, uint32_t candCap,
                                                           uint8_t* __restrict__ candOp) {
    const uint32_t k = ops.intIdx[blockIdx.z];
    alloc_collect(A, ops.depth[k], cam, op_mat(ops.t[k]), op_mat(ops.tinv[k]), cand, candCap, candOp, (uint8_t)k);
}
// In the sequential reference a block allocated for integrate op j does not exist for the ops
// before j. Every candidate was absent when the batch started (the collect pass reads the hash
// before any insert), so after the inserts each one records, per block, the earliest op that asked
// for it: birth = epoch << 8 | (255 - op), kept by atomicMax (newest epoch, then smallest op).
__global__ __launch_bounds__(256) void k_alloc_birth(HashArgs A, const unsigned long long* __restrict__ cand,
                                                     const uint8_t* __restrict__ candOp, uint32_t candCap, uint32_t* birth,
                                                     uint32_t epoch) {
    const uint32_t n = min(A.ctrl[C_CAND], candCap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const i3 b = key_block(cand[i]);
        const int ptr = lookup_ptr(A, b.x, b.y, b.z);
        if (ptr == BF_FREE_ENTRY) continue;  // not inserted (hash / heap full: flagged in ctrl)
        atomicMax(&birth[(uint32_t)ptr], (epoch << 8) | (255u - candOp[i]));
    }
}

__device__ void alloc_overflow_serial(const HashArgs& A, const unsigned long long* ovf);

// allocBlock, VoxelUtilHashSDF.h:549-655 (bucket path), lock-free: global dedup, CAS on the
// slot's ptr, wave-aggregated heap pop.
__global__ __launch_bounds__(256) void k_alloc_insert(HashArgs A, const unsigned long long* __restrict__ cand, uint32_t candCap,
                                                      unsigned long long* candSet, uint32_t setMask, int* candSlot,
                                                      unsigned long long* ovf) {
    const uint32_t n = min(A.ctrl[C_CAND], candCap);
    const uint32_t lane = lane_id();
    const uint32_t waveStride = gridDim.x * blockDim.x;
    unsigned long long allocated = 0;
    for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < n; base += waveStride) {
        const uint32_t i = base + lane;
        const bool valid = i < n;
        const unsigned long long key = valid ? cand[i] : EMPTY_KEY;
        bool owner = false;
        if (valid) {
            uint32_t h = mix_hash(key) & setMask;
            int slot = -1;
            for (int p = 0; p < 64; p++) {
                unsigned long long old = atomicCAS(&candSet[h], EMPTY_KEY, key);
                if (old == EMPTY_KEY) { owner = true; slot = (int)h; break; }
                if (old == key) break;
                h = (h + 1) & setMask;
            }
            if (!owner) {
                // duplicate, unless all probes hit other keys (congested set): flag that
                bool dup = false;
                uint32_t h2 = mix_hash(key) & setMask;
                for (int p = 0; p < 64 && !dup; p++) { dup = (candSet[h2] == key); h2 = (h2 + 1) & setMask; }
                if (!dup) atomicOr(&A.ctrl[C_ERR], 4u);
            }
            candSlot[i] = slot;
        }
        int hslot = -1;
        i3 p = key_block(key);
        if (owner) {
            const uint32_t b = hash_bucket(p.x, p.y, p.z, A.numBuckets);
            for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
                int* ptrp = &A.hash[b * BF_HASH_BUCKET_SIZE + j].ptr;
                if (atomicCAS(ptrp, BF_FREE_ENTRY, BF_LOCK_ENTRY) == BF_FREE_ENTRY) { hslot = (int)(b * BF_HASH_BUCKET_SIZE + j); break; }
            }
            if (hslot < 0) {
                uint32_t o = atomicAdd(&A.ctrl[C_OVF], 1u);
                if (o < OVF_CAP) ovf[o] = key;
                else atomicOr(&A.ctrl[C_ERR], 1u);
            }
        }
        // consumeHeap (VoxelUtilHashSDF.h:535-540), one atomic per wave
        const bool need = hslot >= 0;
        const unsigned long long m = __ballot(need);
        if (m) {
            const int leader = __ffsll((long long)m) - 1;
            const uint32_t cnt = (uint32_t)__popcll(m);
            uint32_t old = 0;
            if ((int)lane == leader) {
                old = atomicSub(&A.ctrl[C_HEAP], cnt);
                if (old >= A.numBlocks) { atomicAdd(&A.ctrl[C_HEAP], cnt); atomicOr(&A.ctrl[C_ERR], 2u); }
                else if (cnt > old + 1) { atomicAdd(&A.ctrl[C_HEAP], cnt - (old + 1)); atomicOr(&A.ctrl[C_ERR], 2u); }
            }
            old = __shfl(old, leader);
            if (need) {
                const uint32_t rank = (uint32_t)__popcll(m & lanemask_lt());
                const bool ok = old < A.numBlocks && rank <= old;
                int4* e = reinterpret_cast<int4*>(A.hash + hslot);
                if (ok) {
                    const uint32_t blk = A.heap[old - rank];
                    e[1] = make_int4(0, 0, 0, 0);
                    e[0] = make_int4(p.x, p.y, p.z, (int)blk);
                    A.blockPos[blk] = make_int4(p.x, p.y, p.z, 1);
                    atomicMax(&A.ctrl[C_HIGHWATER], blk + 1);
                    allocated++;
                } else {
                    e[0] = make_int4(0, 0, 0, BF_FREE_ENTRY);  // release the claimed slot
                }
            }
        }
    }
    flush_stats2(A.stats, S_ALLOC, allocated, -1, 0);
    // the last workgroup to finish replays the bucket-full candidates serially (the collision-
    // list path), so no separate launch is needed: release fence + ticket, acquire on the winner
    __shared__ bool s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        s_last = atomicAdd(&A.ctrl[C_TICKET], 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (s_last && threadIdx.x == 0) {
        __threadfence();
        A.ctrl[C_TICKET] = 0;
        A.ctrl[C_CANDPEAK] = max(A.ctrl[C_CANDPEAK], A.ctrl[C_CAND]);  // candidate demand, against candCap
        if (A.ctrl[C_OVF]) alloc_overflow_serial(A, ovf);
    }
}

// allocBlock collision-list path (VoxelUtilHashSDF.h:573-654), serial: bucket-full candidates
// are rare at the configured load factor; one lane replays the reference insert for each.
__device__ void alloc_overflow_serial(const HashArgs& A, const unsigned long long* ovf) {
    const uint32_t n = min(A.ctrl[C_OVF], OVF_CAP);
    for (uint32_t k = 0; k < n; k++) {
        const i3 pos = key_block(ovf[k]);
        const uint32_t h = hash_bucket(pos.x, pos.y, pos.z, A.numBuckets), hp = h * BF_HASH_BUCKET_SIZE;
        int firstEmpty = -1;
        bool present = false;
        for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
            const BFHashEntry& c = A.hash[hp + j];
            if (c.x == pos.x && c.y == pos.y && c.z == pos.z && c.ptr != BF_FREE_ENTRY) present = true;
            if (firstEmpty == -1 && c.ptr == BF_FREE_ENTRY) firstEmpty = (int)(hp + j);
        }
        const uint32_t last = hp + BF_HASH_BUCKET_SIZE - 1;
        uint32_t i = last;
        for (uint32_t it = 0; it < A.maxList && !present; it++) {
            const BFHashEntry& c = A.hash[i];
            if (c.x == pos.x && c.y == pos.y && c.z == pos.z && c.ptr != BF_FREE_ENTRY) present = true;
            if (c.offset == 0) break;
            i = (last + c.offset) % A.numEntries;
        }
        if (present) continue;
        uint32_t target = 0xFFFFFFFFu, newOffset = 0;
        int offset = 0;
        if (firstEmpty >= 0) {
            target = (uint32_t)firstEmpty;
        } else {
            for (uint32_t it = 0; it < A.maxList;) {
                offset++;
                i = (last + (uint32_t)offset) % A.numEntries;
                if ((offset % BF_HASH_BUCKET_SIZE) == 0) continue;
                if (A.hash[i].ptr == BF_FREE_ENTRY) { target = i; break; }
                it++;
            }
            if (target == 0xFFFFFFFFu) continue;  // no free slot within reach: not allocated (as in the reference)
        }
        const uint32_t old = A.ctrl[C_HEAP];
        if (old >= A.numBlocks) { A.ctrl[C_ERR] |= 2u; continue; }
        A.ctrl[C_HEAP] = old - 1;
        const uint32_t blk = A.heap[old];
        BFHashEntry& e = A.hash[target];
        e.x = pos.x; e.y = pos.y; e.z = pos.z;
        if (firstEmpty >= 0) {
            e.offset = 0;
        } else {
            e.offset = A.hash[last].offset;
            A.hash[last].offset = (uint32_t)offset;
            newOffset = (uint32_t)offset;
        }
        (void)newOffset;
        e.ptr = (int)blk;
        A.blockPos[blk] = make_int4(pos.x, pos.y, pos.z, 1);
        if (blk + 1 > A.ctrl[C_HIGHWATER]) A.ctrl[C_HIGHWATER] = blk + 1;
        A.stats[S_ALLOC]++;
    }
}

__global__ void k_alloc_overflow(HashArgs A, const unsigned long long* ovf) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    alloc_overflow_serial(A, ovf);
}

__global__ void k_alloc_cleanup(const uint32_t* ctrl, uint32_t candCap, const int* candSlot, unsigned long long* candSet) {
    const uint32_t n = min(ctrl[C_CAND], candCap);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int s = candSlot[i];
        if (s >= 0) candSet[s] = EMPTY_KEY;
    }
}

// compactifyHashAllInOneKernel, CUDASceneRepHashSDF.cu:324-366: stream the allocated pool
// prefix [0, highWater), keep the in-frustum blocks; wave ballot + one atomic per wave.
enum CompactMode { CM_FRUSTUM = 0, CM_INTEGRATE = 1 };

// MODE selects the lists a pass builds:
//   CM_FRUSTUM    visible (the API's compactify / the raycaster)
//   CM_INTEGRATE  visible (GC list) + band (integrate's work list); releases the alloc dedup set
template <int MODE>
__global__ __launch_bounds__(256) void k_compactify(HashArgs A, BFDepthCameraParams cam, BFMat4 Tinv, uint32_t candCap,
                                                    const int* __restrict__ candSlot, unsigned long long* candSet) {
    if (MODE == CM_INTEGRATE) {  // release this op's alloc dedup-set slots
        const uint32_t n = min(A.ctrl[C_CAND], candCap);
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            const int sl = candSlot[i];
            if (sl >= 0) candSet[sl] = EMPTY_KEY;
        }
    }
    // one list append per workgroup iteration: wave ballots -> LDS prefix over the 4 waves ->
    // a single atomic per list (instead of one per wave on the hot counter)
    __shared__ uint32_t s_cnt[2][4], s_base[2];
    const uint32_t hw = A.ctrl[C_HIGHWATER];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    unsigned long long scanned = 0, vis = 0, band = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < hw; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        int4 bp = make_int4(0, 0, 0, 0);
        if (i < hw) bp = A.blockPos[i];
        const bool alloc = bp.w != 0;
        const bool inFr = alloc && block_in_frustum_fast(cam, Tinv, bp.x, bp.y, bp.z, A.voxelSize);
        const bool inb = MODE != CM_FRUSTUM && inFr && block_may_update(A, cam, Tinv, bp.x, bp.y, bp.z, A.tiles, A.tiles2);
        const bool keepVis = inFr;
        const unsigned long long m0 = __ballot(keepVis), m1 = __ballot(inb);
        if (lane == 0) {
            s_cnt[0][wv] = (uint32_t)__popcll(m0);
            s_cnt[1][wv] = (uint32_t)__popcll(m1);
        }
        __syncthreads();
        if (threadIdx.x < 2) {
            const uint32_t tot = s_cnt[threadIdx.x][0] + s_cnt[threadIdx.x][1] + s_cnt[threadIdx.x][2] + s_cnt[threadIdx.x][3];
            s_base[threadIdx.x] = tot ? atomicAdd(&A.ctrl[threadIdx.x == 0 ? C_VISIBLE : C_BAND], tot) : 0u;
        }
        __syncthreads();
        uint32_t off0 = s_base[0], off1 = s_base[1];
        for (uint32_t k = 0; k < wv; k++) {
            off0 += s_cnt[0][k];
            off1 += s_cnt[1][k];
        }
        const int4 ent = make_int4(bp.x, bp.y, bp.z, (int)i);
        if (keepVis) A.visible[off0 + __popcll(m0 & lanemask_lt())] = ent;
        if (inb) A.band[off1 + __popcll(m1 & lanemask_lt())] = ent;
        scanned += alloc ? 1 : 0;
        vis += inFr ? 1 : 0;
        band += inb ? 1 : 0;
        __syncthreads();  // s_cnt / s_base reuse
    }
    flush_stats2(A.stats, S_SCANNED, scanned, S_VISIBLE, vis);
    if (MODE != CM_FRUSTUM) {
        __syncthreads();  // thread 0 of the first flush reads its LDS sums before they are reset
        flush_stats2(A.stats, S_BAND, band, -1, 0);
    }
}

// ---- divisions whose result only feeds an integer ------------------------------------------------
// f2i(num / den + m + 0.5f) and roundf(num / den) with the quotient of the reference's IEEE division.
// The quotient is first formed as num * rcp(den) (v_rcp_f32, 1 ulp): |q_approx - q| <= 2^-22 |q|.
// The integer outcome is a step function of the quotient, monotone through the remaining rounded
// additions, so it can only differ when a step (an integer for f2i, a half-integer for roundf) lies
// within that bound plus the rounding of the later additions. Such lanes (~1e-4 of them), and
// non-finite quotients, redo the IEEE division: the result is bit-identical to the plain code.
// The exact division runs only in waves where some lane needs it: the branch is taken on the wave's
// ballot and holds an empty asm statement, so the compiler cannot if-convert (speculate) it.
__device__ __forceinline__ int proj_coord(float num, float den, float m) {
    const float qa = num * __builtin_amdgcn_rcpf(den);
    float t = (qa + m) + 0.5f;
    const float eps = (fabsf(qa) + 2.0f * fabsf(t) + 2.0f) * 0x1p-21f;
    const bool need = !(fabsf(t - rintf(t)) > eps);
    if (__builtin_amdgcn_ballot_w64(need)) {
        asm volatile("" ::: "memory");
        const float te = (num / den + m) + 0.5f;
        t = need ? te : t;
    }
    return f2i(t);
}
__device__ __forceinline__ float round_quot(float num, float den, float rden) {
    float q = num * rden;
    const float aq = fabsf(q);
    const float eps = (aq + 1.0f) * 0x1p-21f;
    const bool need = !(fabsf((aq - floorf(aq)) - 0.5f) > eps);
    if (__builtin_amdgcn_ballot_w64(need)) {
        asm volatile("" ::: "memory");
        const float e = num / den;
        q = need ? e : q;
    }
    return roundf(q);
}

// Integrate colour blend of integrateDepthMapKernel (CUDASceneRepHashSDF.cu:486-496): per channel
// u8(clamp(roundf(0.2f * cu + 0.8f * oc), 0, 254.5)), or the new colour when the voxel is empty. The
// float expression lies within 1e-5 of (cu + 4 oc) / 5, whose fractional part is a multiple of 0.2,
// so its roundf is the integer (2 cu + 8 oc + 5) / 10 = ((2 cu + 8 oc + 5) * 6554) >> 16 (exact for
// all 65536 (cu, oc): checked exhaustively in tests/test_oracle_tsdf.py). Integer ops replace the
// float blend + roundf + clamp.
__device__ __forceinline__ uint32_t blend_channel(uint32_t cu, uint32_t oc, bool empty) {
    const uint32_t m = ((2u * cu + 8u * oc + 5u) * 6554u) >> 16;
    return min(empty ? cu : m, 254u);
}
__device__ __forceinline__ uint32_t blend_color(uint32_t c, uint32_t col, bool empty) {
    return blend_channel(c & 0xFF, col & 0xFF, empty) | (blend_channel((c >> 8) & 0xFF, (col >> 8) & 0xFF, empty) << 8) |
           (blend_channel((c >> 16) & 0xFF, (col >> 16) & 0xFF, empty) << 16) | (255u << 24);
}
// blend_color with packed FP32 arithmetic (the batch pass; BF_BLEND_F=0 builds the integer form:
// 4 VALU fewer per integrate update, k_apply_ops 619 / 618 -> 593 / 596 us, A/B pairs in
// profiles/r5_apply_experiments.txt): (cu + 4 oc) / 5 as (4 oc + cu)
// x 0.2f (operands exact integers, product within 1e-5 of the quotient, whose fraction is a multiple of
// 0.2), rounded by rintf (never a tie), min 254, and packed by v_cvt_pk_u8_f32 (an exact conversion of
// an integral value). An empty voxel takes oc = cu, for which the quotient is cu. Same bytes as
// blend_color for every (cu, oc, empty).
#ifndef BF_BLEND_F
#define BF_BLEND_F 1
#endif
__device__ __forceinline__ uint32_t blend_color_f(uint32_t c, uint32_t col, bool empty) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const uint32_t o = empty ? c : col;
    const f2 cu = {(float)(c & 0xFF), (float)((c >> 8) & 0xFF)}, oc = {(float)(o & 0xFF), (float)((o >> 8) & 0xFF)};
    const f2 t = __builtin_elementwise_fma(oc, f2{4.0f, 4.0f}, cu) * f2{0.2f, 0.2f};
    const float t2 = __builtin_fmaf((float)((o >> 16) & 0xFF), 4.0f, (float)((c >> 16) & 0xFF)) * 0.2f;
    uint32_t r = __builtin_amdgcn_cvt_pk_u8_f32(fminf(rintf(t.x), 254.0f), 0u, 0xFF000000u);
    r = __builtin_amdgcn_cvt_pk_u8_f32(fminf(rintf(t.y), 254.0f), 1u, r);
    return __builtin_amdgcn_cvt_pk_u8_f32(fminf(rintf(t2), 254.0f), 2u, r);
}
// Voxel update of integrateDepthMapKernel (CUDASceneRepHashSDF.cu:486-514), weightUpdate = 1.
__device__ __forceinline__ void voxel_integrate(float& s0, float& w0, uint32_t& col, float sdf, uint32_t c, float weightMax) {
    const float wUpd = 1.0f;
    col = blend_color(c, col, w0 == 0.0f);
    s0 = (sdf * wUpd + s0 * w0) / (wUpd + w0);
    w0 = fminf(weightMax, wUpd + w0);
}
__device__ __forceinline__ void voxel_deintegrate(float& s0, float& w0, uint32_t& col, float sdf, uint32_t c) {
    const float wUpd = 1.0f;
    const float cu0 = (float)(c & 0xFF), cu1 = (float)((c >> 8) & 0xFF), cu2 = (float)((c >> 16) & 0xFF);
    const float oc0 = (float)(col & 0xFF), oc1 = (float)((col >> 8) & 0xFF), oc2 = (float)((col >> 16) & 0xFF);
    const float den = w0 - wUpd, rden = __builtin_amdgcn_rcpf(den);
    float r0 = fmaxf(0.0f, fminf(round_quot(oc0 * w0 - cu0 * wUpd, den, rden), 254.5f));
    float r1 = fmaxf(0.0f, fminf(round_quot(oc1 * w0 - cu1 * wUpd, den, rden), 254.5f));
    float r2 = fmaxf(0.0f, fminf(round_quot(oc2 * w0 - cu2 * wUpd, den, rden), 254.5f));
    col = (uint32_t)(uint8_t)r0 | ((uint32_t)(uint8_t)r1 << 8) | ((uint32_t)(uint8_t)r2 << 16) | (255u << 24);
    s0 = (s0 * w0 - sdf * wUpd) / (w0 - wUpd);
    w0 = fmaxf(0.0f, w0 - wUpd);
    if (w0 <= 0.001f) { s0 = 0.0f; col = 0u; w0 = 0.0f; }
}

// The running-average quotient num / den of the voxel update, den = an integral weight in [0, 1024]:
// rcp, product, one fma residual and one fma correction. Checked bit-identical to the IEEE division
// for every float numerator in [2^-100, 2^100] (both signs) and every divisor 1..1024 on the GPU (the
// update's numerators are 0 or far above 2^-100: sdf and s0 * w0 are multiples of ~1e-9 m); den = 0
// only when a de-integration empties the voxel, whose sdf is then reset to 0.
__device__ __forceinline__ float div_weight(float num, float den) {
    const float r = __builtin_amdgcn_rcpf(den);
    const float q = num * r;
    const float e = __builtin_fmaf(-q, den, num);
    return __builtin_fmaf(e, r, q);
}
__device__ __forceinline__ void voxel_integrate_f(float& s0, float& w0, uint32_t& col, float sdf, uint32_t c, float weightMax) {
    col = blend_color(c, col, w0 == 0.0f);
    s0 = div_weight(sdf * 1.0f + s0 * w0, 1.0f + w0);
    w0 = fminf(weightMax, 1.0f + w0);
}
// De-integrate colour of one channel, u8(clamp(roundf((oc w - cu) / (w - 1)), 0, 254.5)), for an
// integral weight w >= 2 (every weight the update produces: +-1 steps from 0, capped by the integral
// weightMax). With d = w - 1 and delta = oc - cu the quotient is oc + delta / d, so the result is
// oc + floor((2 delta + d) / (2 d)), clamped to [0, 254]; for d > 510 the floor is 0 (|delta| <= 255),
// otherwise the quotient's distance to an integer is 0 or >= 1 / (2 d) >= 1 / 1020, far above the
// rcp product's error (<= 5e-5), so floor(fma(2 delta + d, rcp(2 d), 5e-4)) is exact. 9.3e9 cases
// (w 2..140000 with rcp +-1 ulp, sampled up to 1e8, every oc, cu; the fused and the unfused form)
// checked equal to the IEEE expression (tools/check_deint_color.c). Integer bytes in and out:
// delta and oc + k are 32-bit integer ops, floor + convert is one v_cvt_flr_i32_f32.
// rc = rcp(2 d), or 0 when d > 510; di = (int)d.
__device__ __forceinline__ int cvt_flr(float v) {
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(v));  // floor, saturate, NaN -> 0 (no UB)
    return r;
}
__device__ __forceinline__ uint32_t deint_channel(int oc, int cu, int di, float rc) {
    const int k = cvt_flr(__builtin_fmaf((float)(2 * (oc - cu) + di), rc, 5e-4f));
    return (uint32_t)min(max(oc + k, 0), 254);
}
// The de-integrate colour of the batch pass: deint_channel for integral weights, the reference
// expression otherwise (only an imported scene can hold those).
__device__ __forceinline__ void voxel_deint_color(float w0, uint32_t col, uint32_t c, uint32_t& out) {
    const float den = w0 - 1.0f;
    if (__builtin_amdgcn_ballot_w64(w0 != rintf(w0))) {
        asm volatile("" ::: "memory");
        const float wUpd = 1.0f;
        const float cu0 = (float)(c & 0xFF), cu1 = (float)((c >> 8) & 0xFF), cu2 = (float)((c >> 16) & 0xFF);
        const float oc0 = (float)(col & 0xFF), oc1 = (float)((col >> 8) & 0xFF), oc2 = (float)((col >> 16) & 0xFF);
        float r0 = fmaxf(0.0f, fminf(roundf((oc0 * w0 - cu0 * wUpd) / den), 254.5f));
        float r1 = fmaxf(0.0f, fminf(roundf((oc1 * w0 - cu1 * wUpd) / den), 254.5f));
        float r2 = fmaxf(0.0f, fminf(roundf((oc2 * w0 - cu2 * wUpd) / den), 254.5f));
        out = (uint32_t)(uint8_t)r0 | ((uint32_t)(uint8_t)r1 << 8) | ((uint32_t)(uint8_t)r2 << 16) | (255u << 24);
    } else {
        const float rc = den > 510.0f ? 0.0f : __builtin_amdgcn_rcpf(2.0f * den);
        const int di = cvt_flr(den);  // den is integral (w0 >= 0 here: no saturation matters)
        out = deint_channel((int)(col & 0xFF), (int)(c & 0xFF), di, rc) |
              (deint_channel((int)((col >> 8) & 0xFF), (int)((c >> 8) & 0xFF), di, rc) << 8) |
              (deint_channel((int)((col >> 16) & 0xFF), (int)((c >> 16) & 0xFF), di, rc) << 16) | (255u << 24);
    }
}

// Two voxels of one lane column, (x, y, z) and (x, y, z + 1), projected together: every float
// operation is the scalar path's (xform's ((e0 x + e1 y) + e2 z) + e3, then fx * x, the rcp quotient,
// + m, + 0.5), done elementwise on 2-wide vectors so that it issues as packed-FP32 instructions
// (v_pk_mul_f32 / v_pk_add_f32: two IEEE results per instruction, no contraction). The exactness
// check and the IEEE fallback of proj_coord follow per element.
typedef float f2v __attribute__((ext_vector_type(2)));
// Exactness test of a rounded screen coordinate t = (num * rcp(den) + m) + 0.5 against a bound that
// is constant per launch: eps_c = (3 (max(W, H) + 2) + max(|mx|, |my|) + 3) 2^-21 is at least
// proj_coord's per-lane bound (|qa| + 2 |t| + 2) 2^-21 for every lane with |t| <= max(W, H) + 2.
// Lanes beyond that are off-screen for the fast and the exact quotient alike (their distance to the
// screen exceeds the quotient error), so the pixel decision is the IEEE one everywhere.
__device__ __forceinline__ bool proj_needs_exact(float t, float epsc) { return !(fabsf(t - rintf(t)) > epsc); }
// b_r = e[4r] wx + e[4r+1] wy: the (x, y) part of every row, computed once per lane column and op.
// Outputs the byte offsets of the two voxels' pixels in the op's {depth, colour} image, or
// 0xFFFFFFFF off-screen (wc = 0 forces every pixel off-screen: an op without colour, :441-448);
// uy * W + ux in 24-bit multiplies (the image is far below 2^24 pixels a side).
__device__ __forceinline__ void voxel_pixel2b(const BFDepthCameraParams& cam, const BFMat4& T, const float* b, f2v wz,
                                              uint32_t wc, float epsc, uint32_t& off0, uint32_t& off1, f2v& pz) {
    const float* e = T.m;
    f2v p[3];
#pragma unroll
    for (int r = 0; r < 3; r++) p[r] = (f2v{b[r], b[r]} + f2v{e[4 * r + 2], e[4 * r + 2]} * wz) + f2v{e[4 * r + 3], e[4 * r + 3]};
    const f2v nx = p[0] * f2v{cam.fx, cam.fx}, ny = p[1] * f2v{cam.fy, cam.fy};
    const f2v rz = f2v{__builtin_amdgcn_rcpf(p[2].x), __builtin_amdgcn_rcpf(p[2].y)};
    const f2v qx = nx * rz, qy = ny * rz;
    f2v tx = (qx + f2v{cam.mx, cam.mx}) + f2v{0.5f, 0.5f};
    f2v ty = (qy + f2v{cam.my, cam.my}) + f2v{0.5f, 0.5f};
    const bool nx0 = proj_needs_exact(tx.x, epsc), nx1 = proj_needs_exact(tx.y, epsc);
    const bool ny0 = proj_needs_exact(ty.x, epsc), ny1 = proj_needs_exact(ty.y, epsc);
    if (__builtin_amdgcn_ballot_w64(nx0 | nx1 | ny0 | ny1)) {  // ~1e-4 of lanes: the IEEE quotients
        asm volatile("" ::: "memory");
        if (nx0) tx.x = (nx.x / p[2].x + cam.mx) + 0.5f;
        if (nx1) tx.y = (nx.y / p[2].y + cam.mx) + 0.5f;
        if (ny0) ty.x = (ny.x / p[2].x + cam.my) + 0.5f;
        if (ny1) ty.y = (ny.y / p[2].y + cam.my) + 0.5f;
    }
    const uint32_t ux0 = (uint32_t)f2i(tx.x), ux1 = (uint32_t)f2i(tx.y);
    const uint32_t uy0 = (uint32_t)f2i(ty.x), uy1 = (uint32_t)f2i(ty.y);
    const uint32_t W8 = cam.imageWidth * 8u;
    pz = p[2];
    off0 = ((ux0 < wc) & (uy0 < cam.imageHeight)) ? __umul24(uy0, W8) + (ux0 << 3) : 0xFFFFFFFFu;
    off1 = ((ux1 < wc) & (uy1 < cam.imageHeight)) ? __umul24(uy1, W8) + (ux1 << 3) : 0xFFFFFFFFu;
}

// Band test of one voxel for one pose (CUDASceneRepHashSDF.cu:449-466): sdf clamped to +-truncation.
__device__ __forceinline__ bool voxel_in_band(const HashArgs& A, float dz, float pz, float& sdf) {
    sdf = dz - pz;
    const float tr = A.truncation + A.truncScale * dz;
    const bool in = dz != -INFINITY && dz < A.maxIntegrationDistance && fabsf(sdf) < tr;
    sdf = (sdf >= 0.0f) ? fminf(tr, sdf) : fmaxf(-tr, sdf);
    return in;
}

// integrateDepthMapKernel<deIntegrate>, CUDASceneRepHashSDF.cu:420-521. One wave per block:
// lane = (y, x) of a z-slice, 8 slices. Voxel bytes are touched only inside the band.
template <bool DEINT, int ZC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_integrate(HashArgs A, const float* __restrict__ depthImg,
                                                   const uint32_t* __restrict__ colorImg, BFDepthCameraParams cam,
                                                   BFMat4 Tinv) {
    const uint32_t nvis = A.ctrl[C_BAND];
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    const int lx = lane & 7, ly = lane >> 3;
    const uint32_t W = cam.imageWidth, H = cam.imageHeight;
    const float wUpd = 1.0f;  // weightUpdate forced to 1 (:465-466)
    unsigned long long updated = 0;
    for (uint32_t b = wave; b < nvis; b += nwaves) {
        const int4 e = A.band[b];
        const int bx = e.x * BF_SDF_BLOCK_SIZE + lx, by = e.y * BF_SDF_BLOCK_SIZE + ly, bz = e.z * BF_SDF_BLOCK_SIZE;
        int dcount = 0;
        uint32_t nupd = 0;
        // ZC z-slices per round (8: one round, most ILP; 4: two rounds, fewer VGPRs, more waves)
#pragma unroll
        for (int z0 = 0; z0 < BF_SDF_BLOCK_SIZE; z0 += ZC) {
        // phase 1: project the lane's voxels and issue the depth gathers back to back
        float depth[ZC], pz[ZC];
        uint32_t pix[ZC];
#pragma unroll
        for (int zi = 0; zi < ZC; zi++) {
            const int z = z0 + zi;
            const f3 pf = xform(Tinv, vvox_to_world(bx, by, bz + z, A.voxelSize));
            const uint32_t ux = (uint32_t)proj_coord(pf.x * cam.fx, pf.z, cam.mx);
            const uint32_t uy = (uint32_t)proj_coord(pf.y * cam.fy, pf.z, cam.my);
            const bool on = ux < W && uy < H && colorImg != nullptr;  // colour NULL: no update (:441-448)
            pix[zi] = on ? uy * W + ux : 0xFFFFFFFFu;
            pz[zi] = pf.z;
            depth[zi] = on ? depthImg[pix[zi]] : -INFINITY;
        }
        // phase 2: band test, then issue the in-band voxel and colour loads together
        float sdfv[ZC], osdf[ZC], ow[ZC];
        uint32_t oc[ZC], cc[ZC];
        uint32_t band = 0;
#pragma unroll
        for (int zi = 0; zi < ZC; zi++) {
            const int z = z0 + zi;
            const float dz = depth[zi];
            float sdf = dz - pz[zi];
            const float tr = A.truncation + A.truncScale * dz;
            const bool in = dz != -INFINITY && dz < A.maxIntegrationDistance && fabsf(sdf) < tr;
            sdf = (sdf >= 0.0f) ? fminf(tr, sdf) : fmaxf(-tr, sdf);
            sdfv[zi] = sdf;
            osdf[zi] = 0.0f; ow[zi] = 0.0f; oc[zi] = 0u; cc[zi] = 0u;
            if (in) {
                band |= 1u << zi;
                // one 12-B load per voxel (global_load_dwordx3) instead of three dword loads
                const Vox3 v = *reinterpret_cast<const Vox3*>(A.voxels + (size_t)e.w * BF_VOXELS_PER_BLOCK + (uint32_t)(z * 64 + lane));
                osdf[zi] = __uint_as_float(v.a);
                ow[zi] = __uint_as_float(v.b);
                oc[zi] = v.c;
                cc[zi] = colorImg[pix[zi]];
            }
        }
        // phase 3: running average (integrate) or its inverse (de-integrate), store
#pragma unroll
        for (int zi = 0; zi < ZC; zi++) {
            const int z = z0 + zi;
            if (!(band & (1u << zi))) continue;
            const uint32_t c = cc[zi];
            const float cu0 = (float)(c & 0xFF), cu1 = (float)((c >> 8) & 0xFF), cu2 = (float)((c >> 16) & 0xFF);
            const uint32_t o = oc[zi];
            const float oc0 = (float)(o & 0xFF), oc1 = (float)((o >> 8) & 0xFF), oc2 = (float)((o >> 16) & 0xFF);
            const float w0 = ow[zi], s0 = osdf[zi], sdf = sdfv[zi];
            float r0, r1, r2, nsdf, nw;
            uint32_t ncol;
            if (!DEINT) {
                ncol = blend_color(c, o, w0 == 0.0f);
                nsdf = (sdf * wUpd + s0 * w0) / (wUpd + w0);
                nw = fminf(A.weightMax, wUpd + w0);
            } else {
                const float den = w0 - wUpd, rden = __builtin_amdgcn_rcpf(den);
                r0 = fmaxf(0.0f, fminf(round_quot(oc0 * w0 - cu0 * wUpd, den, rden), 254.5f));
                r1 = fmaxf(0.0f, fminf(round_quot(oc1 * w0 - cu1 * wUpd, den, rden), 254.5f));
                r2 = fmaxf(0.0f, fminf(round_quot(oc2 * w0 - cu2 * wUpd, den, rden), 254.5f));
                ncol = (uint32_t)(uint8_t)r0 | ((uint32_t)(uint8_t)r1 << 8) | ((uint32_t)(uint8_t)r2 << 16) | (255u << 24);
                nsdf = (s0 * w0 - sdf * wUpd) / (w0 - wUpd);
                nw = fmaxf(0.0f, w0 - wUpd);
                if (nw <= 0.001f) { nsdf = 0.0f; ncol = 0u; nw = 0.0f; }
            }
            Vox3 nv;
            nv.a = __float_as_uint(nsdf);
            nv.b = __float_as_uint(nw);
            nv.c = ncol;
            *reinterpret_cast<Vox3*>(A.voxels + (size_t)e.w * BF_VOXELS_PER_BLOCK + (uint32_t)(z * 64 + lane)) = nv;  // dwordx3 store
            // per-block count of voxels with (uint)weight != 0 (GC decision, :606/:625)
            dcount += (int)(nw >= 1.0f) - (int)(w0 >= 1.0f);
            nupd++;
        }
        }  // z0
        const unsigned long long anyChange = __ballot(dcount != 0);
        if (anyChange) {
            for (int off = 32; off > 0; off >>= 1) dcount += __shfl_xor(dcount, off);
            if (lane == 0 && dcount != 0) atomicAdd(&A.blockCount[(uint32_t)e.w], (uint32_t)dcount);
        }
        updated += nupd;
    }
    flush_stats2(A.stats, S_VOXELS, updated, S_RMW, updated);
}

// ---- op batches (Scene::applyOps) ---------------------------------------------------------------
// The batch pass's {depth, colour} image stores depth as bits(d) ^ 0xFF800000 for the depths
// integrateDepthMapKernel accepts (d != MINF, d < maxIntegrationDistance, CUDASceneRepHashSDF.cu:
// 449-452) and 0 for the rest: a decoded invalid depth, like the all-zero word a buffer load returns
// past the image's range, is -inf, for which |d - z| < truncation + truncScale * d is false. The band
// test is then that one comparison, and the clamp of sdf to +-truncation (:458-462) is the identity
// inside the band.
constexpr uint32_t DC_DEPTH_KEY = 0xFF800000u;

// k_apply_ops's grid: rounds of resident workgroups (Scene::Scene)
constexpr int kApplyRounds = 4;
// k_apply_ops's inner step and occupancy (overridable for A/B builds of kernel variants)
#ifndef BF_APPLY_ZC
#define BF_APPLY_ZC 4
#endif
#ifndef BF_APPLY_WPE
#define BF_APPLY_WPE 8
#endif
// k_apply_ops: wave priority while a wave projects an op step's voxels and issues its gathers (0: off;
// see apply_op_slices)
#ifndef BF_APPLY_PRIO
#define BF_APPLY_PRIO 1
#endif
// k_compactify_ops: workgroups per CU, its occupancy (5: <= 96 VGPRs; 4 / 6 measured 49.0 / 47.1 us
// against 44.7, profiles/r11_scan_ab.txt)
#ifndef BF_SCAN_WPC
#define BF_SCAN_WPC 5
#endif
// work-list op mask of a block: which ops may update each z-half (x: voxel z 0..3, y: 4..7)
typedef uint2 OpMask;
constexpr int MASK_PARTS = 2;
__device__ __forceinline__ uint32_t dc_depth_word(float d, float maxDist) {
    return (d != -INFINITY && d < maxDist) ? (__float_as_uint(d) ^ DC_DEPTH_KEY) : 0u;
}

// per-op interleaved {depth, colour} image: the voxel pass gathers both values of a pixel with one
// dwordx2 load from one cache line (two dword gathers from two images before). Ops without colour
// never gather (their pixels are off-screen to integrateDepthMapKernel, :441-448).
__device__ __forceinline__ void pack_dc(const OpTable& ops, uint32_t k, uint32_t i0, uint32_t stride, uint32_t P, float maxDist) {
    if (ops.color[k] == nullptr) return;
    const float* __restrict__ d = ops.depth[k];
    const uint32_t* __restrict__ c = ops.color[k];
    uint2* __restrict__ o = ops.dc[k];
    for (uint32_t i = i0; i < P; i += stride) o[i] = make_uint2(dc_depth_word(d[i], maxDist), c[i]);
}
// per-op 8x8-tile depth bounds and dc image (blockIdx.y = op; workgroups [0, tileBlocks) build the
// tiles, the rest the dc image) + the per-batch counter reset (ops whose frame already has both,
// e.g. a frame-store frame re-integrated before, skip)
__global__ __launch_bounds__(256) void k_begin_ops_tiles(uint32_t* ctrl, unsigned long long* stats, OpTable ops, uint32_t W,
                                                         uint32_t H, uint32_t tilesW, uint32_t tilesH, uint32_t tiles2W,
                                                         uint32_t tiles2H, float maxDist, uint32_t tileBlocks) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        ctrl[C_VISIBLE] = 0;
        ctrl[C_BAND] = 0;
        ctrl[C_CAND] = 0;
        ctrl[C_OVF] = 0;
        stats[S_OPS] += ops.n;
        stats[S_BOPS] += ops.n;
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < Scene::kMaxOps) ctrl[C_OPBIN + threadIdx.x] = 0;
    if (blockIdx.y >= ops.nTile) return;  // a batch whose frames are all cached launches one workgroup
    const uint32_t k = ops.tileIdx[blockIdx.y];
    if (blockIdx.x >= tileBlocks) {
        pack_dc(ops, k, (blockIdx.x - tileBlocks) * blockDim.x + threadIdx.x, (gridDim.x - tileBlocks) * blockDim.x, W * H, maxDist);
        return;
    }
    depth_tile_wave((blockIdx.x * blockDim.x + threadIdx.x) >> 6, ops.depth[k], W, H, tilesW, tilesH, tiles2W, tiles2H,
                    maxDist, ops.tiles[k], ops.tiles2[k]);
}

// One scan of the allocated pool for the whole batch: `visible` = frustum list of the last op (the
// list garbageCollect walks), work list = blocks some op may update, with the op bit mask. Also
// releases the batch's alloc dedup-set slots.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BF_SCAN_WPC))) void k_compactify_ops(HashArgs A, BFDepthCameraParams cam, OpTable ops, uint32_t candCap,
                                                        const int* __restrict__ candSlot, unsigned long long* candSet,
                                                        OpMask* masks, const uint32_t* __restrict__ birth, uint32_t epoch,
                                                        uint32_t binCap) {
    {
        const uint32_t n = min(A.ctrl[C_CAND], candCap);
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            const int sl = candSlot[i];
            if (sl >= 0) candSet[sl] = EMPTY_KEY;
        }
    }
    __shared__ uint32_t s_cnt[4], s_base, s_bcnt[Scene::kMaxOps], s_bbase[Scene::kMaxOps];
    // the band cull runs on the (block, op) pairs that passed the frustum test, compacted per wave:
    // run per lane over its ops, it had every lane of a wave execute it whenever one lane's block
    // passed (the wave's 64 blocks almost always include one), ~3x the VALU of the compacted form
    __shared__ int4 s_bp[256];
    __shared__ uint32_t s_mask[MASK_PARTS][256];  // per z-half (voxel z 0..3 / 4..7) or z-quarter of the block
    __shared__ uint16_t s_q[4][64 * Scene::kMaxOps];  // per wave: lane << 5 | op
    __shared__ float s_tinv[Scene::kMaxOps][12];
    __shared__ const float2* s_tiles[2][Scene::kMaxOps];
    for (uint32_t q = threadIdx.x; q < ops.n * 12; q += blockDim.x) s_tinv[q / 12][q % 12] = ops.tinv[q / 12][q % 12];
    if (threadIdx.x < ops.n) {
        s_tiles[0][threadIdx.x] = ops.tiles[threadIdx.x];
        s_tiles[1][threadIdx.x] = ops.tiles2[threadIdx.x];
    }
    __syncthreads();
    __shared__ float4 s_cull[Scene::kMaxOps][CULL_CONSTS / 4];
    if (threadIdx.x < ops.n) cull_op_consts(s_tinv[threadIdx.x], cam, A.voxelSize, reinterpret_cast<float*>(s_cull[threadIdx.x]));
    __syncthreads();
    const uint32_t hw = A.ctrl[C_HIGHWATER];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    unsigned long long scanned = 0, vis = 0, band = 0, evals = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < hw; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        int4 bp = make_int4(0, 0, 0, 0);
        uint32_t bi = 0;
        if (i < hw) {  // both loads issued together (the birth load waited for the position before)
            bp = A.blockPos[i];
            bi = birth[i];
        }
        const bool alloc = bp.w != 0;
        uint32_t fr = 0;  // ops whose frustum holds the block
        if (alloc) {
            // a block born in this batch at op j exists for ops j.. only (ops before it see no block)
            const uint32_t first = (bi >> 8) == epoch ? 255u - (bi & 255u) : 0u;
            // k runs over every op in every lane (a wave-uniform loop keeps the op's pose in scalar loads)
            for (uint32_t k = 0; k < ops.n; k++) {
                const BFMat4 Ti = op_mat(ops.tinv[k]);
                if (k >= first && block_in_frustum_fast(cam, Ti, bp.x, bp.y, bp.z, A.voxelSize)) fr |= 1u << k;
            }
        }
        // the GC's list: the last op's frustum (a block born in the batch exists for the last op)
        const bool keepVis = (fr >> (ops.n - 1)) & 1u;
        // queue the wave's (block, op) pairs, then every lane takes one pair per round for the band cull
        s_bp[threadIdx.x] = bp;
#pragma unroll
        for (int q = 0; q < MASK_PARTS; q++) s_mask[q][threadIdx.x] = 0u;
        uint32_t qoff = (uint32_t)__popc(fr), qtot = qoff;
        for (int off = 1; off < 64; off <<= 1) {  // inclusive wave scan of the pair counts
            const uint32_t v = (uint32_t)__shfl_up((int)qoff, off);
            if ((int)lane >= off) qoff += v;
        }
        qtot = (uint32_t)__shfl((int)qoff, 63);
        qoff -= (uint32_t)__popc(fr);
        for (uint32_t m = fr; m; m &= m - 1) s_q[wv][qoff++] = (uint16_t)((lane << 5) | (uint32_t)__builtin_ctz(m));
        __syncthreads();
        for (uint32_t r = lane; r < qtot; r += 64) {
            const uint32_t e = s_q[wv][r], src = wv * 64 + (e >> 5), k = e & 31u;
            const int4 b = s_bp[src];
            // the voxel pass applies an op to a block half by half (4 z-slices per round)
#if defined(BF_CULL_DIAG_NOBAND)  // timing diagnostic only (wrong masks): the scan without the band cull
            const uint32_t hb = 3u;
            (void)b;
#else
            float cq[CULL_CONSTS];
#pragma unroll
            for (int c = 0; c < CULL_CONSTS / 4; c++) reinterpret_cast<float4*>(cq)[c] = s_cull[k][c];
            const uint32_t hb = block_may_update_halves_q(A, cam, cq, b.x, b.y, b.z, s_tiles[0][k], s_tiles[1][k]);
#endif
#pragma unroll
            for (int q = 0; q < MASK_PARTS; q++)
                if ((hb >> q) & 1u) atomicOr(&s_mask[q][src], 1u << k);
        }
        __syncthreads();
        const OpMask hm = make_uint2(s_mask[0][threadIdx.x], s_mask[1][threadIdx.x]);
        const uint32_t mask = hm.x | hm.y;
        const uint32_t cost = (uint32_t)(__popc(hm.x) + __popc(hm.y));  // op-halves to apply
        const uint32_t evq = 2u * cost;
        const bool inb = mask != 0;
        // work list: one bin per cost (op-halves, two per bin), so the voxel pass can hand out the
        // costliest blocks first (entry order inside a bin is free: every block is applied by one wave)
        const uint32_t bin = inb ? (cost + 1u) / 2u - 1u : 0u;
        const unsigned long long m0 = __ballot(keepVis);
        if (threadIdx.x < Scene::kMaxOps) s_bcnt[threadIdx.x] = 0;
        if (lane == 0) s_cnt[wv] = (uint32_t)__popcll(m0);
        __syncthreads();
        const uint32_t local = inb ? atomicAdd(&s_bcnt[bin], 1u) : 0u;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
            s_base = tot ? atomicAdd(&A.ctrl[C_VISIBLE], tot) : 0u;
        }
        if (threadIdx.x < ops.n && s_bcnt[threadIdx.x]) s_bbase[threadIdx.x] = atomicAdd(&A.ctrl[C_OPBIN + threadIdx.x], s_bcnt[threadIdx.x]);
        __syncthreads();
        uint32_t off0 = s_base;
        for (uint32_t k = 0; k < wv; k++) off0 += s_cnt[k];
        const int4 ent = make_int4(bp.x, bp.y, bp.z, (int)i);
        if (keepVis) A.visible[off0 + __popcll(m0 & lanemask_lt())] = ent;
        if (inb) {
            const size_t k = (size_t)bin * binCap + s_bbase[bin] + local;
            A.band[k] = ent;
            masks[k] = hm;
        }
        scanned += alloc ? 1 : 0;
        vis += keepVis ? 1 : 0;
        band += inb ? 1 : 0;
        evals += (unsigned long long)evq;
        __syncthreads();
    }
    flush_stats2(A.stats, S_SCANNED, scanned, S_VISIBLE, vis);
    __syncthreads();
    flush_stats2(A.stats, S_BAND, band, S_BBLOCKS, band);
    __syncthreads();
    flush_stats2(A.stats, S_BEVAL, evals * (BF_VOXELS_PER_BLOCK / 4), -1, 0);  // evaluations: 128 voxels per op-quarter
}

// The batch's voxel pass: one wave per work-list block, lane = (x, y), ZC z-slices per round. For
// each op of the block's mask, in sequence order: project, gather depth, band test, then the
// integrate / de-integrate update of integrateDepthMapKernel (CUDASceneRepHashSDF.cu:420-521) on
// the register copy of the voxel. A voxel is loaded when the first op reaches it and stored once.
// The batch work list as one virtual list, costliest bins first (op count n down to 1): position g
// of the list -> its slot. A wave walks g = wave, wave + nwaves, ..., so every wave takes one entry
// per round of a list sorted by cost and all waves end with nearly equal work (with the list in scan
// order a wave's ~9 blocks drew random op counts and the waves that drew many-op blocks set the
// launch's end: 946 -> 824 us per launch at the bench workload).
struct WorkCursor {
    uint32_t bin, lo, hi;  // current bin and its virtual range [lo, hi)
};
__device__ __forceinline__ WorkCursor work_begin(const uint32_t* ctrl, uint32_t nops) {
    const uint32_t b = nops - 1;
    return WorkCursor{b, 0u, ctrl[C_OPBIN + b]};
}
// slot of virtual position g (g never decreases between calls); returns false past the end
__device__ __forceinline__ bool work_slot(const uint32_t* ctrl, WorkCursor& c, uint32_t g, uint32_t binCap, size_t& slot) {
    while (g >= c.hi) {
        if (c.bin == 0) return false;
        c.bin--;
        c.lo = c.hi;
        c.hi += ctrl[C_OPBIN + c.bin];
    }
    slot = (size_t)c.bin * binCap + (g - c.lo);
    return true;
}
// k_apply_ops, the batch's voxel pass: one wave per work-list block, lane = (x, y) column. The lane's
// voxels of ZR z-slices stay in registers while the ops of the block's mask run over them in sequence
// order (the outer loop), ZC z-slices per step (the inner one): project, gather {depth, colour}, band
// test, then the integrate / de-integrate update of integrateDepthMapKernel (CUDASceneRepHashSDF.cu:
// 420-521) on the register copy; each touched voxel is stored once. An op's z-slices project to nearly
// the same pixels, so its gathers follow each other and hit the lines the previous slice fetched (the
// z-round-outer order re-fetched every op's footprint once per round: 888 -> 856 us per launch at the
// bench workload); the op's pose and the (x, y) part of its projection are taken once per ZR slices.
// ZR = 4, ZC = 4 at 8 waves per SIMD (64 VGPRs; measured: ZR 4 / ZC 2 847 us, 7 waves 901 us).
// Voxel updates of the batch pass (integrateDepthMapKernel, :467-514, weightUpdate = 1) on register
// copies, for in-band voxels (sdf unclamped: see above). Weights are non-negative floats here, whose
// bit patterns order like the values: min(1 + w, weightMax) is an integer min of the bits.
__device__ __forceinline__ void batch_integrate(float& s0, float& w0, uint32_t& col, float sdf, uint32_t c, float weightMax) {
    col = BF_BLEND_F ? blend_color_f(c, col, w0 == 0.0f) : blend_color(c, col, w0 == 0.0f);
    s0 = div_weight(sdf * 1.0f + s0 * w0, 1.0f + w0);
    w0 = __uint_as_float(min(__float_as_uint(1.0f + w0), __float_as_uint(weightMax)));
}
__device__ __forceinline__ void batch_deintegrate(float& s0, float& w0, uint32_t& col, float sdf, uint32_t c) {
    uint32_t ncol;
    voxel_deint_color(w0, col, c, ncol);
    const float den = w0 - 1.0f;
    const float ns = div_weight(s0 * w0 - sdf * 1.0f, den);
    // fmaxf(0, w - 1) <= 0.001 exactly when w - 1 <= 0.001: the emptied voxel is reset
    const bool empty = den <= 0.001f;
    s0 = empty ? 0.0f : ns;
    col = empty ? 0u : ncol;
    w0 = empty ? 0.0f : den;
}

// A voxel's register copy in the batch pass: an array of these (not three arrays of floats, which the
// compiler promotes to vectors whose one-element updates cost whole-vector register copies)
struct RegVox {
    float s, w;
    uint32_t c;
};
// One op over the lane's ZR register voxels (see k_apply_ops); deint: the op's direction (wave-
// uniform; a template split of the op body into two directions measured spills at 64 VGPRs).
template <int ZR, int ZC, int TOFF = 0>
__device__ __forceinline__ void apply_op_slices(bool deint, const HashArgs& A, const BFDepthCameraParams& cam, const BFMat4& Ti,
                                                const float* bxy, __amdgpu_buffer_rsrc_t dcRsrc, uint32_t wc, float epsc,
                                                int bzh, RegVox* rv, uint32_t& touched,
                                                uint32_t& nupd, uint32_t& nwav
#ifdef BF_APPLY_DIAG
                                                , uint32_t* diag
#endif
                                                ) {
#pragma unroll
    for (int z0 = 0; z0 < ZR; z0 += ZC) {
        uint32_t pix[ZC], cc[ZC];
        float pz[ZC], d[ZC];
#if BF_APPLY_PRIO
        // the projection at a raised priority, back to normal once the step's gathers are issued: among the
        // SIMD's waves, one that is about to issue loads goes first, so more gathers are in flight while the
        // others run their updates (458 -> 441 us per launch; the raise over the whole kernel, above the
        // bundling kernels' waves, or for the update phase instead measured slower, profiles/r11_prio_ab.txt)
        __builtin_amdgcn_s_setprio(BF_APPLY_PRIO);
#endif
#pragma unroll
        for (int zi = 0; zi < ZC; zi += 2) {
            const f2v wz = f2v{(float)(bzh + z0 + zi), (float)(bzh + z0 + zi + 1)} * f2v{A.voxelSize, A.voxelSize};
            f2v pz2;
            voxel_pixel2b(cam, Ti, bxy, wz, wc, epsc, pix[zi], pix[zi + 1], pz2);
            pz[zi] = pz2.x;
            pz[zi + 1] = pz2.y;
        }
#pragma unroll
        for (int zi = 0; zi < ZC; zi++) {
            // off-screen lanes read past the descriptor's range: {0, 0}
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(dcRsrc, pix[zi], 0, 0);
            d[zi] = __uint_as_float(v[0] ^ DC_DEPTH_KEY);
            cc[zi] = v[1];
        }
#if BF_APPLY_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
#ifdef BF_APPLY_DIAG
        {  // (slice pair, op) wave-slots with no lane in band, and all of them (counted on lane 0)
            unsigned long long b[ZC];
#pragma unroll
            for (int zi = 0; zi < ZC; zi++) b[zi] = __builtin_amdgcn_ballot_w64(fabsf(d[zi] - pz[zi]) < A.truncation + A.truncScale * d[zi]);
            if (lane_id_here() == 0)
#pragma unroll
                for (int zi = 0; zi < ZC; zi += 2) { diag[4] += (b[zi] | b[zi + 1]) == 0; diag[5] += 1; }
        }
#endif
#pragma unroll
        for (int zi = 0; zi < ZC; zi++) {
            const float sd = d[zi] - pz[zi];
            const float tr = A.truncation + A.truncScale * d[zi];
            const bool in = fabsf(sd) < tr;
#ifdef BF_APPLY_DIAG
            {  // measurement build: where the evaluations go (per lane)
                const bool off = pix[zi] == 0xFFFFFFFFu, inval = !off && d[zi] == -INFINITY;
                diag[0] += off;
                diag[1] += inval;
                diag[2] += !off && !inval && sd >= tr;
                diag[3] += !off && !inval && sd <= -tr;
            }
#endif
            // the wave's in-band lanes, counted in uniform control flow (a scalar add inside the
            // divergent branch below would be per lane)
            nupd += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(in));
#ifdef BF_APPLY_COUNT_WAVES
            nwav += __builtin_amdgcn_ballot_w64(in) ? 64u : 0u;  // measurement build: update executions x 64 as voxels_rmw
#endif
            if (!in) continue;
            touched |= 1u << (TOFF + z0 + zi);
            RegVox& v = rv[z0 + zi];
            if (deint) batch_deintegrate(v.s, v.w, v.c, sd, cc[zi]);
            else batch_integrate(v.s, v.w, v.c, sd, cc[zi], A.weightMax);
        }
    }
}

// k_apply_ops, the batch's voxel pass: one wave per work-list block, lane = (x, y) column. The lane's
// voxels of ZR z-slices stay in registers while the ops of the block's mask run over them in sequence
// order (the outer loop), ZC z-slices per step (the inner one): project, gather {depth, colour}, band
// test, then the integrate / de-integrate update of integrateDepthMapKernel (CUDASceneRepHashSDF.cu:
// 420-521) on the register copy; each touched voxel is stored once. An op's z-slices project to nearly
// the same pixels, so its gathers follow each other and hit the lines the previous slice fetched (the
// z-round-outer order re-fetched every op's footprint once per round: 888 -> 856 us per launch at the
// bench workload); the op's pose and the (x, y) part of its projection are taken once per ZR slices.
// ZR = 4, ZC = 4 at 8 waves per SIMD (64 VGPRs; measured: ZR 4 / ZC 2 847 us, 7 waves 901 us). One wave
// per workgroup (a slot is handed on as soon as its wave ends). The kernel sits at neither roof: ~0.5 of the
// VALU issue peak and 0.36 of HBM by the counters at the driver workload (458-461 us per launch), with the
// waves' cycles 22 % issuing, 45.5 % waiting to issue (dependencies) and 32.5 % waiting on memory
// (profiles/r10_apply_sq_pmc.txt): it is dependency / latency bound. Lane-derived values are re-read per
// block instead of kept live (no spills), counters are scalar. The op steps' projections run at a raised
// issue priority (apply_op_slices): 458 -> 441 us.
template <int ZR, int ZC, int WPE, bool XCDRUNS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) void k_apply_ops(
    HashArgs A, BFDepthCameraParams cam, OpTable ops, const OpMask* __restrict__ masks, const int4* __restrict__ band, uint32_t binCap,
    int xcdShift) {
    static_assert(ZR * 2 == BF_SDF_BLOCK_SIZE, "one op mask per z-half of the block");
    const uint32_t nwaves = gridDim.x;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(blockIdx.x);
    // XCDRUNS (BFSceneOptions.applyXcdRun): runs of 2^xcdShift consecutive work-list positions go to one XCD
    // (workgroup i runs on XCD i mod 8), run j to XCD j mod 8; otherwise (a grid that is not a multiple of 8)
    // consecutive positions go to consecutive waves, i.e. every XCD's waves spread over the whole list
    uint32_t v0 = wave, vstep = nwaves, xcd = 0, cmask = 0;
    if constexpr (XCDRUNS) {
        v0 = (uint32_t)__builtin_amdgcn_readfirstlane(blockIdx.x >> 3);
        vstep = nwaves >> 3;
        xcd = blockIdx.x & 7u;
        cmask = (1u << xcdShift) - 1u;
    }
    const float epsc = (3.0f * (float)(max(cam.imageWidth, cam.imageHeight) + 2u) + fmaxf(fabsf(cam.mx), fabsf(cam.my)) + 3.0f) * 0x1p-21f;
    uint32_t updated = 0, rmw = 0, halves = 0;  // per wave and launch: < 2^32
#ifdef BF_APPLY_DIAG
    uint32_t diag[6] = {0, 0, 0, 0, 0, 0}, diagPairs = 0, diagEmpty = 0;
#endif
    WorkCursor cur = work_begin(A.ctrl, ops.n);
    size_t b;
    auto pos = [&](uint32_t v) { return XCDRUNS ? (((v >> xcdShift) << 3 | xcd) << xcdShift) | (v & cmask) : v; };
    // the next block's work-list entry and mask (scalar loads) are issued while this block runs, so a block
    // start waits for its voxel loads alone: 440 -> 435 us per launch (profiles/r11_prio_ab.txt)
    bool have = work_slot(A.ctrl, cur, pos(v0), binCap, b);
    int4 evN = make_int4(0, 0, 0, 0);
    OpMask mhN = make_uint2(0u, 0u);
    if (have) { evN = band[b]; mhN = masks[b]; }
    for (uint32_t v = v0; have;) {
        const int4 ev = evN;
        const OpMask mh = mhN;
        v += vstep;
        have = work_slot(A.ctrl, cur, pos(v), binCap, b);
        if (have) { evN = band[b]; mhN = masks[b]; }
        // wave-uniform: keep the block's coordinates and base in SGPRs
        const int4 e = make_int4(__builtin_amdgcn_readfirstlane(ev.x), __builtin_amdgcn_readfirstlane(ev.y),
                                 __builtin_amdgcn_readfirstlane(ev.z), __builtin_amdgcn_readfirstlane(ev.w));
        const uint32_t blk = (uint32_t)e.w;
        const uint32_t lane = lane_id_here();
        const int lx = lane & 7, ly = lane >> 3;
        const uint32_t maskH[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(mh.x), (uint32_t)__builtin_amdgcn_readfirstlane(mh.y)};
        const int bx = e.x * BF_SDF_BLOCK_SIZE + lx, by = e.y * BF_SDF_BLOCK_SIZE + ly, bz = e.z * BF_SDF_BLOCK_SIZE;
        const float wx = (float)bx * A.voxelSize, wy = (float)by * A.voxelSize;
        Vox3* vp = reinterpret_cast<Vox3*>(A.voxels + (size_t)e.w * BF_VOXELS_PER_BLOCK) + lane;
        int dcount = 0;
        uint32_t nupd = 0, nrmw = 0, nwav = 0;
#pragma unroll
        for (int h = 0; h < BF_SDF_BLOCK_SIZE; h += ZR) {
            // a half no op reaches is neither read nor written (wave-uniform branch on an SGPR mask)
            if (maskH[h / ZR] == 0u) continue;
            halves++;
            RegVox rv[ZR];
            uint32_t pos0 = 0;
#pragma unroll
            for (int z = 0; z < ZR; z++) {
                const Vox3 v = vp[(h + z) * 64];
                rv[z] = RegVox{__uint_as_float(v.a), __uint_as_float(v.b), v.c};
                pos0 |= (uint32_t)(rv[z].w >= 1.0f) << z;
            }
            uint32_t touched = 0;
            for (uint32_t mk = maskH[h / ZR]; mk;) {
                const uint32_t k = (uint32_t)__builtin_ctz(mk);
                mk &= mk - 1;
                const BFMat4 Ti = op_mat(ops.tinv[k]);
                const float bxy[3] = {Ti.m[0] * wx + Ti.m[1] * wy, Ti.m[4] * wx + Ti.m[5] * wy, Ti.m[8] * wx + Ti.m[9] * wy};
                // the op's {depth, colour} image through a buffer descriptor: 32-bit offsets, and an
                // off-screen lane's out-of-range offset reads 0 without a branch
                const int dcBytes = (int)(cam.imageWidth * cam.imageHeight * 8u);
                const __amdgpu_buffer_rsrc_t dcRsrc = __builtin_amdgcn_make_buffer_rsrc((void*)ops.dc[k], (short)0, dcBytes, 0x00020000);
                const uint32_t wc = ops.color[k] != nullptr ? cam.imageWidth : 0u;
#ifdef BF_APPLY_DIAG
                const uint32_t before = nupd;
                apply_op_slices<ZR, ZC>((ops.deintMask >> k) & 1u, A, cam, Ti, bxy, dcRsrc, wc, epsc, bz + h, rv, touched, nupd, nwav, diag);
                diagPairs++;
                diagEmpty += nupd == before;
#else
                apply_op_slices<ZR, ZC>((ops.deintMask >> k) & 1u, A, cam, Ti, bxy, dcRsrc, wc, epsc, bz + h, rv, touched, nupd, nwav);
#endif
            }
#pragma unroll
            for (int z = 0; z < ZR; z++) {
                if (!((touched >> z) & 1u)) continue;
                Vox3 nv;
                nv.a = __float_as_uint(rv[z].s);
                nv.b = __float_as_uint(rv[z].w);
                nv.c = rv[z].c;
                vp[(h + z) * 64] = nv;
                dcount += (int)(rv[z].w >= 1.0f) - (int)((pos0 >> z) & 1u);
                nrmw++;
            }
        }
        if (__ballot(dcount != 0)) {
            const int total = wave_sum(dcount);
            if (lane_id_here() == 0 && total != 0) atomicAdd(&A.blockCount[blk], (uint32_t)total);
        }
        updated += nupd;
#ifdef BF_APPLY_COUNT_WAVES
        rmw += lane_id_here() == 0 ? nwav : 0u;
#else
        rmw += nrmw;
#endif
    }
    // updated is the wave's total (scalar), rmw per lane; one wave per workgroup: its sums go straight to the
    // workgroup's counter slot (no LDS stage, no barriers)
    {
        const unsigned long long rmwW = wave_sum_u64(rmw);
        if (lane_id_here() == 0) {
            unsigned long long* st = A.stats + (size_t)(blockIdx.x % STAT_SLOTS) * STAT_FIELDS;
            if (updated) {
                atomicAdd(&st[S_VOXELS], (unsigned long long)updated);
                atomicAdd(&st[S_BUPD], (unsigned long long)updated);
            }
            if (rmwW) {
                atomicAdd(&st[S_RMW], rmwW);
                atomicAdd(&st[S_BRMW], rmwW);
            }
            if (halves) atomicAdd(&st[S_BHALF], (unsigned long long)halves);
        }
    }
#ifdef BF_APPLY_DIAG
    __syncthreads();
    flush_stats2(A.stats, 20, diag[0], 21, diag[1]);
    __syncthreads();
    flush_stats2(A.stats, 22, diag[2], 23, diag[3]);
    __syncthreads();
    flush_stats2(A.stats, 24, lane_id_here() == 0 ? diagPairs : 0u, 25, lane_id_here() == 0 ? diagEmpty : 0u);
    __syncthreads();
    flush_stats2(A.stats, 26, diag[4], 27, diag[5]);
#endif
}

__device__ void gc_free_list_serial(const HashArgs& A, unsigned long long* listV, uint32_t* locked);

// One launch for the GC pass: garbageCollectIdentifyKernel (:584-631, via the per-block nonzero-weight
// count) and garbageCollectFreeKernel (:648-668). A victim sitting in its bucket with offset == 0 (the
// classification deleteHashEntryElement, VoxelUtilHashSDF.h:739-826, needs) is freed right away by the
// wave that found it: slot cleared, block pushed onto the heap (appendHeap, :541-546), voxels zeroed by
// the wave. Another victim's classification reads only its own entry, which such a free never touches,
// so the identified sets equal the two-kernel form's. Every other victim touches a collision list and is
// queued for the serial path, which the last workgroup to finish runs (release fence + ticket, acquire on
// the winner: the identify / free / list kernels were three launches).
__global__ __launch_bounds__(256) void k_gc(HashArgs A, unsigned long long* listV, uint32_t* errMirror) {
    const uint32_t nvis = A.ctrl[C_VISIBLE];
    const uint32_t lane = lane_id();
    uint32_t freed = 0;
    for (uint32_t base = blockIdx.x * blockDim.x; base < nvis; base += gridDim.x * blockDim.x) {
        const uint32_t b = base + threadIdx.x;
        bool simple = false;
        int slot = -1;
        uint32_t blk = 0;
        if (b < nvis) {
            const int4 e = A.visible[b];
            blk = (uint32_t)e.w;
            if (A.blockCount[blk] == 0 && A.blockPos[blk].w != 0) {  // (pos.w == 0: already freed by an earlier GC)
                const uint32_t h = hash_bucket(e.x, e.y, e.z, A.numBuckets), hp = h * BF_HASH_BUCKET_SIZE;
                uint32_t off = 0;
                for (int j = 0; j < BF_HASH_BUCKET_SIZE; j++) {
                    int4 a, c;
                    load_entry(A.hash, hp + j, a, c);
                    if (a.x == e.x && a.y == e.y && a.z == e.z && a.w != BF_FREE_ENTRY) { slot = (int)(hp + j); off = (uint32_t)c.x; break; }
                }
                simple = slot >= 0 && off == 0;
                if (!simple) {
                    const uint32_t k = atomicAdd(&A.ctrl[C_GC_LIST], 1u);
                    if (k < GC_LIST_CAP) listV[k] = block_key(e.x, e.y, e.z);
                }
            }
        }
        // the wave frees its simple victims one after another, all lanes zeroing each block's voxels
        for (unsigned long long m = __ballot(simple); m; m &= m - 1) {
            const int src = __ffsll((long long)m) - 1;
            const int vSlot = __shfl(slot, src);
            const uint32_t vBlk = (uint32_t)__shfl((int)blk, src);
            if (lane == 0) {
                int4* e = reinterpret_cast<int4*>(A.hash + vSlot);
                e[0] = make_int4(0, 0, 0, BF_FREE_ENTRY);
                e[1] = make_int4(0, 0, 0, 0);
                const uint32_t addr = atomicAdd(&A.ctrl[C_HEAP], 1u);
                A.heap[addr + 1] = vBlk;
                A.blockPos[vBlk] = make_int4(0, 0, 0, 0);
                A.blockCount[vBlk] = 0;
            }
            int4* vz = reinterpret_cast<int4*>(A.voxels + (size_t)vBlk * BF_VOXELS_PER_BLOCK);
            for (int q = lane; q < BF_VOXELS_PER_BLOCK * 12 / 16; q += 64) vz[q] = make_int4(0, 0, 0, 0);
            freed++;
        }
    }
    if (lane == 0 && freed) atomicAdd(&A.stats[S_GCFREED], (unsigned long long)freed);
    __shared__ bool s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        s_last = atomicAdd(&A.ctrl[C_TICKET_GC], 1u) == gridDim.x - 1;
    }
    __syncthreads();
    __shared__ uint32_t s_locked[64];  // the serial path's locked buckets (in LDS: a private array went to scratch)
    if (s_last && threadIdx.x == 0) {
        __threadfence();
        A.ctrl[C_TICKET_GC] = 0;
        gc_free_list_serial(A, listV, s_locked);
        // the scene's sticky error bits, as of this frame's batch, to the host without a synchronization
        if (errMirror) __hip_atomic_store(errMirror, A.ctrl[C_ERR], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// deleteHashEntryElement collision-list cases, serial in ascending block-key order with the
// reference's per-bucket try-lock semantics (one list delete per bucket per GC pass); one thread, after
// every in-bucket free of the pass
__device__ void gc_free_list_serial(const HashArgs& A, unsigned long long* listV, uint32_t* locked) {
    const uint32_t n = min(A.ctrl[C_GC_LIST], GC_LIST_CAP);
    for (uint32_t a = 1; a < n; a++) {  // insertion sort (n is tiny)
        unsigned long long k = listV[a];
        int b = (int)a - 1;
        while (b >= 0 && listV[b] > k) { listV[b + 1] = listV[b]; b--; }
        listV[b + 1] = k;
    }
    uint32_t nlocked = 0;
    auto try_lock = [&](uint32_t h) -> bool {
        for (uint32_t q = 0; q < nlocked; q++)
            if (locked[q] == h) return false;
        if (nlocked < 64) locked[nlocked++] = h;
        return true;
    };
    uint32_t freed = 0;
    for (uint32_t k = 0; k < n; k++) {
        const i3 b = key_block(listV[k]);
        const uint32_t h = hash_bucket(b.x, b.y, b.z, A.numBuckets), hp = h * BF_HASH_BUCKET_SIZE;
        int delPtr = -1;
        bool handled = false;
        for (uint32_t j = 0; j < BF_HASH_BUCKET_SIZE && !handled; j++) {
            const uint32_t i = hp + j;
            BFHashEntry curr = A.hash[i];
            if (curr.x == b.x && curr.y == b.y && curr.z == b.z && curr.ptr != BF_FREE_ENTRY) {
                handled = true;
                if (curr.offset != 0) {
                    if (!try_lock(h)) break;
                    delPtr = curr.ptr;
                    const uint32_t nextIdx = (i + curr.offset) % A.numEntries;
                    A.hash[i] = A.hash[nextIdx];
                    BFHashEntry& nx = A.hash[nextIdx];
                    nx.x = nx.y = nx.z = 0; nx.offset = 0; nx.ptr = BF_FREE_ENTRY;
                } else {
                    delPtr = curr.ptr;
                    BFHashEntry& c = A.hash[i];
                    c.x = c.y = c.z = 0; c.offset = 0; c.ptr = BF_FREE_ENTRY;
                }
            }
        }
        if (!handled) {
            const uint32_t last = hp + BF_HASH_BUCKET_SIZE - 1;
            uint32_t prevIdx = last;
            uint32_t i = (last + A.hash[last].offset) % A.numEntries;
            for (uint32_t it = 0; it < A.maxList; it++) {
                const BFHashEntry curr = A.hash[i];
                if (curr.x == b.x && curr.y == b.y && curr.z == b.z && curr.ptr != BF_FREE_ENTRY) {
                    if (!try_lock(h)) break;
                    delPtr = curr.ptr;
                    BFHashEntry& c = A.hash[i];
                    c.x = c.y = c.z = 0; c.offset = 0; c.ptr = BF_FREE_ENTRY;
                    A.hash[prevIdx].offset = curr.offset;
                    break;
                }
                if (curr.offset == 0) break;
                prevIdx = i;
                i = (last + curr.offset) % A.numEntries;
            }
        }
        if (delPtr >= 0) {
            const uint32_t blk = (uint32_t)delPtr;
            const uint32_t addr = A.ctrl[C_HEAP]++;
            A.heap[addr + 1] = blk;
            A.blockPos[blk] = make_int4(0, 0, 0, 0);
            A.blockCount[blk] = 0;
            int4* vz = reinterpret_cast<int4*>(A.voxels + (size_t)blk * BF_VOXELS_PER_BLOCK);
            for (int q = 0; q < BF_VOXELS_PER_BLOCK * 12 / 16; q++) vz[q] = make_int4(0, 0, 0, 0);
            freed++;
        }
    }
    A.stats[S_GCFREED] += freed;
    // the pass's last kernel re-arms the victim counters for the next GC (zero after a reset, too),
    // so GC needs no counter-reset launch of its own
    A.stats[S_GCBLOCKS] += A.ctrl[C_VISIBLE];
    A.ctrl[C_GC_LIST] = 0;
}

}  // namespace

// ------------------------------------------------------------------------------------
// RN(1 / x) for the divisors div_by_uniform admits ([2^-20, 2^20]), else 0 (the kernels divide in IEEE)
// (BF_ALLOC_UNIFORM_DIV=0 builds the IEEE-only walk setup, for A/B and for the fallback's parity)
#ifndef BF_ALLOC_UNIFORM_DIV
#define BF_ALLOC_UNIFORM_DIV 1
#endif
static float recip_or_zero(float x) { return (BF_ALLOC_UNIFORM_DIV && x >= 0x1p-20f && x <= 0x1p20f) ? 1.0f / x : 0.0f; }
static void set_camera_recips(HashArgs& a, const BFDepthCameraParams& cam) {
    const float rx = recip_or_zero(cam.fx), ry = recip_or_zero(cam.fy);
    a.rFx = (rx != 0.0f && ry != 0.0f) ? rx : 0.0f;
    a.rFy = (rx != 0.0f && ry != 0.0f) ? ry : 0.0f;
}
static HashArgs make_args(const SceneConfig& cfg, BFHashEntry* hash, uint32_t* heap, BFVoxel* vox, int4* bp, uint32_t* bc,
                          int4* vis, uint32_t* ctrl, unsigned long long* st, const uint32_t* bitMask) {
    HashArgs a;
    a.hash = hash; a.heap = heap; a.voxels = vox; a.blockPos = bp; a.blockCount = bc; a.visible = vis; a.ctrl = ctrl; a.stats = st;
    a.band = nullptr; a.tiles = nullptr; a.tilesW = a.tilesH = 0; a.tiles2 = nullptr; a.tiles2W = 0;
    a.numBuckets = cfg.hp.hashNumBuckets;
    a.numEntries = cfg.hp.hashNumBuckets * BF_HASH_BUCKET_SIZE;
    a.numBlocks = cfg.hp.numSDFBlocks;
    a.maxList = cfg.hp.hashMaxCollisionLinkedListSize;
    a.voxelSize = cfg.hp.virtualVoxelSize;
    a.rVoxelSize = recip_or_zero(cfg.hp.virtualVoxelSize);
    a.rFx = a.rFy = 0.0f;  // per batch: set_camera_recips
    a.truncation = cfg.hp.truncation;
    a.truncScale = cfg.hp.truncScale;
    a.maxIntegrationDistance = cfg.hp.maxIntegrationDistance;
    a.weightMax = (float)cfg.hp.integrationWeightMax;
    a.shardCount = cfg.shardCount;
    a.shardIndex = cfg.shardIndex;
    a.allocForceDirect = cfg.allocForceDirect;
    a.shardChunk = cfg.shardChunk > 0 ? cfg.shardChunk : 1.0f;
    a.bitMask = bitMask;
    a.streamExtents = cfg.hp.streamingVoxelExtents;
    a.streamGridDims = cfg.hp.streamingGridDimensions;
    a.streamMinGridPos = cfg.hp.streamingMinGridPos;
    return a;
}

SceneConfig scene_config(const BFHashParams& hp, const BFSceneOptions* so) {
    SceneConfig c{};
    c.hp = hp;
    if (so) {
        c.candCapacity = so->candidateCapacity;
        c.shardCount = so->shardCount;
        c.shardIndex = so->shardIndex;
        c.shardChunk = so->shardChunk;
        c.applyXcdRun = so->applyXcdRun;
        c.applyRounds = so->applyRounds;
        c.allocForceDirect = (so->testFlags & BF_SCENE_TEST_ALLOC_DIRECT) ? 1u : 0u;
        c.splatRowCap = so->splatRowCap;
        BF_REQUIRE((so->testFlags & ~BF_SCENE_TEST_ALLOC_DIRECT) == 0, BF_ERR_ARG, "unknown BFSceneOptions.testFlags bits");
        BF_REQUIRE(so->applyXcdRun == 0 || ((so->applyXcdRun & (so->applyXcdRun - 1)) == 0 && so->applyXcdRun <= 32768u),
                   BF_ERR_ARG, "BFSceneOptions.applyXcdRun must be a power of two <= 32768");
        BF_REQUIRE(so->applyRounds <= 64, BF_ERR_ARG, "BFSceneOptions.applyRounds > 64");
    }
    return c;
}

Scene::Scene(const SceneConfig& cfg, hipStream_t stream) : cfg_(cfg), stream_(stream) {
    BF_REQUIRE(cfg.hp.hashNumBuckets > 0 && cfg.hp.numSDFBlocks > 0, BF_ERR_ARG, "empty hash/heap");
    // HashEntry.ptr holds the heap block index inside the scene (voxel address = ptr * 512 in 64 bits):
    // the reference's int32 voxel index (ptr = block * 512, VoxelUtilHashSDF.h:60,609) stops at 2^22
    // blocks (25.8 GB of voxels); block indices reach 2^31 - 1, beyond what one GPU's HBM holds
    BF_REQUIRE(cfg.hp.numSDFBlocks < (1u << 31), BF_ERR_CAPACITY, "numSDFBlocks exceeds the int block-index range");
    BF_REQUIRE((uint64_t)cfg.hp.hashNumBuckets * BF_HASH_BUCKET_SIZE < (1ull << 31), BF_ERR_CAPACITY, "hash too large");
    BF_REQUIRE(cfg.hp.virtualVoxelSize > 0, BF_ERR_ARG, "voxel size");
    E_ = cfg.hp.hashNumBuckets * BF_HASH_BUCKET_SIZE;
    B_ = cfg.hp.numSDFBlocks;
    if (cfg_.candCapacity == 0) cfg_.candCapacity = 1u << 21;
    if (cfg_.shardCount == 0) cfg_.shardCount = 1;
    uint32_t setSize = 1;
    while (setSize < 2 * cfg_.candCapacity) setSize <<= 1;
    candSetMask_ = setSize - 1;
    hash_.alloc(E_);
    heap_.alloc(B_);
    voxels_.alloc((size_t)B_ * BF_VOXELS_PER_BLOCK);
    blockPos_.alloc(B_);
    visible_.alloc(B_);
    band_.alloc((size_t)kMaxOps * B_);  // op batches: one bin per op count
    blockMask_.alloc((size_t)kMaxOps * B_ * sizeof(OpMask) / sizeof(uint4) + 1);
    blockBirth_.alloc(B_);
    candOp_.alloc(cfg_.candCapacity);
    ctrl_.alloc(C_COUNT);
    stats_.alloc(STAT_SLOTS * STAT_FIELDS);
    cand_.alloc(cfg_.candCapacity);
    candSet_.alloc(setSize);
    candSlot_.alloc(cfg_.candCapacity);
    ovf_.alloc(OVF_CAP);
    gcList_.alloc(GC_LIST_CAP);
    blockCount_.alloc(B_);
    hipDeviceProp_t prop;
    int dev = 0;
    BF_HIP(hipGetDevice(&dev));
    BF_HIP(hipGetDeviceProperties(&prop, dev));
    numCUs_ = prop.multiProcessorCount;
    renderStats_.alloc((size_t)kRenderStatSlots * kRenderStatFields);  // RenderStat counters (raycast.hip)
    BF_HIP(hipMemsetAsync(renderStats_.p, 0, renderStats_.bytes(), stream_));
    // k_integrate walks its block list with a static grid stride: size the grid to exactly the
    // resident workgroups, so every wave gets the same share in one round (no tail round)
    int occ0 = 0, occ1 = 0, occA = 0;
    BF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, k_integrate<false, 4>, 256, 0));
    BF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, k_integrate<true, 4>, 256, 0));
    // One-wave workgroups: a wave's slot is handed on when that wave ends instead of when the slowest of its
    // workgroup's four ends (the waves of a workgroup draw blocks of different cost, and the workgroup's end-of-
    // pass counter flush waited for all four): k_apply_ops 475-477 -> 466-467 us, 1 484-1 487 -> 1 498-1 499
    // frames/s at the bench workload, config 4's stream and the G = 8 rehearsal unchanged
    // (profiles/r10_apply_tpb_ab.txt).
    BF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occA, k_apply_ops<4, BF_APPLY_ZC, BF_APPLY_WPE, true>, 64, 0));
    // sharded: one 256-thread workgroup's worth of slots per CU stays free for the bundling streams' launches
    const int freeSlots = cfg_.shardCount > 1 ? 4 : 0;
    // The grid is applyRounds (4) rounds of resident workgroups, each wave a 1/applyRounds share of the strided
    // list: the dispatcher hands the later rounds' workgroups to the slots the earlier ones free, so the waves
    // that drew costly blocks no longer set the pass's end (one resident round: 537 us per launch at the
    // bench workload; 2 / 4 / 8 rounds: 495 / 480 / 505 us, profiles/r10_apply_rounds_ab.txt), and other
    // streams' kernels find free slots at every round's end instead of the pass's.
    const unsigned rounds = cfg_.applyRounds ? cfg_.applyRounds : (unsigned)kApplyRounds;
    applyGrid_ = (unsigned)std::max(1, occA - freeSlots) * (unsigned)numCUs_ * rounds;
    // the voxel pass hands out runs of 64 consecutive work-list positions per XCD (k_apply_ops<..., true>): the
    // list is in heap order, so a run's blocks lie together and one XCD's L2 serves their depth / colour lines.
    // FETCH per launch at the driver workload: 1.14 GB with 4-position runs (consecutive waves: the plain grid
    // stride), 1.04 / 0.98 / 0.96 / 0.95 / 0.93 GB with 16 / 64 / 128 / 256 / 1024; time 478 µs up to 64, then
    // 480 / 485 / 516 µs as the coarser runs unbalance the XCDs (profiles/r10_apply_xcd_runs.txt).
    const uint32_t run = cfg_.applyXcdRun ? cfg_.applyXcdRun : 64u;
    applyXcdShift_ = -1;
    for (int sh = 0; sh < 16; sh++)
        if (run == (1u << sh)) applyXcdShift_ = sh;
    // the batch scan: 4 workgroups per CU (its occupancy; 5-6 per CU and 2-3 resident rounds measured no faster)
    compactifyGrid_ = (unsigned)numCUs_ * (unsigned)BF_SCAN_WPC;
    integrateGrid_[0] = (unsigned)std::max(1, occ0) * (unsigned)numCUs_;
    integrateGrid_[1] = (unsigned)std::max(1, occ1) * (unsigned)numCUs_;
    BF_HIP(hipMemsetAsync(candSet_.p, 0xFF, candSet_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(blockBirth_.p, 0, blockBirth_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(stats_.p, 0, stats_.bytes(), stream_));
    float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    std::memcpy(T_.m, I, 64);
    std::memcpy(Tinv_.m, I, 64);
    reset();
}

Scene::~Scene() {
    if (errMirror_) {
        (void)hipStreamSynchronize(stream_);  // k_gc may still write it
        (void)hipHostFree(errMirror_);
    }
}

void Scene::enableErrorMirror() {
    if (errMirror_) return;
    BF_HIP(hipHostMalloc((void**)&errMirror_, sizeof(uint32_t), hipHostMallocCoherent));
    *errMirror_ = 0;
}

BFSceneCapacity Scene::capacity() {
    uint32_t c[C_COUNT];
    BF_HIP(hipMemcpyAsync(c, ctrl_.p, sizeof(c), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    BFSceneCapacity o{};
    o.errorFlags = c[C_ERR];
    o.peakCandidates = c[C_CANDPEAK];
    o.candidateCapacity = cfg_.candCapacity;
    o.heapFree = c[C_HEAP] + 1;
    o.numSDFBlocks = B_;
    o.highWater = c[C_HIGHWATER];
    return o;
}

size_t Scene::deviceBytes() const {
    return hash_.bytes() + heap_.bytes() + voxels_.bytes() + blockPos_.bytes() + visible_.bytes() + band_.bytes() +
           blockMask_.bytes() + blockBirth_.bytes() + candOp_.bytes() +
           tiles_.bytes() + tiles2_.bytes() + ctrl_.bytes() +
           stats_.bytes() + cand_.bytes() + candSet_.bytes() + candSlot_.bytes() + ovf_.bytes() +
           gcList_.bytes() + blockCount_.bytes();
}

// CUDASceneRepHashSDF::reset (.h:147-155) -> resetCUDA (.cu:67-111)
void Scene::reset() {
    const unsigned grid = (unsigned)numCUs_ * 8;
    k_reset_hash<<<grid, 256, 0, stream_>>>(hash_.p, E_);
    BF_LAUNCH_CHECK();
    k_reset_heap<<<grid, 256, 0, stream_>>>(heap_.p, blockPos_.p, blockCount_.p, B_, ctrl_.p);
    BF_LAUNCH_CHECK();
    BF_HIP(hipMemsetAsync(voxels_.p, 0, voxels_.bytes(), stream_));
    cfg_.hp.numOccupiedBlocks = 0;
}

void Scene::ensureTiles(size_t fine, size_t coarse) {
    if (fine > tilesCap_) {
        tiles_.alloc(fine);
        tilesCap_ = fine;
    }
    if (coarse > tiles2Cap_) {
        tiles2_.alloc(coarse);
        tiles2Cap_ = coarse;
    }
}

void Scene::beginOp() {
    k_begin_op<<<1, 64, 0, stream_>>>(ctrl_.p, stats_.p);
    BF_LAUNCH_CHECK();
}

void Scene::alloc(const float* depth, const BFDepthCameraParams& cam, const uint32_t* bitMask) {
    HashArgs A = make_args(cfg_, hash_.p, heap_.p, voxels_.p, blockPos_.p, blockCount_.p, visible_.p, ctrl_.p, stats_.p, bitMask);
    set_camera_recips(A, cam);
    dim3 g(div_up(cam.imageWidth, ALLOC_TILE), div_up(cam.imageHeight, ALLOC_TILE));
    k_alloc_collect<<<g, 256, 0, stream_>>>(A, depth, cam, T_, Tinv_, cand_.p, cfg_.candCapacity);
    hostPixels_ += (uint64_t)cam.imageWidth * cam.imageHeight;
    BF_LAUNCH_CHECK();
    // few candidates per op in steady state: a small grid keeps the last-workgroup ticket cheap
    const unsigned grid = 64;
    k_alloc_insert<<<grid, 256, 0, stream_>>>(A, cand_.p, cfg_.candCapacity, candSet_.p, candSetMask_, candSlot_.p, ovf_.p);
    BF_LAUNCH_CHECK();
    // k_alloc_insert's last workgroup runs the serial collision-list inserts; the dedup-set
    // cleanup runs inside the following k_compactify
}

void Scene::compactify(const BFMat4& T, const BFDepthCameraParams& cam) {
    T_ = T;
    Tinv_ = mat4_inverse(T);
    beginOp();
    HashArgs A = make_args(cfg_, hash_.p, heap_.p, voxels_.p, blockPos_.p, blockCount_.p, visible_.p, ctrl_.p, stats_.p, nullptr);
    k_compactify<CM_FRUSTUM><<<(unsigned)numCUs_ * 4, 256, 0, stream_>>>(A, cam, Tinv_, 0u, nullptr, nullptr);
    BF_LAUNCH_CHECK();
}

// CUDASceneRepHashSDF::integrate (.h:65-83) / deIntegrate (.h:85-108)
void Scene::integrate(const BFMat4& T, const float* depth, const uint8_t* color, const BFDepthCameraParams& cam, bool deint,
                      const uint32_t* bitMask) {
    BF_REQUIRE(depth != nullptr, BF_ERR_ARG, "depth is null");
    T_ = T;
    Tinv_ = mat4_inverse(T);
    const uint32_t tw = div_up(cam.imageWidth, DEPTH_TILE), th = div_up(cam.imageHeight, DEPTH_TILE);
    const uint32_t tw2 = div_up(cam.imageWidth, DEPTH_TILE2), th2 = div_up(cam.imageHeight, DEPTH_TILE2);
    ensureTiles(tw * th, tw2 * th2);
    k_begin_op_tiles<<<div_up((size_t)(tw * th + tw2 * th2) * 64, 256), 256, 0, stream_>>>(
        ctrl_.p, stats_.p, depth, cam.imageWidth, cam.imageHeight, tw, th, tw2, th2, cfg_.hp.maxIntegrationDistance, tiles_.p,
        tiles2_.p, 1u);
    BF_LAUNCH_CHECK();
    if (!deint) alloc(depth, cam, bitMask);
    HashArgs A = make_args(cfg_, hash_.p, heap_.p, voxels_.p, blockPos_.p, blockCount_.p, visible_.p, ctrl_.p, stats_.p, bitMask);
    A.band = band_.p;
    A.tiles = tiles_.p;
    A.tilesW = tw;
    A.tilesH = th;
    A.tiles2 = tiles2_.p;
    A.tiles2W = tw2;
    const unsigned grid = (unsigned)numCUs_ * 4;
    k_compactify<CM_INTEGRATE><<<grid, 256, 0, stream_>>>(A, cam, Tinv_, cfg_.candCapacity, candSlot_.p, candSet_.p);
    BF_LAUNCH_CHECK();
    const unsigned igrid = deint ? integrateGrid_[1] : integrateGrid_[0];
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    const bool timed = integrateClock_.enabled();
    if (timed) integrateClock_.slot(ev0, ev1);
    const uint32_t* col = reinterpret_cast<const uint32_t*>(color);
    if (deint)
        hipExtLaunchKernelGGL(k_integrate<true, 4>, dim3(igrid), dim3(256), 0, stream_, ev0, ev1, 0, A, depth, col, cam, Tinv_);
    else
        hipExtLaunchKernelGGL(k_integrate<false, 4>, dim3(igrid), dim3(256), 0, stream_, ev0, ev1, 0, A, depth, col, cam, Tinv_);
    BF_LAUNCH_CHECK();
    if (timed) integrateClock_.commit();
}

// reintegrate() fix of one frame (DepthSensing.cpp:890-895): deIntegrate(Told) + integrate(Tnew) as a
// two-op batch (one alloc, one compactify scan, one voxel pass; same voxels as the two calls)
void Scene::reintegrate(const BFMat4& Told, const BFMat4& Tnew, const float* depth, const uint8_t* color,
                        const BFDepthCameraParams& cam) {
    BF_REQUIRE(depth != nullptr, BF_ERR_ARG, "depth is null");
    VoxelOp ops[2];
    ops[0] = VoxelOp{Told, depth, color, true};
    ops[1] = VoxelOp{Tnew, depth, color, false};
    applyOps(ops, 2, cam);
}

// reintegrate() (DepthSensing.cpp:854-902) fixes of one frame as one pass: see tsdf.h
void Scene::applyOps(const VoxelOp* ops, uint32_t n, const BFDepthCameraParams& cam) {
    if (n == 0) return;
    BF_REQUIRE(n <= kMaxOps, BF_ERR_ARG, "too many ops in one batch");
    OpTable tab;
    std::memset(&tab, 0, sizeof(tab));
    tab.n = n;
    for (uint32_t k = 0; k < n; k++) {
        BF_REQUIRE(ops[k].depth != nullptr, BF_ERR_ARG, "depth is null");
        const BFMat4 Ti = mat4_inverse(ops[k].T);
        std::memcpy(tab.tinv[k], Ti.m, 48);
        std::memcpy(tab.t[k], ops[k].T.m, 48);
        tab.depth[k] = ops[k].depth;
        tab.color[k] = reinterpret_cast<const uint32_t*>(ops[k].color);
        if (ops[k].deint) tab.deintMask |= 1u << k;
        else tab.intIdx[tab.nInt++] = (uint8_t)k;
    }
    const uint32_t tw = div_up(cam.imageWidth, DEPTH_TILE), th = div_up(cam.imageHeight, DEPTH_TILE);
    const uint32_t tw2 = div_up(cam.imageWidth, DEPTH_TILE2), th2 = div_up(cam.imageHeight, DEPTH_TILE2);
    ensureTiles(tw * th * kMaxOps, tw2 * th2 * kMaxOps);
    const size_t P = (size_t)cam.imageWidth * cam.imageHeight;
    bool needScratch = false;
    for (uint32_t k = 0; k < n; k++) needScratch |= ops[k].tiles == nullptr;
    if (needScratch && dcCap_ < P * kMaxOps) {
        dc_.alloc(P * kMaxOps);
        dcCap_ = P * kMaxOps;
    }
    for (uint32_t k = 0; k < n; k++) {
        BF_REQUIRE(ops[k].tiles == nullptr || ops[k].dc != nullptr, BF_ERR_ARG, "a tile cache needs its dc image");
        if (ops[k].tiles) {  // the caller's per-depth-map tile cache (fine level, then the coarse level)
            tab.tiles[k] = ops[k].tiles;
            tab.tiles2[k] = ops[k].tiles + (size_t)tw * th;
            tab.dc[k] = ops[k].dc;
            if (!ops[k].tilesReady) tab.tileMask |= 1u << k;
        } else {
            tab.tiles[k] = tiles_.p + (size_t)k * tw * th;
            tab.tiles2[k] = tiles2_.p + (size_t)k * tw2 * th2;
            tab.dc[k] = dc_.p + (size_t)k * P;
            tab.tileMask |= 1u << k;
        }
    }
    const uint32_t tileBlocks = (uint32_t)div_up((size_t)(tw * th + tw2 * th2) * 64, 256);
    const uint32_t packBlocks = (uint32_t)std::min<size_t>(div_up(P, 256), 1024);
    for (uint32_t k = 0; k < n; k++)
        if ((tab.tileMask >> k) & 1u) tab.tileIdx[tab.nTile++] = (uint8_t)k;
    // grid.y = the ops whose caches are built here (not every op of the batch: most are cached)
    const dim3 tileGrid = tab.nTile ? dim3(tileBlocks + packBlocks, tab.nTile) : dim3(1, 1);
    k_begin_ops_tiles<<<tileGrid, 256, 0, stream_>>>(
        ctrl_.p, stats_.p, tab, cam.imageWidth, cam.imageHeight, tw, th, tw2, th2, cfg_.hp.maxIntegrationDistance, tileBlocks);
    BF_LAUNCH_CHECK();
    HashArgs A = make_args(cfg_, hash_.p, heap_.p, voxels_.p, blockPos_.p, blockCount_.p, visible_.p, ctrl_.p, stats_.p, nullptr);
    set_camera_recips(A, cam);
    if (++batchEpoch_ >= (1u << 24)) {  // birth stamps are epoch << 8: restart the epochs before they wrap
        BF_HIP(hipMemsetAsync(blockBirth_.p, 0, blockBirth_.bytes(), stream_));
        batchEpoch_ = 1;
    }
    const uint32_t epoch = batchEpoch_;
    if (tab.nInt) {
        dim3 g(div_up(cam.imageWidth, ALLOC_TILE), div_up(cam.imageHeight, ALLOC_TILE), tab.nInt);
        k_alloc_collect_ops<<<g, 256, 0, stream_>>>(A, cam, tab, cand_.p, cfg_.candCapacity, candOp_.p);
        hostPixels_ += (uint64_t)cam.imageWidth * cam.imageHeight * tab.nInt;
        BF_LAUNCH_CHECK();
        k_alloc_insert<<<64, 256, 0, stream_>>>(A, cand_.p, cfg_.candCapacity, candSet_.p, candSetMask_, candSlot_.p, ovf_.p);
        BF_LAUNCH_CHECK();
        k_alloc_birth<<<(unsigned)numCUs_, 256, 0, stream_>>>(A, cand_.p, candOp_.p, cfg_.candCapacity, blockBirth_.p, epoch);
        BF_LAUNCH_CHECK();
    }
    A.band = band_.p;
    A.tiles = tiles_.p;
    A.tilesW = tw;
    A.tilesH = th;
    A.tiles2 = tiles2_.p;
    A.tiles2W = tw2;
    k_compactify_ops<<<compactifyGrid_, 256, 0, stream_>>>(A, cam, tab, cfg_.candCapacity, candSlot_.p, candSet_.p,
                                                                  reinterpret_cast<OpMask*>(blockMask_.p), blockBirth_.p, epoch, B_);
    BF_LAUNCH_CHECK();
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    const bool timed = applyClock_.enabled() && applyClock_.slotSampled(ev0, ev1);
    if (applyGrid_ % 8u == 0u)  // workgroup i runs on XCD i mod 8
        hipExtLaunchKernelGGL(k_apply_ops<4, BF_APPLY_ZC, BF_APPLY_WPE, true>, dim3(applyGrid_), dim3(64), 0, stream_, ev0, ev1, 0, A,
                              cam, tab, reinterpret_cast<const OpMask*>(blockMask_.p), static_cast<const int4*>(band_.p), B_,
                              applyXcdShift_);
    else
        hipExtLaunchKernelGGL(k_apply_ops<4, BF_APPLY_ZC, BF_APPLY_WPE, false>, dim3(applyGrid_), dim3(64), 0, stream_, ev0, ev1, 0, A,
                              cam, tab, reinterpret_cast<const OpMask*>(blockMask_.p), static_cast<const int4*>(band_.p), B_, -1);
    BF_LAUNCH_CHECK();
    if (timed) applyClock_.commit();
    T_ = ops[n - 1].T;
    Tinv_ = mat4_inverse(T_);
}

// CUDASceneRepHashSDF::garbageCollect (.h:110-126)
void Scene::garbageCollect() {
    HashArgs A = make_args(cfg_, hash_.p, heap_.p, voxels_.p, blockPos_.p, blockCount_.p, visible_.p, ctrl_.p, stats_.p, nullptr);
    // half a workgroup per CU: every workgroup ends with a fence and a same-address ticket atomic, whose
    // serialisation made 2 per CU cost 21 us a pass against 13.6 at one per two CUs (15.2 at 1, 14.4 at 1/4;
    // profiles/r11_gc_ab.txt); the visible-list walk itself is ~6.5 us
    const unsigned gcGrid = std::max(1u, (unsigned)numCUs_ / 2u);
    k_gc<<<gcGrid, 256, 0, stream_>>>(A, gcList_.p, errMirror_);
    BF_LAUNCH_CHECK();
}

size_t Scene::dcCount(const BFDepthCameraParams& cam) { return (size_t)cam.imageWidth * cam.imageHeight; }

size_t Scene::tileCount(const BFDepthCameraParams& cam) {
    return (size_t)div_up(cam.imageWidth, DEPTH_TILE) * div_up(cam.imageHeight, DEPTH_TILE) +
           (size_t)div_up(cam.imageWidth, DEPTH_TILE2) * div_up(cam.imageHeight, DEPTH_TILE2);
}

uint32_t Scene::heapFreeCount() {
    uint32_t c = 0;
    BF_HIP(hipMemcpyAsync(&c, ctrl_.p + C_HEAP, 4, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    return c + 1;  // .h:168-172
}

uint32_t Scene::numVisible() {
    uint32_t c = 0;
    BF_HIP(hipMemcpyAsync(&c, ctrl_.p + C_VISIBLE, 4, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    return c;
}

uint32_t Scene::errorFlags() {
    uint32_t c = 0;
    BF_HIP(hipMemcpyAsync(&c, ctrl_.p + C_ERR, 4, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    return c;
}

BFTsdfStats Scene::stats() {
    std::vector<unsigned long long> h(STAT_SLOTS * STAT_FIELDS);
    BF_HIP(hipMemcpyAsync(h.data(), stats_.p, stats_.bytes(), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    uint64_t sum[STAT_FIELDS] = {0};
    for (int sl = 0; sl < STAT_SLOTS; sl++)
        for (int f = 0; f < STAT_FIELDS; f++) sum[f] += h[sl * STAT_FIELDS + f];
    BFTsdfStats s;
    static_assert(sizeof(BFTsdfStats) == 18 * 8 && sizeof(BFTsdfStats) <= STAT_FIELDS * 8, "stats layout");
    std::memcpy(&s, sum, sizeof(s));
    s.pixels += hostPixels_;
#ifdef BF_APPLY_DIAG
    fprintf(stderr, "apply diag: offscreen %llu invalid %llu front %llu behind %llu (half,op) pairs %llu empty %llu (slice pair,op) %llu empty %llu\n",
            (unsigned long long)sum[20], (unsigned long long)sum[21], (unsigned long long)sum[22], (unsigned long long)sum[23],
            (unsigned long long)sum[24], (unsigned long long)sum[25], (unsigned long long)sum[27], (unsigned long long)sum[26]);
#endif
    return s;
}

void Scene::resetStats() {
    BF_HIP(hipMemsetAsync(stats_.p, 0, stats_.bytes(), stream_));
    hostPixels_ = 0;
}

// Dumps use the reference's units: ptr = heap block * 512 (the voxel index of the block's first
// voxel), which an int32 holds up to 2^22 blocks; larger scenes dump blocks and voxels by heap block
// (exportBlocks, exportBlockVoxels).
static inline int32_t ref_ptr(int32_t blk) { return blk >= 0 ? blk * BF_VOXELS_PER_BLOCK : blk; }

void Scene::exportState(BFHashEntry* hash, uint32_t* heap, uint32_t* heapCounter, BFVoxel* voxels) {
    BF_REQUIRE(hash == nullptr || (uint64_t)B_ <= (1ull << 22), BF_ERR_CAPACITY,
               "hash dump in the reference's voxel-index ptr needs numSDFBlocks <= 2^22 (use bf_scene_export_blocks)");
    if (hash) BF_HIP(hipMemcpyAsync(hash, hash_.p, hash_.bytes(), hipMemcpyDeviceToHost, stream_));
    if (heap) BF_HIP(hipMemcpyAsync(heap, heap_.p, heap_.bytes(), hipMemcpyDeviceToHost, stream_));
    if (heapCounter) BF_HIP(hipMemcpyAsync(heapCounter, ctrl_.p + C_HEAP, 4, hipMemcpyDeviceToHost, stream_));
    if (voxels) BF_HIP(hipMemcpyAsync(voxels, voxels_.p, voxels_.bytes(), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    if (hash)
        for (uint32_t i = 0; i < E_; i++) hash[i].ptr = ref_ptr(hash[i].ptr);
}

uint32_t Scene::exportBlocks(int4* out, uint32_t cap) {
    uint32_t hw = 0;
    BF_HIP(hipMemcpyAsync(&hw, ctrl_.p + C_HIGHWATER, 4, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    const uint32_t n = std::min(hw, cap);
    if (n && out) BF_HIP(hipMemcpyAsync(out, blockPos_.p, n * sizeof(int4), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    return hw;
}

uint32_t Scene::exportVisible(int4* out, uint32_t cap) {
    BF_REQUIRE((uint64_t)B_ <= (1ull << 22), BF_ERR_CAPACITY, "visible dump in voxel-index ptr needs numSDFBlocks <= 2^22");
    uint32_t n = numVisible();
    n = std::min(n, cap);
    if (n) BF_HIP(hipMemcpyAsync(out, visible_.p, n * sizeof(int4), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    for (uint32_t i = 0; i < n; i++) out[i].w = ref_ptr(out[i].w);
    return n;
}

void Scene::exportBlockVoxels(uint32_t first, uint32_t count, BFVoxel* out) {
    BF_REQUIRE((uint64_t)first + count <= B_, BF_ERR_ARG, "heap block range out of bounds");
    if (count)
        BF_HIP(hipMemcpyAsync(out, voxels_.p + (size_t)first * BF_VOXELS_PER_BLOCK, (size_t)count * BF_VOXELS_PER_BLOCK * sizeof(BFVoxel),
                              hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
}

}  // namespace bf
