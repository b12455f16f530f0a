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
#include <cstdio>
#include <vector>

namespace bf {

BFMat4 mat4_inverse(const BFMat4& M);  // api.cpp

namespace {

const float MINF_F = -__builtin_inff();
enum RenderStat { RS_SAMPLES = 0, RS_LOADS, RS_PROBES, RS_RAYS, RS_QUADS, RS_ATOMICS, RS_RENDERS, RS_PIXELS, RS_WAVESAMPLES, RS_WAVEMAX, RS_LONGWAVES, RS_COUNT };

static_assert(RS_COUNT <= Scene::kRenderStatFields, "render counters per slot");
// Counter updates: one workgroup's counters are summed in LDS and added to one of kRenderStatSlots slots
// (workgroup index mod slots; renderStats sums them). Device-scope atomics on one address serialise: with
// every wave of k_render adding its 7 counters to the same 7 words (34 k atomics per render) the waves
// drained through that queue one after another, and the kernel took 320 us for a march whose fastest waves
// end in 23 us (BF_RENDER_WAVE_LOG, gpurun_out/s36)
__device__ __forceinline__ unsigned long long* rs_slot(unsigned long long* stats) {
    return stats + (size_t)((blockIdx.y * gridDim.x + blockIdx.x) % (uint32_t)Scene::kRenderStatSlots) * Scene::kRenderStatFields;
}

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
    unsigned long long* waveLog;  // diagnostics (BF_RENDER_WAVE_LOG): per wave {start, end, __smid, longest march}
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

// rayIntervalSplatKernel (CUDARayCastSDF.cu:101-190) for both passes + the raster of its quads, binned by screen
// tile, without global atomics: k_splat_quads writes each visible block's covered pixel rectangle and encoded
// depths (one thread per block: the 8 corners projected with cameraToDepthProj, min / max NDC depth rectangles);
// k_splat_tiles gives each workgroup a 64x8 pixel tile that scans its tile row's rectangles, keeps the ones
// overlapping its tile in LDS, and folds them into per-pixel min / max held in registers, then writes each pixel
// once. The first form issued one atomic min and max per covered pixel (8.9 M per render on the bench scene, ~30
// per pixel, all to HBM: 145 us for the splat against 56 us now); here the traffic is the row's rectangle list
// read once per tile (from L2) and one store per pixel, and no clear pass is needed. A pass a block does not take carries the clear value
// (enc(+inf) for min, enc(-inf) for max), which leaves the pixel unchanged, so the result is the same
// order-independent min / max as the atomics'
// 64x8 tiles (2 rows per wave), 8 rectangles per thread per chunk (32 KB of LDS list): 600 workgroups for
// 640x480, two to three per CU. The fold is issue-bound (~40 instructions per rectangle and wave, 140 ns
// each with one wave per SIMD: BF_SPLAT_TILE_LOG), so it wants several waves per SIMD and few rows per wave;
// 64x20 tiles (one workgroup per CU, 5 rows per wave) took 58 us, 64x8 37 us, 64x4 (1 200 workgroups) 38 us
constexpr int ST_W = 64, ST_H = 8, ST_PX = ST_W * ST_H / 256, ST_Q = 8;  // tile, pixels per thread, rectangles per thread per chunk
// Tile rows: each rectangle is also listed under every ST_H-pixel tile row it spans (count in k_splat_quads,
// exclusive scan in k_splat_rows, fill in k_splat_fill), so a tile scans its own row's rectangles instead of
// all of them. Renders taller than ST_ROWS tile rows, or whose row lists would exceed their capacity
// (4 entries per visible block), scan every rectangle.
constexpr int ST_ROWS = 256;
enum SplatBin { SB_COUNT = 0, SB_START = ST_ROWS, SB_LEN = 2 * ST_ROWS, SB_CURSOR = 3 * ST_ROWS, SB_TOTAL = 4 * ST_ROWS,
                SB_OVERFLOW, SB_WORDS };
__device__ __forceinline__ bool quad_rows(const int4 q, int& r0, int& r1) {  // the tile rows a rectangle spans
    const int x0 = q.x & 0xFFFF, x1 = q.y & 0xFFFF;
    r0 = (q.x >> 16) / ST_H;
    r1 = (q.y >> 16) / ST_H;
    return x0 <= x1;
}
__global__ __launch_bounds__(256) void k_splat_quads(const int4* __restrict__ visible, const uint32_t* ctrl, float voxelSize,
                                                     BFDepthCameraParams cam, BFRayCastParams rp, int4* quads,
                                                     unsigned long long* stats, uint32_t* bin) {
    const uint32_t n = ctrl[C_VISIBLE];
    uint32_t nq = 0, npix = 0;
    __shared__ uint32_t s_row[ST_ROWS];
    if (threadIdx.x < ST_ROWS) s_row[threadIdx.x] = 0;
    __syncthreads();
    const BFMat4 V = rp.viewMatrix;
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < n; b += gridDim.x * blockDim.x) {
        int4 out = make_int4(0xFFFF, 0, 0, 0);  // an empty rectangle (x0 > x1)
        const int4 e = visible[b];
        if (block_in_frustum(cam, V, e.x, e.y, e.z, voxelSize)) {
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
            const float dwMin = mn.z * (rp.maxDepth - rp.minDepth) + rp.minDepth;
            const float dwMax = mx.z * (rp.maxDepth - rp.minDepth) + rp.minDepth;
            const bool minOk = mn.z < 1.0f, maxOk = mx.z > 0.0f;
            const float W = (float)rp.width, H = (float)rp.height;
            const float left = (mn.x + 1.0f) * 0.5f * W, right = (mx.x + 1.0f) * 0.5f * W;
            const float top = (1.0f - mx.y) * 0.5f * H, bottom = (1.0f - mn.y) * 0.5f * H;
            if ((minOk || maxOk) && left < right && top < bottom) {
                const float fx0 = ceilf(left - 0.5f), fx1 = ceilf(right - 0.5f) - 1.0f;
                const float fy0 = ceilf(top - 0.5f), fy1 = ceilf(bottom - 0.5f) - 1.0f;
                if (!(fx1 < 0.0f || fy1 < 0.0f || fx0 > W - 1.0f || fy0 > H - 1.0f)) {
                    const int x0 = (int)fmaxf(fx0, 0.0f), x1 = (int)fminf(fx1, W - 1.0f);
                    const int y0 = (int)fmaxf(fy0, 0.0f), y1 = (int)fminf(fy1, H - 1.0f);
                    if (x1 >= x0 && y1 >= y0) {
                        out = make_int4(x0 | (y0 << 16), x1 | (y1 << 16), (int)(minOk ? enc_f(dwMin) : enc_f(__builtin_inff())),
                                        (int)(maxOk ? enc_f(dwMax) : enc_f(-__builtin_inff())));
                        nq++;
                        npix += (uint32_t)(x1 - x0 + 1) * (uint32_t)(y1 - y0 + 1) * ((minOk ? 1u : 0u) + (maxOk ? 1u : 0u));
                    }
                }
            }
        }
        quads[b] = out;
        int r0, r1;
        if (bin && quad_rows(out, r0, r1))
            for (int r = r0; r <= r1; r++) atomicAdd(&s_row[r], 1u);
    }
    __shared__ unsigned long long s_st[2];
    if (threadIdx.x < 2) s_st[threadIdx.x] = 0;
    __syncthreads();
    if (bin && threadIdx.x < ST_ROWS && s_row[threadIdx.x]) atomicAdd(&bin[SB_COUNT + threadIdx.x], s_row[threadIdx.x]);
    nq = wave_sum_u32(nq);
    npix = wave_sum_u32(npix);
    if ((threadIdx.x & 63) == 0 && nq) {
        atomicAdd(&s_st[0], (unsigned long long)nq);
        atomicAdd(&s_st[1], (unsigned long long)npix);
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_st[0]) {
        atomicAdd(&rs_slot(stats)[RS_QUADS], s_st[0]);
        atomicAdd(&rs_slot(stats)[RS_ATOMICS], s_st[1]);
    }
}

// exclusive scan of the row counts (then zeroed for the next render), capacity check
__global__ __launch_bounds__(ST_ROWS) void k_splat_rows(uint32_t* bin, uint32_t cap) {
    __shared__ uint32_t s[ST_ROWS];
    const uint32_t r = threadIdx.x, c = bin[SB_COUNT + r];
    s[r] = c;
    __syncthreads();
    for (uint32_t o = 1; o < (uint32_t)ST_ROWS; o <<= 1) {
        const uint32_t v = r >= o ? s[r - o] : 0u;
        __syncthreads();
        s[r] += v;
        __syncthreads();
    }
    const uint32_t incl = s[r];
    bin[SB_START + r] = incl - c;
    bin[SB_CURSOR + r] = incl - c;
    bin[SB_LEN + r] = c;
    bin[SB_COUNT + r] = 0;
    if (r == ST_ROWS - 1) {
        bin[SB_TOTAL] = incl;
        bin[SB_OVERFLOW] = incl > cap ? 1u : 0u;
    }
}
// the row lists: a workgroup counts its rectangles per row, takes each row's range with one atomic, and hands
// the slots out in LDS (same grid as k_splat_quads, so the same rectangles per workgroup)
__global__ __launch_bounds__(256) void k_splat_fill(const int4* __restrict__ quads, const uint32_t* ctrl, uint32_t* bin,
                                                    uint32_t* rowIdx, uint32_t cap) {
    const uint32_t n = ctrl[C_VISIBLE];
    __shared__ uint32_t s_row[ST_ROWS];
    if (threadIdx.x < ST_ROWS) s_row[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < n; b += gridDim.x * blockDim.x) {
        int r0, r1;
        if (quad_rows(quads[b], r0, r1))
            for (int r = r0; r <= r1; r++) atomicAdd(&s_row[r], 1u);
    }
    __syncthreads();
    if (threadIdx.x < ST_ROWS && s_row[threadIdx.x]) s_row[threadIdx.x] = atomicAdd(&bin[SB_CURSOR + threadIdx.x], s_row[threadIdx.x]);
    __syncthreads();
    if (bin[SB_OVERFLOW]) return;  // the tiles scan every rectangle
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < n; b += gridDim.x * blockDim.x) {
        int r0, r1;
        if (quad_rows(quads[b], r0, r1))
            for (int r = r0; r <= r1; r++) {
                const uint32_t slot = atomicAdd(&s_row[r], 1u);
                if (slot < cap) rowIdx[slot] = b;
            }
    }
}

__global__ __launch_bounds__(256) void k_splat_tiles(const int4* __restrict__ quads, const uint32_t* ctrl, uint32_t W, uint32_t H,
                                                     uint32_t* smin, uint32_t* smax, const uint32_t* __restrict__ bin,
                                                     const uint32_t* __restrict__ rowIdx, unsigned long long* tileLog) {
    const long long tStart = tileLog ? wall_clock64() : 0;
    uint32_t folded = 0;  // diagnostics (BF_SPLAT_TILE_LOG): rectangles folded by this tile
    // binned: this tile row's rectangles (indices into quads), else every rectangle
    const bool binned = bin && bin[SB_OVERFLOW] == 0u;
    const uint32_t n = binned ? bin[SB_LEN + blockIdx.y] : ctrl[C_VISIBLE];
    const uint32_t* idxs = binned ? rowIdx + bin[SB_START + blockIdx.y] : nullptr;
    const int tx0 = (int)blockIdx.x * ST_W, ty0 = (int)blockIdx.y * ST_H;
    const int tx1 = min(tx0 + ST_W, (int)W) - 1, ty1 = min(ty0 + ST_H, (int)H) - 1;
    // a wave owns ST_PX consecutive rows of the tile (rows py0 .. py0 + ST_PX - 1, lane = column): a rectangle's
    // row range is wave-uniform, so a wave skips the rectangles outside its rows with one uniform test and
    // tests only the column per lane (interleaved rows made every wave fold every rectangle of the tile)
    const int px = tx0 + (int)(threadIdx.x & 63);
    const int py0 = __builtin_amdgcn_readfirstlane(ty0 + ST_PX * (int)(threadIdx.x >> 6));  // scalar: row tests are SALU
    uint32_t mn[ST_PX], mx[ST_PX];
#pragma unroll
    for (int i = 0; i < ST_PX; i++) { mn[i] = enc_f(__builtin_inff()); mx[i] = enc_f(-__builtin_inff()); }
    __shared__ int4 s_list[256 * ST_Q];
    __shared__ uint32_t s_cnt;
    // the next chunk's rectangles are loaded while this chunk's are folded (the scan is L2-latency bound otherwise)
    // (a load from a clamped index, then a select: `idx < n ? quads[idx] : EMPTY` became a select between a global
    // and a private address, i.e. flat loads and a scratch copy of EMPTY)
    int4 q[ST_Q];
    const uint32_t last = n ? n - 1u : 0u;
    auto fetch = [&](uint32_t idx) {
        const uint32_t i = min(idx, last);
        const int4 v = quads[binned ? (n ? idxs[i] : 0u) : i];
        return idx < n ? v : make_int4(0xFFFF, 0, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < ST_Q; i++) q[i] = fetch((uint32_t)i * 256u + threadIdx.x);
    // the barriers order LDS only: __syncthreads() also waits for every outstanding global load, which made each
    // chunk wait for the next chunk's prefetch (one L2 round trip per chunk: 133 us per render)
    auto lds_barrier = [] {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    };
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t base = 0; base < n; base += 256u * ST_Q) {
        if (threadIdx.x == 0) s_cnt = 0;
        lds_barrier();
#pragma unroll
        for (int i = 0; i < ST_Q; i++) {
            const int x0 = q[i].x & 0xFFFF, y0 = q[i].x >> 16, x1 = q[i].y & 0xFFFF, y1 = q[i].y >> 16;
            const bool hit = x0 <= tx1 && x1 >= tx0 && y0 <= ty1 && y1 >= ty0;
            const unsigned long long m = __ballot(hit);  // one LDS atomic per wave and rectangle slot that has hits
            if (m) {
                const uint32_t first = (uint32_t)__builtin_ctzll(m);
                uint32_t at = 0;
                if (lane == first) at = atomicAdd(&s_cnt, (uint32_t)__builtin_popcountll(m));
                at = (uint32_t)__shfl((int)at, (int)first);
                if (hit) s_list[at + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull))] = q[i];
            }
        }
        const uint32_t next = base + 256u * ST_Q;
#pragma unroll
        for (int i = 0; i < ST_Q; i++) q[i] = fetch(next + (uint32_t)i * 256u + threadIdx.x);
        lds_barrier();
        const uint32_t c = s_cnt;
        folded += c;
        auto fold = [&](const int4 r) {
            const int y0 = __builtin_amdgcn_readfirstlane(r.x >> 16), y1 = __builtin_amdgcn_readfirstlane(r.y >> 16);
            if (y1 < py0 || y0 > py0 + ST_PX - 1) return;  // wave-uniform
            const int x0 = r.x & 0xFFFF, x1 = r.y & 0xFFFF;
            const bool inx = px >= x0 && px <= x1;
            // branch-free: a pixel outside the rectangle takes a value that leaves it unchanged (a branch per row
            // cost ~8 exec-mask instructions: 137 ns per folded rectangle, BF_SPLAT_TILE_LOG)
            const uint32_t zmin = inx ? (uint32_t)r.z : 0xFFFFFFFFu, zmax = inx ? (uint32_t)r.w : 0u;
#pragma unroll
            for (int i = 0; i < ST_PX; i++) {
                if (py0 + i >= y0 && py0 + i <= y1) {  // wave-uniform (scalar branch)
                    mn[i] = min(mn[i], zmin);
                    mx[i] = max(mx[i], zmax);
                }
            }
        };
        uint32_t e = 0;
        for (; e + 4u <= c; e += 4u) {  // four list reads in flight per wait
            const int4 r0 = s_list[e], r1 = s_list[e + 1], r2 = s_list[e + 2], r3 = s_list[e + 3];
            fold(r0); fold(r1); fold(r2); fold(r3);
        }
        for (; e < c; e++) fold(s_list[e]);
        lds_barrier();  // every wave has read s_cnt and the list before the next chunk resets them
    }
    if (tileLog && threadIdx.x == 0) {
        unsigned long long* w = tileLog + 4ull * (blockIdx.y * gridDim.x + blockIdx.x);
        w[0] = (unsigned long long)tStart;
        w[1] = (unsigned long long)wall_clock64();
        w[2] = __smid();
        w[3] = folded | ((unsigned long long)n << 32);
    }
    if (px >= (int)W) return;
#pragma unroll
    for (int i = 0; i < ST_PX; i++) {
        const int py = py0 + i;
        if (py < (int)H) {
            smin[(uint32_t)py * W + (uint32_t)px] = mn[i];
            smax[(uint32_t)py * W + (uint32_t)px] = mx[i];
        }
    }
}

// getVoxel(worldPos) (VoxelUtilHashSDF.h:406-417)'s block lookup with a two-entry per-thread block cache: a
// trilinear sample's corners straddle a block face about a third of the time, and a one-entry cache re-probed
// the hash as the corners alternated between the two blocks
#ifndef BF_RENDER_CACHE
#define BF_RENDER_CACHE 1  // per-thread register cache entries (A/B builds: 2)
#endif
struct BlockCache {
    int ax = INT_MIN, ay = 0, az = 0, ap = BF_FREE_ENTRY;  // entry A
#if BF_RENDER_CACHE == 2
    int bx = INT_MIN, by = 0, bz = 0, bp = BF_FREE_ENTRY;  // entry B
    bool replaceB = false;  // the entry a miss replaces (the one not used last)
#endif
    uint32_t samples = 0, loads = 0, probes = 0;  // render statistics (trilinear samples, voxel loads, hash probes)
    unsigned long long* table = nullptr;  // the workgroup's LDS block table (nullptr: probe every miss)
    __device__ __forceinline__ int lookup(const RayArgs& R, i3 b) {
        // hits and updates as register selects: written as branches on the two entries, the compiler kept the
        // pair {ap, bp} in scratch and read it back on every hit (a memory round trip per corner lookup)
        const bool hitA = b.x == ax && b.y == ay && b.z == az;
#if BF_RENDER_CACHE == 2
        const bool hitB = b.x == bx && b.y == by && b.z == bz;
        if (hitA || hitB) {
            replaceB = hitA;
            return hitA ? ap : bp;
        }
#else
        if (hitA) return ap;
#endif
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
#if BF_RENDER_CACHE == 2
        const bool toB = replaceB;
        bx = toB ? b.x : bx; by = toB ? b.y : by; bz = toB ? b.z : bz; bp = toB ? p : bp;
        ax = toB ? ax : b.x; ay = toB ? ay : b.y; az = toB ? az : b.z; ap = toB ? ap : p;
        replaceB = !replaceB;
#else
        ax = b.x; ay = b.y; az = b.z; ap = p;
#endif
        return p;
    }
};
__device__ __forceinline__ int local_mod(int v) {  // v mod SDF_BLOCK_SIZE in [0, 8) (getVoxel's virtualVoxelPosToLocalSDFBlockIndex)
    int l = v % BF_SDF_BLOCK_SIZE;
    return l < 0 ? l + BF_SDF_BLOCK_SIZE : l;
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
    // the 8 corners' voxels located first (hash probes only where the block changes), then loaded together: the
    // reference reads them one after another and stops at the first zero weight, which made each load wait for
    // the previous one; the sums below keep its order and its stop.
    // Corner k is posDual + offs(k), added per component, so its virtual voxel takes on each axis either corner
    // 000's coordinate or corner 111's: the sample touches the blocks b0 + {0, 1}^3 on the axes where 000's and
    // 111's blocks differ (mask sm), one block usually, two across a face. Corner 000's block is located first
    // (in a free block the reference's first read has weight 0 and the sample ends: no other lookups in free
    // space); each lane then resolves its own other blocks in a loop, so a wave waits for the largest count on
    // one lane (one lookup, usually) instead of one lookup round trip per corner any lane missed (up to seven)
    const i3 v0 = world_to_vvox(posDual + offs(0), R.voxelSize), v7 = world_to_vvox(posDual + offs(7), R.voxelSize);
    const i3 b0 = vvox_to_block(v0), b7 = vvox_to_block(v7);
    int pj[8];
    pj[0] = c.lookup(R, b0);
    if (pj[0] == BF_FREE_ENTRY) return false;
    const uint32_t sm = (b7.x != b0.x ? 1u : 0u) | (b7.y != b0.y ? 2u : 0u) | (b7.z != b0.z ? 4u : 0u);
#pragma unroll
    for (int j = 1; j < 8; j++) pj[j] = pj[0];
    uint32_t pend = 0u;  // the nonzero subsets of sm
#pragma unroll
    for (uint32_t j = 1; j < 8; j++) pend |= (j & ~sm) == 0u ? 1u << j : 0u;
    while (pend) {
        const uint32_t j = (uint32_t)__builtin_ctz(pend);
        pend &= pend - 1u;
        const int p = c.lookup(R, i3{(j & 1u) ? b7.x : b0.x, (j & 2u) ? b7.y : b0.y, (j & 4u) ? b7.z : b0.z});
#pragma unroll
        for (uint32_t jj = 1; jj < 8; jj++) pj[jj] = (jj & sm) == j ? p : pj[jj];
    }
    const int l0x = local_mod(v0.x), l0y = local_mod(v0.y), l0z = local_mod(v0.z);
    const int l7x = local_mod(v7.x), l7y = local_mod(v7.y), l7z = local_mod(v7.z);
    float vs[8], vw[8];
    uint32_t vc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const bool kx = k == 1 || k == 4 || k == 6 || k == 7, ky = k == 2 || k == 4 || k == 5 || k == 7,
                   kz = k == 3 || k == 5 || k == 6 || k == 7;
        const int ptr = pj[(kx ? 1 : 0) | (ky ? 2 : 0) | (kz ? 4 : 0)];
        vs[k] = 0.0f; vw[k] = 0.0f; vc[k] = 0u;
        if (ptr != BF_FREE_ENTRY) {
            const int lx = kx ? l7x : l0x, ly = ky ? l7y : l0y, lz = kz ? l7z : l0z;
            const BFVoxel* vp = R.voxels + (size_t)ptr * BF_VOXELS_PER_BLOCK +
                                (lz * BF_SDF_BLOCK_SIZE * BF_SDF_BLOCK_SIZE + ly * BF_SDF_BLOCK_SIZE + lx);
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
template <bool GRAD>
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
                        if (GRAD) {
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
// Occupancy: a render is 4 800 waves. At 4 waves per SIMD (105-121 VGPRs) the 4 096 slots took them in two
// rounds, each a whole march long (the march is bound by memory latency, not by issue); the kernel without the
// gradient path fits 96 VGPRs (5 waves per SIMD: every wave of a 640x480 render resident at once) when the
// per-thread block cache holds one block (the sample's own corners no longer need two: trilinear resolves them
// per sample) and the two pointers it spills are reloaded once per pixel. useGradients renders take the kernel
// instantiated with the gradient path (its six extra samples need 17 more VGPRs).
#ifndef BF_RENDER_WPE  // A/B builds: waves per SIMD asked of the compiler for the kernel without gradients
#define BF_RENDER_WPE 5
#endif
template <int TPB, bool GRAD>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(GRAD ? 4 : BF_RENDER_WPE))) void k_render(RayArgs R, BFRayCastParams rp, const uint32_t* __restrict__ smin,
                                                const uint32_t* __restrict__ smax, float* d_depth, float4* d_depth4,
                                                float4* d_normals, float4* d_colors, float* outMin, float* outMax,
                                                unsigned long long* stats) {
    constexpr uint32_t TILE = TPB == 256 ? 16u : 8u;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t x = blockIdx.x * TILE + (wv & 1u) * 8u + (lane & 7u), y = blockIdx.y * TILE + (wv >> 1) * 8u + (lane >> 3);
    const long long tStart = R.waveLog ? wall_clock64() : 0;
    __shared__ unsigned long long s_table[RC_SLOTS];
    for (uint32_t i = threadIdx.x; i < (uint32_t)RC_SLOTS; i += TPB) s_table[i] = RC_EMPTY;
    __syncthreads();
    BlockCache cache;
    if (R.ldsTable) cache.table = s_table;
    bool rayed = false;
    if (x < rp.width && y < rp.height)
        render_pixel<GRAD>(R, rp, cache, x, y, smin, smax, d_depth, d_depth4, d_normals, d_colors, outMin, outMax, rayed);
    const uint32_t s = wave_sum_u32(cache.samples), l = wave_sum_u32(cache.loads), p = wave_sum_u32(cache.probes);
    const uint32_t r = wave_sum_u32(rayed ? 1u : 0u);
    uint32_t wmax = cache.samples;  // the wave's longest march
    for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off));
    __shared__ unsigned long long s_st[RS_COUNT];
    if (threadIdx.x < RS_COUNT) s_st[threadIdx.x] = 0;
    __syncthreads();
    if (lane == 0) {
        atomicAdd(&s_st[RS_SAMPLES], (unsigned long long)s);
        atomicAdd(&s_st[RS_LOADS], (unsigned long long)l);
        atomicAdd(&s_st[RS_PROBES], (unsigned long long)p);
        atomicAdd(&s_st[RS_RAYS], (unsigned long long)r);
        atomicAdd(&s_st[RS_WAVESAMPLES], 64ull * wmax);
        atomicMax(&s_st[RS_WAVEMAX], (unsigned long long)wmax);
        if (wmax > 32u) atomicAdd(&s_st[RS_LONGWAVES], 1ull);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long* st = rs_slot(stats);
        if (blockIdx.x == 0 && blockIdx.y == 0) {
            atomicAdd(&st[RS_RENDERS], 1ull);
            atomicAdd(&st[RS_PIXELS], (unsigned long long)rp.width * rp.height);
        }
        if (s_st[RS_SAMPLES]) {
            atomicAdd(&st[RS_SAMPLES], s_st[RS_SAMPLES]);
            atomicAdd(&st[RS_LOADS], s_st[RS_LOADS]);
            atomicAdd(&st[RS_PROBES], s_st[RS_PROBES]);
            atomicAdd(&st[RS_WAVESAMPLES], s_st[RS_WAVESAMPLES]);
            atomicMax(&st[RS_WAVEMAX], s_st[RS_WAVEMAX]);
        }
        if (s_st[RS_RAYS]) atomicAdd(&st[RS_RAYS], s_st[RS_RAYS]);
        if (s_st[RS_LONGWAVES]) atomicAdd(&st[RS_LONGWAVES], s_st[RS_LONGWAVES]);
    }
    if (lane == 0) {
        if (R.waveLog) {
            unsigned long long* w = R.waveLog + 4ull * ((blockIdx.y * gridDim.x + blockIdx.x) * (TPB / 64u) + wv);
            w[0] = (unsigned long long)tStart;
            w[1] = (unsigned long long)wall_clock64();
            w[2] = __smid();
            w[3] = wmax;
        }
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
    std::vector<uint64_t> all((size_t)kRenderStatSlots * kRenderStatFields);
    BF_HIP(hipMemcpyAsync(all.data(), renderStats_.p, all.size() * 8, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    uint64_t c[RS_COUNT] = {};
    for (int sl = 0; sl < kRenderStatSlots; sl++)
        for (int f = 0; f < RS_COUNT; f++) {
            const uint64_t v = all[(size_t)sl * kRenderStatFields + f];
            c[f] = f == RS_WAVEMAX ? std::max(c[f], v) : c[f] + v;
        }
    out.samples = c[RS_SAMPLES]; out.voxelLoads = c[RS_LOADS]; out.hashProbes = c[RS_PROBES]; out.rays = c[RS_RAYS];
    out.splatBlocks = c[RS_QUADS]; out.splatAtomics = c[RS_ATOMICS]; out.renders = c[RS_RENDERS]; out.pixels = c[RS_PIXELS];
    out.waveSamples = c[RS_WAVESAMPLES];
    out.waveSamplesMax = c[RS_WAVEMAX];
    out.longWaves = c[RS_LONGWAVES];
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
    if (!splatQuads_.p) splatQuads_.alloc(B_);
    const bool timed = renderClock_.enabled();
    if (timed) {
        if (!splatClock_.enabled()) splatClock_.enable(true);
        splatClock_.start(stream_);
    }
    {
        BF_REQUIRE(rp.width <= 0xFFFFu && rp.height <= 0x7FFFu, BF_ERR_ARG, "raycast size (16-bit splat rectangles)");
        const bool rows = div_up(rp.height, ST_H) <= (unsigned)ST_ROWS;
        const uint32_t rowCap = cfg_.splatRowCap ? cfg_.splatRowCap : 4u * B_;
        if (rows && !splatBin_.p) {
            splatBin_.alloc(SB_WORDS);
            BF_HIP(hipMemsetAsync(splatBin_.p, 0, splatBin_.bytes(), stream_));
            splatRowIdx_.alloc(rowCap);
        }
        uint32_t* bin = rows ? splatBin_.p : nullptr;
        const unsigned qgrid = (unsigned)numCUs_;  // one workgroup per CU: few same-address row-count atomics
        k_splat_quads<<<qgrid, 256, 0, stream_>>>(visible_.p, ctrl_.p, cfg_.hp.virtualVoxelSize, cam, rp, splatQuads_.p,
                                                   renderStats_.p, bin);
        BF_LAUNCH_CHECK();
        if (rows) {
            k_splat_rows<<<1, ST_ROWS, 0, stream_>>>(bin, rowCap);
            BF_LAUNCH_CHECK();
            k_splat_fill<<<qgrid, 256, 0, stream_>>>(splatQuads_.p, ctrl_.p, bin, splatRowIdx_.p, rowCap);
            BF_LAUNCH_CHECK();
        }
        const dim3 tg(div_up(rp.width, ST_W), div_up(rp.height, ST_H));
        const size_t nTiles = (size_t)tg.x * tg.y;
#ifdef BF_RENDER_DIAG  // diagnostics build: BF_SPLAT_TILE_LOG=path, per tile {start, end, __smid, rectangles folded | scanned << 32}
        static const char* tileLogPath = std::getenv("BF_SPLAT_TILE_LOG");
#else
        static const char* tileLogPath = nullptr;
#endif
        if (tileLogPath && tileLog_.n < 4 * nTiles) tileLog_.alloc(4 * nTiles);
        k_splat_tiles<<<tg, 256, 0, stream_>>>(splatQuads_.p, ctrl_.p, rp.width, rp.height, splatMin_.p, splatMax_.p, bin,
                                               splatRowIdx_.p, tileLogPath ? tileLog_.p : nullptr);
        if (tileLogPath) {
            std::vector<unsigned long long> h(4 * nTiles);
            BF_HIP(hipMemcpyAsync(h.data(), tileLog_.p, h.size() * 8, hipMemcpyDeviceToHost, stream_));
            BF_HIP(hipStreamSynchronize(stream_));
            if (FILE* f = std::fopen(tileLogPath, "ab")) {
                const unsigned long long nt = nTiles;
                std::fwrite(&nt, 8, 1, f);
                std::fwrite(h.data(), 8, h.size(), f);
                std::fclose(f);
            }
        }
    }
    BF_LAUNCH_CHECK();
    if (timed) splatClock_.stop(stream_);
    RayArgs R;
    R.hash = hash_.p;
    R.voxels = voxels_.p;
    R.numBuckets = cfg_.hp.hashNumBuckets;
    R.numEntries = E_;
    R.maxList = cfg_.hp.hashMaxCollisionLinkedListSize;
    R.voxelSize = cfg_.hp.virtualVoxelSize;
    R.ldsTable = cfg_.hp.numSDFBlocks < 0xFFFFFFu ? 1u : 0u;
#ifdef BF_RENDER_DIAG  // diagnostics build: BF_RENDER_WAVE_LOG=path, every render appends {waves, then per wave start /
                       // end wall clock (100 MHz), __smid, longest per-lane march}, synchronising the stream after it
    static const char* waveLogPath = std::getenv("BF_RENDER_WAVE_LOG");
#else
    static const char* waveLogPath = nullptr;
#endif
    const size_t nWaves = (size_t)div_up(rp.width, 16) * div_up(rp.height, 16) * 4;  // >= the 8x8 squares of either tile shape
    R.waveLog = nullptr;
    if (waveLogPath) {
        if (waveLog_.n < 4 * nWaves) waveLog_.alloc(4 * nWaves);
        R.waveLog = waveLog_.p;
    }
    const dim3 g(div_up(rp.width, 16), div_up(rp.height, 16));
    if (timed) renderClock_.start(stream_);
    auto launch = [&](auto kern) {
        kern<<<g, 256, 0, stream_>>>(R, rp, splatMin_.p, splatMax_.p, depth, depth4, normals, colors, rayMin, rayMax,
                                     renderStats_.p);
    };
    rp.useGradients ? launch(k_render<256, true>) : launch(k_render<256, false>);
    BF_LAUNCH_CHECK();
    if (timed) renderClock_.stop(stream_);
    if (waveLogPath) {
        std::vector<unsigned long long> h(4 * nWaves);
        BF_HIP(hipMemcpyAsync(h.data(), waveLog_.p, h.size() * 8, hipMemcpyDeviceToHost, stream_));
        BF_HIP(hipStreamSynchronize(stream_));
        if (FILE* f = std::fopen(waveLogPath, "ab")) {
            const unsigned long long n = nWaves;
            std::fwrite(&n, 8, 1, f);
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
        }
    }
    if (!rp.useGradients) {
        k_normals<<<g, 256, 0, stream_>>>(normals, depth4, rp.width, rp.height);
        BF_LAUNCH_CHECK();
    }
}

}  // namespace bf
