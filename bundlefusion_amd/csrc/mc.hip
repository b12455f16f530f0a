// mc.hip — gfx950 marching-cubes mesh extraction of the voxel-hash TSDF (replaces
// CUDAMarchingCubesHashSDF::extractIsoSurface, /root/reference/FriedLiver/Source/DepthSensing/
// CUDAMarchingCubesHashSDF.cpp:107-118, extractIsoSurfaceKernel (CUDAMarchingCubesSDF.cu:15-27) and
// MarchingCubesData::extractIsoSurfaceAtPosition (MarchingCubesSDFUtil.h:119-227)).
//
//  * Work list: the allocated heap blocks [0, highWater) (blockPos.w != 0), one workgroup of 512
//    threads per block, thread = voxel (z*64 + y*8 + x, the reference's 8x8x8 thread block). The
//    reference launches one workgroup per hash ENTRY (4 * numBuckets, 33.5 M at the bench's 2^23
//    buckets) and returns from the free ones.
//  * The 27 blocks around the workgroup's block are looked up once into LDS; every getVoxel of the
//    8 trilinear corner samples (64 voxel fetches per voxel) resolves its block there (a full hash
//    lookup only if float rounding ever leaves that neighbourhood).
//  * A voxel whose own weight is 0 emits nothing: every corner sample's 2x2x2 footprint contains
//    the voxel itself (posDual + off rounds to it), so each of the reference's trilinear calls would
//    fail. This early-out is exact and skips the 64 fetches for empty space.
//  * Deterministic output: a count pass (triangles per block), a scan, and an emit pass that
//    writes each block's triangles at its offset in (block, voxel, triTable) order. The reference
//    appends with atomicAdd (order varies run to run) and drops triangles past m_maxNumTriangles;
//    here the first maxNumTriangles of the fixed order are kept and the total is reported.
#include "hash_dev.h"
#include "mc_tables.h"
#include "tsdf.h"

namespace bf {

namespace {

__constant__ McTables c_mc = make_mc_tables();

__constant__ uint8_t c_edgeA[12] = {0, 1, 2, 3, 4, 5, 6, 7, 0, 1, 2, 3};
__constant__ uint8_t c_edgeB[12] = {1, 2, 3, 0, 5, 6, 7, 4, 4, 5, 6, 7};

constexpr int MC_WG = 512;        // one thread per voxel of a block
constexpr int MC_SCAN_CHUNK = 1024;

struct McArgs {
    const BFHashEntry* hash;
    const BFVoxel* voxels;
    const int4* blockPos;
    uint32_t numBuckets, numEntries, maxList;
    float voxelSize;
    float thresh, thresh2;
    uint32_t box;
    f3 bmin, bmax;
};

struct Nbhd {  // LDS: pointers of the 3x3x3 blocks around the workgroup's block
    int ptr[27];
    i3 base;
};

// getVoxel(worldPos) (VoxelUtilHashSDF.h:406-417)
__device__ __forceinline__ void mc_voxel(const McArgs& A, const Nbhd& nb, f3 pos, float& sdf, float& weight,
                                         uint32_t& color) {
    const i3 v = world_to_vvox(pos, A.voxelSize);
    const i3 b = vvox_to_block(v);
    const int dx = b.x - nb.base.x + 1, dy = b.y - nb.base.y + 1, dz = b.z - nb.base.z + 1;
    int ptr;
    if ((unsigned)dx < 3u && (unsigned)dy < 3u && (unsigned)dz < 3u) ptr = nb.ptr[dz * 9 + dy * 3 + dx];
    else ptr = hash_lookup(A.hash, A.numBuckets, A.numEntries, A.maxList, b.x, b.y, b.z);
    if (ptr == BF_FREE_ENTRY) {  // deleteVoxel
        sdf = 0.0f; weight = 0.0f; color = 0u;
        return;
    }
    int lx = v.x % BF_SDF_BLOCK_SIZE, ly = v.y % BF_SDF_BLOCK_SIZE, lz = v.z % BF_SDF_BLOCK_SIZE;
    if (lx < 0) lx += BF_SDF_BLOCK_SIZE;
    if (ly < 0) ly += BF_SDF_BLOCK_SIZE;
    if (lz < 0) lz += BF_SDF_BLOCK_SIZE;
    const BFVoxel* vp = A.voxels + (size_t)ptr * BF_VOXELS_PER_BLOCK + (lz * BF_SDF_BLOCK_SIZE * BF_SDF_BLOCK_SIZE + ly * BF_SDF_BLOCK_SIZE + lx);
    sdf = vp->sdf;
    weight = vp->weight;
    color = *reinterpret_cast<const uint32_t*>(vp->color);
}

__device__ __forceinline__ float mc_frac(float v) { return v - floorf(v); }

// trilinearInterpolationSimpleFastFast (RayCastSDFUtil.h:96-116); only dist is used by marching cubes
__device__ __forceinline__ bool mc_trilinear(const McArgs& A, const Nbhd& nb, f3 pos, float& dist) {
    const float oSet = A.voxelSize;
    const f3 posDual = pos - mk3(oSet / 2.0f, oSet / 2.0f, oSet / 2.0f);
    const f3 vv = pos / A.voxelSize;
    const f3 w = mk3(mc_frac(vv.x), mc_frac(vv.y), mc_frac(vv.z));
    dist = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const f3 off = mk3((k == 1 || k == 4 || k == 6 || k == 7) ? oSet : 0.0f, (k == 2 || k == 4 || k == 5 || k == 7) ? oSet : 0.0f,
                           (k == 3 || k == 5 || k == 6 || k == 7) ? oSet : 0.0f);
        float sdf, wt;
        uint32_t col;
        mc_voxel(A, nb, posDual + off, sdf, wt, col);
        if (wt == 0.0f) return false;
        const float a = (k == 1 || k == 4 || k == 6 || k == 7) ? w.x : 1.0f - w.x;
        const float bq = (k == 2 || k == 4 || k == 5 || k == 7) ? w.y : 1.0f - w.y;
        const float cq = (k == 3 || k == 5 || k == 6 || k == 7) ? w.z : 1.0f - w.z;
        dist += a * bq * cq * sdf;
    }
    return true;
}

// The per-voxel part of extractIsoSurfaceAtPosition up to the case lookup: returns the cube index
// (or -1 when the voxel emits nothing) with the 8 corner positions / distances in cubeindex-bit
// order (0 p010, 1 p110, 2 p100, 3 p000, 4 p011, 5 p111, 6 p101, 7 p001).
__device__ __forceinline__ int mc_case(const McArgs& A, const Nbhd& nb, f3 worldPos, f3* cp, float* cd) {
    if (A.box) {  // isInBoxAA (:229-237)
        if (worldPos.x < A.bmin.x || worldPos.x > A.bmax.x) return -1;
        if (worldPos.y < A.bmin.y || worldPos.y > A.bmax.y) return -1;
        if (worldPos.z < A.bmin.z || worldPos.z > A.bmax.z) return -1;
    }
    const float P = A.voxelSize / 2.0f;
    const float M = -P;
    // corner c's offset signs in cubeindex order
    const float ox[8] = {M, P, P, M, M, P, P, M};
    const float oy[8] = {P, P, M, M, P, P, M, M};
    const float oz[8] = {M, M, M, M, P, P, P, P};
#pragma unroll
    for (int c = 0; c < 8; c++) {
        cp[c] = worldPos + mk3(ox[c], oy[c], oz[c]);
        if (!mc_trilinear(A, nb, cp[c], cd[c])) return -1;
    }
    int cubeindex = 0;
#pragma unroll
    for (int c = 0; c < 8; c++)
        if (cd[c] < 0.0f) cubeindex |= 1 << c;
    const float thres = A.thresh;
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
        for (int l = 0; l < 8; l++) {
            if (cd[k] * cd[l] < 0.0f) {
                if (fabsf(cd[k]) + fabsf(cd[l]) > thres) return -1;
            } else {
                if (fabsf(cd[k] - cd[l]) > thres) return -1;
            }
        }
#pragma unroll
    for (int c = 0; c < 8; c++)
        if (fabsf(cd[c]) > A.thresh2) return -1;
    const uint32_t e = c_mc.edges[cubeindex];
    if (e == 0 || e == 255) return -1;
    return cubeindex;
}

// vertexInterp (MarchingCubesSDFUtil.h:205-227) with c1 == c2 == the voxel's colour
__device__ __forceinline__ BFMcVertex mc_interp(f3 p1, f3 p2, float d1, float d2, uint32_t col) {
    const float cx = (float)(col & 0xFF), cy = (float)((col >> 8) & 0xFF), cz = (float)((col >> 16) & 0xFF);
    BFMcVertex r;
    const float isolevel = 0.0f;
    f3 p = p1;
    float mu = 0.0f;
    bool lerp = true;
    if (fabsf(isolevel - d1) < 0.00001f) lerp = false;
    else if (fabsf(isolevel - d2) < 0.00001f) { p = p2; lerp = false; }
    else if (fabsf(d1 - d2) < 0.00001f) lerp = false;
    if (lerp) {
        mu = (isolevel - d1) / (d2 - d1);
        p = mk3(p1.x + mu * (p2.x - p1.x), p1.y + mu * (p2.y - p1.y), p1.z + mu * (p2.z - p1.z));
        r.c[0] = (float)(cx + mu * 0.0f) / 255.f;  // (c1 + mu * (c2 - c1)) / 255 with c2 == c1
        r.c[1] = (float)(cy + mu * 0.0f) / 255.f;
        r.c[2] = (float)(cz + mu * 0.0f) / 255.f;
    } else {
        r.c[0] = cx / 255.f;
        r.c[1] = cy / 255.f;
        r.c[2] = cz / 255.f;
    }
    r.p[0] = p.x; r.p[1] = p.y; r.p[2] = p.z;
    return r;
}

__device__ __forceinline__ void load_nbhd(const McArgs& A, Nbhd& nb, int4 bp) {
    if (threadIdx.x == 0) nb.base = i3{bp.x, bp.y, bp.z};
    if (threadIdx.x < 27) {
        const int t = threadIdx.x;
        const int dx = t % 3 - 1, dy = (t / 3) % 3 - 1, dz = t / 9 - 1;
        nb.ptr[t] = hash_lookup(A.hash, A.numBuckets, A.numEntries, A.maxList, bp.x + dx, bp.y + dy, bp.z + dz);
    }
    __syncthreads();
}

__device__ __forceinline__ f3 mc_world_pos(int4 bp, float vs) {
    const int t = threadIdx.x;
    const int x = bp.x * BF_SDF_BLOCK_SIZE + (t & 7), y = bp.y * BF_SDF_BLOCK_SIZE + ((t >> 3) & 7),
              z = bp.z * BF_SDF_BLOCK_SIZE + (t >> 6);
    return vvox_to_world(x, y, z, vs);  // virtualVoxelPosToWorld(SDFBlockToVirtualVoxelPos + threadIdx)
}

// own voxel weight (exact early-out, see the header)
__device__ __forceinline__ bool mc_own_empty(const McArgs& A, uint32_t blk) {
    return A.voxels[(size_t)blk * 512 + threadIdx.x].weight == 0.0f;
}

// exclusive prefix over the workgroup (512 threads = 8 waves); returns the workgroup total in *total
__device__ __forceinline__ uint32_t wg_exclusive(uint32_t v, uint32_t* sWave, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t n = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += n;
    }
    if (lane == 63) sWave[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < MC_WG / 64; w++) {
        const uint32_t s = sWave[w];
        before += (w < wave) ? s : 0u;
        all += s;
    }
    *total = all;
    return before + incl - v;
}

__global__ __launch_bounds__(MC_WG) void k_mc_count(McArgs A, uint32_t* __restrict__ counts) {
    __shared__ Nbhd nb;
    __shared__ uint32_t sWave[MC_WG / 64];
    const uint32_t blk = blockIdx.x;
    const int4 bp = A.blockPos[blk];
    if (bp.w == 0) {
        if (threadIdx.x == 0) counts[blk] = 0;
        return;
    }
    load_nbhd(A, nb, bp);
    uint32_t n = 0;
    if (!mc_own_empty(A, blk)) {
        f3 cp[8];
        float cd[8];
        const int ci = mc_case(A, nb, mc_world_pos(bp, A.voxelSize), cp, cd);
        if (ci >= 0) n = c_mc.ntri[ci];
    }
    uint32_t total;
    wg_exclusive(n, sWave, &total);
    if (threadIdx.x == 0) counts[blk] = total;
}

// per-chunk exclusive scan of the block counts; chunk totals to chunkSum
__global__ __launch_bounds__(MC_SCAN_CHUNK) void k_mc_scan_chunks(const uint32_t* __restrict__ counts, uint32_t n,
                                                                 uint32_t* __restrict__ prefix, uint32_t* __restrict__ chunkSum) {
    __shared__ uint32_t sWave[MC_SCAN_CHUNK / 64];
    const uint32_t i = blockIdx.x * MC_SCAN_CHUNK + threadIdx.x;
    const uint32_t v = i < n ? counts[i] : 0u;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += t;
    }
    if (lane == 63) sWave[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < MC_SCAN_CHUNK / 64; w++) {
        const uint32_t s = sWave[w];
        before += (w < wave) ? s : 0u;
        all += s;
    }
    if (i < n) prefix[i] = before + incl - v;
    if (threadIdx.x == 0) chunkSum[blockIdx.x] = all;
}

// exclusive scan of the chunk totals (one workgroup, serial over rounds of 1024); total to out[nChunks]
__global__ __launch_bounds__(MC_SCAN_CHUNK) void k_mc_scan_top(uint32_t* __restrict__ chunkSum, uint32_t nChunks) {
    __shared__ uint32_t sWave[MC_SCAN_CHUNK / 64];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t r = 0; r < nChunks; r += MC_SCAN_CHUNK) {
        const uint32_t i = r + threadIdx.x;
        const uint32_t v = i < nChunks ? chunkSum[i] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o);
            if (lane >= (uint32_t)o) incl += t;
        }
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (uint32_t w = 0; w < MC_SCAN_CHUNK / 64; w++) {
            const uint32_t s = sWave[w];
            before += (w < wave) ? s : 0u;
            all += s;
        }
        const uint32_t c = carry;
        if (i < nChunks) chunkSum[i] = c + before + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) carry = c + all;
        __syncthreads();
    }
    if (threadIdx.x == 0) chunkSum[nChunks] = carry;
}

__global__ __launch_bounds__(MC_WG) void k_mc_emit(McArgs A, const uint32_t* __restrict__ prefix,
                                                   const uint32_t* __restrict__ chunkSum, BFMcTriangle* __restrict__ out,
                                                   uint32_t cap) {
    __shared__ Nbhd nb;
    __shared__ uint32_t sWave[MC_WG / 64];
    const uint32_t blk = blockIdx.x;
    const int4 bp = A.blockPos[blk];
    if (bp.w == 0) return;
    const uint32_t base = chunkSum[blk / MC_SCAN_CHUNK] + prefix[blk];
    if (base >= cap) return;  // workgroup-uniform
    load_nbhd(A, nb, bp);
    int ci = -1;
    const f3 worldPos = mc_world_pos(bp, A.voxelSize);
    if (!mc_own_empty(A, blk)) {
        f3 cp[8];
        float cd[8];
        ci = mc_case(A, nb, worldPos, cp, cd);
    }
    const uint32_t n = ci >= 0 ? c_mc.ntri[ci] : 0u;
    uint32_t total;
    const uint32_t at = base + wg_exclusive(n, sWave, &total);
    if (n == 0 || at >= cap) return;
    // Voxel v = hashData.getVoxel(worldPos): its colour for every vertex (:178)
    float sdf, w;
    uint32_t col;
    mc_voxel(A, nb, worldPos, sdf, w, col);
    // vertlist[edge] = vertexInterp(corner a, corner b) (:180-192), evaluated per triangle corner: the
    // corner positions and samples are recomputed (pure functions of the voxel), which keeps the
    // kernel in registers instead of a scratch-resident vertex list
    const uint32_t nv = 3u * (at + n <= cap ? n : cap - at);
    BFMcVertex* ov = reinterpret_cast<BFMcVertex*>(out + at);
#pragma unroll 1
    for (uint32_t j = 0; j < nv; j++) {
        const int ed = c_mc.tri[ci][j];
        const int a = c_edgeA[ed], b = c_edgeB[ed];
        const float P = A.voxelSize / 2.0f, M = -P;
        const f3 pa = worldPos + mk3((0x66 >> a) & 1 ? P : M, (0x33 >> a) & 1 ? P : M, a >= 4 ? P : M);
        const f3 pb = worldPos + mk3((0x66 >> b) & 1 ? P : M, (0x33 >> b) & 1 ? P : M, b >= 4 ? P : M);
        float da, db;  // the corner samples again (a pure function of the position)
        mc_trilinear(A, nb, pa, da);
        mc_trilinear(A, nb, pb, db);
        ov[j] = mc_interp(pa, pb, da, db, col);
    }
}

}  // namespace

uint32_t Scene::extractMesh(const BFMarchingCubesParams& p, BFMcTriangle* out, uint32_t cap, uint32_t* total) {
    BF_REQUIRE(p.threshMarchingCubes > 0.0f && p.threshMarchingCubes2 > 0.0f, BF_ERR_ARG, "marching-cubes thresholds must be > 0");
    BF_REQUIRE(out != nullptr || cap == 0, BF_ERR_ARG, "triangle buffer is NULL");
    uint32_t hw = 0;
    BF_HIP(hipMemcpyAsync(&hw, ctrl_.p + C_HIGHWATER, 4, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    BF_REQUIRE(hw <= B_, BF_ERR_INTERNAL, "heap high-water mark beyond the block pool");
    if (hw == 0) {
        if (total) *total = 0;
        return 0;
    }
    McArgs A{};
    A.hash = hash_.p;
    A.voxels = voxels_.p;
    A.blockPos = blockPos_.p;
    A.numBuckets = cfg_.hp.hashNumBuckets;
    A.numEntries = E_;
    A.maxList = cfg_.hp.hashMaxCollisionLinkedListSize;
    A.voxelSize = cfg_.hp.virtualVoxelSize;
    A.thresh = p.threshMarchingCubes;
    A.thresh2 = p.threshMarchingCubes2;
    A.box = p.boxEnabled ? 1u : 0u;
    A.bmin = mk3(p.minCorner[0], p.minCorner[1], p.minCorner[2]);
    A.bmax = mk3(p.maxCorner[0], p.maxCorner[1], p.maxCorner[2]);
    const uint32_t nChunks = (hw + MC_SCAN_CHUNK - 1) / MC_SCAN_CHUNK;
    DevBuf<uint32_t> counts, prefix, chunkSum;
    counts.alloc(hw);
    prefix.alloc(hw);
    chunkSum.alloc(nChunks + 1);
    k_mc_count<<<hw, MC_WG, 0, stream_>>>(A, counts.p);
    BF_HIP(hipGetLastError());
    k_mc_scan_chunks<<<nChunks, MC_SCAN_CHUNK, 0, stream_>>>(counts.p, hw, prefix.p, chunkSum.p);
    k_mc_scan_top<<<1, MC_SCAN_CHUNK, 0, stream_>>>(chunkSum.p, nChunks);
    BF_HIP(hipGetLastError());
    if (cap > 0) {
        k_mc_emit<<<hw, MC_WG, 0, stream_>>>(A, prefix.p, chunkSum.p, out, cap);
        BF_HIP(hipGetLastError());
    }
    uint32_t tot = 0;
    BF_HIP(hipMemcpyAsync(&tot, chunkSum.p + nChunks, 4, hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    if (total) *total = tot;
    return tot < cap ? tot : cap;
}

}  // namespace bf
