// corr.hip — EntryJ producer from depth maps and poses: the stand-in for the SiftGPU front end
// (feature detection / matching are out of scope) that lets the global bundle
// adjuster run on .sens input. Its output is what AddCurrToResidualsCU
// (/root/reference/FriedLiver/Source/SiftGPU/SIFTImageManager.cu:610-686) appends for the current
// frame: per image pair (i, cur), i in [startFrame, cur), up to maxPerPair
// (MAX_MATCHES_PER_IMAGE_PAIR_FILTERED = 25) EntryJ {i, cur, pos_i, pos_j} with
// pos = intrinsicsInv * (depth * (u, v, 1)) in each frame's camera space.
//
// A "match" is a grid pixel of frame i whose back-projection, carried by the poses into frame cur,
// lands on a pixel whose depth agrees within depthThresh. Candidates are visited in a fixed
// permutation of the sampling grid (spreads the matches over the image) and the first maxPerPair
// valid ones are kept, so the output is deterministic: pair order, then candidate order. The
// reference appends each pair's block at an atomic offset (order varies run to run).
//
// One workgroup per pair: 256 candidates per round, ballot + prefix in LDS keep the first ones.
// k_corr_pairs writes each pair's matches to a fixed slot array; k_corr_pack (one workgroup) packs
// the slots in pair order.
#include <hip/hip_runtime.h>

#include "../../include/bf/bf.h"
#include "bf_math.h"
#include "bf_runtime.h"
#include "corr.h"

#include <vector>

namespace bf {

namespace {

constexpr int CORR_WG = 256;
constexpr uint32_t MAX_PER_PAIR = 64;

__host__ __device__ __forceinline__ uint32_t corr_perm(uint32_t k, uint32_t n) {
    return (uint32_t)(((uint64_t)k * 2654435761ull) % n);  // prime multiplier > n: a permutation of [0, n)
}

// float4x4 * float3 with w = 1 (cuda_SimpleMatrixUtil.h:937-945), from a device row-major array
__device__ __forceinline__ f3 xform_p(const float* e, f3 v) {
    return mk3(e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * 1.0f, e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * 1.0f,
               e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * 1.0f);
}

struct CorrArgs {
    const float* const* depth;
    const float* T;     // [n][16] camera -> world
    const float* Tinv;  // [n][16] world -> camera
    float kinv[16];     // intrinsicsInv (row-major float4x4)
    float fx, fy, cx, cy;
    uint32_t W, H, gridW, gridH, maxPerPair, cur, start;
    float minDepth, maxDepth, depthThresh;
    BFEntryJ* slots;    // [pairs][maxPerPair]
    uint32_t* counts;   // [pairs]
    const uint2* list;  // (i, cur) per pair, or null: pair p = (start + p, cur)
};

__global__ __launch_bounds__(CORR_WG) void k_corr_pairs(CorrArgs A) {
    __shared__ uint32_t sWave[CORR_WG / 64];
    __shared__ uint32_t sTaken;
    const uint32_t p = blockIdx.x;
    const uint32_t i = A.list ? A.list[p].x : A.start + p;
    const uint32_t cur = A.list ? A.list[p].y : A.cur;
    if (threadIdx.x == 0) sTaken = 0;
    __syncthreads();
    const uint32_t N = A.gridW * A.gridH;
    const float* di = A.depth[i];
    const float* dj = A.depth[cur];
    const float* Ti = A.T + 16 * (size_t)i;
    const float* Tj = A.Tinv + 16 * (size_t)cur;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t r = 0; r < N; r += CORR_WG) {
        const uint32_t k = r + threadIdx.x;
        bool ok = false;
        BFEntryJ e{};
        if (k < N && i != cur) {
            const uint32_t g = corr_perm(k, N);
            const uint32_t gx = g % A.gridW, gy = g / A.gridW;
            const uint32_t u = gx * (A.W / A.gridW) + (A.W / A.gridW) / 2, v = gy * (A.H / A.gridH) + (A.H / A.gridH) / 2;
            const float d = di[v * A.W + u];
            if (d != -INFINITY && d >= A.minDepth && d <= A.maxDepth) {
                const f3 pi = xform_p(A.kinv, mk3(d * (float)u, d * (float)v, d * 1.0f));
                const f3 pj = xform_p(Tj, xform_p(Ti, pi));
                if (pj.z > 0.0f) {
                    const int uj = f2i(pj.x * A.fx / pj.z + A.cx + 0.5f), vj = f2i(pj.y * A.fy / pj.z + A.cy + 0.5f);
                    if (uj >= 0 && vj >= 0 && uj < (int)A.W && vj < (int)A.H) {
                        const float d2 = dj[vj * A.W + uj];
                        if (d2 != -INFINITY && d2 >= A.minDepth && d2 <= A.maxDepth && fabsf(d2 - pj.z) <= A.depthThresh) {
                            const f3 q = xform_p(A.kinv, mk3(d2 * (float)uj, d2 * (float)vj, d2 * 1.0f));
                            e.imgIdx_i = i;
                            e.imgIdx_j = cur;
                            e.pos_i.x = pi.x; e.pos_i.y = pi.y; e.pos_i.z = pi.z;
                            e.pos_j.x = q.x; e.pos_j.y = q.y; e.pos_j.z = q.z;
                            ok = true;
                        }
                    }
                }
            }
        }
        // keep the first valid candidates of this round in candidate order
        const unsigned long long m = __ballot(ok);
        if (lane == 0) sWave[wave] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (uint32_t w = 0; w < CORR_WG / 64; w++) {
            before += (w < wave) ? sWave[w] : 0u;
            all += sWave[w];
        }
        const uint32_t taken = sTaken;
        const uint32_t at = taken + before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (ok && at < A.maxPerPair) A.slots[(size_t)p * A.maxPerPair + at] = e;
        __syncthreads();
        if (threadIdx.x == 0) sTaken = min(taken + all, A.maxPerPair);
        __syncthreads();
        if (sTaken >= A.maxPerPair) break;  // workgroup-uniform
    }
    if (threadIdx.x == 0) A.counts[p] = sTaken;
}

// pair order: exclusive scan of the counts (one workgroup), then each thread copies its pair's slots
// (a pair with fewer than minPerPair matches contributes none: the matcher's s_minNumMatches filter)
__global__ __launch_bounds__(1024) void k_corr_pack(const BFEntryJ* __restrict__ slots, const uint32_t* __restrict__ counts,
                                                    uint32_t pairs, uint32_t maxPerPair, uint32_t minPerPair, BFEntryJ* out,
                                                    uint32_t cap, uint32_t* total) {
    __shared__ uint32_t sWave[16];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t r = 0; r < pairs; r += 1024) {
        const uint32_t p = r + threadIdx.x;
        uint32_t c = p < pairs ? counts[p] : 0u;
        if (c < minPerPair) c = 0;
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(incl, o);
            if (lane >= (uint32_t)o) incl += t;
        }
        if (lane == 63) sWave[wave] = incl;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (uint32_t w = 0; w < 16; w++) {
            before += (w < wave) ? sWave[w] : 0u;
            all += sWave[w];
        }
        const uint32_t base = carry + before + incl - c;
        for (uint32_t k = 0; k < c; k++)
            if (base + k < cap) out[base + k] = slots[(size_t)p * maxPerPair + k];
        __syncthreads();
        if (threadIdx.x == 0) carry += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

}  // namespace

void CorrScratch::reserve(uint32_t npairs, uint32_t maxPerPair) {
    const size_t need = (size_t)std::max(npairs, 1u) * maxPerPair;
    if (slots.n < need) slots.alloc(need + need / 2);
    if (counts.n < npairs) counts.alloc(npairs + npairs / 2 + 1);
    if (pairs.n < npairs) pairs.alloc(npairs + npairs / 2 + 1);
    if (!total.n) total.alloc(1);
    if (!hostTotal) BF_HIP(hipHostMalloc((void**)&hostTotal, sizeof(uint32_t), hipHostMallocDefault));
}

namespace {
uint32_t corr_run(CorrArgs A, uint32_t pairs, const BFCorrOptions& o, BFEntryJ* out, uint32_t cap, uint32_t* total,
                  hipStream_t s, CorrScratch& sc) {
    A.slots = sc.slots.p;
    A.counts = sc.counts.p;
    k_corr_pairs<<<pairs, CORR_WG, 0, s>>>(A);
    BF_LAUNCH_CHECK();
    k_corr_pack<<<1, 1024, 0, s>>>(sc.slots.p, sc.counts.p, pairs, o.maxPerPair, o.minPerPair, out, cap, sc.total.p);
    BF_LAUNCH_CHECK();
    BF_HIP(hipMemcpyAsync(sc.hostTotal, sc.total.p, 4, hipMemcpyDeviceToHost, s));
    BF_HIP(hipStreamSynchronize(s));
    const uint32_t t = *sc.hostTotal;
    if (total) *total = t;
    return t < cap ? t : cap;
}
CorrArgs corr_args(const float* const* depth, const float* T, const float* Tinv, const BFCorrOptions& o) {
    CorrArgs A{};
    A.depth = depth;
    A.T = T;
    A.Tinv = Tinv;
    for (int k = 0; k < 16; k++) A.kinv[k] = o.intrinsicsInv[k];
    A.fx = o.intrinsics[0]; A.fy = o.intrinsics[1]; A.cx = o.intrinsics[2]; A.cy = o.intrinsics[3];
    A.W = o.width; A.H = o.height;
    A.gridW = o.width / o.stride; A.gridH = o.height / o.stride;
    // candidate permutation: k -> k * 2654435761 mod N is a bijection (the multiplier is a prime > N)
    A.maxPerPair = o.maxPerPair;
    A.minDepth = o.minDepth; A.maxDepth = o.maxDepth; A.depthThresh = o.depthThresh;
    return A;
}
void corr_check(const BFCorrOptions& o, const BFEntryJ* out, uint32_t cap) {
    BF_REQUIRE(o.width > 0 && o.height > 0 && o.stride > 0 && o.stride <= o.width && o.stride <= o.height, BF_ERR_ARG,
               "image size / stride");
    BF_REQUIRE(o.maxPerPair > 0 && o.maxPerPair <= MAX_PER_PAIR, BF_ERR_ARG, "maxPerPair 1..64");
    BF_REQUIRE(out != nullptr || cap == 0, BF_ERR_ARG, "null output");
}
}  // namespace

uint32_t corr_from_pairs(const float* const* depth, const float* T, const float* Tinv, const uint2* list, uint32_t npairs,
                         const BFCorrOptions& o, BFEntryJ* out, uint32_t cap, uint32_t* total, hipStream_t stream,
                         CorrScratch& sc) {
    BF_REQUIRE(depth && T && Tinv && list, BF_ERR_ARG, "null input");
    corr_check(o, out, cap);
    if (total) *total = 0;
    if (npairs == 0) return 0;
    sc.reserve(npairs, o.maxPerPair);
    BF_HIP(hipMemcpyAsync(sc.pairs.p, list, sizeof(uint2) * npairs, hipMemcpyHostToDevice, stream));
    CorrArgs A = corr_args(depth, T, Tinv, o);
    A.list = sc.pairs.p;
    return corr_run(A, npairs, o, out, cap, total, stream, sc);
}

// host entry (bf_corr_from_depth): pairs (start .. cur - 1, cur), with its own scratch, on the null stream, so
// it is ordered after the caller's work on the legacy stream (depth, poses, the pointer table) as the reference's
// AddCurrToResidualsCU on the default stream is; corr_run waits for its count before returning
uint32_t corr_from_depth(const float* const* depth, const float* T, const float* Tinv, uint32_t cur, uint32_t start,
                         const BFCorrOptions& o, BFEntryJ* out, uint32_t cap, uint32_t* total) {
    BF_REQUIRE(depth && T && Tinv, BF_ERR_ARG, "null input");
    BF_REQUIRE(start <= cur, BF_ERR_ARG, "startFrame > curFrame");
    corr_check(o, out, cap);
    const uint32_t pairs = cur - start;
    if (total) *total = 0;
    if (pairs == 0) return 0;
    CorrScratch sc;
    sc.reserve(pairs, o.maxPerPair);
    CorrArgs A = corr_args(depth, T, Tinv, o);
    A.cur = cur;
    A.start = start;
    return corr_run(A, pairs, o, out, cap, total, nullptr, sc);
}

}  // namespace bf
