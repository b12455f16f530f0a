// ba.hip — gfx950 kernels + host class for the bundle adjuster (see ba.h for the layout).
//
// Reference: Source/Solver/SolverBundling.cu, SolverBundlingEquationsLie.h,
// SolverBundlingDenseUtil.h, LieDerivUtil.h (cited per kernel below).
//
// The sparse term is rewritten around two identities of the reference's Lie Jacobian
// (evalLie_dAlpha/dBeta/dGamma, LieDerivUtil.h:231-242):
//   da*w.x + db*w.y + dc*w.z = w x P      and      (da.g, db.g, dc.g) = P x g
// so with P_s = T_self p_self and P_o = T_other p_other fixed for a GN iteration, one row entry of
// image v contributes   g = w[(pRot_v x P_s + pTrans_v) - (pRot_o x P_o + pTrans_o)],
//   Ap_rot(v) += P_s x g,   Ap_trans(v) += g
// (applyJDevice + applyJTDevice, SolverBundlingEquationsLie.h:154-228, with the +-1 sign of the
// row folded in). The PCG loop streams 32 B per row entry and gathers only the N-sized p vector.
#include "ba.h"
#include "lie.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace bf {

namespace {

constexpr float FLOAT_EPSILON = 0.000001f;  // Source/SolverUtil.h:9
constexpr int WG = 256;
static_assert(Solver::kSmallPersistImages == 2 * WG + 1, "the small persistent route (one finisher, 2 rows per thread)");
constexpr uint32_t TILE = 256;  // correspondences per table-build tile, per 256 images (a.tile)
// tile size for n images: the [n][nTiles] count matrix stays ~nCorr entries at any image count (a
// fixed 256 made it 8 x nCorr at 2 001 images: 955 us of strided count writes per solve)
__host__ __device__ constexpr uint32_t tile_for(uint32_t n) { return TILE * (n > 256u ? (n + 255u) / 256u : 1u); }
constexpr int CH = 512;        // row entries per chunk: the work unit of one wave in the GN/PCG kernels
constexpr int CPL = CH / 64;   // chunk entries per lane

enum VecField { V_DELTA = 0, V_R, V_Z, V_P, V_AP, V_M, V_NUM };
enum CtrlWord {
    K_TICKET = 0, K_PCG_DONE, K_GN_DONE, K_GN_ITERS, K_PCG_ITERS, K_RDOTZ, K_NPAIRS, K_LAST_W,
    K_MAXRES, K_MAXIDX, K_ENERGY, K_HIGHCOUNT, K_ERROR, K_USE_DENSE, K_RM_I, K_RM_J,
    K_SKIPPED,      // the solve's gate was 0: nothing ran (an invalidated local submap's global solve)
    K_VERIFY_USED,  // useVerification said yes: the dense pair check ran
    K_VERIFY_OK,    // VerifyTrajectoryCU's d_validOpt (1 unless a pair failed)
    K_COUNT,
    K_NCHUNK = K_COUNT, K_NPAIRS_A,
    K_PCG_ITERS0,  // K_PCG_ITERS before the GN step's PCG (k_pair_init): the timeout recovery (pcg_recover) restarts from it
    K_CTRL_WORDS = 32  // words past K_COUNT are solver-internal (not part of the result)
};
static_assert(K_COUNT == Solver::kResultWords, "result words");

struct BA {
    BFEntryJ* corr;
    uint32_t nCorr;
    const int* valid;
    uint32_t N, maxN, cap;
    int *rowCount, *rowStart, *rowLen, *rowTmp, *rowIdx;
    int* tileCnt;  // [N][nTiles]
    uint32_t nTiles, tile;
    int *rowChunk, *chunkRow;  // chunks of row v: [rowChunk[v], rowChunk[v+1]); chunk -> row
    float4* chunkPart;         // [chunk][3] per-chunk partial sums
    uint32_t* sync;            // last_block_sharded: 8 shard counters + top counter (+ flag words), 64 B apart
    float4* entries;
    float* vec;
    float* img;
    float* T;
    float* Tinv;
    uint32_t* ctrl;
    float* part;
    int* partIdx;
    float* rot;
    float* trans;
    uint2* pairs;
    float* pairW;
    float* pairBlk;
    float* diag;
    float* jtr;
    // dense term in a fixed order (no float atomics, so two solves of one problem agree bit for bit):
    uint32_t* pairFlag;  // [N][N] overlap flag of (i, j), i < j (k_dense_overlap)
    float* pairAcc;      // [maxPairs][54] a pair's J_i^T J_i | J_j^T J_j upper triangles (21 + 21), J_i^T r | J_j^T r
    float* pairProd;     // [N][8] per PCG iteration: image v's dense off-diagonal Ap rows [trans | rot]
    uint32_t* imgPairs;  // [N][N] pairs of image v in pair order: k << 1 | (v is the pair's j)
    uint32_t* imgPairN;  // [N]
    uint32_t maxPairs;
    const BFCachedFrame* cache;
    uint32_t cw, ch;
    float fx, fy, mx, my;
    float distT, normT, colT, gradMin, dmin, dmax, verifyT;
    uint32_t sub;
    // assembled normal equations (pair mode)
    int *rowSorted, *rowOther, *rowSeg, *rowDeg, *rowNA, *pairStart, *rowPairStart, *pairA, *pairB;
    int2 *pairCorr, *rowPair;
    uint32_t entTail;  // float4 offset of k_pair_gather's float2 tail in entries (2 maxCorr + 1)
    double *pstat, *dstat;
    float *apPair, *rzPart;
    uint2* aGran;  // [2][maxN][6] {value bits, tag}: k_pcg_persist's Ap hand-off
    uint2* fxGran; // [2][8] {block partial, tag}: the four-workgroup finisher's p.Ap / r.z partials
    uint32_t pairMode, shardCount, shardIndex, pairBound;
    uint32_t earlyOut;  // ENABLE_EARLY_OUT (SolverBundling.cu:7): PCG |p.Ap| < 5e-7 and GN max|delta| < 0.005 exits
    float* poseBak;     // [maxN][6] rot | trans at the GN step's start (k_pair_init), for the timeout recovery (pcg_recover)
    unsigned long long spinTicks;  // bound of every k_pcg_persist wait (s_memrealtime ticks, 100 MHz)
};

__device__ __forceinline__ unsigned lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ float* vptr(const BA& a, int field, uint32_t v) { return a.vec + ((size_t)field * a.maxN + v) * 8; }
__device__ __forceinline__ void vload(const BA& a, int field, uint32_t v, f3& r, f3& t) {
    const float4* p = reinterpret_cast<const float4*>(vptr(a, field, v));
    float4 x = p[0], y = p[1];
    r = mk3(x.x, x.y, x.z);
    t = mk3(y.x, y.y, y.z);
}
__device__ __forceinline__ void vstore(const BA& a, int field, uint32_t v, f3 r, f3 t) {
    float4* p = reinterpret_cast<float4*>(vptr(a, field, v));
    p[0] = make_float4(r.x, r.y, r.z, 0.0f);
    p[1] = make_float4(t.x, t.y, t.z, 0.0f);
}
// Fixed-order wave sums (all 64 lanes active): adjacent lanes, quads, half rows and rows through DPP
// (after each step every lane of the group holds the same value, so the mirrors pair groups exactly as
// an xor butterfly would), then the four row sums as (r0 + r1) + (r2 + r3), read into scalars. Every
// lane returns the same value; no LDS round trips.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true)); }
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);  // row_half_mirror
    v += dpp_f<0x140>(v);  // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}
__device__ __forceinline__ float ctrlf(const uint32_t* c, int k) { return __uint_as_float(c[k]); }
__device__ __forceinline__ m4 loadm4(const float* p) {
    m4 m;
    const float4* q = reinterpret_cast<const float4*>(p);
    for (int r = 0; r < 4; r++) {
        float4 v = q[r];
        m.e[r * 4 + 0] = v.x; m.e[r * 4 + 1] = v.y; m.e[r * 4 + 2] = v.z; m.e[r * 4 + 3] = v.w;
    }
    return m;
}
__device__ __forceinline__ bool corr_valid(const BFEntryJ& e) { return e.imgIdx_i != BF_INVALID_IMAGE; }

// In-launch hand-offs (MI355X_MICROARCH.md §inter-workgroup visibility, "valid forms" row 1): the
// producer stores its payload write-through (sc1: 8-B agent-scope atomic stores to global memory),
// drains its stores (s_waitcnt vmcnt(0)) and then adds to an agent-scope counter; the adder that
// draws the last ticket reads the payload with sc1 loads (which bypass this CU's L1). No release or
// acquire fence is needed, so the hand-off costs no L2 write-back per wave.
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void st_wt(float4* p, float4 v) {
    gu64* q = (gu64*)(p);
    __hip_atomic_store(q, ((uint64_t)__float_as_uint(v.y) << 32) | __float_as_uint(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, ((uint64_t)__float_as_uint(v.w) << 32) | __float_as_uint(v.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld_wt(const float4* p) {
    gu64* q = (gu64*)(p);
    const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)), __uint_as_float((uint32_t)b),
                       __uint_as_float((uint32_t)(b >> 32)));
}
__device__ __forceinline__ void st_wt(uint32_t* p, uint32_t v) { __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t ld_wt(const uint32_t* p) { return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void st_wt(float* p, float v) { st_wt(reinterpret_cast<uint32_t*>(p), __float_as_uint(v)); }
// k_pcg_persist's flag word: {count, alpha bits} as one 8-B store / load (the workers get alpha with
// the flag instead of one more dependent load after it)
__device__ __forceinline__ void st_wt64(uint32_t* p, uint32_t lo, uint32_t hi) {
    __hip_atomic_store((gu64*)p, ((uint64_t)hi << 32) | lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_wt64(const uint32_t* p) { return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_wtf(const float* p) { return __uint_as_float(ld_wt(reinterpret_cast<const uint32_t*>(p))); }
__device__ __forceinline__ uint32_t ticket_add(uint32_t* p) {
    return __hip_atomic_fetch_add((gu32*)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// vector fields through write-through (WT) or plain accesses
template <bool WT>
__device__ __forceinline__ void vload_t(const BA& a, int field, uint32_t v, f3& r, f3& t) {
    if (WT) {
        const float4* p = reinterpret_cast<const float4*>(vptr(a, field, v));
        const float4 x = ld_wt(p), y = ld_wt(p + 1);
        r = mk3(x.x, x.y, x.z);
        t = mk3(y.x, y.y, y.z);
    } else {
        vload(a, field, v, r, t);
    }
}
template <bool WT>
__device__ __forceinline__ void vstore_t(const BA& a, int field, uint32_t v, f3 r, f3 t) {
    if (WT) {
        float4* p = reinterpret_cast<float4*>(vptr(a, field, v));
        st_wt(p, make_float4(r.x, r.y, r.z, 0.0f));
        st_wt(p + 1, make_float4(t.x, t.y, t.z, 0.0f));
    } else {
        vstore(a, field, v, r, t);
    }
}

// "Last workgroup" hand-off: every wave drains its write-through stores, one lane takes a ticket;
// the workgroup holding the last ticket continues (and reads the hand-off with ld_wt).
__device__ bool last_block(uint32_t* ticket) {
    __shared__ int isLast;
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) isLast = (ticket_add(ticket) == gridDim.x * gridDim.y - 1) ? 1 : 0;
    __syncthreads();
    return isLast != 0;
}

// Two-level arrival for grid-wide hand-offs with many workgroups (MI355X_MICROARCH.md: one counter
// with hundreds of arrivers serialises at ~11 ns per atomic): workgroups are split into 8 shards by
// blockIdx % 8 (the dispatcher's round-robin XCD: a placement guess for speed only, correctness does
// not depend on it); a shard's last arriver adds to the top counter. Counters grow monotonically
// within a launch, so round `epoch` (1-based) completes at epoch * arrivers.
constexpr int SYNC_LINE = 16;  // words per 64-B line
constexpr int SYNC_TOP = 8 * SYNC_LINE, SYNC_FLAG = 9 * SYNC_LINE, SYNC_ALPHA = 17 * SYNC_LINE;  // alpha: 256 words
// k_pcg_persist's flag in PP_NFLAG replicas 256 B apart (one per 64-word stride): 500 workgroups polling
// one word took 5.9 us from the finisher's store to the last of them seeing it (1.0 at 126)
constexpr int PP_NFLAG = 16, PP_FLAG_STRIDE = 64;
constexpr int SYNC_FLAGR = SYNC_ALPHA + 256;
constexpr int SYNC_WORDS = SYNC_FLAGR + PP_NFLAG * PP_FLAG_STRIDE + SYNC_LINE;
__device__ bool last_block_sharded(uint32_t* sync, uint32_t epoch) {
    __shared__ int isLast;
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x, sh = blockIdx.x & 7u;
        const uint32_t ns = (G + 7u - sh) / 8u, nShards = G < 8u ? G : 8u;
        int last = 0;
        if (ticket_add(&sync[sh * SYNC_LINE]) == epoch * ns - 1u) last = ticket_add(&sync[SYNC_TOP]) == epoch * nShards - 1u;
        isLast = last;
    }
    __syncthreads();
    return isLast != 0;
}

// deterministic block reduction of one float per thread: fixed butterfly per wave, then the wave
// sums in wave order
__device__ float block_sum(float v, float* sh) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = 0.0f;
    for (uint32_t w = 0; w < (blockDim.x >> 6); w++) r += sh[w];
    __syncthreads();
    return r;
}

// ---- correspondence table (BuildVariablesToCorrespondencesTableDevice, SolverBundling.cu:1226-1248) ----
// The reference appends (image -> correspondence) pairs with atomics and drops an append once the row
// holds maxCorrPerImage entries. The deterministic replay here is a stable counting sort: rows list
// their correspondences in ascending index order (the serial order of that loop), an entry ranked
// >= cap in either of its rows invalidates the correspondence. Three passes over tiles of TILE
// consecutive correspondences: per-tile row histograms, a per-row scan over tiles, and a placement
// pass that ranks each entry inside its tile with wave ballots (no global atomics, no row sort).
__device__ __forceinline__ bool corr_rows(const BA& a, uint32_t c, uint32_t& i, uint32_t& j) {
    const uint2 ij = *reinterpret_cast<const uint2*>(&a.corr[c].imgIdx_i);
    i = ij.x; j = ij.y;
    return i != BF_INVALID_IMAGE && i < a.N && j < a.N;
}
__global__ __launch_bounds__(64) void k_tile_count(BA a) {
    extern __shared__ int hist[];  // [N]
    const uint32_t t = blockIdx.x;
    for (uint32_t r = threadIdx.x; r < a.N; r += 64) hist[r] = 0;
    __syncthreads();
    const uint32_t c1 = min((t + 1) * a.tile, a.nCorr);
    for (uint32_t c = t * a.tile + threadIdx.x; c < c1; c += 64) {
        uint32_t i, j;
        if (!corr_rows(a, c, i, j)) continue;
        atomicAdd(&hist[i], 1);
        atomicAdd(&hist[j], 1);
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < a.N; r += 64) a.tileCnt[(size_t)r * a.nTiles + t] = hist[r];
}
// one workgroup per row: exclusive scan of the row's tile counts (in place), rowCount = total
__global__ __launch_bounds__(WG) void k_tile_scan(BA a) {
    __shared__ int sh[WG];
    const uint32_t r = blockIdx.x;
    int* cnt = a.tileCnt + (size_t)r * a.nTiles;
    int carry = 0;
    for (uint32_t base = 0; base < a.nTiles; base += WG) {
        const uint32_t t = base + threadIdx.x;
        const int c = t < a.nTiles ? cnt[t] : 0;
        sh[threadIdx.x] = c;
        __syncthreads();
        for (int off = 1; off < WG; off <<= 1) {
            const int x = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
            __syncthreads();
            sh[threadIdx.x] += x;
            __syncthreads();
        }
        if (t < a.nTiles) cnt[t] = carry + sh[threadIdx.x] - c;
        carry += sh[WG - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) a.rowCount[r] = carry;
}
__global__ void k_scan(BA a) {  // one workgroup: exclusive scan of rowCount -> rowStart
    __shared__ int sh[WG];
    int carry = 0;
    for (uint32_t base = 0; base < a.N; base += WG) {
        const uint32_t v = base + threadIdx.x;
        const int c = v < a.N ? a.rowCount[v] : 0;
        sh[threadIdx.x] = c;
        __syncthreads();
        for (int off = 1; off < WG; off <<= 1) {
            int t = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
            __syncthreads();
            sh[threadIdx.x] += t;
            __syncthreads();
        }
        if (v < a.N) a.rowStart[v] = carry + sh[threadIdx.x] - c;
        carry += sh[WG - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) a.rowStart[a.N] = carry;
}
// placement: one wave per tile, 64 correspondences per step. Each distinct row key of the step is
// resolved in one ballot round: an entry's slot = row start + the row's tile offset + entries of
// that row placed earlier in this tile + lower lanes of this step holding the same row (an i entry
// precedes the j entry of the same correspondence).
__global__ __launch_bounds__(64) void k_tile_fill(BA a) {
    extern __shared__ int run[];  // [N] entries placed so far in this tile, per row
    const uint32_t t = blockIdx.x, lane = threadIdx.x;
    for (uint32_t r = lane; r < a.N; r += 64) run[r] = 0;
    __syncthreads();
    const uint64_t lower = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t c1 = min((t + 1) * a.tile, a.nCorr);
    for (uint32_t c0 = t * a.tile; c0 < c1; c0 += 64) {
        const uint32_t c = c0 + lane;
        uint32_t i = BF_INVALID_IMAGE, j = BF_INVALID_IMAGE;
        const bool ok = c < c1 && corr_rows(a, c, i, j);
        uint64_t pendI = __ballot(ok), pendJ = pendI;
        int posI = -1, posJ = -1;
        while (pendI | pendJ) {
            const int src = pendI ? __ffsll((unsigned long long)pendI) - 1 : __ffsll((unsigned long long)pendJ) - 1;
            const uint32_t key = __shfl(pendI ? i : j, src);
            const bool hi = ok && i == key, hj = ok && j == key;
            const uint64_t mi = __ballot(hi), mj = __ballot(hj);
            const int base = a.rowStart[key] + a.tileCnt[(size_t)key * a.nTiles + t] + run[key];
            const int below = __popcll(mi & lower) + __popcll(mj & lower);
            if (hi) posI = base + below;
            if (hj) posJ = base + below + (hi ? 1 : 0);
            __syncthreads();
            if (lane == 0) run[key] += __popcll(mi) + __popcll(mj);
            __syncthreads();
            pendI &= ~mi;
            pendJ &= ~mj;
        }
        if (ok) {
            a.rowTmp[posI] = (int)c;
            a.rowTmp[posJ] = (int)c;
            // setInvalid (SolverBundling.cu:1241-1245) for an entry past the per-image cap
            if (posI - a.rowStart[i] >= (int)a.cap || posJ - a.rowStart[j] >= (int)a.cap) {
                a.corr[c].imgIdx_i = BF_INVALID_IMAGE;
                a.corr[c].imgIdx_j = BF_INVALID_IMAGE;
            }
        }
    }
}
// keep the entries that survived the cap (stable), rowLen = kept count
__global__ __launch_bounds__(WG) void k_compact_rows(BA a) {
    __shared__ int base;
    const uint32_t v = blockIdx.x;
    if (v >= a.N) return;
    const int n = min(a.rowCount[v], (int)a.cap), s0 = a.rowStart[v];
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += WG) {
        const int k = k0 + threadIdx.x;
        bool keep = false;
        int c = 0;
        if (k < n) { c = a.rowTmp[s0 + k]; keep = corr_valid(a.corr[c]); }
        __shared__ int cnt[WG / 64];
        const unsigned long long m = __ballot(keep);
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) cnt[w] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int q = 0; q < w; q++) off += cnt[q];
        const unsigned l = lane_id();
        if (keep) a.rowIdx[s0 + off + __popcll(m & ((l == 0) ? 0ull : (~0ull >> (64 - l))))] = c;
        __syncthreads();
        if (threadIdx.x == 0) { int t = 0; for (int q = 0; q < WG / 64; q++) t += cnt[q]; base += t; }
        __syncthreads();
    }
    if (threadIdx.x == 0) a.rowLen[v] = base;
}

// chunk table: row v (v >= 1; image 0 is fixed) is cut into ceil(rowLen / CH) chunks of CH entries
__global__ void k_chunks(BA a) {  // one workgroup
    __shared__ int sh[WG];
    int carry = 0;
    for (uint32_t base = 0; base < a.N; base += WG) {
        const uint32_t v = base + threadIdx.x;
        const int c = (v >= 1 && v < a.N) ? (a.rowLen[v] + CH - 1) / CH : 0;
        sh[threadIdx.x] = c;
        __syncthreads();
        for (int off = 1; off < WG; off <<= 1) {
            const int x = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
            __syncthreads();
            sh[threadIdx.x] += x;
            __syncthreads();
        }
        const int s = carry + sh[threadIdx.x] - c;
        if (v < a.N) {
            a.rowChunk[v] = s;
            for (int q = 0; q < c; q++) a.chunkRow[s + q] = (int)v;
        }
        carry += sh[WG - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        a.rowChunk[a.N] = carry;
        a.ctrl[K_NCHUNK] = (uint32_t)carry;
    }
}
__device__ __forceinline__ void chunk_range(const BA& a, uint32_t c, uint32_t& v, int& k0, int& k1) {
    v = (uint32_t)a.chunkRow[c];
    const int s0 = a.rowStart[v];
    k0 = s0 + ((int)c - a.rowChunk[v]) * CH;
    k1 = min(s0 + a.rowLen[v], k0 + CH);
}

// ---- assembled normal equations (pair mode) ---------------------------------------------------
// The reference applies J^T J matrix-free: every PCG iteration streams all correspondences
// (applyJDevice / applyJTDevice, SolverBundlingEquationsLie.h:154-228). For a sparse-only solve the
// same operator is a sum over image pairs of 6x6 blocks, and with A_v = [-[P_v]x | I] (P_v = T_v p_v,
// the world point of a correspondence in image v) every block is fixed by a few sums over the pair's
// correspondences (a < b, P_a / P_b the two world points):
//   M = sum P_b P_a^T (9), s_a = sum P_a, s_b = sum P_b, n, Q_a = sum P_a P_a^T, Q_b = sum P_b P_b^T (6 each)
//   sum A_a^T A_b = [[tr(M) I - M, [s_a]x], [-[s_b]x, n I]]          (off-diagonal, row a)
//   sum A_v^T A_v = [[tr(Q) I - Q, [s]x], [-[s]x, n I]]              (diagonal, summed over v's pairs)
//   sum A_v^T r  = (-/+ (sum P_a x P_b), s_v - s_u)                     (J^T F, r = P_v - P_u)
// The statistics are accumulated in fp64 (products of fp32 points are exact in fp64), so the
// blocks keep the cancellation D_v p_v - sum_u B_vu p_u accurate. A PCG iteration then reads 128 B
// per (row, pair) entry instead of 64 B per (row, correspondence) entry. Pair p is built by shard
// p % shardCount; every other shard writes zeros, so the RCCL sum over shards reproduces the
// single-GPU statistics bit for bit (x + 0 = x), and the replicated PCG that follows is identical on
// every GPU (one all-reduce per GN iteration).
constexpr int PSTAT = 28;        // doubles per pair: M[9] s_a[3] s_b[3] n Q_a[6] Q_b[6]
constexpr int DSTAT = 10;        // doubles per image: Q[6] s[3] n
constexpr uint32_t SORT_MAX = 4096;  // >= maxCorrPerImage (4000)
constexpr uint32_t ROW_POS_BITS = 12;
constexpr uint32_t PAIR_A_FLAG = 0x80000000u;

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | lo);
}
__device__ __forceinline__ double wave_sum_d(double v) {  // wave_sum's order in fp64
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// per row v: the row's entries ordered by (other image, position) — position order is ascending
// correspondence index — with the row's distinct partners counted (rowDeg) and those above v (rowNA)
__global__ __launch_bounds__(WG) void k_pair_sort(BA a) {
    __shared__ uint32_t key[SORT_MAX];
    __shared__ int shd[WG / 64], sha[WG / 64];
    const uint32_t v = blockIdx.x;
    const int n = a.rowLen[v], s0 = a.rowStart[v];
    uint32_t P = 1;
    while (P < (uint32_t)n) P <<= 1;
    for (uint32_t t = threadIdx.x; t < P; t += WG) {
        uint32_t k = 0xFFFFFFFFu;
        if ((int)t < n) {
            const int c = a.rowIdx[s0 + t];
            const uint2 ij = *reinterpret_cast<const uint2*>(&a.corr[c].imgIdx_i);
            const uint32_t u = (ij.x == v) ? ij.y : ij.x;
            k = (u << ROW_POS_BITS) | t;
        }
        key[t] = k;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= P; size <<= 1) {  // bitonic sort, ascending
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t t = threadIdx.x; t < P / 2; t += WG) {
                const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
                const uint32_t x = key[i], y = key[j];
                if ((x > y) == ((i & size) == 0)) { key[i] = y; key[j] = x; }
            }
            __syncthreads();
        }
    }
    int deg = 0, na = 0;
    for (uint32_t t = threadIdx.x; t < (uint32_t)n; t += WG) {
        const uint32_t k = key[t], u = k >> ROW_POS_BITS;
        a.rowSorted[s0 + t] = a.rowIdx[s0 + (k & ((1u << ROW_POS_BITS) - 1))];
        a.rowOther[s0 + t] = (int)u;
        const bool head = (t == 0 || (key[t - 1] >> ROW_POS_BITS) != u) && u != v;  // self pairs are skipped
        int len = 0;
        if (head) {  // run length of partner u, from the sorted keys in LDS
            uint32_t e = t + 1;
            while (e < (uint32_t)n && (key[e] >> ROW_POS_BITS) == u) e++;
            len = (int)(e - t);
        }
        a.rowSeg[s0 + t] = len;
        deg += head ? 1 : 0;
        na += (head && u > v) ? 1 : 0;
    }
    for (int off = 32; off > 0; off >>= 1) { deg += __shfl_xor(deg, off); na += __shfl_xor(na, off); }
    if ((threadIdx.x & 63) == 0) { shd[threadIdx.x >> 6] = deg; sha[threadIdx.x >> 6] = na; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int d = 0, m = 0;
        for (int w = 0; w < WG / 64; w++) { d += shd[w]; m += sha[w]; }
        a.rowDeg[v] = d;
        a.rowNA[v] = m;
    }
}
// one workgroup: exclusive scans rowNA -> pairStart (pairs (a, b > a) numbered in (a, b) order) and
// rowDeg -> rowPairStart (each row's incident pairs)
__device__ void block_exclusive_scan(const int* in, int* out, uint32_t n, int* sh) {
    int carry = 0;
    for (uint32_t base = 0; base < n; base += WG) {
        const uint32_t v = base + threadIdx.x;
        const int c = v < n ? in[v] : 0;
        sh[threadIdx.x] = c;
        __syncthreads();
        for (int off = 1; off < WG; off <<= 1) {
            const int x = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
            __syncthreads();
            sh[threadIdx.x] += x;
            __syncthreads();
        }
        if (v < n) out[v] = carry + sh[threadIdx.x] - c;
        carry += sh[WG - 1];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[n] = carry;
    __syncthreads();
}
__global__ void k_pair_scan(BA a) {
    __shared__ int sh[WG];
    block_exclusive_scan(a.rowNA, a.pairStart, a.N, sh);
    block_exclusive_scan(a.rowDeg, a.rowPairStart, a.N, sh);
    if (threadIdx.x == 0) a.ctrl[K_NPAIRS_A] = (uint32_t)a.pairStart[a.N];
}
// one wave per row: segments (runs of one partner u) of the sorted row. Row a numbers its pairs with
// u > a and records their correspondence runs; the row entries of pairs with u < a are filled by
// k_pair_rows once every pair has its number.
__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) { return lane == 0 ? 0ull : (~0ull >> (64 - lane)); }
template <bool OWN>
__device__ void pair_segments(const BA& a, uint32_t v) {
    const uint32_t lane = lane_id();
    const int n = a.rowLen[v], s0 = a.rowStart[v];
    int seg = 0, segA = 0;
    for (int base = 0; base < n; base += 64) {
        const int t = base + (int)lane;
        const int u = t < n ? a.rowOther[s0 + t] : -1;
        const int prev = (t > 0 && t < n) ? a.rowOther[s0 + t - 1] : -1;
        const bool head = t < n && u != prev && u != (int)v;
        const uint64_t mh = __ballot(head), ma = __ballot(head && u > (int)v);
        const int rank = seg + __popcll(mh & lanes_below(lane));
        if (head) {
            if (OWN && u > (int)v) {
                const int p = a.pairStart[v] + segA + __popcll(ma & lanes_below(lane));
                a.pairA[p] = (int)v;
                a.pairB[p] = u;
                a.pairCorr[p] = make_int2(s0 + t, a.rowSeg[s0 + t]);
                a.rowPair[a.rowPairStart[v] + rank] = make_int2(p, (int)((uint32_t)u | PAIR_A_FLAG));
            } else if (!OWN && u < (int)v) {  // pair (u, v): binary search v in u's partner list
                int lo = a.pairStart[u], hi = a.pairStart[u + 1] - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (a.pairB[mid] < (int)v) lo = mid + 1; else hi = mid;
                }
                a.rowPair[a.rowPairStart[v] + rank] = make_int2(lo, u);
            }
        }
        seg += __popcll(mh);
        segA += __popcll(ma);
    }
}
__global__ __launch_bounds__(64) void k_pair_fill(BA a) { pair_segments<true>(a, blockIdx.x); }
__global__ __launch_bounds__(64) void k_pair_rows(BA a) { pair_segments<false>(a, blockIdx.x); }

// once per solve (pair mode): each pair's correspondence points, oriented (a, b), copied into the
// pair's run order — k_pair_stats then streams them contiguously on every GN iteration instead of
// gathering 48-B EntryJ records through rowSorted three times (the entries buffer is free in pair mode)
__global__ __launch_bounds__(WG) void k_pair_gather(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t np = a.ctrl[K_NPAIRS_A];
    float2* tail = reinterpret_cast<float2*>(a.entries + a.entTail);
    for (uint32_t p = wave; p < np; p += nw) {
        if (p % a.shardCount != a.shardIndex) continue;
        const uint32_t pa = (uint32_t)a.pairA[p];
        const int2 run = a.pairCorr[p];
        for (int k = (int)lane; k < run.y; k += 64) {
            const BFEntryJ e = a.corr[a.rowSorted[run.x + k]];
            const bool aIsI = e.imgIdx_i == pa;
            const f3 pA = aIsI ? mk3(e.pos_i.x, e.pos_i.y, e.pos_i.z) : mk3(e.pos_j.x, e.pos_j.y, e.pos_j.z);
            const f3 pB = aIsI ? mk3(e.pos_j.x, e.pos_j.y, e.pos_j.z) : mk3(e.pos_i.x, e.pos_i.y, e.pos_i.z);
            a.entries[run.x + k] = make_float4(pA.x, pA.y, pA.z, pB.x);
            tail[run.x + k] = make_float2(pB.y, pB.z);
        }
    }
}

// per GN iteration: the sufficient statistics of every pair of this shard (one wave per pair,
// lanes over its correspondences in ascending index order, fixed butterfly); pairs of other shards
// and slots in [nPairs, pairBound) are written as zeros
__global__ __launch_bounds__(WG) void k_pair_stats(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t np = a.ctrl[K_NPAIRS_A];
    const uint32_t bound = a.pairBound > np ? a.pairBound : np;
    if (a.pairBound && np > a.pairBound && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&a.ctrl[K_ERROR], 4u);
    for (uint32_t p = wave; p < bound; p += nw) {
        double* out = a.pstat + (size_t)p * PSTAT;
        if (p >= np || p % a.shardCount != a.shardIndex) {
            if (lane < PSTAT) out[lane] = 0.0;
            continue;
        }
        const uint32_t pa = (uint32_t)a.pairA[p], pb = (uint32_t)a.pairB[p];
        const int2 run = a.pairCorr[p];
        const m4 Ta = loadm4(a.T + (size_t)pa * 16), Tb = loadm4(a.T + (size_t)pb * 16);
        double M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, sa[3] = {0, 0, 0}, sb[3] = {0, 0, 0}, cnt = 0.0;
        double qa[6] = {0, 0, 0, 0, 0, 0}, qb[6] = {0, 0, 0, 0, 0, 0};
        const float2* tail = reinterpret_cast<const float2*>(a.entries + a.entTail);
        for (int k = (int)lane; k < run.y; k += 64) {
            const float4 x = a.entries[run.x + k];  // k_pair_gather's copy, contiguous per pair
            const float2 y = tail[run.x + k];
            const f3 pA = mk3(x.x, x.y, x.z), pB = mk3(x.w, y.x, y.y);
            const f3 A3 = xf(Ta, pA), B3 = xf(Tb, pB);  // the world points of k_entries
            const double A[3] = {A3.x, A3.y, A3.z}, B[3] = {B3.x, B3.y, B3.z};
#pragma unroll
            for (int r = 0; r < 3; r++) {
#pragma unroll
                for (int c = 0; c < 3; c++) M[r * 3 + c] += B[r] * A[c];
                sa[r] += A[r];
                sb[r] += B[r];
            }
            qa[0] += A[0] * A[0]; qa[1] += A[0] * A[1]; qa[2] += A[0] * A[2];
            qa[3] += A[1] * A[1]; qa[4] += A[1] * A[2]; qa[5] += A[2] * A[2];
            qb[0] += B[0] * B[0]; qb[1] += B[0] * B[1]; qb[2] += B[0] * B[2];
            qb[3] += B[1] * B[1]; qb[4] += B[1] * B[2]; qb[5] += B[2] * B[2];
            cnt += 1.0;
        }
        double s[PSTAT];
#pragma unroll
        for (int q = 0; q < 9; q++) s[q] = M[q];
#pragma unroll
        for (int q = 0; q < 3; q++) { s[9 + q] = sa[q]; s[12 + q] = sb[q]; }
        s[15] = cnt;
#pragma unroll
        for (int q = 0; q < 6; q++) { s[16 + q] = qa[q]; s[22 + q] = qb[q]; }
#pragma unroll
        for (int q = 0; q < PSTAT; q++) s[q] = wave_sum_d(s[q]) + 0.0;  // + 0.0: no -0 (exact shard sums)
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < PSTAT; q += 2) *reinterpret_cast<double2*>(out + q) = make_double2(s[q], s[q + 1]);
        }
    }
}

// B_vu p_u for the row entry (pair p, orientation): rot = tr(M) w - M w + s_v x t, trans = -s_u x w + n t,
// with M = sum P_u P_v^T (the pair's M for v = a, its transpose for v = b)
__device__ __forceinline__ void pair_block_apply(const double* st, bool vIsA, const double w[3], const double t[3],
                                                 double o[6]) {
    double M[9];
#pragma unroll
    for (int q = 0; q < 9; q++) M[q] = st[q];
    const double* sv = vIsA ? st + 9 : st + 12;
    const double* su = vIsA ? st + 12 : st + 9;
    const double n = st[15];
    const double tr = M[0] + M[4] + M[8];
    double Mw[3];
#pragma unroll
    for (int r = 0; r < 3; r++)
        Mw[r] = vIsA ? (M[r * 3] * w[0] + M[r * 3 + 1] * w[1] + M[r * 3 + 2] * w[2])
                     : (M[r] * w[0] + M[3 + r] * w[1] + M[6 + r] * w[2]);
    o[0] = tr * w[0] - Mw[0] + (sv[1] * t[2] - sv[2] * t[1]);
    o[1] = tr * w[1] - Mw[1] + (sv[2] * t[0] - sv[0] * t[2]);
    o[2] = tr * w[2] - Mw[2] + (sv[0] * t[1] - sv[1] * t[0]);
    o[3] = -(su[1] * w[2] - su[2] * w[1]) + n * t[0];
    o[4] = -(su[2] * w[0] - su[0] * w[2]) + n * t[1];
    o[5] = -(su[0] * w[1] - su[1] * w[0]) + n * t[2];
}
// D_v p_v from the image statistics Q (xx xy xz yy yz zz), s, n
__device__ __forceinline__ void diag_apply(const double* d, const double w[3], const double t[3], double o[6]) {
    const double Q[9] = {d[0], d[1], d[2], d[1], d[3], d[4], d[2], d[4], d[5]};
    const double* s = d + 6;
    const double n = d[9], tr = d[0] + d[3] + d[5];
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = tr * w[r] - (Q[r * 3] * w[0] + Q[r * 3 + 1] * w[1] + Q[r * 3 + 2] * w[2]);
    o[0] += s[1] * t[2] - s[2] * t[1];
    o[1] += s[2] * t[0] - s[0] * t[2];
    o[2] += s[0] * t[1] - s[1] * t[0];
    o[3] = -(s[1] * w[2] - s[2] * w[1]) + n * t[0];
    o[4] = -(s[2] * w[0] - s[0] * w[2]) + n * t[1];
    o[5] = -(s[0] * w[1] - s[1] * w[0]) + n * t[2];
}

// ---- per GN iteration -------------------------------------------------------------------------
// convertLiePosesToMatricesCU (SolverBundling.cu:1114-1121); also resets the PCG state of this
// GN iteration. gated: no-op once the GN loop converged on the device.
__device__ __forceinline__ void transforms_rows(const BA& a, uint32_t first, uint32_t stride) {
    for (uint32_t v = first; v < a.N; v += stride) {
        const m4 T = pose_to_matrix(mk3(a.rot[3 * v], a.rot[3 * v + 1], a.rot[3 * v + 2]),
                                    mk3(a.trans[3 * v], a.trans[3 * v + 1], a.trans[3 * v + 2]));
        const m4 Ti = inverse44(T);
        float4* t = reinterpret_cast<float4*>(a.T + (size_t)v * 16);
        float4* ti = reinterpret_cast<float4*>(a.Tinv + (size_t)v * 16);
        for (int r = 0; r < 4; r++) {
            t[r] = make_float4(T.e[r * 4], T.e[r * 4 + 1], T.e[r * 4 + 2], T.e[r * 4 + 3]);
            ti[r] = make_float4(Ti.e[r * 4], Ti.e[r * 4 + 1], Ti.e[r * 4 + 2], Ti.e[r * 4 + 3]);
        }
    }
}
__global__ void k_transforms(BA a, float wSparse, int useDense, int gated, int setState) {
    if (gated && a.ctrl[K_GN_DONE]) return;
    transforms_rows(a, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
    if (setState && blockIdx.x == 0 && threadIdx.x == 0) {
        a.ctrl[K_PCG_DONE] = 0;
        a.ctrl[K_TICKET] = 0;
        a.ctrl[K_LAST_W] = __float_as_uint(wSparse);
        a.ctrl[K_USE_DENSE] = (uint32_t)useDense;
    }
}

// chunk partials are handed to the finishing workgroup write-through (see last_block)
__device__ __forceinline__ void put_part(const BA& a, uint32_t c, int f, f3 s) {
    st_wt(a.chunkPart + (size_t)c * 3 + f, make_float4(s.x, s.y, s.z, 0.0f));
}
// PCGInit per row: r = -Jtr, Jacobi preconditioner, p = M r; returns r.z
__device__ float init_row_cnt(const BA& a, uint32_t v, f3 rr, f3 rt, f3 pr, float cnt, float wSparse, int useDense) {
    f3 resR = mk3(-wSparse * rr.x, -wSparse * rr.y, -wSparse * rr.z);
    f3 resT = mk3(-wSparse * rt.x, -wSparse * rt.y, -wSparse * rt.z);
    if (useDense) {
        const float* j = a.jtr + (size_t)v * 6;
        resR = resR - mk3(j[3], j[4], j[5]);
        resT = resT - mk3(j[0], j[1], j[2]);
    }
    auto inv = [](float x) { return x > FLOAT_EPSILON ? 1.0f / x : 1.0f; };
    const f3 mR = mk3(inv(pr.x), inv(pr.y), inv(pr.z));
    const f3 mT = mk3(inv(cnt), inv(cnt), inv(cnt));
    const f3 pR = mul3(mR, resR), pT = mul3(mT, resT);
    vstore(a, V_M, v, mR, mT);
    vstore(a, V_R, v, resR, resT);
    vstore(a, V_P, v, pR, pT);
    vstore(a, V_DELTA, v, mk3(0, 0, 0), mk3(0, 0, 0));
    return dot3(resR, pR) + dot3(resT, pT);
}
__device__ float init_row(const BA& a, uint32_t v, f3 rr, f3 rt, f3 pr, float wSparse, int useDense) {
    return init_row_cnt(a, v, rr, rt, pr, (float)a.rowLen[v], wSparse, useDense);
}

// world points of every row entry for this GN iteration: {T_self p_self, other}, {T_other p_other}
__global__ __launch_bounds__(WG) void k_entries(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t nch = a.ctrl[K_NCHUNK];
    for (uint32_t c = wave; c < nch; c += nw) {
        uint32_t v;
        int k0, k1;
        chunk_range(a, c, v, k0, k1);
        const m4 Tv = loadm4(a.T + (size_t)v * 16);
        int idx[CPL];
#pragma unroll
        for (int u = 0; u < CPL; u++) idx[u] = a.rowIdx[min(k0 + (int)lane + 64 * u, k1 - 1)];
        BFEntryJ ev[CPL];
#pragma unroll
        for (int u = 0; u < CPL; u++) ev[u] = a.corr[idx[u]];
#pragma unroll
        for (int u = 0; u < CPL; u++) {
            const int k = k0 + (int)lane + 64 * u;
            if (k >= k1) break;
            const BFEntryJ e = ev[u];
            const bool isI = (e.imgIdx_i == v);
            const uint32_t other = isI ? e.imgIdx_j : e.imgIdx_i;
            const f3 ps = isI ? mk3(e.pos_i.x, e.pos_i.y, e.pos_i.z) : mk3(e.pos_j.x, e.pos_j.y, e.pos_j.z);
            const f3 po = isI ? mk3(e.pos_j.x, e.pos_j.y, e.pos_j.z) : mk3(e.pos_i.x, e.pos_i.y, e.pos_i.z);
            const f3 Ps = xf(Tv, ps);
            const f3 Po = xf(loadm4(a.T + (size_t)other * 16), po);
            a.entries[2 * k] = make_float4(Ps.x, Ps.y, Ps.z, __uint_as_float(other));
            a.entries[2 * k + 1] = make_float4(Po.x, Po.y, Po.z, 0.0f);
        }
    }
}

// evalMinusJTFDevice (SolverBundlingEquationsLie.h:63-148) + PCGInit_Kernel1/2 (SolverBundling.cu:755-794).
// Every wave reduces one chunk; the last workgroup sums each row's chunk partials (chunk order),
// initialises the row and sums r.z.
__global__ __launch_bounds__(WG) void k_init(BA a, float wSparse) {
    __shared__ float sh[WG];
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t nch = a.ctrl[K_NCHUNK];
    const int useDense = (int)a.ctrl[K_USE_DENSE];
    for (uint32_t c = wave; c < nch; c += nw) {
        uint32_t v;
        int k0, k1;
        chunk_range(a, c, v, k0, k1);
        float rr[3] = {0, 0, 0}, rt[3] = {0, 0, 0}, pr[3] = {0, 0, 0};
        float4 A[CPL], B[CPL];
#pragma unroll
        for (int u = 0; u < CPL; u++) {
            const int k = min(k0 + (int)lane + 64 * u, k1 - 1);
            A[u] = a.entries[2 * k];
            B[u] = a.entries[2 * k + 1];
        }
#pragma unroll
        for (int u = 0; u < CPL; u++) {
            f3 Ps = mk3(A[u].x, A[u].y, A[u].z), Po = mk3(B[u].x, B[u].y, B[u].z);
            if (k0 + (int)lane + 64 * u >= k1) { Ps = mk3(0, 0, 0); Po = Ps; }
            const f3 r = Ps - Po;         // sign * (T_i p_i - T_j p_j)
            const f3 cr = cross3(Ps, r);  // (dot(da,r), dot(db,r), dot(dc,r)) of P_s
            rr[0] += cr.x; rr[1] += cr.y; rr[2] += cr.z;
            rt[0] += r.x; rt[1] += r.y; rt[2] += r.z;
            pr[0] += Ps.z * Ps.z + Ps.y * Ps.y;  // |dAlpha|^2
            pr[1] += Ps.z * Ps.z + Ps.x * Ps.x;  // |dBeta|^2
            pr[2] += Ps.y * Ps.y + Ps.x * Ps.x;  // |dGamma|^2
        }
        for (int q = 0; q < 3; q++) { rr[q] = wave_sum(rr[q]); rt[q] = wave_sum(rt[q]); pr[q] = wave_sum(pr[q]); }
        if (lane == 0) {
            put_part(a, c, 0, mk3(rr[0], rr[1], rr[2]));
            put_part(a, c, 1, mk3(rt[0], rt[1], rt[2]));
            put_part(a, c, 2, mk3(pr[0], pr[1], pr[2]));
        }
    }
    if (!last_block(&a.ctrl[K_TICKET])) return;
    float s = 0.0f;
    for (uint32_t v = 1 + threadIdx.x; v < a.N; v += blockDim.x) {
        f3 sR = mk3(0, 0, 0), sT = sR, sP = sR;
        for (int c = a.rowChunk[v]; c < a.rowChunk[v + 1]; c++) {
            const float4 x = ld_wt(a.chunkPart + (size_t)c * 3), y = ld_wt(a.chunkPart + (size_t)c * 3 + 1),
                         z = ld_wt(a.chunkPart + (size_t)c * 3 + 2);
            sR = sR + mk3(x.x, x.y, x.z);
            sT = sT + mk3(y.x, y.y, y.z);
            sP = sP + mk3(z.x, z.y, z.z);
        }
        s += init_row(a, v, sR, sT, sP, wSparse, useDense);
    }
    s = block_sum(s, sh);
    if (threadIdx.x == 0) {
        a.ctrl[K_RDOTZ] = __float_as_uint(s);
        a.ctrl[K_TICKET] = 0;
        for (int w = 0; w < SYNC_WORDS; w += SYNC_LINE) a.sync[w] = 0;  // the PCG launches' arrival counters
        vstore(a, V_P, 0, mk3(0, 0, 0), mk3(0, 0, 0));  // image 0 is fixed: its p stays 0
    }
}

// sparse JtJp partial of every chunk (one wave per chunk), handed over write-through
template <bool WT>
__device__ __forceinline__ void pcg_sparse_chunks(const BA& a, float wSparse, uint32_t wave, uint32_t nw, uint32_t nch) {
    const uint32_t lane = lane_id();
    for (uint32_t c = wave; c < nch; c += nw) {
        uint32_t v;
        int k0, k1;
        chunk_range(a, c, v, k0, k1);
        f3 pRv, pTv;
        vload_t<WT>(a, V_P, v, pRv, pTv);
        float ar[3] = {0, 0, 0}, at[3] = {0, 0, 0};
        // all CH/64 entries of this lane are loaded before any is used (clamped indices, masked
        // sums: no per-entry branch), so a chunk costs one HBM round trip plus one L2 gather
        float4 A[CPL], B[CPL];
#pragma unroll
        for (int u = 0; u < CPL; u++) {
            const int k = min(k0 + (int)lane + 64 * u, k1 - 1);
            A[u] = a.entries[2 * k];
            B[u] = a.entries[2 * k + 1];
        }
#pragma unroll
        for (int u = 0; u < CPL; u++) {
            const f3 Ps = mk3(A[u].x, A[u].y, A[u].z), Po = mk3(B[u].x, B[u].y, B[u].z);
            const uint32_t o = __float_as_uint(A[u].w);
            f3 pRo, pTo;
            vload_t<WT>(a, V_P, o, pRo, pTo);
            f3 g = (cross3(pRv, Ps) + pTv - (cross3(pRo, Po) + pTo)) * wSparse;
            f3 cr = cross3(Ps, g);
            if (k0 + (int)lane + 64 * u >= k1) { g = mk3(0, 0, 0); cr = g; }
            ar[0] += cr.x; ar[1] += cr.y; ar[2] += cr.z;
            at[0] += g.x; at[1] += g.y; at[2] += g.z;
        }
        for (int q = 0; q < 3; q++) { ar[q] = wave_sum(ar[q]); at[q] = wave_sum(at[q]); }
        if (lane == 0) { put_part(a, c, 0, mk3(ar[0], ar[1], ar[2])); put_part(a, c, 1, mk3(at[0], at[1], at[2])); }
    }
}

// Ap of row v for the finisher: the sparse part handed over by the row's last chunk wave, plus the
// dense diagonal block and the dense off-diagonal atomics (reset for the next iteration)
__device__ __forceinline__ void pcg_ap(const BA& a, uint32_t v, uint32_t nch, int useDense, f3 pR, f3 pT, f3& aR, f3& aT) {
    aR = mk3(0, 0, 0);
    aT = mk3(0, 0, 0);
    if (a.pairMode) {  // assembled normal equations: sparse Ap of the row, handed over by its wave
        const float4* q = reinterpret_cast<const float4*>(a.apPair + (size_t)v * 8);
        const float4 x = ld_wt(q), y = ld_wt(q + 1);
        aR = mk3(x.x, x.y, x.z);
        aT = mk3(y.x, y.y, y.z);
    } else if (nch) {  // sparse part: the row's chunk partials, in chunk order
        const int c1 = a.rowChunk[v + 1];
#pragma unroll 4
        for (int c = a.rowChunk[v]; c < c1; c++) {
            const float4 x = ld_wt(a.chunkPart + (size_t)c * 3), y = ld_wt(a.chunkPart + (size_t)c * 3 + 1);
            aR = aR + mk3(x.x, x.y, x.z);
            aT = aT + mk3(y.x, y.y, y.z);
        }
    }
    if (useDense) {  // diagonal block [trans | rot] x [pTrans | pRot]
        const float* D = a.diag + (size_t)v * 36;
        const float pv[6] = {pT.x, pT.y, pT.z, pR.x, pR.y, pR.z};
        float o6[6];
        for (int r = 0; r < 6; r++) {
            float s = 0.0f;
            for (int c = 0; c < 6; c++) s += D[r * 6 + c] * pv[c];
            o6[r] = s;
        }
        aT = aT + mk3(o6[0], o6[1], o6[2]);
        aR = aR + mk3(o6[3], o6[4], o6[5]);
        // off-diagonal blocks: the row's sum over its pairs of this launch (pcg_dense_offdiag, write-through)
        const float* pp = a.pairProd + (size_t)v * 8;
        aT = aT + mk3(ld_wtf(pp), ld_wtf(pp + 1), ld_wtf(pp + 2));
        aR = aR + mk3(ld_wtf(pp + 3), ld_wtf(pp + 4), ld_wtf(pp + 5));
    }
}

// PCG finisher with each thread's R rows held in registers: all loads issue up front, then the
// two block reductions, then the stores (z and Ap never go to memory). Same arithmetic as the
// multi-pass form below.
// R = 8 (514..2 049 images): the two dot products are summed as FIN_GROUPS block sums of two rows per
// thread each (rows q = 2g, 2g + 1), added in group order: the order of k_pcg_persist's four-workgroup
// finisher (pcg_persist_finisher_x4), so the persistent and the per-launch solves agree bit for bit
constexpr int FIN_GROUPS = 4;
template <int R>
__device__ __forceinline__ float grouped_sum(const float* e, float* sh) {
    if (R != 8) return block_sum(e[0], sh);
    float t = 0.0f;
#pragma unroll
    for (int g = 0; g < FIN_GROUPS; g++) t += block_sum(e[g], sh);
    return t;
}
template <int R, bool WT>
__device__ float pcg_finish_regs(const BA& a, float* sh, uint32_t nch, int useDense, int iter, int nLin, bool& lastOut) {
    f3 pR[R], pT[R], aR[R], aT[R], dR[R], dT[R], rR[R], rT[R], mR[R], mT[R];
    constexpr int NG = R == 8 ? FIN_GROUPS : 1;
    float d[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) d[g] = 0.0f;
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t v = 1 + threadIdx.x + q * WG;
        if (v < a.N) {
            vload_t<WT>(a, V_P, v, pR[q], pT[q]);
            vload_t<WT>(a, V_DELTA, v, dR[q], dT[q]);
            vload_t<WT>(a, V_R, v, rR[q], rT[q]);
            vload_t<WT>(a, V_M, v, mR[q], mT[q]);
            pcg_ap(a, v, nch, useDense, pR[q], pT[q], aR[q], aT[q]);
            d[NG > 1 ? q / 2 : 0] += dot3(pR[q], aR[q]) + dot3(pT[q], aT[q]);
        }
    }
    const float pAp = grouped_sum<R>(d, sh);
    const float rDotzOld = WT ? __uint_as_float(ld_wt(&a.ctrl[K_RDOTZ])) : ctrlf(a.ctrl, K_RDOTZ);
    const float alpha = (pAp > FLOAT_EPSILON) ? rDotzOld / pAp : 0.0f;
    float b[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) b[g] = 0.0f;
#pragma unroll
    for (int q = 0; q < R; q++) {
        if (1 + threadIdx.x + q * WG < a.N) {
            dR[q] = dR[q] + alpha * pR[q];
            dT[q] = dT[q] + alpha * pT[q];
            rR[q] = rR[q] - alpha * aR[q];
            rT[q] = rT[q] - alpha * aT[q];
            mR[q] = mul3(mR[q], rR[q]);  // z
            mT[q] = mul3(mT[q], rT[q]);
            b[NG > 1 ? q / 2 : 0] += dot3(mR[q], rR[q]) + dot3(mT[q], rT[q]);
        }
    }
    const float rDotzNew = grouped_sum<R>(b, sh);
    const bool last = (iter == nLin - 1) || (a.earlyOut && fabsf(pAp) < 5e-7f);
    const float beta = (rDotzOld > FLOAT_EPSILON) ? rDotzNew / rDotzOld : 0.0f;
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t v = 1 + threadIdx.x + q * WG;
        if (v < a.N) {
            vstore_t<WT>(a, V_DELTA, v, dR[q], dT[q]);
            vstore_t<WT>(a, V_R, v, rR[q], rT[q]);
            vstore_t<WT>(a, V_P, v, mR[q] + beta * pR[q], mT[q] + beta * pT[q]);
            if (last) {  // computeLieUpdate (LieDerivUtil.h:301-307)
                f3 nr, nt;
                lie_update(dR[q], dT[q], mk3(a.rot[3 * v], a.rot[3 * v + 1], a.rot[3 * v + 2]),
                           mk3(a.trans[3 * v], a.trans[3 * v + 1], a.trans[3 * v + 2]), nr, nt);
                a.rot[3 * v] = nr.x; a.rot[3 * v + 1] = nr.y; a.rot[3 * v + 2] = nr.z;
                a.trans[3 * v] = nt.x; a.trans[3 * v + 1] = nt.y; a.trans[3 * v + 2] = nt.z;
            }
        }
    }
    lastOut = last;
    return rDotzNew;
}

// dense off-diagonal blocks, per image v (one wave each): Σ over v's pairs, in pair order, of B p_i
// (v = the pair's j) or B^T p_j (v = its i), [trans | rot] rows. Lanes form 10 groups of 6 (one lane
// per output row); group g takes the list entries g, g + 10, ...; the groups' partial sums are then
// added in group order, so the sum is the same on every run. Stored write-through for the finisher.
__device__ __forceinline__ unsigned long long rtc() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz
constexpr unsigned long long PP_SPIN_TICKS = 200000000ull;  // 2 s at 100 MHz (BFSolverOptions.pcgSpinLimitUs = 0)
__device__ __forceinline__ bool pp_timed_out(unsigned long long t0, unsigned long long lim) { return rtc() - t0 > lim; }
// Data-tagged granules for k_pcg_persist's Ap hand-off (MI355X_MICROARCH.md's handoff-1to1 row): one
// 8-B {value, tag} per float, written by ONE 8-B agent-scope atomic store and read by 8-B agent-scope
// atomic loads, so a granule is never torn and its tag says which iteration wrote it; the consumer
// polls the granules themselves (no drain, no arrival counter). Tags are epoch * 256 + iteration + 1:
// the epoch counts persistent launches on this solver, so no granule of an earlier launch matches.
// (Moving p to the workers the same way — 500 waves polling their partners' granules — ran 2x
// slower than the polled flag: the polls' load traffic swamps the hand-off.)
__device__ __forceinline__ void gran_store(uint2* g, float v, uint32_t tag) {
    __hip_atomic_store((gu64*)g, ((uint64_t)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gran_load(const uint2* g) {
    return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Waits until the granules g[i][0..5] (i < NR) all carry `tag`: every load of every row in flight at
// once, and all of them reloaded after a short sleep while any is stale (no per-granule branches, so
// the loaded values do not multiply into merge copies). Every pointer must be valid and written with
// this tag (a lane without a row of its own polls a row that is). Returns 1, or -1 on timeout.
template <int NR>
__device__ __forceinline__ int gran_rows(const uint2* const* g, uint32_t tag, float out[][6], unsigned long long t0,
                                         unsigned long long lim) {
    uint64_t x[NR][6];
    for (;;) {
#pragma unroll
        for (int r = 0; r < NR; r++)
#pragma unroll
            for (int q = 0; q < 6; q++) x[r][q] = gran_load(g[r] + q);
        bool all = true;
#pragma unroll
        for (int r = 0; r < NR; r++)
#pragma unroll
            for (int q = 0; q < 6; q++) all = all && (uint32_t)(x[r][q] >> 32) == tag;
        if (all) break;
        if (pp_timed_out(t0, lim)) return -1;
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int r = 0; r < NR; r++)
#pragma unroll
        for (int q = 0; q < 6; q++) out[r][q] = __uint_as_float((uint32_t)x[r][q]);
    return 1;
}

// granTag != 0 (k_pcg_persist): the products go out as Ap granules of that tag
template <bool WT>
__device__ void pcg_dense_offdiag_row(const BA& a, uint32_t v, uint32_t granTag = 0) {
    const uint32_t lane = lane_id();
    const uint32_t grp = lane / 6, row = lane % 6;
    const uint32_t* L = a.imgPairs + (size_t)v * a.maxN;
    const uint32_t nL = a.imgPairN[v];
    float o = 0.0f;
    if (grp < 10) {
        for (uint32_t q = grp; q < nL; q += 10) {
            const uint32_t e = L[q], k = e >> 1;
            const uint2 pr = a.pairs[k];
            const float* Bk = a.pairBlk + (size_t)k * 36;  // rows: image pr.y, columns: image pr.x
            f3 r, t;
            vload_t<WT>(a, V_P, (e & 1u) ? pr.x : pr.y, r, t);
            const float pv[6] = {t.x, t.y, t.z, r.x, r.y, r.z};
            float s = 0.0f;
            if (e & 1u) { for (int c = 0; c < 6; c++) s += Bk[row * 6 + c] * pv[c]; }
            else { for (int rr = 0; rr < 6; rr++) s += Bk[rr * 6 + row] * pv[rr]; }
            if ((e & 1u) ? pr.x > 0 : pr.y > 0) o += s;  // p_0 = 0 (image 0 fixed)
        }
    }
    float tot = 0.0f;
    for (uint32_t g = 0; g < 10; g++) tot += __shfl(o, (int)(g * 6 + row));
    if (lane < 6) {
        if (granTag) gran_store(a.aGran + ((size_t)a.maxN + v) * 6 + lane, tot, granTag);  // k_pcg_persist
        else st_wt(reinterpret_cast<uint32_t*>(a.pairProd) + (size_t)v * 8 + lane, __float_as_uint(tot));
    }
}
__device__ void pcg_dense_offdiag(const BA& a, uint32_t wave, uint32_t nw) {
    for (uint32_t v = 1 + wave; v < a.N; v += nw) pcg_dense_offdiag_row<false>(a, v);
}

#ifdef BF_PCG_TIMING
// measurement build: per PCG launch (iteration index mod 1024) the earliest workgroup start, the
// latest phase-A end, the finisher's start and end (s_memrealtime, 100 MHz)
__device__ unsigned long long g_pcgT[1024][4];
__device__ unsigned long long g_pcgS[1024][6];  // the last-arriving workgroup's stage stamps (wave 0)
__device__ unsigned long long g_pcgW[64][1024][2];  // k_pcg_persist: per iteration (< 64) and worker WG: flag seen, arrival
#endif
// PCG finisher (one workgroup): Kernel1b, Kernel2, the host early-out test, Kernel3
template <int RB = 2>
__device__ void pcg_finisher(const BA& a, float* sh, uint32_t nch, int useDense, int iter, int nLin, float& rDotzNew,
                             bool& last) {
    if (a.N <= RB * WG + 1) {
        rDotzNew = pcg_finish_regs<RB, false>(a, sh, nch, useDense, iter, nLin, last);
    } else {
        float d = 0.0f;
        for (uint32_t v = 1 + threadIdx.x; v < a.N; v += blockDim.x) {
            f3 pR, pT, aR, aT;
            vload(a, V_P, v, pR, pT);
            pcg_ap(a, v, nch, useDense, pR, pT, aR, aT);
            vstore(a, V_AP, v, aR, aT);
            d += dot3(pR, aR) + dot3(pT, aT);
        }
        const float pAp = block_sum(d, sh);
        const float rDotzOld = ctrlf(a.ctrl, K_RDOTZ);
        const float alpha = (pAp > FLOAT_EPSILON) ? rDotzOld / pAp : 0.0f;
        float b = 0.0f;
        for (uint32_t v = 1 + threadIdx.x; v < a.N; v += blockDim.x) {
            f3 dR, dT, pR, pT, rR, rT, aR, aT, mR, mT;
            vload(a, V_DELTA, v, dR, dT);
            vload(a, V_P, v, pR, pT);
            vload(a, V_R, v, rR, rT);
            vload(a, V_AP, v, aR, aT);
            vload(a, V_M, v, mR, mT);
            dR = dR + alpha * pR;
            dT = dT + alpha * pT;
            rR = rR - alpha * aR;
            rT = rT - alpha * aT;
            const f3 zR = mul3(mR, rR), zT = mul3(mT, rT);
            vstore(a, V_DELTA, v, dR, dT);
            vstore(a, V_R, v, rR, rT);
            vstore(a, V_Z, v, zR, zT);
            b += dot3(zR, rR) + dot3(zT, rT);
        }
        const float rDotzNew_ = block_sum(b, sh);
        const bool last_ = (iter == nLin - 1) || (a.earlyOut && fabsf(pAp) < 5e-7f);
        const float beta = (rDotzOld > FLOAT_EPSILON) ? rDotzNew_ / rDotzOld : 0.0f;
        for (uint32_t v = 1 + threadIdx.x; v < a.N; v += blockDim.x) {
            f3 zR, zT, pR, pT;
            vload(a, V_Z, v, zR, zT);
            vload(a, V_P, v, pR, pT);
            vstore(a, V_P, v, zR + beta * pR, zT + beta * pT);
            if (last_) {  // computeLieUpdate (LieDerivUtil.h:301-307)
                f3 dR, dT;
                vload(a, V_DELTA, v, dR, dT);
                f3 nr, nt;
                lie_update(dR, dT, mk3(a.rot[3 * v], a.rot[3 * v + 1], a.rot[3 * v + 2]),
                           mk3(a.trans[3 * v], a.trans[3 * v + 1], a.trans[3 * v + 2]), nr, nt);
                a.rot[3 * v] = nr.x; a.rot[3 * v + 1] = nr.y; a.rot[3 * v + 2] = nr.z;
                a.trans[3 * v] = nt.x; a.trans[3 * v + 1] = nt.y; a.trans[3 * v + 2] = nt.z;
            }
        }
        rDotzNew = rDotzNew_;
        last = last_;
    }
}

// One PCG iteration (PCGIteration, SolverBundling.cu:1024-1108) in one launch: every wave
// computes the sparse JtJp partial of its chunks; waves also apply the dense off-diagonal pair
// blocks. The last workgroup then sums each row's partials in chunk order, adds the dense diagonal
// block, does the global dot products and the alpha / beta updates (Kernel1b, Kernel2, Kernel3) and
// the Lie update on the exiting iteration.
__global__ __launch_bounds__(WG) void k_pcg(BA a, float wSparse, int iter, int nLin) {
    __shared__ float sh[WG];
    if (a.ctrl[K_GN_DONE] || a.ctrl[K_PCG_DONE]) return;
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    const int useDense = (int)a.ctrl[K_USE_DENSE];
    const uint32_t nch = (wSparse > 0.0f) ? a.ctrl[K_NCHUNK] : 0u;
    pcg_sparse_chunks<false>(a, wSparse, wave, nw, nch);
    if (useDense) pcg_dense_offdiag(a, wave, nw);
    if (!last_block_sharded(a.sync, 1u)) return;
    if (threadIdx.x < 9) a.sync[threadIdx.x * SYNC_LINE] = 0;  // counters of the next launch
    // ---- finisher (one workgroup): Kernel1b, Kernel2, host early-out test, Kernel3 ----
    float rDotzNew;
    bool last;
    pcg_finisher(a, sh, nch, useDense, iter, nLin, rDotzNew, last);
    if (threadIdx.x == 0) {
        a.ctrl[K_RDOTZ] = __float_as_uint(rDotzNew);
        a.ctrl[K_PCG_ITERS]++;
        if (last) a.ctrl[K_PCG_DONE] = 1;
        a.ctrl[K_TICKET] = 0;
    }
}

// Pair mode, per GN iteration after the exchange: one wave per image row v >= 1 sums its incident
// pairs (in partner order) into D_v (the diagonal block statistics), J^T F and the Jacobi
// preconditioner, then initialises the row as PCGInit does (evalMinusJTFDevice + PCGInit_Kernel1,
// SolverBundlingEquationsLie.h:63-148, SolverBundling.cu:755-794); the last workgroup sums r.z.
// Row v (one wave); lane 0 also keeps the row's pose as it was before the GN step (a.poseBak, the
// state pcg_recover restarts from)
__device__ void pair_init_row(const BA& a, float wSparse, uint32_t v, bool backup) {
    const uint32_t lane = lane_id();
    {
        const int e0 = a.rowPairStart[v], e1 = a.rowPairStart[v + 1];
        double d[DSTAT + 6];
#pragma unroll
        for (int q = 0; q < DSTAT + 6; q++) d[q] = 0.0;
        for (int k = e0 + (int)lane; k < e1; k += 64) {
            const int2 rp = a.rowPair[k];
            const bool vIsA = ((uint32_t)rp.y & PAIR_A_FLAG) != 0;
            const double* st = a.pstat + (size_t)rp.x * PSTAT;
            const double* qv = st + (vIsA ? 16 : 22);
            const double* sv = st + (vIsA ? 9 : 12);
            const double* su = st + (vIsA ? 12 : 9);
#pragma unroll
            for (int q = 0; q < 6; q++) d[q] += qv[q];
#pragma unroll
            for (int q = 0; q < 3; q++) d[6 + q] += sv[q];
            d[9] += st[15];
            // sum P_v x (P_v - P_u) = -/+ sum P_a x P_b, the antisymmetric part of M = sum P_b P_a^T
            const double sg = vIsA ? -1.0 : 1.0;
            d[10] += sg * (st[7] - st[5]);
            d[11] += sg * (st[2] - st[6]);
            d[12] += sg * (st[3] - st[1]);
#pragma unroll
            for (int q = 0; q < 3; q++) d[13 + q] += sv[q] - su[q];
        }
#pragma unroll
        for (int q = 0; q < DSTAT + 6; q++) d[q] = wave_sum_d(d[q]);
        if (lane == 0) {
            double* ds = a.dstat + (size_t)v * DSTAT;
#pragma unroll
            for (int q = 0; q < DSTAT; q += 2) *reinterpret_cast<double2*>(ds + q) = make_double2(d[q], d[q + 1]);
            const f3 rr = mk3((float)d[10], (float)d[11], (float)d[12]);
            const f3 rt = mk3((float)d[13], (float)d[14], (float)d[15]);
            // |dAlpha|^2, |dBeta|^2, |dGamma|^2 summed: (Qyy + Qzz, Qxx + Qzz, Qxx + Qyy)
            const f3 pr = mk3((float)(d[3] + d[5]), (float)(d[0] + d[5]), (float)(d[0] + d[3]));
            st_wt(&a.rzPart[v], init_row_cnt(a, v, rr, rt, pr, (float)d[9], wSparse, (int)a.ctrl[K_USE_DENSE]));
        }
        if (backup && lane < 6) a.poseBak[(size_t)v * 6 + lane] = lane < 3 ? a.rot[3 * v + lane] : a.trans[3 * v + lane - 3];
    }
}
// r.z summed over the rows by one workgroup (k_pair_init's last), PCG counters reset, p_0 = 0
__device__ void pair_init_finish(const BA& a, float* sh) {
    float s = 0.0f;
    for (uint32_t v = 1 + threadIdx.x; v < a.N; v += blockDim.x) s += ld_wtf(&a.rzPart[v]);
    s = block_sum(s, sh);
    if (threadIdx.x == 0) {
        a.ctrl[K_RDOTZ] = __float_as_uint(s);
        a.ctrl[K_TICKET] = 0;
        for (int w = 0; w < SYNC_WORDS; w += SYNC_LINE) a.sync[w] = 0;
        vstore(a, V_P, 0, mk3(0, 0, 0), mk3(0, 0, 0));  // image 0 is fixed: its p stays 0
    }
}
__global__ __launch_bounds__(WG) void k_pair_init(BA a, float wSparse) {
    __shared__ float sh[WG];
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = 1 + wave; v < a.N; v += nw) pair_init_row(a, wSparse, v, true);
    if (!last_block(&a.ctrl[K_TICKET])) return;
    if (threadIdx.x == 0) a.ctrl[K_PCG_ITERS0] = a.ctrl[K_PCG_ITERS];
    pair_init_finish(a, sh);
}

// Ap of row v (one wave), handed to the finisher write-through: k_pcg_pairs and pcg_recover
__device__ void pair_row_ap(const BA& a, float wSparse, uint32_t v, unsigned long long* stg) {
    const uint32_t lane = lane_id();
    (void)stg;
    {
        const int e0 = a.rowPairStart[v], e1 = a.rowPairStart[v + 1];
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); stg[0] = rtc() + (unsigned long long)(e0 & 0); }
#endif
        // the row's own p and image statistics, loaded beside the pair loop (lane 0 uses them)
        f3 pvR, pvT;
        vload(a, V_P, v, pvR, pvT);
        double dst[DSTAT];
#pragma unroll
        for (int q = 0; q < DSTAT; q++) dst[q] = a.dstat[(size_t)v * DSTAT + q];
        double o[6] = {0, 0, 0, 0, 0, 0};
        // two entries per lane per round (k and k + 64), every load of both issued before either is
        // used: one round of dependent loads (entry, then partner p + pair statistics) per 128 entries;
        // each lane still adds its entries in ascending k, so the sums equal the one-entry loop's
        for (int kb = e0; kb < e1; kb += 128) {
            const int k0 = kb + (int)lane, k1 = k0 + 64;
            const int2 rp0 = a.rowPair[min(k0, e1 - 1)], rp1 = a.rowPair[min(k1, e1 - 1)];
            const uint32_t u0 = (uint32_t)rp0.y & ~PAIR_A_FLAG, u1 = (uint32_t)rp1.y & ~PAIR_A_FLAG;
            f3 pr0, pt0, pr1, pt1;
            vload(a, V_P, u0, pr0, pt0);
            vload(a, V_P, u1, pr1, pt1);
            double st0[16], st1[16];
#pragma unroll
            for (int q = 0; q < 16; q += 2) {
                const double2 x0 = *reinterpret_cast<const double2*>(a.pstat + (size_t)rp0.x * PSTAT + q);
                const double2 x1 = *reinterpret_cast<const double2*>(a.pstat + (size_t)rp1.x * PSTAT + q);
                st0[q] = x0.x; st0[q + 1] = x0.y;
                st1[q] = x1.x; st1[q + 1] = x1.y;
            }
            if (k0 < e1 && u0 != 0) {  // p_0 = 0 (image 0 fixed)
                const double w[3] = {pr0.x, pr0.y, pr0.z}, t[3] = {pt0.x, pt0.y, pt0.z};
                double b[6];
                pair_block_apply(st0, ((uint32_t)rp0.y & PAIR_A_FLAG) != 0, w, t, b);
#pragma unroll
                for (int q = 0; q < 6; q++) o[q] += b[q];
            }
            if (k1 < e1 && u1 != 0) {
                const double w[3] = {pr1.x, pr1.y, pr1.z}, t[3] = {pt1.x, pt1.y, pt1.z};
                double b[6];
                pair_block_apply(st1, ((uint32_t)rp1.y & PAIR_A_FLAG) != 0, w, t, b);
#pragma unroll
                for (int q = 0; q < 6; q++) o[q] += b[q];
            }
        }
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) stg[1] = rtc() + (unsigned long long)(o[0] != o[0]);
#endif
#pragma unroll
        for (int q = 0; q < 6; q++) o[q] = wave_sum_d(o[q]);
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) stg[2] = rtc() + (unsigned long long)(o[5] != o[5]);
#endif
        if (lane == 0) {
            const f3 pr = pvR, pt = pvT;
            const double w[3] = {pr.x, pr.y, pr.z}, t[3] = {pt.x, pt.y, pt.z};
            double dp[6];
            diag_apply(dst, w, t, dp);
            const double ws = wSparse;
            float4* q = reinterpret_cast<float4*>(a.apPair + (size_t)v * 8);
            st_wt(q, make_float4((float)(ws * (dp[0] - o[0])), (float)(ws * (dp[1] - o[1])), (float)(ws * (dp[2] - o[2])), 0.0f));
            st_wt(q + 1, make_float4((float)(ws * (dp[3] - o[3])), (float)(ws * (dp[4] - o[4])), (float)(ws * (dp[5] - o[5])), 0.0f));
        }
    }
}

// Pair mode PCG iteration: one wave per row v >= 1, Ap_v = w (D_v p_v - sum_u B_vu p_u) in fp64 over
// the row's pairs (the same operator as applyJ / applyJT; no second w, SolverBundlingEquationsLie.h:
// 154-228), handed to the finisher write-through; then the finisher of k_pcg.
// RB: image rows per finisher thread held in registers (2: up to 513 images; 8: up to 2 049, the
// host picks it from the solve's image count; beyond, the finisher's multi-pass form)
template <int RB>
__global__ __launch_bounds__(WG) void k_pcg_pairs(BA a, float wSparse, int iter, int nLin) {
    __shared__ float sh[WG];
    if (a.ctrl[K_GN_DONE] || a.ctrl[K_PCG_DONE]) return;
#ifdef BF_PCG_TIMING
    const unsigned long long tStart = rtc();
    unsigned long long stg[3] = {0, 0, 0};
#endif
    const uint32_t lane = lane_id();
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t v = 1 + wave; v < a.N; v += nw) {
#ifdef BF_PCG_TIMING
        pair_row_ap(a, wSparse, v, stg);
#else
        pair_row_ap(a, wSparse, v, nullptr);
#endif
    }
    const int useDense = (int)a.ctrl[K_USE_DENSE];
    if (useDense) pcg_dense_offdiag(a, wave, nw);
#ifdef BF_PCG_TIMING
    if (threadIdx.x == 0) {
        atomicMin(&g_pcgT[iter & 1023][0], tStart);
        atomicMax(&g_pcgT[iter & 1023][1], rtc());
    }
#endif
    if (!last_block_sharded(a.sync, 1u)) return;
#ifdef BF_PCG_TIMING
    if (threadIdx.x == 0) {
        g_pcgT[iter & 1023][2] = rtc();
        unsigned long long* S = g_pcgS[iter & 1023];
        S[0] = tStart; S[1] = stg[0]; S[2] = stg[1]; S[3] = stg[2]; S[4] = g_pcgT[iter & 1023][2];
    }
#endif
    if (threadIdx.x < 9) a.sync[threadIdx.x * SYNC_LINE] = 0;  // counters of the next launch
    float rDotzNew;
    bool last;
    pcg_finisher<RB>(a, sh, 0u, useDense, iter, nLin, rDotzNew, last);
#ifdef BF_PCG_TIMING
    __syncthreads();
    if (threadIdx.x == 0) g_pcgT[iter & 1023][3] = rtc();
#endif
    if (threadIdx.x == 0) {
        a.ctrl[K_RDOTZ] = __float_as_uint(rDotzNew);
        a.ctrl[K_PCG_ITERS]++;
        if (last) a.ctrl[K_PCG_DONE] = 1;
        a.ctrl[K_TICKET] = 0;
    }
}

// Pair mode, all PCG iterations of one GN step in ONE launch (64 < N <= 2 WG + 1 images): the
// same arithmetic as k_pcg_pairs<2> + pcg_finish_regs<2> (bit-identical results), without a launch
// per iteration. Workgroup 0 is the finisher: its threads keep their rows' delta, r, M and p in
// registers across iterations. Workgroups 1.. are workers, one wave per image row, each holding its
// row's first PP_CPL x 64 pair entries and their pair statistics in registers across iterations.
// Per iteration the workers gather the partners' p (sc1 loads), apply the pair blocks in fp64 in the
// order of k_pcg_pairs, hand Ap_v over write-through (sc1, drained) and add to their shard's arrival
// counter; the finisher polls the 8 shards, runs Kernel1b / 2 / 3 (SolverBundling.cu:930-1022), stores
// p write-through (drained) and publishes the iteration on a flag word the workers poll: two hand-offs
// per iteration of MI355X_MICROARCH.md's first valid form, instead of a kernel boundary plus a
// last-workgroup election and two reloads of every vector. Every wait is bounded (2 s of s_memrealtime):
// a timeout sets result error bit 3 and releases every workgroup. The grid must be co-resident: the
// host launches it only when the occupancy query admits it with room to spare.
#ifndef BF_PCG_PRIO
#define BF_PCG_PRIO 2  // k_pcg_persist's wave priority (0: off)
#endif
#ifndef BF_PCG_PERSISTENT
#define BF_PCG_PERSISTENT 1  // 0: one k_pcg_pairs launch per PCG iteration (A/B builds)
#endif
constexpr int PP_CPL = 3;                 // cached entries per lane: rows up to 192 partner pairs stay in registers
constexpr uint32_t PP_SHADOW = 256;       // the workgroup without rows (see the workers)
constexpr int PP_OV = 4;                  // further entries per lane whose pair refs stay in registers (rows up to 448)
constexpr uint32_t PP_DONE = 0x80000000u; // flag bit: the PCG loop ended (last iteration or timeout)
constexpr uint32_t PP_ERR_TIMEOUT = 8u;   // K_ERROR bit 3 (BF_SOLVE_ERR_PCG_TIMEOUT)
constexpr uint32_t PP_RECOVERED = 16u;    // K_ERROR bit 4 (BF_SOLVE_PCG_RECOVERED): pcg_recover redid the step

// The finisher workgroup of k_pcg_persist: R image rows per thread (R = 2: up to 513 images, every
// vector in registers; R = 8: up to 2 049, p and r in registers, the preconditioner M in LDS (sM,
// [6][8 WG] floats), delta read and written in memory by the thread that owns the row and z recomputed
// from M r: the same operations in the same order, so the result matches the per-launch finisher's bit
// for bit; the kernel stays within 256 VGPRs, i.e. two workgroups per CU for a 501-workgroup grid). The
// dense term is taken by R = 2 only (the host routes larger dense steps to one launch per iteration).
// The workers' gathers of p: two 16-B buffer loads per row with the sc1 (agent-coherent) cache policy
// — the policy of the agent-scope atomic loads in vload_t<true>, at half the L2 requests (four 8-B
// atomics per row). Tearing cannot matter: p is complete (drained, then flagged) before any gather.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t p_rsrc(const BA& a) {
    return __builtin_amdgcn_make_buffer_rsrc(a.vec + (size_t)V_P * a.maxN * 8, (short)0, (int)(a.maxN * 32u), 0x00020000);
}
__device__ __forceinline__ void pload_coh(__amdgpu_buffer_rsrc_t rs, uint32_t u, f3& r, f3& t) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, u * 32u, 0, 16);  // 16: sc1
    const auto y = __builtin_amdgcn_raw_buffer_load_b128(rs, u * 32u + 16u, 0, 16);
    r = mk3(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]));
    t = mk3(__uint_as_float(y[0]), __uint_as_float(y[1]), __uint_as_float(y[2]));
}
// the finisher's publication of p: 16-B write-through (sc1) stores, [r | 0][t | 0] (the
// MI355X_MICROARCH.md hand-off table: 16-B sc1 stores ~ plain, 8-B ones 2.7x the time per byte)
__device__ __forceinline__ void pstore_coh(__amdgpu_buffer_rsrc_t rs, uint32_t u, f3 r, f3 t) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const u4 x = {__float_as_uint(r.x), __float_as_uint(r.y), __float_as_uint(r.z), 0u};
    const u4 y = {__float_as_uint(t.x), __float_as_uint(t.y), __float_as_uint(t.z), 0u};
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, u * 32u, 0, 16);  // 16: sc1
    __builtin_amdgcn_raw_buffer_store_b128(y, rs, u * 32u + 16u, 0, 16);
}

// The p hand-off of sparse solves, without the finisher's drain and barrier: each 16-B half carries its
// iteration's tag in the pad word (16-B sc1 halves are observed untorn, MI355X_MICROARCH.md R2), the
// flag only says when to start gathering, and a worker re-gathers a half whose tag is stale (standalone
// K = 500 GN iteration 1.016 / 1.050 -> 1.008 / 1.003 ms, A/B pairs; BF_PCG_PTAG=0 builds the drained
// form, which the dense solves keep: their off-diagonal products gather p untagged).
#ifndef BF_PCG_PTAG
#define BF_PCG_PTAG 1
#endif
__device__ __forceinline__ void pstore_tag(__amdgpu_buffer_rsrc_t rs, uint32_t u, f3 r, f3 t, uint32_t tag) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const u4 x = {__float_as_uint(r.x), __float_as_uint(r.y), __float_as_uint(r.z), tag};
    const u4 y = {__float_as_uint(t.x), __float_as_uint(t.y), __float_as_uint(t.z), tag};
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, u * 32u, 0, 16);  // 16: sc1
    __builtin_amdgcn_raw_buffer_store_b128(y, rs, u * 32u + 16u, 0, 16);
}
// gathers p of row u; true when both halves carry `tag`
__device__ __forceinline__ bool pload_tag(__amdgpu_buffer_rsrc_t rs, uint32_t u, f3& r, f3& t, uint32_t tag) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, u * 32u, 0, 16);  // 16: sc1
    const auto y = __builtin_amdgcn_raw_buffer_load_b128(rs, u * 32u + 16u, 0, 16);
    r = mk3(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]));
    t = mk3(__uint_as_float(y[0]), __uint_as_float(y[1]), __uint_as_float(y[2]));
    return x[3] == tag && y[3] == tag;
}
// pload_tag until the tag matches (check = false: p of an earlier launch, no tag); a timeout sets the
// error bit and leaves the last values
__device__ __forceinline__ void pload_wait(const BA& a, __amdgpu_buffer_rsrc_t rs, uint32_t u, f3& r, f3& t, uint32_t tag, bool check,
                                           unsigned long long t0) {
    while (!pload_tag(rs, u, r, t, tag) && check) {
        if (pp_timed_out(t0, a.spinTicks)) { atomicOr(&a.ctrl[K_ERROR], PP_ERR_TIMEOUT); break; }
        __builtin_amdgcn_s_sleep(1);
    }
}
// Row q of this finisher thread, opaque to the compiler at every use: otherwise the addresses of all
// R rows in all five vectors are hoisted out of the PCG loop and held in registers (R = 8: ~100 VGPRs).
__device__ __forceinline__ uint32_t fin_row(int q) {
    uint32_t v = 1 + threadIdx.x + q * WG;
    asm volatile("" : "+v"(v));
    return v;
}
template <int R>
__device__ void pcg_persist_finisher(const BA& a, float* sh, float* sM, int useDense, int nLin, uint32_t tagBase,
                                     uint32_t* flag, unsigned long long t0) {
    constexpr bool REGS = R <= 2;
    constexpr int SMR = R * WG;  // sM row stride (R > 2)
    f3 pR[R], pT[R], rR[R], rT[R];
    f3 mR[REGS ? R : 1], mT[REGS ? R : 1];
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t v = fin_row(q);
        if (v < a.N) {
            vload(a, V_P, v, pR[q], pT[q]);
            vload(a, V_R, v, rR[q], rT[q]);
            if (REGS) {
                vload(a, V_M, v, mR[REGS ? q : 0], mT[REGS ? q : 0]);
            } else {
                f3 mr, mt;
                vload(a, V_M, v, mr, mt);
                const int i = (int)threadIdx.x + q * WG;
                sM[i] = mr.x; sM[SMR + i] = mr.y; sM[2 * SMR + i] = mr.z;
                sM[3 * SMR + i] = mt.x; sM[4 * SMR + i] = mt.y; sM[5 * SMR + i] = mt.z;
            }
        }
    }
    // M of row q (registers, or this thread's own LDS slots)
    auto getM = [&](int q, f3& mr, f3& mt) {
        if (REGS) { mr = mR[REGS ? q : 0]; mt = mT[REGS ? q : 0]; }
        else {
            const int i = (int)threadIdx.x + q * WG;
            mr = mk3(sM[i], sM[SMR + i], sM[2 * SMR + i]);
            mt = mk3(sM[3 * SMR + i], sM[4 * SMR + i], sM[5 * SMR + i]);
        }
    };
    float rz = ctrlf(a.ctrl, K_RDOTZ);
    const __amdgpu_buffer_rsrc_t prs = p_rsrc(a);
    int it = 0;
    bool last = false;
    float lastAlpha = 0.0f;
    for (;; it++) {
        // the rows' Ap granules (sparse part, then the dense off-diagonal products), all polled at once
        constexpr int NG = REGS ? 2 * R : R;
        const uint2* g[NG];
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t v = fin_row(q);
            const uint32_t vv = v < a.N ? v : 1u;  // image 1's granules: written every iteration (N >= 2)
            g[q] = a.aGran + (size_t)vv * 6;
            if (REGS) g[(R + q) % NG] = useDense ? a.aGran + ((size_t)a.maxN + vv) * 6 : g[q];
        }
        float x[NG][6];
        int ok;
        if (REGS && useDense) ok = gran_rows<NG>(g, tagBase + (uint32_t)it + 1u, x, t0, a.spinTicks);
        else if (REGS) ok = gran_rows<R>(g, tagBase + (uint32_t)it + 1u, x, t0, a.spinTicks);  // no dense granules to poll
        else {  // R = 8: two halves of four rows (half the in-flight registers)
            constexpr int H = NG / 2 > 0 ? NG / 2 : 1;
            ok = gran_rows<H>(g, tagBase + (uint32_t)it + 1u, x, t0, a.spinTicks);
            if (ok > 0) ok = gran_rows<H>(g + H, tagBase + (uint32_t)it + 1u, x + H, t0, a.spinTicks);
        }
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) g_pcgT[it & 1023][2] = rtc();
#endif
        float d = 0.0f;
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t v = fin_row(q);
            if (v < a.N) {  // pcg_ap's order of additions; x[q] becomes Ap of the row
                f3 aR = mk3(x[q][0], x[q][1], x[q][2]), aT = mk3(x[q][3], x[q][4], x[q][5]);
                if (REGS && useDense) {  // diagonal block [trans | rot] x [pTrans | pRot], then the off-diagonal products
                    const float* D = a.diag + (size_t)v * 36;
                    const float pv[6] = {pT[q].x, pT[q].y, pT[q].z, pR[q].x, pR[q].y, pR[q].z};
                    float o6[6];
                    for (int r = 0; r < 6; r++) {
                        float sm = 0.0f;
                        for (int c = 0; c < 6; c++) sm += D[r * 6 + c] * pv[c];
                        o6[r] = sm;
                    }
                    aT = aT + mk3(o6[0], o6[1], o6[2]);
                    aR = aR + mk3(o6[3], o6[4], o6[5]);
                    aT = aT + mk3(x[(R + q) % NG][0], x[(R + q) % NG][1], x[(R + q) % NG][2]);
                    aR = aR + mk3(x[(R + q) % NG][3], x[(R + q) % NG][4], x[(R + q) % NG][5]);
                }
                x[q][0] = aR.x; x[q][1] = aR.y; x[q][2] = aR.z;
                x[q][3] = aT.x; x[q][4] = aT.y; x[q][5] = aT.z;
                d += dot3(pR[q], aR) + dot3(pT[q], aT);
            }
        }
        // pAp and the timeout vote in one reduction (block_sum's order; the vote rides in the same pass)
        float pAp;
        {
            const float wsum = wave_sum(d);
            const bool wok = __all(ok > 0);
            if ((threadIdx.x & 63) == 0) { sh[threadIdx.x >> 6] = wsum; sh[WG / 64 + (threadIdx.x >> 6)] = wok ? 1.0f : 0.0f; }
            __syncthreads();
            float r = 0.0f;
            bool all = true;
            for (uint32_t w = 0; w < WG / 64; w++) { r += sh[w]; all = all && sh[WG / 64 + w] != 0.0f; }
            // no trailing barrier: sh[0, 8) is rewritten next iteration, after every wave passed the rz barrier
            if (!all) break;  // timeout: released below
            pAp = r;
        }
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) g_pcgS[it & 1023][0] = rtc();
#endif
        const float alpha = (pAp > FLOAT_EPSILON) ? rz / pAp : 0.0f;
        // delta += alpha p is the workers' (each on its own row, from the p it gathered): alpha goes out
        // in the flag word
        lastAlpha = alpha;
        float b = 0.0f;
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t v = fin_row(q);
            if (v < a.N) {
                const f3 aR = mk3(x[q][0], x[q][1], x[q][2]), aT = mk3(x[q][3], x[q][4], x[q][5]);
                f3 mr, mt;
                getM(q, mr, mt);
                rR[q] = rR[q] - alpha * aR;
                rT[q] = rT[q] - alpha * aT;
                const f3 zR = mul3(mr, rR[q]), zT = mul3(mt, rT[q]);
                b += dot3(zR, rR[q]) + dot3(zT, rT[q]);
            }
        }
        float rzNew;
        {   // block_sum's order in sh[16, 20): its next writer is behind the next iteration's pAp barrier
            const float wsum = wave_sum(b);
            if ((threadIdx.x & 63) == 0) sh[2 * (WG / 64) + (threadIdx.x >> 6)] = wsum;
            __syncthreads();
            float r = 0.0f;
            for (uint32_t w = 0; w < WG / 64; w++) r += sh[2 * (WG / 64) + w];
            rzNew = r;
        }
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) g_pcgS[it & 1023][1] = rtc();
#endif
        last = (it == nLin - 1) || (a.earlyOut && fabsf(pAp) < 5e-7f);
        const float beta = (rz > FLOAT_EPSILON) ? rzNew / rz : 0.0f;
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t v = fin_row(q);
            if (v < a.N) {
                f3 mr, mt;
                getM(q, mr, mt);
                const f3 zR = mul3(mr, rR[q]), zT = mul3(mt, rT[q]);
                pR[q] = zR + beta * pR[q];
                pT[q] = zT + beta * pT[q];
#if BF_PCG_PTAG
                if (!last) pstore_tag(prs, v, pR[q], pT[q], tagBase + (uint32_t)it + 2u);  // iteration it + 1's p
#else
                if (!last) pstore_coh(prs, v, pR[q], pT[q]);  // the workers' next gathers
#endif
            }
        }
        rz = rzNew;
        if (last) break;
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) g_pcgS[it & 1023][2] = rtc();
#endif
        // p is read by ~N x 92 gathers: published write-through, drained, then one flag word
        // (p as polled granules ran 20 % slower: the workers' polls swamp the hand-off)
        if (!BF_PCG_PTAG || useDense) {  // (the dense products gather p untagged: drained hand-off)
            drain_stores();
            __syncthreads();
        }
        if (threadIdx.x < PP_NFLAG) st_wt64(flag + threadIdx.x * PP_FLAG_STRIDE, (uint32_t)(it + 1), __float_as_uint(lastAlpha));  // one instruction
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0) g_pcgT[it & 1023][3] = rtc();
#endif
    }
    // final state (later launches read it plainly across the kernel boundary); delta and the Lie
    // update are the workers'
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t v = fin_row(q);
        if (v < a.N) {
            vstore(a, V_R, v, rR[q], rT[q]);
            vstore(a, V_P, v, pR[q], pT[q]);
        }
    }
    if (threadIdx.x == 0) {
        if (!last) atomicOr(&a.ctrl[K_ERROR], PP_ERR_TIMEOUT);
        a.ctrl[K_RDOTZ] = __float_as_uint(rz);
        a.ctrl[K_PCG_ITERS] += (uint32_t)(it + (last ? 1 : 0));
        a.ctrl[K_PCG_DONE] = 1;
    }
    if (threadIdx.x < 64) {  // wave 0: the final flag carries the last iteration's alpha (valid when last)
        drain_stores();
        if (threadIdx.x < PP_NFLAG)
            st_wt64(flag + threadIdx.x * PP_FLAG_STRIDE, PP_DONE | (uint32_t)(it + (last ? 1 : 0)), __float_as_uint(lastAlpha));
    }
}

// The finisher of wide sparse solves (514..2 017 images) as PP_NF workgroups instead of one with 8 rows per
// thread (whose serial per-row work and polls were 8 of the 11.7 us of a K = 2 001 iteration,
// profiles/r8h_pcg_phase_timing.txt): workgroup g owns rows 1 + t + (2g + q) WG, q = 0, 1, in registers (the
// R = 2 form), and the two dot products go through a hand-off: each workgroup publishes its block partial
// as a tagged granule, every workgroup adds the PP_NF partials in workgroup order (the grouped order of
// pcg_finish_regs<8>, so the result equals the per-launch solve's bit for bit). Workgroup 0 sets the
// flag (p halves carry their iteration's tag; workers re-gather a stale one) and the control words.
constexpr int PP_NF = FIN_GROUPS;
// the rows the wide finishers own, 1 .. 2 PP_NF WG: the host's wide-route bound on numImages (Solver::solve)
static_assert(2 * PP_NF * WG + 1 == 2049, "wide persistent finishers cover rows 1..2048");
constexpr int SH_FX = 64;  // the finisher's LDS slots of the exchanged totals
__device__ __forceinline__ float fx_exchange(const BA& a, float* sh, int kind, uint32_t g, float S, uint32_t tag,
                                             unsigned long long t0, bool& ok) {
    if (threadIdx.x == 0) gran_store(a.fxGran + kind * 8 + g, S, tag);
    if (threadIdx.x < 64) {
        const uint32_t l = threadIdx.x;
        uint64_t x = 0;
        bool got = l >= (uint32_t)PP_NF;
        for (;;) {
            if (!got) {
                x = gran_load(a.fxGran + kind * 8 + l);
                got = (uint32_t)(x >> 32) == tag;
            }
            if (__all(got)) break;
            if (pp_timed_out(t0, a.spinTicks)) break;
            __builtin_amdgcn_s_sleep(1);
        }
        const bool all = __all(got);
        float tot = 0.0f;
#pragma unroll
        for (int k = 0; k < PP_NF; k++) tot += __shfl(__uint_as_float((uint32_t)x), k);  // workgroup order
        if (l == 0) {
            sh[SH_FX + 2 * kind] = tot;
            sh[SH_FX + 2 * kind + 1] = all ? 1.0f : 0.0f;
        }
    }
    __syncthreads();
    ok = sh[SH_FX + 2 * kind + 1] != 0.0f;
    return sh[SH_FX + 2 * kind];
}
__device__ __forceinline__ uint32_t fin_row_g(int q, uint32_t g) {
    uint32_t v = 1 + threadIdx.x + (2 * g + (uint32_t)q) * WG;
    asm volatile("" : "+v"(v));
    return v;
}
__device__ void pcg_persist_finisher_x4(const BA& a, float* sh, int nLin, uint32_t tagBase, uint32_t* flag, unsigned long long t0,
                                        uint32_t g) {
    constexpr int R = 2;
    f3 pR[R], pT[R], rR[R], rT[R], mR[R], mT[R];
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t v = fin_row_g(q, g);
        if (v < a.N) {
            vload(a, V_P, v, pR[q], pT[q]);
            vload(a, V_R, v, rR[q], rT[q]);
            vload(a, V_M, v, mR[q], mT[q]);
        }
    }
    float rz = ctrlf(a.ctrl, K_RDOTZ);
    const __amdgpu_buffer_rsrc_t prs = p_rsrc(a);
    int it = 0;
    bool last = false;
    float lastAlpha = 0.0f;
    for (;; it++) {
        const uint32_t tag = tagBase + (uint32_t)it + 1u;
        const uint2* gp[R];
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t v = fin_row_g(q, g);
            gp[q] = a.aGran + (size_t)(v < a.N ? v : 1u) * 6;  // image 1's granules: written every iteration
        }
        float x[R][6];
        const int got = gran_rows<R>(gp, tag, x, t0, a.spinTicks);
#ifdef BF_PCG_TIMING
        if (g == 0 && threadIdx.x == 0) g_pcgT[it & 1023][2] = rtc();
#endif
        float d = 0.0f;
#pragma unroll
        for (int q = 0; q < R; q++)
            if (fin_row_g(q, g) < a.N) d += dot3(pR[q], mk3(x[q][0], x[q][1], x[q][2])) + dot3(pT[q], mk3(x[q][3], x[q][4], x[q][5]));
        float S;
        bool all = true;
        {   // block_sum's order, with the timeout vote in the same pass
            const float wsum = wave_sum(d);
            const bool wok = __all(got > 0);
            if ((threadIdx.x & 63) == 0) { sh[threadIdx.x >> 6] = wsum; sh[WG / 64 + (threadIdx.x >> 6)] = wok ? 1.0f : 0.0f; }
            __syncthreads();
            S = 0.0f;
            for (uint32_t w = 0; w < WG / 64; w++) { S += sh[w]; all = all && sh[WG / 64 + w] != 0.0f; }
        }
        if (!all) break;
        bool ok;
        const float pAp = fx_exchange(a, sh, 0, g, S, tag, t0, ok);
        if (!ok) break;
#ifdef BF_PCG_TIMING
        if (g == 0 && threadIdx.x == 0) g_pcgS[it & 1023][0] = rtc();
#endif
        const float alpha = (pAp > FLOAT_EPSILON) ? rz / pAp : 0.0f;
        lastAlpha = alpha;
        float b = 0.0f;
#pragma unroll
        for (int q = 0; q < R; q++) {
            if (fin_row_g(q, g) < a.N) {
                rR[q] = rR[q] - alpha * mk3(x[q][0], x[q][1], x[q][2]);
                rT[q] = rT[q] - alpha * mk3(x[q][3], x[q][4], x[q][5]);
                const f3 zR = mul3(mR[q], rR[q]), zT = mul3(mT[q], rT[q]);
                b += dot3(zR, rR[q]) + dot3(zT, rT[q]);
            }
        }
        float S2;
        {
            const float wsum = wave_sum(b);
            if ((threadIdx.x & 63) == 0) sh[2 * (WG / 64) + (threadIdx.x >> 6)] = wsum;
            __syncthreads();
            S2 = 0.0f;
            for (uint32_t w = 0; w < WG / 64; w++) S2 += sh[2 * (WG / 64) + w];
        }
        const float rzNew = fx_exchange(a, sh, 1, g, S2, tag, t0, ok);
        if (!ok) break;
#ifdef BF_PCG_TIMING
        if (g == 0 && threadIdx.x == 0) g_pcgS[it & 1023][1] = rtc();
#endif
        last = (it == nLin - 1) || (a.earlyOut && fabsf(pAp) < 5e-7f);
        const float beta = (rz > FLOAT_EPSILON) ? rzNew / rz : 0.0f;
#pragma unroll
        for (int q = 0; q < R; q++) {
            const uint32_t v = fin_row_g(q, g);
            if (v < a.N) {
                const f3 zR = mul3(mR[q], rR[q]), zT = mul3(mT[q], rT[q]);
                pR[q] = zR + beta * pR[q];
                pT[q] = zT + beta * pT[q];
                if (!last) pstore_tag(prs, v, pR[q], pT[q], tagBase + (uint32_t)it + 2u);  // iteration it + 1's p
            }
        }
        rz = rzNew;
        if (last) break;
#ifdef BF_PCG_TIMING
        if (g == 0 && threadIdx.x == 0) g_pcgS[it & 1023][2] = rtc();
#endif
        // the flag only says when to start gathering: the p halves of the other finishers' rows carry
        // their tag, and a worker re-gathers a stale one
        if (g == 0 && threadIdx.x < PP_NFLAG) st_wt64(flag + threadIdx.x * PP_FLAG_STRIDE, (uint32_t)(it + 1), __float_as_uint(lastAlpha));
#ifdef BF_PCG_TIMING
        if (g == 0 && threadIdx.x == 0) g_pcgT[it & 1023][3] = rtc();
#endif
    }
#pragma unroll
    for (int q = 0; q < R; q++) {
        const uint32_t v = fin_row_g(q, g);
        if (v < a.N) {
            vstore(a, V_R, v, rR[q], rT[q]);
            vstore(a, V_P, v, pR[q], pT[q]);
        }
    }
    if (threadIdx.x == 0) {
        if (!last) atomicOr(&a.ctrl[K_ERROR], PP_ERR_TIMEOUT);
        if (g == 0) {
            a.ctrl[K_RDOTZ] = __float_as_uint(rz);
            a.ctrl[K_PCG_ITERS] += (uint32_t)(it + (last ? 1 : 0));
            a.ctrl[K_PCG_DONE] = 1;
        }
    }
    if (g == 0 && threadIdx.x < 64) {
        drain_stores();
        if (threadIdx.x < PP_NFLAG)
            st_wt64(flag + threadIdx.x * PP_FLAG_STRIDE, PP_DONE | (uint32_t)(it + (last ? 1 : 0)), __float_as_uint(lastAlpha));
    }
}

// NF finisher workgroups: 1 (the R-rows-per-thread finisher) or PP_NF (pcg_persist_finisher_x4, R = 2)
template <int R, int NF = 1>
__global__ __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(2))) void k_pcg_persist(BA a, float wSparse, int nLin, uint32_t epoch) {
    __shared__ float sh[WG];
    __shared__ float sM[R > 2 ? 6 * R * WG : 1];  // the R = 8 finisher's preconditioner (48 KB)
    __shared__ double sD[WG / 64][DSTAT];          // each worker wave's image statistics
    if (a.ctrl[K_GN_DONE] || a.ctrl[K_PCG_DONE]) return;  // uniform over the grid (set by earlier launches)
    const uint32_t lane = lane_id();
#if BF_PCG_PRIO
    // above the voxel pass's waves on the same CU (its op steps run at 1): an iteration's critical path is
    // this kernel's compute between hand-offs, and its waits sleep (s_sleep), so the raise costs the voxel
    // pass little: in-loop time per PCG iteration 7.67 -> 6.43 us (1.46x -> 1.23x standalone), frame rate
    // 1 576 -> 1 587 at the driver workload (profiles/r11_prio_ab.txt)
    __builtin_amdgcn_s_setprio(BF_PCG_PRIO);
#endif
    const int useDense = (int)a.ctrl[K_USE_DENSE];
    const unsigned long long t0 = rtc();
    uint32_t* flag = &a.sync[SYNC_FLAGR];
    const uint32_t tagBase = epoch << 8;  // iteration it's Ap granules carry tagBase + it + 1
    if (blockIdx.x < NF) {
        if (NF == 1) pcg_persist_finisher<R>(a, sh, sM, useDense, nLin, tagBase, flag, t0);
        else pcg_persist_finisher_x4(a, sh, nLin, tagBase, flag, t0, blockIdx.x);
        return;
    }
    const uint32_t* myFlag = flag + ((blockIdx.x * (WG / 64) + (threadIdx.x >> 6)) % PP_NFLAG) * PP_FLAG_STRIDE;
    // ---- workers: one wave per row ----
    // Workgroup PP_SHADOW is dispatched onto the finisher's CU (256 CUs, round-robin) and holds no rows:
    // there, the finisher's granule polls held its rows' gathers up 2.4x (8 us of the 3.4 us others took)
    // (the NF workgroups dispatched onto the finishers' CUs hold none)
    const bool shadow = blockIdx.x >= PP_SHADOW && blockIdx.x < PP_SHADOW + NF;
    const uint32_t wb = blockIdx.x - NF - (blockIdx.x >= PP_SHADOW + NF ? NF : 0);
    const uint32_t v = 1 + wb * (WG / 64) + (threadIdx.x >> 6);
    const bool hasRow = !shadow && v < a.N;
    f3 dlR = mk3(0, 0, 0), dlT = dlR, pvR = dlR, pvT = dlR;  // the row's delta (every lane), the p it gathered
    int e0 = 0, e1 = 0;
    int2 rp[PP_CPL], rq[PP_OV];
    double st[PP_CPL][16];
    double* dst = sD[threadIdx.x >> 6];
    if (hasRow) {
        e0 = a.rowPairStart[v];
        e1 = a.rowPairStart[v + 1];
#pragma unroll
        for (int c = 0; c < PP_CPL; c++) {
            const int k = e0 + (int)lane + 64 * c;
            rp[c] = k < e1 ? a.rowPair[k] : make_int2(0, (int)v);  // idle lanes gather the wave's own row, not one hot row 0
        }
#pragma unroll
        for (int c = 0; c < PP_OV; c++) {
            const int k = e0 + (int)lane + 64 * (PP_CPL + c);
            rq[c] = k < e1 ? a.rowPair[k] : make_int2(0, (int)v);
        }
#pragma unroll
        for (int c = 0; c < PP_CPL; c++) {
            const bool ok = e0 + (int)lane + 64 * c < e1;
#pragma unroll
            for (int q = 0; q < 16; q += 2) {
                const double2 x = ok ? *reinterpret_cast<const double2*>(a.pstat + (size_t)rp[c].x * PSTAT + q) : make_double2(0.0, 0.0);
                st[c][q] = x.x;
                st[c][q + 1] = x.y;
            }
        }
        if (lane < DSTAT) dst[lane] = a.dstat[(size_t)v * DSTAT + lane];
        vload(a, V_DELTA, v, dlR, dlT);
    }
    __syncthreads();
    if (!hasRow) return;  // the row-less waves (the shadow workgroup, rows past N) have nothing to wait for
    const __amdgpu_buffer_rsrc_t prs = p_rsrc(a);
    for (uint32_t it = 0;; it++) {
        if (hasRow) {
            // p of iteration it (the previous launch's, or the finisher's write-through stores)
            f3 pr[PP_CPL], pt[PP_CPL];
            const uint32_t tag = tagBase + it + 1u;
#if BF_PCG_PTAG
            {   // every gather in flight at once, then all of them again while any is stale (rows u = 0,
                // whose p is never written, and p of an earlier launch, it = 0, carry no tag)
                const bool chk = it > 0 && !useDense;
                for (;;) {
                    bool ok = pload_tag(prs, v, pvR, pvT, tag) || !chk;
#pragma unroll
                    for (int c = 0; c < PP_CPL; c++) {
                        const uint32_t u = (uint32_t)rp[c].y & ~PAIR_A_FLAG;
                        ok = (pload_tag(prs, u, pr[c], pt[c], tag) || !chk || u == 0) && ok;
                    }
                    if (ok) break;
                    if (pp_timed_out(t0, a.spinTicks)) { atomicOr(&a.ctrl[K_ERROR], PP_ERR_TIMEOUT); break; }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
#else
#pragma unroll
            for (int c = 0; c < PP_CPL; c++) pload_coh(prs, (uint32_t)rp[c].y & ~PAIR_A_FLAG, pr[c], pt[c]);
            pload_coh(prs, v, pvR, pvT);
#endif
            double o[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int c = 0; c < PP_CPL; c++) {
                const uint32_t u = (uint32_t)rp[c].y & ~PAIR_A_FLAG;
                if (e0 + (int)lane + 64 * c < e1 && u != 0) {  // p_0 = 0 (image 0 fixed)
                    const double w[3] = {pr[c].x, pr[c].y, pr[c].z}, t[3] = {pt[c].x, pt[c].y, pt[c].z};
                    double bb[6];
                    pair_block_apply(st[c], ((uint32_t)rp[c].y & PAIR_A_FLAG) != 0, w, t, bb);
#pragma unroll
                    for (int q = 0; q < 6; q++) o[q] += bb[q];
                }
            }
            // entries beyond the cached ones (rows with more than PP_CPL x 64 partners): the next PP_OV
            // per lane with their pair refs in registers (one dependent load round fewer), then from memory
#pragma unroll
            for (int c = 0; c < PP_OV; c++) {
                if (e0 + (int)lane + 64 * (PP_CPL + c) >= e1) break;
                const uint32_t u = (uint32_t)rq[c].y & ~PAIR_A_FLAG;
                if (u == 0) continue;
                f3 qr, qt;
#if BF_PCG_PTAG
                pload_wait(a, prs, u, qr, qt, tag, it > 0 && !useDense, t0);
#else
                pload_coh(prs, u, qr, qt);
#endif
                const double w[3] = {qr.x, qr.y, qr.z}, t[3] = {qt.x, qt.y, qt.z};
                double bb[6];
                // the pair's statistics address formed here, each iteration: hoisted out of the loop it was spilled
                // (255 VGPRs) and reloaded from scratch every iteration
                int px = rq[c].x;
                asm volatile("" : "+v"(px));
                pair_block_apply(a.pstat + (size_t)px * PSTAT, ((uint32_t)rq[c].y & PAIR_A_FLAG) != 0, w, t, bb);
#pragma unroll
                for (int q = 0; q < 6; q++) o[q] += bb[q];
            }
            for (int k = e0 + (int)lane + 64 * (PP_CPL + PP_OV); k < e1; k += 64) {
                const int2 r2 = a.rowPair[k];
                const uint32_t u = (uint32_t)r2.y & ~PAIR_A_FLAG;
                if (u == 0) continue;
                f3 qr, qt;
#if BF_PCG_PTAG
                pload_wait(a, prs, u, qr, qt, tag, it > 0 && !useDense, t0);
#else
                pload_coh(prs, u, qr, qt);
#endif
                const double w[3] = {qr.x, qr.y, qr.z}, t[3] = {qt.x, qt.y, qt.z};
                double bb[6];
                pair_block_apply(a.pstat + (size_t)r2.x * PSTAT, ((uint32_t)r2.y & PAIR_A_FLAG) != 0, w, t, bb);
#pragma unroll
                for (int q = 0; q < 6; q++) o[q] += bb[q];
            }
#pragma unroll
            for (int q = 0; q < 6; q++) o[q] = wave_sum_d(o[q]);
            if (lane < 6) {  // Ap_v = w (D_v p_v - sum_u B_vu p_u): one granule per lane, [rot | trans]
                const double w[3] = {pvR.x, pvR.y, pvR.z}, t[3] = {pvT.x, pvT.y, pvT.z};
                double dp[6];
                diag_apply(dst, w, t, dp);
                const double ws = wSparse;
                float y = 0.0f;
#pragma unroll
                for (int q = 0; q < 6; q++)
                    if ((int)lane == q) y = (float)(ws * (dp[q] - o[q]));
                gran_store(a.aGran + (size_t)v * 6 + lane, y, tag);
            }
            if (useDense) pcg_dense_offdiag_row<true>(a, v, tag);
        }
        // every wave polls its own flag replica (no workgroup barrier per iteration): one load per poll
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0 && it < 64 && blockIdx.x < 1024) g_pcgW[it][blockIdx.x][1] = rtc();  // plain per-WG stamps
#endif
        uint32_t f, fa = 0;
        for (;;) {
            const uint64_t fw = ld_wt64(myFlag);
            f = __builtin_amdgcn_readfirstlane((uint32_t)fw);
            fa = __builtin_amdgcn_readfirstlane((uint32_t)(fw >> 32));
            if ((f & PP_DONE) || f >= it + 1) break;
            if (pp_timed_out(t0, a.spinTicks)) { f = PP_DONE; break; }
            __builtin_amdgcn_s_sleep(1);
        }
#ifdef BF_PCG_TIMING
        if (threadIdx.x == 0 && !(f & PP_DONE) && it + 1 < 64 && blockIdx.x < 1024) g_pcgW[it + 1][blockIdx.x][0] = rtc();
#endif
        // alpha of this iteration, in the flag word (PP_DONE carries how many iterations ran: the
        // flag seen here is exactly iteration it's, as the finisher's next one needs this row's Ap)
        const bool haveAlpha = !(f & PP_DONE) || (f & ~PP_DONE) > it;
        if (hasRow && haveAlpha) {  // delta += alpha p (the finisher's order of operations)
            const float alpha = __uint_as_float(fa);
            dlR = dlR + alpha * pvR;
            dlT = dlT + alpha * pvT;
        }
        if (f & PP_DONE) {
            if (hasRow && lane == 0) {
                vstore(a, V_DELTA, v, dlR, dlT);
                if (haveAlpha && (f & PP_DONE)) {  // the PCG loop ended normally: computeLieUpdate (LieDerivUtil.h:301-307)
                    f3 nr, nt;
                    lie_update(dlR, dlT, mk3(a.rot[3 * v], a.rot[3 * v + 1], a.rot[3 * v + 2]),
                               mk3(a.trans[3 * v], a.trans[3 * v + 1], a.trans[3 * v + 2]), nr, nt);
                    a.rot[3 * v] = nr.x; a.rot[3 * v + 1] = nr.y; a.rot[3 * v + 2] = nr.z;
                    a.trans[3 * v] = nt.x; a.trans[3 * v + 1] = nt.y; a.trans[3 * v + 2] = nt.z;
                }
            }
            return;
        }
    }
}

// Inside the k_gn_end that follows every k_pcg_persist launch (one workgroup; a uniform test of the
// error word unless the launch timed out): a persistent launch that timed out (a hand-off never arrived, e.g. the grid was not
// co-resident) redoes the GN step's PCG here, from the state k_pair_init left: the poses it saved are
// restored (the timed-out launch may have applied a partial Lie update), the rows are initialised
// again, and every PCG iteration runs as k_pcg_pairs<RB> + its finisher would, in one workgroup (the
// row order of the per-row work does not enter any sum, and the finisher is the same code), so the
// step's result is bit-identical to BFSolverOptions.pcgLaunch = 1. Bit 3 of the result's error word is
// then cleared and bit 4 set: the solve's result is valid and says that it took this path.
template <int RB>
__device__ __forceinline__ void pcg_recover(const BA& a, float* sh, float wSparse, int nLin) {
    const uint32_t wave = threadIdx.x >> 6, nw = WG / 64;
    for (uint32_t v = 1 + threadIdx.x; v < a.N; v += WG) {
        const float* b = a.poseBak + (size_t)v * 6;
        a.rot[3 * v] = b[0]; a.rot[3 * v + 1] = b[1]; a.rot[3 * v + 2] = b[2];
        a.trans[3 * v] = b[3]; a.trans[3 * v + 1] = b[4]; a.trans[3 * v + 2] = b[5];
    }
    __syncthreads();
    for (uint32_t v = 1 + wave; v < a.N; v += nw) pair_init_row(a, wSparse, v, false);
    __syncthreads();
    pair_init_finish(a, sh);
    if (threadIdx.x == 0) {
        a.ctrl[K_PCG_DONE] = 0;
        a.ctrl[K_PCG_ITERS] = a.ctrl[K_PCG_ITERS0];
    }
    __syncthreads();
    const int useDense = (int)a.ctrl[K_USE_DENSE];
    for (int iter = 0; iter < nLin; iter++) {
        for (uint32_t v = 1 + wave; v < a.N; v += nw) pair_row_ap(a, wSparse, v, nullptr);
        if (useDense) pcg_dense_offdiag(a, wave, nw);
        __syncthreads();
        float rDotzNew;
        bool last;
        pcg_finisher<RB>(a, sh, 0u, useDense, iter, nLin, rDotzNew, last);
        if (threadIdx.x == 0) {
            a.ctrl[K_RDOTZ] = __float_as_uint(rDotzNew);
            a.ctrl[K_PCG_ITERS]++;
            if (last) a.ctrl[K_PCG_DONE] = 1;
        }
        __syncthreads();
        if (last) break;  // uniform: from block sums
    }
    if (threadIdx.x == 0) a.ctrl[K_ERROR] = (a.ctrl[K_ERROR] & ~PP_ERR_TIMEOUT) | PP_RECOVERED;
}

// Small solves (N <= 64 images: the 11-frame local submaps, early global solves): every PCG
// iteration of the GN step in ONE workgroup. p lives in LDS; each wave applies the assembled
// operator to its rows (sparse pair blocks in fp64, dense blocks of BuildDenseSystem in fp32: the
// diagonal block and the off-diagonal pair blocks, with the [trans | rot] order of the dense system,
// SolverBundlingDenseUtil.h:371-411); wave 0 holds one row per lane for the vector updates and the
// two dot products (PCGIteration Kernel1b/2/3, SolverBundling.cu:930-1022) with fixed butterflies.
// No grid-wide hand-off and no launch per iteration.
constexpr int SMALL_N = 64;
constexpr int SMALL_WG = 1024;
__global__ __launch_bounds__(SMALL_WG) void k_pcg_small(BA a, float wSparse, int nLin) {
    __shared__ float sP[SMALL_N][6], sAp[SMALL_N][6];
    // wave 0's per-row vectors live in LDS between iterations: held in registers by every wave of the 16, one
    // of them was spilled and reloaded from scratch each iteration
    __shared__ f3 sV[SMALL_N][6];  // dR, dT, rR, rT, mR, mT
    __shared__ int sLast;
    if (a.ctrl[K_GN_DONE] || a.ctrl[K_PCG_DONE]) return;
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6, nw = SMALL_WG / 64;
    const int useDense = (int)a.ctrl[K_USE_DENSE];
    const uint32_t npD = useDense ? a.ctrl[K_NPAIRS] : 0u;
    // wave 0, lane v: row v's vectors (row 0 and rows >= N stay zero)
    const bool own = wave == 0 && lane >= 1 && lane < a.N;
    if (wave == 0) {
        f3 dR = mk3(0, 0, 0), dT = dR, rR = dR, rT = dR, mR = dR, mT = dR, pR = dR, pT = dR;
        if (own) {
            vload(a, V_DELTA, lane, dR, dT);
            vload(a, V_R, lane, rR, rT);
            vload(a, V_M, lane, mR, mT);
            vload(a, V_P, lane, pR, pT);
        }
        sV[lane][0] = dR; sV[lane][1] = dT; sV[lane][2] = rR; sV[lane][3] = rT; sV[lane][4] = mR; sV[lane][5] = mT;
        if (lane < a.N) {
            sP[lane][0] = pR.x; sP[lane][1] = pR.y; sP[lane][2] = pR.z;
            sP[lane][3] = pT.x; sP[lane][4] = pT.y; sP[lane][5] = pT.z;
        }
    }
    float rz = ctrlf(a.ctrl, K_RDOTZ);
    int iters = 0;
    __syncthreads();
    for (int iter = 0; iter < nLin; iter++) {
        for (uint32_t v = 1 + wave; v < a.N; v += nw) {
            double o[6] = {0, 0, 0, 0, 0, 0};
            const int e0 = a.rowPairStart[v], e1 = a.rowPairStart[v + 1];
            for (int k = e0 + (int)lane; k < e1; k += 64) {
                const int2 rp = a.rowPair[k];
                const uint32_t u = (uint32_t)rp.y & ~PAIR_A_FLAG;
                if (u == 0) continue;
                const double w[3] = {sP[u][0], sP[u][1], sP[u][2]}, t[3] = {sP[u][3], sP[u][4], sP[u][5]};
                double b[6];
                pair_block_apply(a.pstat + (size_t)rp.x * PSTAT, ((uint32_t)rp.y & PAIR_A_FLAG) != 0, w, t, b);
#pragma unroll
                for (int q = 0; q < 6; q++) o[q] += b[q];
            }
            float od[6] = {0, 0, 0, 0, 0, 0};  // dense part, [trans | rot] rows
            for (uint32_t k = lane; k < npD; k += 64) {
                if (a.pairW[k] == 0.0f) continue;
                const uint2 pr = a.pairs[k];
                const float* Bk = a.pairBlk + (size_t)k * 36;  // rows: image pr.y, columns: image pr.x
                if (pr.y == v && pr.x > 0) {
                    const float pv[6] = {sP[pr.x][3], sP[pr.x][4], sP[pr.x][5], sP[pr.x][0], sP[pr.x][1], sP[pr.x][2]};
                    for (int r = 0; r < 6; r++) {
                        float s = 0.0f;
                        for (int c = 0; c < 6; c++) s += Bk[r * 6 + c] * pv[c];
                        od[r] += s;
                    }
                } else if (pr.x == v && pr.y > 0) {
                    const float pv[6] = {sP[pr.y][3], sP[pr.y][4], sP[pr.y][5], sP[pr.y][0], sP[pr.y][1], sP[pr.y][2]};
                    for (int c = 0; c < 6; c++) {
                        float s = 0.0f;
                        for (int r = 0; r < 6; r++) s += Bk[r * 6 + c] * pv[r];
                        od[c] += s;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 6; q++) o[q] = wave_sum_d(o[q]);
            if (useDense) {
#pragma unroll
                for (int q = 0; q < 6; q++) od[q] = wave_sum(od[q]);
            }
            if (lane == 0) {
                const double w[3] = {sP[v][0], sP[v][1], sP[v][2]}, t[3] = {sP[v][3], sP[v][4], sP[v][5]};
                double dp[6];
                diag_apply(a.dstat + (size_t)v * DSTAT, w, t, dp);
                const double ws = wSparse;
                float ap[6];
#pragma unroll
                for (int q = 0; q < 6; q++) ap[q] = (float)(ws * (dp[q] - o[q]));
                if (useDense) {
                    const float* D = a.diag + (size_t)v * 36;
                    const float pv[6] = {sP[v][3], sP[v][4], sP[v][5], sP[v][0], sP[v][1], sP[v][2]};
                    float o6[6];
                    for (int r = 0; r < 6; r++) {
                        float s = 0.0f;
                        for (int c = 0; c < 6; c++) s += D[r * 6 + c] * pv[c];
                        o6[r] = s;
                    }
                    for (int q = 0; q < 3; q++) {
                        ap[3 + q] += o6[q] + od[q];      // trans
                        ap[q] += o6[3 + q] + od[3 + q];  // rot
                    }
                }
#pragma unroll
                for (int q = 0; q < 6; q++) sAp[v][q] = ap[q];
            }
        }
        __syncthreads();
        if (wave == 0) {
            const f3 aR = own ? mk3(sAp[lane][0], sAp[lane][1], sAp[lane][2]) : mk3(0, 0, 0);
            const f3 aT = own ? mk3(sAp[lane][3], sAp[lane][4], sAp[lane][5]) : mk3(0, 0, 0);
            f3 pR = own ? mk3(sP[lane][0], sP[lane][1], sP[lane][2]) : mk3(0, 0, 0);
            f3 pT = own ? mk3(sP[lane][3], sP[lane][4], sP[lane][5]) : mk3(0, 0, 0);
            f3 dR = sV[lane][0], dT = sV[lane][1], rR = sV[lane][2], rT = sV[lane][3];
            const f3 mR = sV[lane][4], mT = sV[lane][5];
            const float pAp = wave_sum(dot3(pR, aR) + dot3(pT, aT));
            const float alpha = (pAp > FLOAT_EPSILON) ? rz / pAp : 0.0f;
            dR = dR + alpha * pR;
            dT = dT + alpha * pT;
            rR = rR - alpha * aR;
            rT = rT - alpha * aT;
            const f3 zR = mul3(mR, rR), zT = mul3(mT, rT);
            const float rzNew = wave_sum(dot3(zR, rR) + dot3(zT, rT));
            const bool last = (iter == nLin - 1) || (a.earlyOut && fabsf(pAp) < 5e-7f);
            const float beta = (rz > FLOAT_EPSILON) ? rzNew / rz : 0.0f;
            if (own) {
                pR = zR + beta * pR;
                pT = zT + beta * pT;
                sP[lane][0] = pR.x; sP[lane][1] = pR.y; sP[lane][2] = pR.z;
                sP[lane][3] = pT.x; sP[lane][4] = pT.y; sP[lane][5] = pT.z;
            }
            sV[lane][0] = dR; sV[lane][1] = dT; sV[lane][2] = rR; sV[lane][3] = rT;
            rz = rzNew;
            if (lane == 0) sLast = last ? 1 : 0;
        }
        iters++;
        __syncthreads();
        if (sLast) break;
    }
    if (own) {
        const f3 dR = sV[lane][0], dT = sV[lane][1];
        vstore(a, V_DELTA, lane, dR, dT);
        vstore(a, V_R, lane, sV[lane][2], sV[lane][3]);
        vstore(a, V_P, lane, mk3(sP[lane][0], sP[lane][1], sP[lane][2]), mk3(sP[lane][3], sP[lane][4], sP[lane][5]));
        // computeLieUpdate (LieDerivUtil.h:301-307) on the exiting iteration
        f3 nr, nt;
        lie_update(dR, dT, mk3(a.rot[3 * lane], a.rot[3 * lane + 1], a.rot[3 * lane + 2]),
                   mk3(a.trans[3 * lane], a.trans[3 * lane + 1], a.trans[3 * lane + 2]), nr, nt);
        a.rot[3 * lane] = nr.x; a.rot[3 * lane + 1] = nr.y; a.rot[3 * lane + 2] = nr.z;
        a.trans[3 * lane] = nt.x; a.trans[3 * lane + 1] = nt.y; a.trans[3 * lane + 2] = nt.z;
    }
    if (threadIdx.x == 0) {
        a.ctrl[K_RDOTZ] = __float_as_uint(rz);
        a.ctrl[K_PCG_ITERS] += (uint32_t)iters;
        a.ctrl[K_PCG_DONE] = 1;
    }
}

// EvalGNConvergence (SolverBundling.cu:694-749) + the early-out test of solveBundlingStub (:1204-1210).
// After a persistent PCG launch (recoverRB = its finisher's rows per thread) it first redoes a GN step
// whose launch timed out (pcg_recover; one uniform test otherwise, no launch of its own).
template <int recoverRB>
// nextW > 0: the next GN step is a sparse pair-mode step of weight nextW, whose k_transforms this launch
// does when the loop goes on (one launch fewer per GN step)
__global__ __launch_bounds__(WG) void k_gn_end(BA a, int gnIndex, int nNonLin, float wSparse, int nLin, float nextW) {
    __shared__ float sh[WG];
    if (a.ctrl[K_GN_DONE]) return;
    if (recoverRB && (a.ctrl[K_ERROR] & PP_ERR_TIMEOUT)) {
        pcg_recover<recoverRB ? recoverRB : 2>(a, sh, wSparse, nLin);
        __syncthreads();
    }
    float m = 0.0f;
    for (uint32_t v = 1 + threadIdx.x; v < a.N; v += blockDim.x) {
        if (a.valid[v] == 0) continue;
        f3 dR, dT;
        vload(a, V_DELTA, v, dR, dT);
        const float r = fmaxf(fmaxf(fmaxf(fabsf(dR.x), fabsf(dT.x)), fmaxf(fabsf(dR.y), fabsf(dT.y))), fmaxf(fabsf(dR.z), fabsf(dT.z)));
        m = fmaxf(m, r);
    }
    sh[threadIdx.x] = m;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) sh[threadIdx.x] = fmaxf(sh[threadIdx.x], sh[threadIdx.x + s]);
        __syncthreads();
    }
    const bool done = a.earlyOut && gnIndex < nNonLin - 1 && sh[0] < 0.005f;
    if (threadIdx.x == 0) {
        a.ctrl[K_GN_ITERS]++;
        if (done) a.ctrl[K_GN_DONE] = 1;
    }
    if (nextW > 0.0f && !done) {  // k_transforms(a, nextW, 0, 1, 1) of the next step
        transforms_rows(a, threadIdx.x, blockDim.x);
        if (threadIdx.x == 0) {
            a.ctrl[K_PCG_DONE] = 0;
            a.ctrl[K_TICKET] = 0;
            a.ctrl[K_LAST_W] = __float_as_uint(nextW);
            a.ctrl[K_USE_DENSE] = 0u;
        }
    }
}

// ---- dense term (BuildDenseSystem, SolverBundling.cu:308-471) ----------------------------------
__device__ __forceinline__ f3 d2c(const BA& a, int x, int y, float depth) {  // CUDACameraUtil.h:15-19
    const float xx = ((float)x - a.mx) / a.fx, yy = ((float)y - a.my) / a.fy;
    return mk3(depth * xx, depth * yy, depth);
}
__device__ __forceinline__ void bilinear(const BA& a, float x, float y, const float* img, int comp, float* out) {
    const int W = (int)a.cw, H = (int)a.ch;
    const int px = (int)floorf(x), py = (int)floorf(y);
    const float alpha = x - (float)px, beta = y - (float)py;
    float s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, w0 = 0, w1 = 0;
    const int qx[4] = {px, px + 1, px, px + 1}, qy[4] = {py, py, py + 1, py + 1};
    const float wt[4] = {1.0f - alpha, alpha, 1.0f - alpha, alpha};
    for (int t = 0; t < 4; t++) {
        if ((unsigned)qx[t] < (unsigned)W && (unsigned)qy[t] < (unsigned)H) {
            const float* v = img + ((size_t)qy[t] * W + qx[t]) * comp;
            if (v[0] != -INFINITY) {
                float* s = t < 2 ? s0 : s1;
                for (int k = 0; k < comp; k++) s[k] += wt[t] * v[k];
                if (t < 2) w0 += wt[t]; else w1 += wt[t];
            }
        }
    }
    float ss[4] = {0, 0, 0, 0}, ww = 0;
    if (w0 > 0.0f) { for (int k = 0; k < comp; k++) ss[k] += (1.0f - beta) * (s0[k] / w0); ww += (1.0f - beta); }
    if (w1 > 0.0f) { for (int k = 0; k < comp; k++) ss[k] += beta * (s1[k] / w1); ww += beta; }
    for (int k = 0; k < comp; k++) out[k] = (ww > 0.0f) ? ss[k] / ww : -INFINITY;
}

__global__ void k_dense_reset(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < a.N * a.N; k += gridDim.x * blockDim.x) a.pairFlag[k] = 0u;
}

// FindImageImageCorr_Kernel<true> (SolverBundling.cu:29-79), one wave per (i, j), i < j
__global__ void k_dense_overlap(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t i = blockIdx.x, j = blockIdx.y;
    if (i >= j || j >= a.N) return;
    if (a.valid[i] == 0 || a.valid[j] == 0) return;
    const m4 t = mul44(loadm4(a.Tinv + (size_t)i * 16), loadm4(a.T + (size_t)j * 16));
    // computeAngleDiff (SolverBundlingDenseUtil.h:416-424)
    const f3 x1 = normalize3(mk3(1.0f, 1.0f, 1.0f));
    const f3 v1 = mul3v(rot_of(t), x1);
    if (!(fabsf(acosf(fmaxf(-1.0f, fminf(dot3(x1, v1), 1.0f)))) < 0.52f)) return;
    const uint32_t W = a.cw, H = a.ch, subW = W / a.sub;
    const float* tgt = a.cache[i].depth;
    const float* src = a.cache[j].depth;
    int found = 0;
    for (uint32_t tid = threadIdx.x; tid < 512; tid += blockDim.x) {
        const uint32_t x = (tid % subW) * a.sub, y = (tid / subW) * a.sub, idx = y * W + x;
        if (idx >= W * H) continue;
        const f3 cj = d2c(a, (int)x, (int)y, src[idx]);  // findDenseCorr depth-only (:22-42)
        if (!(cj.z > a.dmin && cj.z < a.dmax)) continue;
        const f3 s2t = xf(t, cj);
        const float u = s2t.x * a.fx / s2t.z + a.mx, vv = s2t.y * a.fy / s2t.z + a.my;
        const int tx = (int)roundf(u), ty = (int)roundf(vv);
        if (!(tx >= 0 && ty >= 0 && tx < (int)W && ty < (int)H)) continue;
        const f3 ct = d2c(a, tx, ty, tgt[ty * W + tx]);
        if (!(ct.z > a.dmin && ct.z < a.dmax)) continue;
        if (length3(s2t - ct) <= a.distT) found++;
    }
    for (int off = 32; off > 0; off >>= 1) found += __shfl_xor(found, off);
    if (threadIdx.x == 0 && found > 10) a.pairFlag[(size_t)i * a.N + j] = 1u;
}

// The overlapping pairs in (i, j) order (the reference appends them at atomic offsets): one workgroup
// compacts the flag matrix with wave ballots; K_NPAIRS = all pairs found, the first maxPairs are kept.
__global__ __launch_bounds__(256) void k_dense_compact(BA a) {
    __shared__ uint32_t sCnt[4], sBase;
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6, NN = a.N * a.N;
    if (threadIdx.x == 0) sBase = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < NN; b0 += 256) {
        const uint32_t idx = b0 + threadIdx.x;
        const bool f = idx < NN && a.pairFlag[idx] != 0u;
        const unsigned long long m = __ballot(f);
        if (lane == 0) sCnt[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t off = sBase;
        for (uint32_t w = 0; w < wv; w++) off += sCnt[w];
        off += (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (f && off < a.maxPairs) a.pairs[off] = make_uint2(idx / a.N, idx % a.N);
        __syncthreads();
        if (threadIdx.x == 0) for (uint32_t w = 0; w < 4; w++) sBase += sCnt[w];
        __syncthreads();
    }
    if (threadIdx.x == 0) a.ctrl[K_NPAIRS] = sBase;
}

// FindDenseCorrespondences_Kernel (:92-160, uchar4-normal variant :152-184) + WeightDenseCorrespondences (:162-180)
__global__ void k_dense_count(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t np = min(a.ctrl[K_NPAIRS], a.maxPairs);
    for (uint32_t k = blockIdx.x; k < np; k += gridDim.x) {
        const uint2 pr = a.pairs[k];
        const m4 t = mul44(loadm4(a.Tinv + (size_t)pr.x * 16), loadm4(a.T + (size_t)pr.y * 16));
        const m3 R = rot_of(t);
        const BFCachedFrame fi = a.cache[pr.x], fj = a.cache[pr.y];
        const uint32_t W = a.cw, H = a.ch;
        int count = 0;
        for (uint32_t idx = threadIdx.x; idx < W * H; idx += blockDim.x) {
            const int x = (int)(idx % W), y = (int)(idx / W);
            const f3 cj = d2c(a, x, y, fj.depth[idx]);
            if (!(cj.z > a.dmin && cj.z < a.dmax)) continue;
            const uint32_t nj = reinterpret_cast<const uint32_t*>(fj.normalsU8)[idx];
            if (nj == 0) continue;
            f3 nrmj = mk3((float)(nj & 0xFF), (float)((nj >> 8) & 0xFF), (float)((nj >> 16) & 0xFF)) / 255.0f * 2.0f - mk3(1.0f, 1.0f, 1.0f);
            nrmj = mul3v(R, nrmj);
            const f3 s2t = xf(t, cj);
            const float u = s2t.x * a.fx / s2t.z + a.mx, vv = s2t.y * a.fy / s2t.z + a.my;
            const int tx = (int)roundf(u), ty = (int)roundf(vv);
            if (!(tx >= 0 && ty >= 0 && tx < (int)W && ty < (int)H)) continue;
            const f3 ct = d2c(a, tx, ty, fi.depth[ty * W + tx]);
            if (!(ct.z > a.dmin && ct.z < a.dmax)) continue;
            const uint32_t ni = reinterpret_cast<const uint32_t*>(fi.normalsU8)[ty * W + tx];
            if (ni == 0) continue;
            const f3 nrmi = mk3((float)(ni & 0xFF), (float)((ni >> 8) & 0xFF), (float)((ni >> 16) & 0xFF)) / 255.0f * 2.0f - mk3(1.0f, 1.0f, 1.0f);
            if (dot3(nrmj, nrmi) >= a.normT && length3(s2t - ct) <= a.distT) count++;
        }
        for (int off = 32; off > 0; off >>= 1) count += __shfl_xor(count, off);
        __shared__ int wc[WG / 64];
        if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = count;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (uint32_t q = 0; q < blockDim.x / 64; q++) tot += wc[q];
            float x = (float)tot;
            if (x > 0) x = (x < 800) ? 0.0f : 1.0f / fminf(logf(x), 9.0f);
            a.pairW[k] = x;
        }
        __syncthreads();
    }
}

// BuildDenseSystem_Kernel<depth, color> (:182-306): one workgroup per overlapping pair; every
// thread accumulates its pixels' 6x6 outer products (addToLocalSystem, DenseUtil.h:229-288) in
// registers, then one workgroup reduction and one set of global adds per pair.
__global__ __launch_bounds__(WG) void k_dense_build(BA a, float wDepth, float wColor) {
    __shared__ float red[WG / 64][90];
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t np = min(a.ctrl[K_NPAIRS], a.maxPairs);
    const bool useDepth = wDepth > 0.0f;
    const bool useColor = !useDepth || wColor > 0.0f;
    for (uint32_t k = blockIdx.x; k < np; k += gridDim.x) {
        const float pw = a.pairW[k];
        if (pw == 0.0f) continue;  // uniform per workgroup
        const uint2 pr = a.pairs[k];
        const uint32_t i = pr.x, j = pr.y;
        const m4 Ti = loadm4(a.T + (size_t)i * 16), Tj = loadm4(a.T + (size_t)j * 16);
        const m4 Tiinv = loadm4(a.Tinv + (size_t)i * 16), Tjinv = loadm4(a.Tinv + (size_t)j * 16);
        const m4 t = mul44(Tiinv, Tj);
        const BFCachedFrame fi = a.cache[i], fj = a.cache[j];
        float acc[90];  // [0,21) ii upper, [21,42) jj upper, [42,78) ij (row b of i . col c of j), [78,84) jtr_i, [84,90) jtr_j
#pragma unroll
        for (int q = 0; q < 90; q++) acc[q] = 0.0f;
        const uint32_t W = a.cw, H = a.ch;
        for (uint32_t src = threadIdx.x; src < W * H; src += blockDim.x) {
            // findDenseCorr with camera positions + float4 normals (DenseUtil.h:79-113)
            const float4 cp = reinterpret_cast<const float4*>(fj.campos)[src];
            if (!(cp.z > a.dmin && cp.z < a.dmax)) continue;
            const f3 cps = mk3(cp.x, cp.y, cp.z);
            const float4 nj = reinterpret_cast<const float4*>(fj.normals)[src];
            if (nj.x == -INFINITY) continue;
            const f3 nrmj = mk3(t.e[0] * nj.x + t.e[1] * nj.y + t.e[2] * nj.z + t.e[3] * nj.w,
                                t.e[4] * nj.x + t.e[5] * nj.y + t.e[6] * nj.z + t.e[7] * nj.w,
                                t.e[8] * nj.x + t.e[9] * nj.y + t.e[10] * nj.z + t.e[11] * nj.w);
            const float nrmjw = t.e[12] * nj.x + t.e[13] * nj.y + t.e[14] * nj.z + t.e[15] * nj.w;
            const f3 s2t = xf(t, cps);
            const float u = s2t.x * a.fx / s2t.z + a.mx, vv = s2t.y * a.fy / s2t.z + a.my;
            const int tx = (int)roundf(u), ty = (int)roundf(vv);
            if (!(tx >= 0 && ty >= 0 && tx < (int)W && ty < (int)H)) continue;
            float ci[4], ni[4];
            bilinear(a, u, vv, fi.campos, 4, ci);
            if (!(ci[2] > a.dmin && ci[2] < a.dmax)) continue;
            bilinear(a, u, vv, fi.normals, 4, ni);
            if (ni[0] == -INFINITY) continue;
            const f3 cpt = mk3(ci[0], ci[1], ci[2]), nT = mk3(ni[0], ni[1], ni[2]);
            const float dn = nrmj.x * ni[0] + nrmj.y * ni[1] + nrmj.z * ni[2] + nrmjw * ni[3];
            if (!(dn >= a.normT && length3(s2t - cpt) <= a.distT)) continue;
            // rows of the two terms; accumulate J^T W J and J^T W r (every loop over acc unrolled: with a
            // run-time index the 90 accumulators lived in scratch, one memory round trip per update)
#pragma unroll
            for (int term = 0; term < 2; term++) {
                float Ji[6] = {0, 0, 0, 0, 0, 0}, Jj[6] = {0, 0, 0, 0, 0, 0};
                float res = 0.0f, w = 0.0f;
                if (term == 0) {
                    if (!useDepth) continue;
                    res = dot3(cpt - s2t, nT);
                    w = wDepth * pw * powf(fmaxf(0.0f, 1.0f - cpt.z / 2.0f), 2.5f);
                    if (i > 0) { const m36 J = deriv_i(Tjinv, Ti, cps); for (int c = 0; c < 6; c++) Ji[c] = -dot3(mk3(J.e[c], J.e[6 + c], J.e[12 + c]), nT); }
                    if (j > 0) { const m36 J = deriv_j(Tiinv, Tj, cps); for (int c = 0; c < 6; c++) Jj[c] = -dot3(mk3(J.e[c], J.e[6 + c], J.e[12 + c]), nT); }
                } else {
                    if (!useColor) continue;
                    float dI[2], It;
                    bilinear(a, u, vv, fi.intensityDeriv, 2, dI);
                    bilinear(a, u, vv, fi.intensity, 1, &It);
                    res = It - fj.intensity[src];
                    if (!(dI[0] != -INFINITY && fabsf(res) < a.colT && sqrtf(dI[0] * dI[0] + dI[1] * dI[1]) > a.gradMin)) continue;
                    const float wSq = s2t.z * s2t.z;
                    const float d00 = a.fx / s2t.z, d11 = a.fy / s2t.z, d02 = -a.fx * s2t.x / wSq, d12 = -a.fy * s2t.y / wSq;
                    if (i > 0) {
                        const m36 J = deriv_i(Tjinv, Ti, cps);
                        for (int c = 0; c < 6; c++) Ji[c] = dI[0] * (d00 * J.e[c] + 0.0f * J.e[6 + c] + d02 * J.e[12 + c]) + dI[1] * (0.0f * J.e[c] + d11 * J.e[6 + c] + d12 * J.e[12 + c]);
                    }
                    if (j > 0) {
                        const m36 J = deriv_j(Tiinv, Tj, cps);
                        for (int c = 0; c < 6; c++) Jj[c] = dI[0] * (d00 * J.e[c] + 0.0f * J.e[6 + c] + d02 * J.e[12 + c]) + dI[1] * (0.0f * J.e[c] + d11 * J.e[6 + c] + d12 * J.e[12 + c]);
                    }
                    w = wColor * pw * fmaxf(0.0f, 1.0f - fabsf(res) / (1.15f * a.colT));
                }
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int c = r; c < 6; c++) {
                        const int q = r * 6 - r * (r - 1) / 2 + (c - r);  // row-major upper triangle
                        acc[q] += Ji[r] * Ji[c] * w;
                        acc[21 + q] += Jj[r] * Jj[c] * w;
                    }
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int c = 0; c < 6; c++) acc[42 + r * 6 + c] += Ji[r] * Jj[c] * w;
#pragma unroll
                for (int r = 0; r < 6; r++) { acc[78 + r] += Ji[r] * res * w; acc[84 + r] += Jj[r] * res * w; }
            }
        }
#pragma unroll
        for (int q = 0; q < 90; q++) {
            const float s = wave_sum(acc[q]);
            if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][q] = s;
        }
        __syncthreads();
        if (threadIdx.x < 90) {
            float s = 0.0f;
            for (uint32_t wv = 0; wv < blockDim.x / 64; wv++) s += red[wv][threadIdx.x];
            const int q = threadIdx.x;
            if (q < 42) {  // diagonal-block upper triangles of images i (q < 21) and j: summed per image by k_dense_lists
                a.pairAcc[(size_t)k * 54 + q] = s;
            } else if (q < 78) {  // B(row j-index c, col i-index r) = (J_i^T W J_j)^T
                const int r = (q - 42) / 6, c = (q - 42) % 6;
                a.pairBlk[(size_t)k * 36 + c * 6 + r] = s;
            } else {  // J_i^T r (q < 84), J_j^T r
                a.pairAcc[(size_t)k * 54 + 42 + (q - 78)] = s;
            }
        }
        __syncthreads();
    }
}

// Per image v (one wave): its pairs in pair order (pairW != 0), and its dense diagonal block and J^T r
// summed over them in that order (the reference adds them with float atomics in arrival order).
__global__ __launch_bounds__(64) void k_dense_lists(BA a) {
    if (a.ctrl[K_GN_DONE]) return;
    const uint32_t v = blockIdx.x, lane = lane_id();
    const uint32_t np = min(a.ctrl[K_NPAIRS], a.maxPairs);
    uint32_t* L = a.imgPairs + (size_t)v * a.maxN;
    uint32_t n = 0;
    float s = 0.0f;  // lane < 21: upper-triangle entry of the diagonal block, 21..26: J^T r
    for (uint32_t b0 = 0; b0 < np; b0 += 64) {
        const uint32_t k = b0 + lane;
        uint32_t e = 0;
        bool in = false;
        if (k < np && a.pairW[k] != 0.0f) {
            const uint2 pr = a.pairs[k];
            in = pr.x == v || pr.y == v;
            e = (k << 1) | (pr.y == v ? 1u : 0u);
        }
        const unsigned long long m = __ballot(in);
        if (in) L[n + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = e;
        n += (uint32_t)__popcll(m);
        for (unsigned long long mm = m; mm; mm &= mm - 1ull) {  // this chunk's pairs of v, ascending
            const uint32_t ek = (uint32_t)__shfl((int)e, (int)__builtin_ctzll(mm));
            const float* acc = a.pairAcc + (size_t)(ek >> 1) * 54;
            if (lane < 21) s += acc[((ek & 1u) ? 21 : 0) + lane];
            else if (lane < 27) s += acc[42 + ((ek & 1u) ? 6 : 0) + (lane - 21)];
        }
    }
    if (lane == 0) a.imgPairN[v] = n;
    if (lane < 21) {
        int r = 0, c = 0, t2 = 0;
        for (r = 0; r < 6; r++) { if ((int)lane < t2 + (6 - r)) { c = r + ((int)lane - t2); break; } t2 += 6 - r; }
        a.diag[(size_t)v * 36 + r * 6 + c] = s;
        a.diag[(size_t)v * 36 + c * 6 + r] = s;
    } else if (lane < 27) {
        a.jtr[(size_t)v * 6 + (lane - 21)] = s;
    }
}

// ---- residual analysis (EvalMaxResidual :511-564, EvalResidual :570-614, CountHighResiduals :657-687) ----
__global__ __launch_bounds__(WG) void k_residuals(BA a) {
    __shared__ float shv[WG];
    __shared__ int shi[WG];
    __shared__ float she[WG];
    __shared__ int shc[WG];
    if (a.ctrl[K_SKIPPED]) return;  // gated-off solve: no residual analysis, hence no removal
    const float w = ctrlf(a.ctrl, K_LAST_W);
    float best = 0.0f, e = 0.0f;
    int bi = 0x7FFFFFFF, cnt = 0;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < a.nCorr; c += gridDim.x * blockDim.x) {
        const BFEntryJ x = a.corr[c];
        if (!corr_valid(x)) continue;
        const f3 r = xf(loadm4(a.T + (size_t)x.imgIdx_i * 16), mk3(x.pos_i.x, x.pos_i.y, x.pos_i.z)) -
                     xf(loadm4(a.T + (size_t)x.imgIdx_j * 16), mk3(x.pos_j.x, x.pos_j.y, x.pos_j.z));
        const f3 ar = mk3(fabsf(r.x), fabsf(r.y), fabsf(r.z)) * w;
        const float m = fmaxf(ar.z, fmaxf(ar.x, ar.y));  // evalAbsMaxResidualDevice (EquationsLie.h:27-40)
        if (m > best || (m == best && (int)c < bi)) { best = m; bi = (int)c; }
        e += w * dot3(r, r);                              // evalFDevice (:42-57)
        if (m > a.verifyT) cnt++;
    }
    shv[threadIdx.x] = best; shi[threadIdx.x] = bi; she[threadIdx.x] = e; shc[threadIdx.x] = cnt;
    __syncthreads();
    for (int s = WG / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            const float v2 = shv[threadIdx.x + s];
            const int i2 = shi[threadIdx.x + s];
            if (v2 > shv[threadIdx.x] || (v2 == shv[threadIdx.x] && i2 < shi[threadIdx.x])) { shv[threadIdx.x] = v2; shi[threadIdx.x] = i2; }
            she[threadIdx.x] += she[threadIdx.x + s];
            shc[threadIdx.x] += shc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        st_wt(&a.part[blockIdx.x * 2], shv[0]);
        st_wt(&a.part[blockIdx.x * 2 + 1], she[0]);
        st_wt(reinterpret_cast<uint32_t*>(&a.partIdx[blockIdx.x * 2]), (uint32_t)shi[0]);
        st_wt(reinterpret_cast<uint32_t*>(&a.partIdx[blockIdx.x * 2 + 1]), (uint32_t)shc[0]);
    }
    if (!last_block(&a.ctrl[K_TICKET])) return;
    // all threads fold the per-workgroup partials, then one fixed tree (deterministic)
    float mv = 0.0f, en = 0.0f;
    int mi = 0x7FFFFFFF, hc = 0;
    for (uint32_t b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
        const float v2 = ld_wtf(&a.part[b * 2]);
        const int i2 = (int)ld_wt(reinterpret_cast<const uint32_t*>(&a.partIdx[b * 2]));
        if (v2 > mv || (v2 == mv && i2 < mi)) { mv = v2; mi = i2; }
        en += ld_wtf(&a.part[b * 2 + 1]);
        hc += (int)ld_wt(reinterpret_cast<const uint32_t*>(&a.partIdx[b * 2 + 1]));
    }
    shv[threadIdx.x] = mv; shi[threadIdx.x] = mi; she[threadIdx.x] = en; shc[threadIdx.x] = hc;
    __syncthreads();
    for (int s = WG / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            const float v2 = shv[threadIdx.x + s];
            const int i2 = shi[threadIdx.x + s];
            if (v2 > shv[threadIdx.x] || (v2 == shv[threadIdx.x] && i2 < shi[threadIdx.x])) { shv[threadIdx.x] = v2; shi[threadIdx.x] = i2; }
            she[threadIdx.x] += she[threadIdx.x + s];
            shc[threadIdx.x] += shc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        mv = shv[0]; mi = shi[0]; en = she[0]; hc = shc[0];
        if (!(w > 0.0f) || mi == 0x7FFFFFFF) { mv = 0.0f; mi = 0; }
        a.ctrl[K_MAXRES] = __float_as_uint(mv);
        a.ctrl[K_MAXIDX] = (uint32_t)mi;
        a.ctrl[K_ENERGY] = __float_as_uint(en);
        a.ctrl[K_HIGHCOUNT] = (uint32_t)hc;
        a.ctrl[K_TICKET] = 0;
    }
}

__global__ void k_solve_begin(uint32_t* ctrl, const int* gate) {
    const uint32_t off = (gate && *gate == 0) ? 1u : 0u;
    const uint32_t t = threadIdx.x;
    if (t < K_COUNT)  // the error word too: every solve reports its own
        ctrl[t] = (t == K_RM_I || t == K_RM_J) ? BF_INVALID_IMAGE : (t == K_GN_DONE || t == K_SKIPPED) ? off : 0u;
}

// ---- local-submap verification (SBA.cpp:106-109 -> CUDASolverBundling::useVerification,
// CUDASolverBundling.cpp:454-476 -> Bundler::optimize, Bundler.cpp:259-274) ----------------------
struct VerifyArgs {
    const float* T;
    const int* valid;
    uint32_t N;
    const BFCachedFrame* cache;
    uint32_t W, H;
    float K[16];  // cache intrinsics as the reference's float4x4 (MatrixConversion::toCUDA(getIntrinsics()))
    float distT, normT, errT, corrT, dmin, dmax, percentT;
    uint32_t nCorr, always;
    uint32_t* ctrl;
    float* stats;
};
// useVerification: the pair check runs when the solve left >= 5 % of its correspondences with a
// max-norm residual above verifyOptDistThresh (K_HIGHCOUNT, counted by k_residuals)
__global__ void k_verify_begin(VerifyArgs v) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const bool used = v.always || ((float)v.ctrl[K_HIGHCOUNT] / (float)v.nCorr >= v.percentT);
    v.ctrl[K_VERIFY_USED] = used ? 1u : 0u;
    v.ctrl[K_VERIFY_OK] = 1u;
}
__device__ __forceinline__ float4 m4x4(const m4& m, float4 p) {  // float4x4 * float4 (cuda_SimpleMatrixUtil.h:925-933)
    const float* e = m.e;
    return make_float4(e[0] * p.x + e[1] * p.y + e[2] * p.z + e[3] * p.w, e[4] * p.x + e[5] * p.y + e[6] * p.z + e[7] * p.w,
                       e[8] * p.x + e[9] * p.y + e[10] * p.z + e[11] * p.w, e[12] * p.x + e[13] * p.y + e[14] * p.z + e[15] * p.w);
}
// computeProjError, CUDACACHE_FLOAT_NORMALS branch (SIFTImageManager.cu:418-487; CUDACacheUtil.h:7-8
// defines both normal formats, the float one is the branch compiled): {residual, weight, 1} of input
// pixel idx carried by `tr` into the model frame, or 0
__device__ f3 proj_error(const VerifyArgs& v, uint32_t idx, const m4& tr, const BFCachedFrame& in, const BFCachedFrame& model) {
    const float4 pIn = reinterpret_cast<const float4*>(in.campos)[idx];
    float4 nIn = reinterpret_cast<const float4*>(in.normals)[idx];
    nIn.w = 0.0f;
    const float dIn = in.depth[idx];
    if (!(pIn.x != -INFINITY && nIn.x != -INFINITY && dIn >= v.dmin && dIn <= v.dmax)) return mk3(0, 0, 0);
    const float4 pT = m4x4(tr, pIn), nT = m4x4(tr, nIn);
    const float* K = v.K;
    const f3 q = mk3(K[0] * pT.x + K[1] * pT.y + K[2] * pT.z + K[3] * 1.0f, K[4] * pT.x + K[5] * pT.y + K[6] * pT.z + K[7] * 1.0f,
                     K[8] * pT.x + K[9] * pT.y + K[10] * pT.z + K[11] * 1.0f);
    const int sx = f2i(roundf(q.x / q.z)), sy = f2i(roundf(q.y / q.z));
    if (!(sx >= 0 && sy >= 0 && sx < (int)v.W && sy < (int)v.H)) return mk3(0, 0, 0);
    const uint32_t t = (uint32_t)sy * v.W + (uint32_t)sx;
    const float4 pTg = reinterpret_cast<const float4*>(model.campos)[t];
    const float4 nTg = reinterpret_cast<const float4*>(model.normals)[t];
    if (!(pTg.x != -INFINITY && nTg.x != -INFINITY)) return mk3(0, 0, 0);
    const float dx = pT.x - pTg.x, dy = pT.y - pTg.y, dz = pT.z - pTg.z, dw = pT.w - pTg.w;
    const float d = sqrtf(dx * dx + dy * dy + dz * dz + dw * dw);  // length(float4)
    const float dN = nT.x * nTg.x + nT.y * nTg.y + nT.z * nTg.z;
    const float tgtDepth = model.depth[t];
    if (!(tgtDepth >= v.dmin && tgtDepth <= v.dmax)) return mk3(0, 0, 0);
    const bool bad = (tgtDepth != -INFINITY && pT.z < tgtDepth) && d > v.distT;  // known bad match
    if (!((dN >= v.normT && d <= v.distT) || bad)) return mk3(0, 0, 0);
    const float camZ = (pT.z - v.dmin) / (v.dmax - v.dmin);
    const float w = fmaxf(0.0f, 0.5f * ((1.0f - d / v.distT) + (1.0f - camZ)));
    return mk3(d, w, 1.0f);
}
// VerifyTrajectoryCU_Kernel (SIFTImageManager.cu:1036-1127): one workgroup per image pair i < j,
// both directions of every cache pixel. Sums per thread in pixel order (t, t + 256, ...), then a fixed
// tree per wave and the 4 waves in order (the reference's warp sums + shared float atomics have no
// fixed order; the oracle restates this one).
__global__ __launch_bounds__(WG) void k_verify_pairs(VerifyArgs v) {
    __shared__ float sh[3][WG / 64];
    if (!v.ctrl[K_VERIFY_USED]) return;
    const uint32_t i = blockIdx.x / v.N, j = blockIdx.x % v.N;
    if (i >= j) return;
    if (v.valid[i] == 0 || v.valid[j] == 0) return;
    const m4 tr = mul44(inverse44(loadm4(v.T + (size_t)j * 16)), loadm4(v.T + (size_t)i * 16));
    const m4 trInv = inverse44(tr);
    const BFCachedFrame in = v.cache[i], model = v.cache[j];
    float sr = 0.0f, sw = 0.0f, sn = 0.0f;
    for (uint32_t idx = threadIdx.x; idx < v.W * v.H; idx += WG) {
        const f3 a = proj_error(v, idx, tr, in, model);
        const f3 b = proj_error(v, idx, trInv, model, in);
        sr += a.x + b.x;
        sw += a.y + b.y;
        sn += a.z + b.z;
    }
    for (int off = 32; off > 0; off >>= 1) {
        sr += __shfl_down(sr, off);
        sw += __shfl_down(sw, off);
        sn += __shfl_down(sn, off);
    }
    if ((threadIdx.x & 63) == 0) {
        sh[0][threadIdx.x >> 6] = sr;
        sh[1][threadIdx.x >> 6] = sw;
        sh[2][threadIdx.x >> 6] = sn;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    float s[3];
    for (int q = 0; q < 3; q++) s[q] = ((sh[q][0] + sh[q][1]) + sh[q][2]) + sh[q][3];
    if (v.stats)
        for (int q = 0; q < 3; q++) v.stats[((size_t)i * v.N + j) * 3 + q] = s[q];
    const float err = s[0] / s[1];
    const float corr = 0.5f * s[2] / (float)(v.W * v.H);
    if (corr < v.corrT || err > v.errT || isnan(err)) v.ctrl[K_VERIFY_OK] = 0u;  // every failing pair writes 0
}

// ---- SBA.cu / SIFTImageManager.cu helpers ----
__global__ void k_m2p(const float* T, uint32_t n, float* rot, float* trans, const int* valid) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && valid[i]) {
        m4 M;
        for (int k = 0; k < 16; k++) M.e[k] = T[(size_t)i * 16 + k];
        f3 r, t;
        matrix_to_pose(M, r, t);
        rot[3 * i] = r.x; rot[3 * i + 1] = r.y; rot[3 * i + 2] = r.z;
        trans[3 * i] = t.x; trans[3 * i + 1] = t.y; trans[3 * i + 2] = t.z;
    }
}
__global__ void k_p2m(const float* rot, const float* trans, uint32_t n, float* T, const int* valid) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && valid[i]) {
        const m4 M = pose_to_matrix(mk3(rot[3 * i], rot[3 * i + 1], rot[3 * i + 2]), mk3(trans[3 * i], trans[3 * i + 1], trans[3 * i + 2]));
        for (int k = 0; k < 16; k++) T[(size_t)i * 16 + k] = M.e[k];
    }
}
__global__ void k_invalidate_pair(BFEntryJ* corr, uint32_t n, uint32_t i, uint32_t j) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n && corr[c].imgIdx_i == i && corr[c].imgIdx_j == j) { corr[c].imgIdx_i = BF_INVALID_IMAGE; corr[c].imgIdx_j = BF_INVALID_IMAGE; }
}
__global__ void k_check_frames(const int* numEntries, int* valid, uint32_t numImages, BFEntryJ* corr, uint32_t nCorr, int comprehensive) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < numImages && numEntries[t] == 0) valid[t] = 0;
    if (comprehensive) {
        for (uint32_t c = t; c < nCorr; c += gridDim.x * blockDim.x) {
            const BFEntryJ e = corr[c];
            if (corr_valid(e) && (numEntries[e.imgIdx_i] == 0 || numEntries[e.imgIdx_j] == 0)) {
                corr[c].imgIdx_i = BF_INVALID_IMAGE;
                corr[c].imgIdx_j = BF_INVALID_IMAGE;
            }
        }
    }
}

// initNextGlobalTransformCU (OnlineBundler.cu:112-140): keyframe s+1 = global[s] * local[last]; when the
// submap's gate is 0 (invalid local) Bundler::initializeNextTransformUnknown instead (Bundler.h:75-79,
// via addInvalidFrame, Bundler.cpp:362-368): keyframe s+1 = keyframe s
__global__ void k_seed_keyframe(const float* localRot, const float* localTrans, uint32_t last, float* rot, float* trans,
                                uint32_t s, const int* gate) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (gate && *gate == 0) {
        for (int k = 0; k < 3; k++) { rot[3 * (s + 1) + k] = rot[3 * s + k]; trans[3 * (s + 1) + k] = trans[3 * s + k]; }
        return;
    }
    const m4 G = pose_to_matrix(mk3(rot[3 * s], rot[3 * s + 1], rot[3 * s + 2]), mk3(trans[3 * s], trans[3 * s + 1], trans[3 * s + 2]));
    const m4 L = pose_to_matrix(mk3(localRot[3 * last], localRot[3 * last + 1], localRot[3 * last + 2]),
                                mk3(localTrans[3 * last], localTrans[3 * last + 1], localTrans[3 * last + 2]));
    f3 r, t;
    matrix_to_pose(mul44(G, L), r, t);
    rot[3 * (s + 1)] = r.x; rot[3 * (s + 1) + 1] = r.y; rot[3 * (s + 1) + 2] = r.z;
    trans[3 * (s + 1)] = t.x; trans[3 * (s + 1) + 1] = t.y; trans[3 * (s + 1) + 2] = t.z;
}
__global__ void k_set_gate(int* gate, const int* src) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *gate = src ? *src : 1;
}
// An invalidated local submap becomes an invalid global frame with no features
// (OnlineBundler.cpp:351-360: addInvalidFrame; :399-401: invalidateLastFrame): its keyframe is marked
// invalid and no correspondence of the global list may reference it (the reference's matcher finds
// none for a frame with 0 SIFT keys; here the list is an input, so its entries are invalidated)
__global__ void k_invalidate_local(const int* gate, uint32_t s, int* valid, BFEntryJ* corr, uint32_t n) {
    if (*gate != 0) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) valid[s] = 0;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x)
        if (corr[c].imgIdx_i == s || corr[c].imgIdx_j == s) { corr[c].imgIdx_i = BF_INVALID_IMAGE; corr[c].imgIdx_j = BF_INVALID_IMAGE; }
}

// SBA::removeMaxResidualCUDA (SBA.cpp:164-203) + getMaxResidual (CUDASolverBundling.cpp:429-452) on
// the device: pick the pair of the max residual when it exceeds the threshold and is not (0, <10)
__global__ void k_pick_maxres_pair(uint32_t* ctrl, const BFEntryJ* corr, float thresh) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t pi = BF_INVALID_IMAGE, pj = BF_INVALID_IMAGE;
    const float mr = __uint_as_float(ctrl[K_MAXRES]);
    if (mr > thresh) {
        const BFEntryJ e = corr[ctrl[K_MAXIDX]];
        if (e.imgIdx_i != BF_INVALID_IMAGE && !(e.imgIdx_i == 0 && e.imgIdx_j < 10)) {
            pi = e.imgIdx_i;
            pj = e.imgIdx_j;
        }
    }
    ctrl[K_RM_I] = pi;
    ctrl[K_RM_J] = pj;
}
__global__ void k_invalidate_picked_pair(const uint32_t* ctrl, BFEntryJ* corr, uint32_t n) {
    const uint32_t i = ctrl[K_RM_I], j = ctrl[K_RM_J];
    if (i == BF_INVALID_IMAGE) return;
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x)
        if (corr[c].imgIdx_i == i && corr[c].imgIdx_j == j) { corr[c].imgIdx_i = BF_INVALID_IMAGE; corr[c].imgIdx_j = BF_INVALID_IMAGE; }
}
// CheckForInvalidFramesSimpleCU (SIFTImageManager.cu:725-745), only after a removal
__global__ void k_check_frames_if_removed(const uint32_t* ctrl, const int* numEntries, int* valid, uint32_t numImages) {
    if (ctrl[K_RM_I] == BF_INVALID_IMAGE) return;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < numImages && numEntries[t] == 0) valid[t] = 0;
}

// one per device: orders the persistent PCG launches of all solvers on it (Solver::solve)
struct PersistGate {
    std::mutex mu;
    hipEvent_t ev = nullptr;
    hipStream_t stream = nullptr;
};
PersistGate& persist_gate() {
    static PersistGate gates[64];
    int dev = 0;
    BF_HIP(hipGetDevice(&dev));
    return gates[dev & 63];
}

}  // namespace

// zParametersBundlingDefault.txt defaults for every option left 0
SolverConfig make_solver_config(uint32_t maxImages, uint32_t maxCorr, const BFSolverOptions* o) {
    SolverConfig cfg{};
    cfg.maxImages = maxImages;
    cfg.maxCorr = maxCorr;
    cfg.denseDistThresh = (o && o->denseDistThresh > 0) ? o->denseDistThresh : 0.15f;
    cfg.denseNormalThresh = (o && o->denseNormalThresh > 0) ? o->denseNormalThresh : 0.97f;
    cfg.denseColorThresh = (o && o->denseColorThresh > 0) ? o->denseColorThresh : 0.1f;
    cfg.denseColorGradientMin = (o && o->denseColorGradientMin > 0) ? o->denseColorGradientMin : 0.005f;
    cfg.denseDepthMin = (o && o->denseDepthMin > 0) ? o->denseDepthMin : 0.5f;
    cfg.denseDepthMax = (o && o->denseDepthMax > 0) ? o->denseDepthMax : 4.0f;
    cfg.denseOverlapSubsample = (o && o->denseOverlapSubsample) ? o->denseOverlapSubsample : 4;
    cfg.verifyOptDistThresh = (o && o->verifyOptDistThresh > 0) ? o->verifyOptDistThresh : 0.02f;
    cfg.normalEquations = o ? o->normalEquations : 0;
    cfg.earlyOut = !(o && o->disableEarlyOut);
    cfg.pcgLaunch = o ? o->pcgLaunch : 0;
    cfg.pcgSpinLimitUs = o ? o->pcgSpinLimitUs : 0u;
    return cfg;
}

VerifyParams verify_params(const BFVerifyOptions* o) {
    VerifyParams p{};
    if (!o) return p;
    if (o->projCorrDistThresh > 0) p.distThresh = o->projCorrDistThresh;
    if (o->projCorrNormalThresh > 0) p.normalThresh = o->projCorrNormalThresh;
    if (o->verifyOptErrThresh > 0) p.errThresh = o->verifyOptErrThresh;
    if (o->verifyOptCorrThresh > 0) p.corrThresh = o->verifyOptCorrThresh;
    if (o->verifyOptPercentThresh > 0) p.percentThresh = o->verifyOptPercentThresh;
    if (o->sensorDepthMin > 0) p.depthMin = o->sensorDepthMin;
    if (o->sensorDepthMax > 0) p.depthMax = o->sensorDepthMax;
    p.always = o->always != 0;
    return p;
}

// ------------------------------------------------------------------------------------------------
Solver::Solver(const SolverConfig& cfg, hipStream_t stream) : cfg_(cfg), stream_(stream) {
    BF_REQUIRE(cfg.maxImages >= 2 && cfg.maxCorr >= 1, BF_ERR_ARG, "solver capacity");
    // maxCorrPerImage = clamp(maxRes / maxImages, 1000, 4000) (CUDASolverBundling.cpp:37)
    maxCorrPerImage_ = std::min(4000u, std::max(1000u, cfg.maxCorr / cfg.maxImages));
    maxPairs_ = cfg.maxImages * (cfg.maxImages - 1) / 2;
    const uint32_t N = cfg.maxImages;
    rowCount_.alloc(N + 1);
    rowStart_.alloc(N + 1);
    rowLen_.alloc(N + 1);
    BF_REQUIRE(cfg.maxImages <= 16384, BF_ERR_CAPACITY, "maxImages > 16384 (LDS row histograms)");
    maxTiles_ = div_up(cfg.maxCorr, TILE);  // tiles at <= 256 images; tileCnt_ holds any n x div_up(nCorr, tile_for(n))
    maxChunks_ = div_up(2 * (size_t)cfg.maxCorr, (size_t)CH) + N;
    tileCnt_.alloc((size_t)maxTiles_ * std::min(N, 256u) + (size_t)cfg.maxCorr + N + TILE + 1);
    rowChunk_.alloc(N + 1);
    chunkRow_.alloc(maxChunks_ + 1);
    chunkPart_.alloc(3 * (size_t)maxChunks_ + 3);
    rowTmp_.alloc(2 * (size_t)cfg.maxCorr + 1);
    rowIdx_.alloc(2 * (size_t)cfg.maxCorr + 1);
    entries_.alloc(4 * (size_t)cfg.maxCorr + 2);
    vec_.alloc((size_t)V_NUM * N * 8);
    img_.alloc(2 * (size_t)N);
    T_.alloc((size_t)N * 16);
    Tinv_.alloc((size_t)N * 16);
    ctrl_.alloc(K_CTRL_WORDS);
    sync_.alloc(SYNC_WORDS);
    part_.alloc(2 * 4096);
    partIdx_.alloc(2 * 4096);
    pairs_.alloc(maxPairs_);
    pairW_.alloc(maxPairs_);
    pairBlk_.alloc((size_t)maxPairs_ * 36);
    diag_.alloc((size_t)N * 36);
    jtr_.alloc((size_t)N * 6);
    pairFlag_.alloc((size_t)N * N);
    pairAcc_.alloc((size_t)maxPairs_ * 54);
    pairProd_.alloc((size_t)N * 8);
    imgPairs_.alloc((size_t)N * N);
    imgPairN_.alloc(N);
    // assembled normal equations: a pair has >= 1 correspondence, so pairs <= min(N(N-1)/2, maxCorr)
    maxPairsA_ = (uint32_t)std::min<size_t>((size_t)N * (N - 1) / 2, (size_t)cfg.maxCorr);
    rowSorted_.alloc(2 * (size_t)cfg.maxCorr + 1);
    rowOther_.alloc(2 * (size_t)cfg.maxCorr + 1);
    rowSeg_.alloc(2 * (size_t)cfg.maxCorr + 1);
    rowDeg_.alloc(N + 1);
    rowNA_.alloc(N + 1);
    pairStart_.alloc(N + 1);
    rowPairStart_.alloc(N + 1);
    pairA_.alloc(maxPairsA_ + 1);
    pairB_.alloc(maxPairsA_ + 1);
    pairCorr_.alloc(maxPairsA_ + 1);
    rowPair_.alloc(2 * (size_t)maxPairsA_ + 1);
    pstat_.alloc(((size_t)maxPairsA_ + 1) * PSTAT);
    dstat_.alloc((size_t)N * DSTAT);
    apPair_.alloc((size_t)N * 8);
    aGran_.alloc((size_t)N * 12);  // [2][N][6]: sparse Ap rows, then the dense off-diagonal products
    fxGran_.alloc(16);
    rzPart_.alloc(N);
    poseBak_.alloc((size_t)N * 6);
    int dev = 0;
    hipDeviceProp_t prop;
    BF_HIP(hipGetDevice(&dev));
    BF_HIP(hipGetDeviceProperties(&prop, dev));
    numCUs_ = prop.multiProcessorCount;
    int occP = 0, occP8 = 0;
    BF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occP, k_pcg_persist<2>, WG, 0));
    BF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occP8, k_pcg_persist<2, PP_NF>, WG, 0));
    persistCapacity_ = (unsigned)std::max(std::min(occP, occP8), 0) * (unsigned)numCUs_;
#ifdef BF_PCG_TIMING
    fprintf(stderr, "k_pcg_persist occupancy: <2> %d, <8> %d workgroups per CU, %d CUs\n", occP, occP8, numCUs_);
#endif
    BF_HIP(hipMemsetAsync(vec_.p, 0, vec_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(ctrl_.p, 0, ctrl_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(sync_.p, 0, sync_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(aGran_.p, 0, aGran_.bytes(), stream_));  // tag 0 is never awaited
    BF_HIP(hipMemsetAsync(fxGran_.p, 0, fxGran_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(imgPairN_.p, 0, imgPairN_.bytes(), stream_));
    BF_HIP(hipMemsetAsync(rowCount_.p, 0, rowCount_.bytes(), stream_));
}

Solver::~Solver() {}

size_t Solver::deviceBytes() const {
    return rowCount_.bytes() * 3 + tileCnt_.bytes() + rowChunk_.bytes() + chunkRow_.bytes() + chunkPart_.bytes() + rowTmp_.bytes() + rowIdx_.bytes() + entries_.bytes() + vec_.bytes() + img_.bytes() +
           T_.bytes() + Tinv_.bytes() + pairs_.bytes() + pairW_.bytes() + pairBlk_.bytes() + diag_.bytes() + jtr_.bytes() +
           rowSorted_.bytes() * 2 + pairA_.bytes() * 2 + pairCorr_.bytes() + rowPair_.bytes() + pstat_.bytes() + dstat_.bytes();
}

void Solver::setShard(uint32_t count, uint32_t index, Comm* comm) {
    BF_REQUIRE(count >= 1 && index < count, BF_ERR_ARG, "shard index / count");
    BF_REQUIRE(!comm || (comm->size() == (int)count && comm->rank() == (int)index), BF_ERR_ARG,
               "communicator size / rank must equal the shard count / index");
    shardCount_ = count;
    shardIndex_ = index;
    comm_ = comm;
}

uint32_t Solver::exportPairs(double* stats, int* pairAB, uint32_t cap) {
    BF_HIP(hipStreamSynchronize(stream_));
    uint32_t np = 0;
    if (lastPairMode_) BF_HIP(hipMemcpy(&np, ctrl_.p + K_NPAIRS_A, 4, hipMemcpyDeviceToHost));
    const uint32_t n = std::min(np, cap);
    if (n && stats) BF_HIP(hipMemcpy(stats, pstat_.p, sizeof(double) * PSTAT * n, hipMemcpyDeviceToHost));
    if (n && pairAB) {
        std::vector<int> A(n), B(n);
        BF_HIP(hipMemcpy(A.data(), pairA_.p, 4 * n, hipMemcpyDeviceToHost));
        BF_HIP(hipMemcpy(B.data(), pairB_.p, 4 * n, hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < n; k++) { pairAB[2 * k] = A[k]; pairAB[2 * k + 1] = B[k]; }
    }
    return np;
}

// CUDASolverBundling::solve (CUDASolverBundling.cpp:187-284) -> solveBundlingStub (SolverBundling.cu:1137-1220)
void Solver::solve(const SolveArgs& s) {
    BF_REQUIRE(s.numImages > 1 && s.numImages <= cfg_.maxImages, BF_ERR_ARG, "numImages out of range");
    BF_REQUIRE(s.numCorr <= cfg_.maxCorr, BF_ERR_CAPACITY, "numCorr exceeds solver capacity");
    BF_REQUIRE(s.nNonLin > 0 && s.wSparse, BF_ERR_ARG, "nNonLin / weights");
    BA a{};
    a.corr = s.corr; a.nCorr = s.numCorr; a.valid = s.valid; a.N = s.numImages; a.maxN = cfg_.maxImages; a.cap = maxCorrPerImage_;
    a.rowCount = rowCount_.p; a.rowStart = rowStart_.p; a.rowLen = rowLen_.p; a.rowTmp = rowTmp_.p; a.rowIdx = rowIdx_.p;
    a.entries = entries_.p; a.entTail = 2u * cfg_.maxCorr + 1u; a.vec = vec_.p; a.img = img_.p; a.T = T_.p; a.Tinv = Tinv_.p; a.ctrl = ctrl_.p;
    a.part = part_.p; a.partIdx = partIdx_.p; a.rot = s.rot; a.trans = s.trans;
    a.pairs = pairs_.p; a.pairW = pairW_.p; a.pairBlk = pairBlk_.p; a.diag = diag_.p; a.jtr = jtr_.p;
    a.pairFlag = pairFlag_.p; a.pairAcc = pairAcc_.p; a.pairProd = pairProd_.p; a.imgPairs = imgPairs_.p; a.imgPairN = imgPairN_.p;
    a.maxPairs = s.numImages * (s.numImages - 1) / 2;
    a.tileCnt = tileCnt_.p; a.tile = tile_for(s.numImages); a.nTiles = div_up(s.numCorr, a.tile);
    a.rowChunk = rowChunk_.p; a.chunkRow = chunkRow_.p; a.chunkPart = chunkPart_.p; a.sync = sync_.p;
    a.cache = s.cache; a.cw = s.cacheW; a.ch = s.cacheH;
    a.fx = s.intrinsics[0]; a.fy = s.intrinsics[1]; a.mx = s.intrinsics[2]; a.my = s.intrinsics[3];
    a.distT = cfg_.denseDistThresh; a.normT = cfg_.denseNormalThresh; a.colT = cfg_.denseColorThresh;
    a.gradMin = cfg_.denseColorGradientMin; a.dmin = cfg_.denseDepthMin; a.dmax = cfg_.denseDepthMax;
    a.sub = cfg_.denseOverlapSubsample ? cfg_.denseOverlapSubsample : 4;
    a.verifyT = cfg_.verifyOptDistThresh;
    a.rowSorted = rowSorted_.p; a.rowOther = rowOther_.p; a.rowSeg = rowSeg_.p; a.rowDeg = rowDeg_.p; a.rowNA = rowNA_.p;
    a.pairStart = pairStart_.p; a.rowPairStart = rowPairStart_.p; a.pairA = pairA_.p; a.pairB = pairB_.p;
    a.pairCorr = pairCorr_.p; a.rowPair = rowPair_.p; a.pstat = pstat_.p; a.dstat = dstat_.p;
    a.apPair = apPair_.p; a.rzPart = rzPart_.p;
    a.aGran = aGran_.p;
    a.fxGran = fxGran_.p;
    a.shardCount = shardCount_; a.shardIndex = shardIndex_; a.pairBound = 0;
    a.earlyOut = cfg_.earlyOut ? 1u : 0u;
    a.poseBak = poseBak_.p;
    a.spinTicks = cfg_.pcgSpinLimitUs ? 100ull * cfg_.pcgSpinLimitUs : PP_SPIN_TICKS;
    // assembled normal equations for sparse-only solves (auto) unless the matrix-free path is forced
    bool denseAny = false;
    for (uint32_t it = 0; it < s.nNonLin && s.cache; it++)
        denseAny = denseAny || (s.wDenseDepth && s.wDenseDepth[it] > 0.0f) || (s.wDenseColor && s.wDenseColor[it] > 0.0f);
    (void)denseAny;
    const bool pairMode = cfg_.normalEquations != 1;
    BF_REQUIRE(pairMode || shardCount_ == 1, BF_ERR_ARG, "sharded solves use the assembled normal equations");
    a.pairMode = pairMode ? 1u : 0u;
    lastPairMode_ = pairMode;

    const unsigned corrGrid = std::max(1u, std::min(div_up(s.numCorr, WG), (unsigned)numCUs_ * 8));
    // chunk kernels: one wave per chunk of CH row entries, up to 16 waves per CU
    const size_t chunkBound = div_up(2 * (size_t)s.numCorr, (size_t)CH) + s.numImages;
    const unsigned rowGrid = std::max(1u, std::min(div_up(chunkBound, (size_t)(WG / 64)), (unsigned)numCUs_ * 4));
    const bool timed = solveClock_.enabled();
    if (timed) solveClock_.start(stream_);
    k_solve_begin<<<1, 64, 0, stream_>>>(ctrl_.p, s.gate);
    BF_LAUNCH_CHECK();
    if (s.rebuildJT) {
        const size_t lds = sizeof(int) * s.numImages;
        if (a.nTiles) k_tile_count<<<a.nTiles, 64, lds, stream_>>>(a);
        k_tile_scan<<<s.numImages, WG, 0, stream_>>>(a);
        k_scan<<<1, WG, 0, stream_>>>(a);
        if (a.nTiles) k_tile_fill<<<a.nTiles, 64, lds, stream_>>>(a);
        k_compact_rows<<<s.numImages, WG, 0, stream_>>>(a);
        k_chunks<<<1, WG, 0, stream_>>>(a);
        BF_LAUNCH_CHECK();
        pairTable_ = false;
    }
    uint32_t bound = 0;
    if (pairMode) {
        if (!pairTable_) {
            k_pair_sort<<<s.numImages, WG, 0, stream_>>>(a);
            k_pair_scan<<<1, WG, 0, stream_>>>(a);
            k_pair_fill<<<s.numImages, 64, 0, stream_>>>(a);
            k_pair_rows<<<s.numImages, 64, 0, stream_>>>(a);
            BF_LAUNCH_CHECK();
            pairTable_ = true;
            pairCountHost_ = 0;
        }
        if (comm_ && comm_->size() > 1) {
            // the all-reduce count must be known on the host: the caller's bound, or the pair count
            // read back once per table build
            if (s.pairBound) {
                bound = s.pairBound;
            } else {
                if (!pairCountHost_) {
                    BF_HIP(hipMemcpyAsync(&pairCountHost_, ctrl_.p + K_NPAIRS_A, 4, hipMemcpyDeviceToHost, stream_));
                    BF_HIP(hipStreamSynchronize(stream_));
                }
                bound = std::max(pairCountHost_, 1u);
            }
            BF_REQUIRE(bound <= maxPairsA_, BF_ERR_CAPACITY, "pair bound exceeds the solver's pair capacity");
            a.pairBound = bound;
        }
    }
    if (pairMode) k_pair_gather<<<(unsigned)numCUs_ * 4, WG, 0, stream_>>>(a);
    const unsigned pairRowGrid = std::max(1u, std::min(div_up(s.numImages, WG / 64), (unsigned)numCUs_ * 4));
    bool transformsDone = false;
    for (uint32_t it = 0; it < s.nNonLin; it++) {
        const float wS = s.wSparse[it];
        const float wD = s.wDenseDepth ? s.wDenseDepth[it] : 0.0f;
        const float wC = s.wDenseColor ? s.wDenseColor[it] : 0.0f;
        const bool dense = (wD > 0.0f || wC > 0.0f) && s.cache != nullptr;
        // the next sparse pair-mode step's transforms come from this step's k_gn_end
        const bool nextDense = it + 1 < s.nNonLin && s.cache != nullptr &&
                               ((s.wDenseDepth && s.wDenseDepth[it + 1] > 0.0f) || (s.wDenseColor && s.wDenseColor[it + 1] > 0.0f));
        const float nextW = (pairMode && it + 1 < s.nNonLin && !nextDense && s.wSparse[it + 1] > 0.0f) ? s.wSparse[it + 1] : 0.0f;
        if (!transformsDone) k_transforms<<<div_up(s.numImages, 64), 64, 0, stream_>>>(a, wS, dense ? 1 : 0, 1, 1);
        transformsDone = nextW > 0.0f;
        if (pairMode) {
            if (dense) {
                k_dense_reset<<<64, WG, 0, stream_>>>(a);
                k_dense_overlap<<<dim3(s.numImages, s.numImages), 64, 0, stream_>>>(a);
                k_dense_compact<<<1, 256, 0, stream_>>>(a);
                k_dense_count<<<std::min(a.maxPairs, (uint32_t)numCUs_ * 8), WG, 0, stream_>>>(a);
                k_dense_build<<<std::min(a.maxPairs, (uint32_t)numCUs_ * 4), WG, 0, stream_>>>(a, wD, wC);
                k_dense_lists<<<s.numImages, 64, 0, stream_>>>(a);
                BF_LAUNCH_CHECK();
            }
            k_pair_stats<<<(unsigned)numCUs_ * 4, WG, 0, stream_>>>(a);
            BF_LAUNCH_CHECK();
            if (comm_ && comm_->size() > 1) comm_->allreduceSum(pstat_.p, (size_t)bound * PSTAT, stream_);
            k_pair_init<<<pairRowGrid, WG, 0, stream_>>>(a, wS);
            int recoverRB = 0;  // the finisher form of a persistent launch this GN step
            if (s.numImages <= (uint32_t)SMALL_N) {
                if (s.nLin) k_pcg_small<<<1, SMALL_WG, 0, stream_>>>(a, wS, (int)s.nLin);
            } else {
                // one launch for the GN step's PCG loop when its grid is co-resident: up to 513 images
                // (one finisher workgroup, rows in registers, dense term included) with room to spare; up
                // to 2 017 sparse-only (config 4's 2 001 keyframes) with PP_NF finisher workgroups within
                // the occupancy query's capacity (persistent launches are serialized per device, below)
                const bool smallN = s.numImages <= 2u * WG + 1u;
                const unsigned nF = smallN ? 1u : (unsigned)PP_NF;
                const unsigned nW = div_up(s.numImages - 1u, (unsigned)(WG / 64));
                unsigned persistGrid = nF + nW;
                if (persistGrid > PP_SHADOW) persistGrid += nF;  // the row-less workgroups on the finishers' CUs
                const bool small = smallN && persistGrid * 2u <= persistCapacity_;
                // the PP_NF finishers own rows 1 .. 2 * PP_NF * WG: beyond that no finisher would tag a row's p
                const bool wide = !smallN && !dense && s.numImages <= 2u * (unsigned)PP_NF * WG + 1u &&
                                  persistGrid <= persistCapacity_;
                if (BF_PCG_PERSISTENT && cfg_.pcgLaunch == 0 && s.nLin < 255u && s.numImages >= 2u && (small || wide)) {
#ifdef BF_PCG_TIMING
                    {
                        std::vector<unsigned long long> z(1024 * 4, 0ull);
                        BF_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_pcgT), z.data(), z.size() * 8, 0, hipMemcpyHostToDevice, stream_));
                    }
#endif
                    if (s.nLin) {
                        // ranks of a loopback group (one GPU) issue their persistent launches in rank order
                        struct Turn {
                            Comm* c;
                            explicit Turn(Comm* x) : c(x) { if (c) c->orderedLaunchBegin(); }
                            ~Turn() { if (c) c->orderedLaunchEnd(); }
                        } turn(comm_ && comm_->size() > 1 ? comm_ : nullptr);
                        // persistent launches of every solver on this device run one at a time: two
                        // partly resident persistent grids could each wait on the other's workgroups
                        PersistGate& pg = persist_gate();
                        std::lock_guard<std::mutex> lk(pg.mu);
                        // always wait, on the same stream too: a destroyed solver's stream handle may be
                        // reused by a new solver whose launch must still follow the old one (cheap in order)
                        if (pg.ev) BF_HIP(hipStreamWaitEvent(stream_, pg.ev, 0));
                        // dispatch-stamped events (pcgClock): the launch's own device time, for the in-loop
                        // time per PCG iteration beside the standalone one
                        hipEvent_t e0 = nullptr, e1 = nullptr;
                        const bool timed = pcgClock_.enabled();
                        if (timed) pcgClock_.slot(e0, e1);
                        if (small)
                            hipExtLaunchKernelGGL(k_pcg_persist<2>, dim3(persistGrid), dim3(WG), 0, stream_, e0, e1, 0, a, wS,
                                                  (int)s.nLin, pcgEpoch_);
                        else
                            hipExtLaunchKernelGGL((k_pcg_persist<2, PP_NF>), dim3(persistGrid), dim3(WG), 0, stream_, e0, e1, 0, a,
                                                  wS, (int)s.nLin, pcgEpoch_);
                        BF_LAUNCH_CHECK();
                        if (timed) pcgClock_.commit();
                        if (!pg.ev) BF_HIP(hipEventCreateWithFlags(&pg.ev, hipEventDisableTiming));
                        BF_HIP(hipEventRecord(pg.ev, stream_));
                        pg.stream = stream_;
                        pcgEpoch_ = (pcgEpoch_ + 1) & 0xFFFFFFu;
                        recoverRB = s.numImages <= 2u * WG + 1u ? 2 : 8;  // k_gn_end redoes a timed-out step
                    }
#ifdef BF_PCG_TIMING
                    {
                        std::vector<unsigned long long> t(1024 * 4);
                        BF_HIP(hipMemcpyFromSymbolAsync(t.data(), HIP_SYMBOL(g_pcgT), t.size() * 8, 0, hipMemcpyDeviceToHost, stream_));
                        BF_HIP(hipStreamSynchronize(stream_));
                        {   // per-WG stamps (iterations < 64): maxima into t[.][0..1]; spread and per-WG work time
                            std::vector<unsigned long long> W(64 * 1024 * 2);
                            BF_HIP(hipMemcpyFromSymbol(W.data(), HIP_SYMBOL(g_pcgW), W.size() * 8));
                            double spreadSeen = 0, spreadArr = 0, meanWork = 0, maxWork = 0; int nq = 0;
                            for (uint32_t q = 1; q < 63 && q + 2 < s.nLin; q++) {
                                unsigned long long s0 = ~0ull, s1 = 0, a0 = ~0ull, a1 = 0; double wsum = 0, wmax = 0; int nw = 0, bmax = 0;
                                for (uint32_t b = 1; b < persistGrid && b < 1024; b++) {
                                    if (b == PP_SHADOW) continue;  // no rows
                                    const unsigned long long fs = W[(q * 1024 + b) * 2], ar = W[(q * 1024 + b) * 2 + 1];
                                    if (!fs || !ar) continue;
                                    s0 = std::min(s0, fs); s1 = std::max(s1, fs); a0 = std::min(a0, ar); a1 = std::max(a1, ar);
                                    if ((double)ar - (double)fs > wmax) bmax = (int)b;
                                    wsum += (double)ar - (double)fs; wmax = std::max(wmax, (double)ar - (double)fs); nw++;
                                }
                                if (!nw) continue;
                                if (q < 6) {  // the slowest workgroups of a few iterations
                                    std::vector<std::pair<double, int>> v;
                                    for (uint32_t b = 1; b < persistGrid && b < 1024; b++) {
                                    if (b == PP_SHADOW) continue;  // no rows
                                        const unsigned long long fs = W[(q * 1024 + b) * 2], ar = W[(q * 1024 + b) * 2 + 1];
                                        if (fs && ar) v.push_back({((double)ar - (double)fs) / 100, (int)b});
                                    }
                                    std::sort(v.rbegin(), v.rend());
                                    fprintf(stderr, "  iteration %u slowest WGs (us:block):", q);
                                    for (size_t k = 0; k < v.size() && k < 8; k++) fprintf(stderr, " %.2f:%d", v[k].first, v[k].second);
                                    fprintf(stderr, "\n");
                                    std::vector<std::pair<double, int>> fsv;
                                    for (uint32_t b = 1; b < persistGrid && b < 1024; b++) {
                                    if (b == PP_SHADOW) continue;  // no rows
                                        const unsigned long long fs = W[(q * 1024 + b) * 2];
                                        if (fs) fsv.push_back({((double)fs - (double)s0) / 100, (int)b});
                                    }
                                    std::sort(fsv.rbegin(), fsv.rend());
                                    fprintf(stderr, "  iteration %u latest flag-seen WGs (us after first:block):", q);
                                    for (size_t k = 0; k < fsv.size() && k < 12; k++) fprintf(stderr, " %.2f:%d", fsv[k].first, fsv[k].second);
                                    int late = 0;
                                    for (auto& e : fsv) late += e.first > 2.0;
                                    fprintf(stderr, "  (%d WGs > 2 us)\n", late);
                                }
                                (void)bmax;
                                t[q * 4] = s1; t[q * 4 + 1] = a1;
                                spreadSeen += (double)(s1 - s0); spreadArr += (double)(a1 - a0); meanWork += wsum / nw; maxWork += wmax; nq++;
                            }
                            for (uint32_t q = 64; q < 1024; q++) t[q * 4] = t[q * 4 + 1] = 0;
                            if (nq) fprintf(stderr, "  workers (us, iterations 1-62): flag-seen spread %.2f  arrival spread %.2f  per-WG work mean %.2f  max %.2f\n",
                                            spreadSeen / nq / 100, spreadArr / nq / 100, meanWork / nq / 100, maxWork / nq / 100);
                        }
                        // per iteration q: [0] latest worker saw the flag of q, [1] latest worker arrival of q,
                        // [2] finisher saw all arrivals of q, [3] finisher published q + 1
                        double w = 0, ar = 0, fi = 0, bc = 0; int n = 0;
                        for (uint32_t q = 1; q + 2 < s.nLin && q < 1023; q++) {
                            const unsigned long long* r = &t[q * 4];
                            const unsigned long long* nx = &t[(q + 1) * 4];
                            if (!r[0] || !r[1] || !r[2] || !r[3] || !nx[0]) continue;
                            w += (double)r[1] - (double)r[0]; ar += (double)r[2] - (double)r[1];
                            fi += (double)r[3] - (double)r[2]; bc += (double)nx[0] - (double)r[3]; n++;
                        }
                        if (n) fprintf(stderr, "persistent pcg (us, mean over %d iterations): workers flag->arrive %.2f  arrival->finisher %.2f  finisher %.2f  flag->last worker %.2f  total %.2f\n",
                                       n, w / n / 100, ar / n / 100, fi / n / 100, bc / n / 100, (w + ar + fi + bc) / n / 100);
                        std::vector<unsigned long long> g(1024 * 6);
                        BF_HIP(hipMemcpyFromSymbol(g.data(), HIP_SYMBOL(g_pcgS), g.size() * 8));
                        double f0 = 0, f1 = 0, f2 = 0, f3v = 0; int m = 0;
                        for (uint32_t q = 1; q + 2 < s.nLin && q < 1023; q++) {
                            const unsigned long long* r = &t[q * 4];
                            const unsigned long long* G = &g[q * 6];
                            if (!r[2] || !r[3] || !G[0] || !G[1] || !G[2]) continue;
                            f0 += (double)G[0] - (double)r[2]; f1 += (double)G[1] - (double)G[0];
                            f2 += (double)G[2] - (double)G[1]; f3v += (double)r[3] - (double)G[2]; m++;
                        }
                        if (m) fprintf(stderr, "  finisher (us): Ap + pAp sum %.2f  delta/r/z + rz sum %.2f  p + stores %.2f  drain + flag %.2f\n",
                                       f0 / m / 100, f1 / m / 100, f2 / m / 100, f3v / m / 100);
                        std::vector<int> rps(s.numImages + 1);
                        BF_HIP(hipMemcpy(rps.data(), rowPairStart_.p, rps.size() * 4, hipMemcpyDeviceToHost));
                        int dmax = 0, over192 = 0, over448 = 0;
                        for (uint32_t q = 1; q < s.numImages; q++) {
                            const int dg = rps[q + 1] - rps[q];
                            dmax = std::max(dmax, dg); over192 += dg > 192; over448 += dg > 448;
                        }
                        fprintf(stderr, "  row degrees: mean %.1f  max %d  rows > 192: %d  > 448: %d\n",
                                (double)(rps[s.numImages] - rps[1]) / (s.numImages - 1), dmax, over192, over448);
                    }
#endif
                } else if (s.numImages <= 2u * WG + 1u) {
#ifdef BF_PCG_TIMING
                    {
                        std::vector<unsigned long long> init(1024 * 4);
                        for (int q = 0; q < 1024; q++) { init[q * 4] = ~0ull; init[q * 4 + 1] = 0; init[q * 4 + 2] = 0; init[q * 4 + 3] = 0; }
                        BF_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_pcgT), init.data(), init.size() * 8, 0, hipMemcpyHostToDevice, stream_));
                    }
#endif
                    for (uint32_t li = 0; li < s.nLin; li++) k_pcg_pairs<2><<<pairRowGrid, WG, 0, stream_>>>(a, wS, (int)li, (int)s.nLin);
#ifdef BF_PCG_TIMING
                    {
                        std::vector<unsigned long long> t(1024 * 4);
                        BF_HIP(hipMemcpyFromSymbolAsync(t.data(), HIP_SYMBOL(g_pcgT), t.size() * 8, 0, hipMemcpyDeviceToHost, stream_));
                        BF_HIP(hipStreamSynchronize(stream_));
                        double sA = 0, sW = 0, sF = 0, sAll = 0; int n = 0;
                        for (uint32_t q = 1; q + 1 < s.nLin && q < 1024; q++) {
                            const unsigned long long* r = &t[q * 4];
                            const unsigned long long* nx = &t[(q + 1) * 4];
                            if (!r[3] || !nx[3] || r[0] == ~0ull) continue;
                            sA += (double)(r[1] - r[0]); sW += (double)(r[2] - r[1]); sF += (double)(r[3] - r[2]);
                            sAll += (double)(nx[0] - r[0]); n++;
                        }
                        if (n) fprintf(stderr, "pcg timing (us, mean over %d launches): phase A %.2f  arrival %.2f  finisher %.2f  start-to-next-start %.2f\n",
                                       n, sA / n / 100.0, sW / n / 100.0, sF / n / 100.0, sAll / n / 100.0);
                        std::vector<unsigned long long> g(1024 * 6);
                        BF_HIP(hipMemcpyFromSymbol(g.data(), HIP_SYMBOL(g_pcgS), g.size() * 8));
                        double d0 = 0, d1 = 0, d2 = 0, d3 = 0, sk = 0; int m = 0;
                        for (uint32_t q = 1; q + 1 < s.nLin && q < 1024; q++) {
                            const unsigned long long* G = &g[q * 6];
                            if (!G[4] || !G[1] || !G[2] || !G[3]) continue;
                            sk += (double)(G[0] - t[q * 4]); d0 += (double)(G[1] - G[0]); d1 += (double)(G[2] - G[1]);
                            d2 += (double)(G[3] - G[2]); d3 += (double)(G[4] - G[3]); m++;
                        }
                        if (m) fprintf(stderr, "  last WG (us): start skew %.2f  row start loads %.2f  pair loop %.2f  wave sums %.2f  diag+store+arrival %.2f\n",
                                       sk / m / 100.0, d0 / m / 100.0, d1 / m / 100.0, d2 / m / 100.0, d3 / m / 100.0);
                    }
#endif
                } else {
                    for (uint32_t li = 0; li < s.nLin; li++) k_pcg_pairs<8><<<pairRowGrid, WG, 0, stream_>>>(a, wS, (int)li, (int)s.nLin);
                }
            }
            BF_LAUNCH_CHECK();
            if (recoverRB == 2) k_gn_end<2><<<1, WG, 0, stream_>>>(a, (int)it, (int)s.nNonLin, wS, (int)s.nLin, nextW);
            else if (recoverRB == 8) k_gn_end<8><<<1, WG, 0, stream_>>>(a, (int)it, (int)s.nNonLin, wS, (int)s.nLin, nextW);
            else k_gn_end<0><<<1, WG, 0, stream_>>>(a, (int)it, (int)s.nNonLin, wS, (int)s.nLin, nextW);
            BF_LAUNCH_CHECK();
            continue;
        }
        if (dense) {
            k_dense_reset<<<64, WG, 0, stream_>>>(a);
            k_dense_overlap<<<dim3(s.numImages, s.numImages), 64, 0, stream_>>>(a);
            k_dense_compact<<<1, 256, 0, stream_>>>(a);
            k_dense_count<<<std::min(a.maxPairs, (uint32_t)numCUs_ * 8), WG, 0, stream_>>>(a);
            k_dense_build<<<std::min(a.maxPairs, (uint32_t)numCUs_ * 4), WG, 0, stream_>>>(a, wD, wC);
            k_dense_lists<<<s.numImages, 64, 0, stream_>>>(a);
            BF_LAUNCH_CHECK();
        }
        k_entries<<<rowGrid, WG, 0, stream_>>>(a);
        k_init<<<rowGrid, WG, 0, stream_>>>(a, wS);
        BF_LAUNCH_CHECK();
        for (uint32_t li = 0; li < s.nLin; li++) k_pcg<<<rowGrid, WG, 0, stream_>>>(a, wS, (int)li, (int)s.nLin);
        BF_LAUNCH_CHECK();
        k_gn_end<0><<<1, WG, 0, stream_>>>(a, (int)it, (int)s.nNonLin, wS, (int)s.nLin, 0.0f);
        BF_LAUNCH_CHECK();
        transformsDone = false;
    }
    if (s.findMaxResidual) {
        // T from the final poses (ctrl untouched), then computeMaxResidual with the weightSparse of
        // the last GN iteration that ran (CUDASolverBundling.cpp:313-427)
        k_transforms<<<div_up(s.numImages, 64), 64, 0, stream_>>>(a, 0.0f, 0, 0, 0);
        k_residuals<<<corrGrid, WG, 0, stream_>>>(a);
        BF_LAUNCH_CHECK();
    }
    if (timed) solveClock_.stop(stream_);
}

SolveResult Solver::result() {
    uint32_t c[K_COUNT];
    BF_HIP(hipMemcpyAsync(c, ctrl_.p, sizeof(c), hipMemcpyDeviceToHost, stream_));
    BF_HIP(hipStreamSynchronize(stream_));
    return decodeResult(c);
}

void Solver::resultAsync(uint32_t* pinnedCtrl) {
    BF_HIP(hipMemcpyAsync(pinnedCtrl, ctrl_.p, sizeof(uint32_t) * K_COUNT, hipMemcpyDeviceToHost, stream_));
}

void Solver::removeMaxResidualAsync(BFEntryJ* corr, uint32_t n, int* valid, uint32_t numImages, float thresh) {
    k_pick_maxres_pair<<<1, 64, 0, stream_>>>(ctrl_.p, corr, thresh);
    BF_LAUNCH_CHECK();
    if (n) k_invalidate_picked_pair<<<std::max(1u, std::min(div_up(n, 256), 1024u)), 256, 0, stream_>>>(ctrl_.p, corr, n);
    k_check_frames_if_removed<<<div_up(numImages, 64), 64, 0, stream_>>>(ctrl_.p, rowCount_.p, valid, numImages);
    BF_LAUNCH_CHECK();
}

SolveResult Solver::decodeResult(const uint32_t* c) {
    SolveResult r{};
    r.gnIterations = c[K_GN_ITERS];
    r.pcgIterations = c[K_PCG_ITERS];
    std::memcpy(&r.maxResidual, &c[K_MAXRES], 4);
    r.maxResidualIndex = (int32_t)c[K_MAXIDX];
    std::memcpy(&r.energy, &c[K_ENERGY], 4);
    r.highResidualCount = c[K_HIGHCOUNT];
    r.numDensePairs = c[K_NPAIRS];
    r.error = c[K_ERROR];
    r.removedI = c[K_RM_I];
    r.removedJ = c[K_RM_J];
    r.skipped = c[K_SKIPPED];
    r.verifyUsed = c[K_VERIFY_USED];
    r.verifyOk = c[K_VERIFY_OK];
    return r;
}

void Solver::verify(const VerifyParams& p) {
    BF_REQUIRE(p.numImages >= 1 && p.numImages <= cfg_.maxImages, BF_ERR_ARG, "verify: numImages out of range");
    BF_REQUIRE(p.cache && p.T && p.valid, BF_ERR_ARG, "verify: trajectory, valid flags and cache frames are required");
    VerifyArgs v{};
    v.T = p.T; v.valid = p.valid; v.N = p.numImages; v.cache = p.cache; v.W = p.cacheW; v.H = p.cacheH;
    for (int k = 0; k < 16; k++) v.K[k] = 0.0f;  // mat4f intrinsics of the cache (CUDACache.cpp:20-24)
    v.K[0] = p.intrinsics[0]; v.K[2] = p.intrinsics[2];
    v.K[5] = p.intrinsics[1]; v.K[6] = p.intrinsics[3];
    v.K[10] = 1.0f; v.K[15] = 1.0f;
    v.distT = p.distThresh; v.normT = p.normalThresh; v.errT = p.errThresh; v.corrT = p.corrThresh;
    v.dmin = p.depthMin; v.dmax = p.depthMax; v.percentT = p.percentThresh;
    v.nCorr = p.numCorr; v.always = p.always ? 1u : 0u; v.ctrl = ctrl_.p; v.stats = p.pairStats;
    k_verify_begin<<<1, 64, 0, stream_>>>(v);
    if (p.numImages >= 2) k_verify_pairs<<<p.numImages * p.numImages, WG, 0, stream_>>>(v);
    BF_LAUNCH_CHECK();
}

const int* Solver::verifyFlag() const { return reinterpret_cast<const int*>(ctrl_.p + K_VERIFY_OK); }

void seed_keyframe(const float* localRot, const float* localTrans, uint32_t last, float* rot, float* trans, uint32_t s,
                   hipStream_t st, const int* gate) {
    k_seed_keyframe<<<1, 64, 0, st>>>(localRot, localTrans, last, rot, trans, s, gate);
    BF_LAUNCH_CHECK();
}
void set_gate(int* gate, const int* src, hipStream_t st) {
    k_set_gate<<<1, 64, 0, st>>>(gate, src);
    BF_LAUNCH_CHECK();
}
void invalidate_local(const int* gate, uint32_t s, int* valid, BFEntryJ* corr, uint32_t n, hipStream_t st) {
    k_invalidate_local<<<std::max(1u, std::min(div_up(n, 256), 1024u)), 256, 0, st>>>(gate, s, valid, corr, n);
    BF_LAUNCH_CHECK();
}

void matrices_to_poses(const float* T, uint32_t n, float* rot, float* trans, const int* valid, hipStream_t s) {
    if (!n) return;
    k_m2p<<<div_up(n, 64), 64, 0, s>>>(T, n, rot, trans, valid);
    BF_LAUNCH_CHECK();
}
void poses_to_matrices(const float* rot, const float* trans, uint32_t n, float* T, const int* valid, hipStream_t s) {
    if (!n) return;
    k_p2m<<<div_up(n, 64), 64, 0, s>>>(rot, trans, n, T, valid);
    BF_LAUNCH_CHECK();
}
void invalidate_image_pair(BFEntryJ* corr, uint32_t n, uint32_t i, uint32_t j, hipStream_t s) {
    if (!n) return;
    k_invalidate_pair<<<div_up(n, 128), 128, 0, s>>>(corr, n, i, j);
    BF_LAUNCH_CHECK();
}
void check_invalid_frames(const int* numEntries, int* valid, uint32_t numImages, BFEntryJ* corr, uint32_t nCorr,
                          bool comprehensive, hipStream_t s) {
    const uint32_t n = std::max(numImages, comprehensive ? nCorr : 0u);
    k_check_frames<<<std::max(1u, std::min(div_up(n, 256), 4096u)), 256, 0, s>>>(numEntries, valid, numImages, corr, nCorr,
                                                                                  comprehensive ? 1 : 0);
    BF_LAUNCH_CHECK();
}

}  // namespace bf
