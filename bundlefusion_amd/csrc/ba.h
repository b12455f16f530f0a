// ba.h — MI355X sparse-then-dense bundle adjuster (replaces CUDASolverBundling,
// Source/Solver/CUDASolverBundling.h/.cpp, and solveBundlingStub, Source/Solver/SolverBundling.cu).
//
// Device layout (all resident in HBM, sized for maxImages / maxCorr at construction):
//   rowCount/rowStart/rowLen   per-image CSR of correspondence indices, built deterministically
//                              (ascending correspondence index, as a serial replay of the
//                              reference's atomic table build, SolverBundling.cu:1226-1248) by a
//                              tiled stable counting sort (tileCnt: per-row, per-tile counts)
//   chunks                     every row cut into chunks of CH entries: the work unit of one wave
//                              in the GN/PCG kernels; chunk partials are summed per row in chunk
//                              order by the finishing workgroup (deterministic, no float atomics)
//   entries                    per row entry, rebuilt each GN iteration: {T_self*p_self, other},
//                              {T_other*p_other} — 32 B, streamed contiguously by the PCG loop
//   vec                        per-image 8-float vectors: x is the caller's (rot, trans);
//                              delta, r, z, p, Ap, M (Jacobi preconditioner)
//   dense                      block-sparse JtJ: per-image 6x6 diagonal blocks, per-pair 6x6
//                              off-diagonal blocks, Jtr (instead of the reference's (6N)^2 matrix)
//   ctrl                       device-resident solver state (tickets, early-exit flags, scalars)
// A solve is enqueued asynchronously on the solver's stream: PCG early exit and GN convergence
// are evaluated on the device, so there is no host round trip inside solve (the reference
// copies scanAlpha to the host every PCG iteration, SolverBundling.cu:1089).
#pragma once
#include <vector>
#include "../../include/bf/bf.h"
#include "bf_math.h"
#include "bf_runtime.h"
#include "comm.h"

namespace bf {

struct SolverConfig {
    uint32_t maxImages;
    uint32_t maxCorr;
    float denseDistThresh;        // s_denseDistThresh 0.15
    float denseNormalThresh;      // s_denseNormalThresh 0.97
    float denseColorThresh;       // s_denseColorThresh 0.1
    float denseColorGradientMin;  // s_denseColorGradientMin 0.005
    float denseDepthMin;          // s_denseDepthMin 0.5
    float denseDepthMax;          // s_denseDepthMax 4.0
    uint32_t denseOverlapSubsample;  // s_denseOverlapCheckSubsampleFactor 4
    float verifyOptDistThresh;    // 0.02 (CUDASolverBundling.cpp:34)
    int normalEquations;          // 0 auto (assembled for sparse-only solves), 1 matrix-free, 2 assembled
    bool earlyOut = true;         // the reference's ENABLE_EARLY_OUT build (SolverBundling.cu:7)
    int pcgLaunch = 0;            // 0 auto (persistent PCG launch when it fits), 1 one launch per iteration
    uint32_t pcgSpinLimitUs = 0;  // bound of each persistent-PCG wait (0: 2 s); tests force the recovery path with it
};

struct SolveArgs {
    BFEntryJ* corr;
    uint32_t numCorr;
    const int* valid;
    uint32_t numImages;
    uint32_t nNonLin, nLin;
    const float* wSparse;  // host arrays [nNonLin]
    const float* wDenseDepth;
    const float* wDenseColor;
    const BFCachedFrame* cache;  // device array [numImages] or null
    uint32_t cacheW, cacheH;
    float intrinsics[4];
    float* rot;    // device float3[numImages], in/out
    float* trans;  // device float3[numImages], in/out
    bool rebuildJT;
    bool findMaxResidual;
    uint32_t pairBound = 0;  // host-known upper bound on image pairs (sharded solves; 0: read it back)
    // device int read when the solve starts: 0 skips the whole solve (no pose change, no residual
    // analysis, so no max-residual removal). The reconstruction loop gates a submap's global solve on
    // its local verification (OnlineBundler.cpp:351-360, :399-405: an invalid local is not solved).
    const int* gate = nullptr;
};

// Local-submap verification: CUDASolverBundling::useVerification (CUDASolverBundling.cpp:454-476)
// -> Bundler::optimize (Bundler.cpp:259-274) -> SIFTImageManager::VerifyTrajectoryCU
// (SiftGPU/SIFTImageManager.cu:1036-1159), defaults of zParametersBundlingDefault.txt:55-64.
struct VerifyParams {
    const float* T;              // device float4x4[n] camera -> world (the solved trajectory)
    const int* valid;            // device int[n]
    uint32_t numImages;
    const BFCachedFrame* cache;  // device array [n]
    uint32_t cacheW, cacheH;
    float intrinsics[4];         // fx fy mx my of the cache frames
    float distThresh = 0.15f;    // s_projCorrDistThres
    float normalThresh = 0.97f;  // s_projCorrNormalThres
    float errThresh = 0.05f;     // s_verifyOptErrThresh
    float corrThresh = 0.001f;   // s_verifyOptCorrThresh
    float percentThresh = 0.05f; // m_verifyOptPercentThresh (CUDASolverBundling.cpp:36)
    float depthMin = 0.1f, depthMax = 3.0f;  // Bundler.cpp:267
    uint32_t numCorr = 0;        // the solve's correspondence count (useVerification's denominator)
    bool always = false;         // true: skip useVerification and check every pair
    float* pairStats = nullptr;  // optional device float[n*n*3]: {sum residual, sum weight, #corr} per pair i < j
};

struct SolveResult {
    uint32_t gnIterations;
    uint32_t pcgIterations;
    float maxResidual;
    int32_t maxResidualIndex;
    float energy;
    uint32_t highResidualCount;
    uint32_t numDensePairs;
    uint32_t error;
    uint32_t removedI = 0xFFFFFFFFu, removedJ = 0xFFFFFFFFu;  // pair invalidated by removeMaxResidualAsync
    uint32_t skipped = 0;      // the solve's gate was 0
    uint32_t verifyUsed = 0;   // the last verify ran its pair check
    uint32_t verifyOk = 0;     // ... and its outcome (1 valid)
};

class Solver {
public:
    Solver(const SolverConfig& cfg, hipStream_t stream);
    ~Solver();
    void solve(const SolveArgs& a);       // async
    SolveResult result();                 // synchronizes
    // async variants for the reconstruction loop: copy the result words into pinned host memory
    // (kResultWords words) and decode them once the stream has passed that point
    void resultAsync(uint32_t* pinnedCtrl);
    static SolveResult decodeResult(const uint32_t* ctrl);
    static constexpr uint32_t kResultWords = 19;
    // image count up to which a persistent global PCG runs with one finisher workgroup (2 rows per
    // thread): its grid, about N / 4 + 2 workgroups, takes at most a quarter of the device's slots
    static constexpr uint32_t kSmallPersistImages = 2 * 256 + 1;
    // device-side SBA::removeMaxResidualCUDA after a solve with findMaxResidual
    void removeMaxResidualAsync(BFEntryJ* corr, uint32_t n, int* valid, uint32_t numImages, float thresh);
    // async local verification after a solve with findMaxResidual (its high-residual count decides
    // whether the pair check runs); the outcome is the device int verifyFlag() (1 valid, 0 invalid)
    void verify(const VerifyParams& p);
    const int* verifyFlag() const;
    const int* numEntriesPerRow() const { return rowCount_.p; }  // getVarToCorrNumEntriesPerRow
    hipStream_t stream() const { return stream_; }
    // moves the solver's later work to another stream (the caller orders it after this one's)
    void setStream(hipStream_t s) { stream_ = s; }
    const SolverConfig& config() const { return cfg_; }
    size_t deviceBytes() const;
    // sharded global solve: this handle builds the normal-equation blocks of the
    // image pairs p with p % count == index; comm (may be null: no exchange, tests) sums them
    void setShard(uint32_t count, uint32_t index, Comm* comm);
    // assembled normal equations of the last GN iteration: per pair (a, b) the 28 sufficient
    // statistics (see ba.hip, k_pair_stats); synchronizes
    uint32_t exportPairs(double* stats, int* pairAB, uint32_t cap);
    KernelClock& solveClock() { return solveClock_; }  // whole-solve device time (ms/GN-iter)
    KernelClock& pcgClock() { return pcgClock_; }      // device time of the persistent PCG launches

private:
    KernelClock solveClock_;
    KernelClock pcgClock_;
    SolverConfig cfg_;
    hipStream_t stream_;
    uint32_t maxCorrPerImage_;
    uint32_t maxPairs_;
    int numCUs_;
    unsigned persistCapacity_ = 0;  // co-resident workgroups of k_pcg_persist (occupancy query x CUs)
    uint32_t maxTiles_;
    size_t maxChunks_;
    DevBuf<int> rowCount_, rowStart_, rowLen_;
    DevBuf<int> tileCnt_, rowChunk_, chunkRow_;
    DevBuf<float4> chunkPart_;
    DevBuf<uint32_t> sync_;  // grid hand-off counters / flags (64 B apart)
    DevBuf<int> rowTmp_, rowIdx_;
    DevBuf<float4> entries_;
    DevBuf<float> vec_;     // [N][8] per field
    DevBuf<float> img_;     // per-image scalars [2][N]
    DevBuf<float> T_;       // [N][16]
    DevBuf<float> Tinv_;    // [N][16]
    DevBuf<uint32_t> ctrl_;
    DevBuf<float> part_;    // per-workgroup partials
    DevBuf<int> partIdx_;
    DevBuf<uint2> pairs_;
    DevBuf<float> pairW_;
    DevBuf<float> pairBlk_;  // [maxPairs][36]
    DevBuf<float> diag_;     // [N][36]
    DevBuf<float> jtr_;      // [N][6]
    DevBuf<uint32_t> pairFlag_;  // [N][N]
    DevBuf<float> pairAcc_;      // [maxPairs][54]
    DevBuf<float> pairProd_;     // [N][8]
    DevBuf<uint32_t> imgPairs_;  // [N][N]
    DevBuf<uint32_t> imgPairN_;  // [N]
    // assembled (pair) normal equations
    uint32_t maxPairsA_ = 0;
    uint32_t shardCount_ = 1, shardIndex_ = 0;
    Comm* comm_ = nullptr;
    bool pairTable_ = false;       // pair table built for the current row table
    uint32_t pairCountHost_ = 0;   // read back once per table build when a sharded solve needs it
    bool lastPairMode_ = false;
    DevBuf<int> rowSorted_, rowOther_, rowSeg_, rowDeg_, rowNA_, pairStart_, rowPairStart_, pairA_, pairB_;
    DevBuf<int2> pairCorr_, rowPair_;
    DevBuf<double> pstat_, dstat_;
    DevBuf<float> apPair_, rzPart_, poseBak_;
    DevBuf<uint2> aGran_;           // k_pcg_persist: Ap rows as {value, tag} granules
    DevBuf<uint2> fxGran_;          // k_pcg_persist's four-workgroup finisher: its exchanged partials
    uint32_t pcgEpoch_ = 0;          // tag base of the next persistent launch
};

SolverConfig make_solver_config(uint32_t maxImages, uint32_t maxCorr, const BFSolverOptions* opts);
VerifyParams verify_params(const BFVerifyOptions* o);  // defaults for fields left 0

// initNextGlobalTransformCU: rot/trans[s+1] = log(exp(rot/trans[s]) * exp(localRot/Trans[last])), or
// rot/trans[s] when the device int *gate is 0 (invalid local submap, Bundler.h:75-79)
void seed_keyframe(const float* localRot, const float* localTrans, uint32_t last, float* rot, float* trans, uint32_t s,
                   hipStream_t st, const int* gate = nullptr);
// *gate = *src (1 when src is null), on the stream
void set_gate(int* gate, const int* src, hipStream_t st);
// *gate == 0: keyframe s invalid and every correspondence with image s invalidated (OnlineBundler.cpp:351-360)
void invalidate_local(const int* gate, uint32_t s, int* valid, BFEntryJ* corr, uint32_t n, hipStream_t st);

// SBA.cu:75-119 — float4x4 <-> (rot, trans) for valid images
void matrices_to_poses(const float* T, uint32_t n, float* rot, float* trans, const int* valid, hipStream_t s);
void poses_to_matrices(const float* rot, const float* trans, uint32_t n, float* T, const int* valid, hipStream_t s);
// SIFTImageManager.cu:692-793
void invalidate_image_pair(BFEntryJ* corr, uint32_t n, uint32_t i, uint32_t j, hipStream_t s);
void check_invalid_frames(const int* numEntries, int* valid, uint32_t numImages, BFEntryJ* corr, uint32_t nCorr,
                          bool comprehensive, hipStream_t s);

}  // namespace bf
