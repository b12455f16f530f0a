// recon.cpp — see recon.h.
#include "recon.h"

#include "host_pool.h"

#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <string>
#include <cstdio>
#include <cstring>
#include <limits>
#include <unordered_set>

namespace bf {

#ifdef BF_HOST_PROFILE  // diagnostic build (tools/build_variant.sh): host time per loop section
namespace {
enum HostSec { HS_PRE, HS_CACHE, HS_PENDING, HS_SUBMAP, HS_QUEUE, HS_SCENE, HS_GC, HS_ALL, HS_N };
const char* kHostSecName[HS_N] = {"preprocess", "cache", "applyPending", "endSubmap", "queue", "applyOps", "gc", "processFrame"};
double g_hostSec[HS_N];
uint64_t g_hostFrames;
struct HostTimer {
    HostSec s;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    explicit HostTimer(HostSec x) : s(x) {}
    ~HostTimer() { g_hostSec[s] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count(); }
};
}  // namespace
#define BF_HOST_T(sec) HostTimer bf_host_timer_(sec)
#else
#define BF_HOST_T(sec) ((void)0)
#endif

BFMat4 mat4_mul(const BFMat4& a, const BFMat4& b);  // api.cpp

namespace {
const float NEG_INF = -std::numeric_limits<float>::infinity();
constexpr uint32_t RING = 8;  // bundling results in flight before the loop waits for the oldest
BFMat4 ninf_mat() {
    BFMat4 m;
    for (float& v : m.m) v = NEG_INF;
    return m;
}
BFMat4 identity() {
    BFMat4 m{};
    m.m[0] = m.m[5] = m.m[10] = m.m[15] = 1.0f;
    return m;
}
template <class T>
T or_default(T v, T d) { return v ? v : d; }
BFSolveResult to_abi(const SolveResult& r) {
    BFSolveResult o{};
    o.gnIterations = r.gnIterations;
    o.pcgIterations = r.pcgIterations;
    o.maxResidual = r.maxResidual;
    o.maxResidualIndex = r.maxResidualIndex;
    o.energy = r.energy;
    o.highResidualCount = r.highResidualCount;
    o.numDensePairs = r.numDensePairs;
    o.error = r.error;
    o.skipped = r.skipped;
    o.verifyUsed = r.verifyUsed;
    o.verifyOk = r.verifyOk;
    return o;
}
template <class T>
T* pinned(size_t n) {
    void* p = nullptr;
    BF_HIP(hipHostMalloc(&p, sizeof(T) * std::max<size_t>(n, 1), hipHostMallocDefault));
    return static_cast<T*>(p);
}
}  // namespace

Recon::Recon(const BFHashParams& hp, const BFSceneOptions* so, const BFDepthCameraParams& cam, const BFReconOptions& o)
    : opt_(o), cam_(cam) {
    opt_.submapSize = or_default(o.submapSize, 10u);
    opt_.maxFrameFixes = or_default(o.maxFrameFixes, 10u);
    opt_.topNActive = or_default(o.topNActive, 30u);
    opt_.localNonLin = or_default(o.localNonLin, 2u);
    opt_.localLin = or_default(o.localLin, 100u);
    opt_.globalNonLin = or_default(o.globalNonLin, 3u);
    opt_.globalLin = or_default(o.globalLin, 150u);
    opt_.maxResidualThresh = o.maxResidualThresh > 0 ? o.maxResidualThresh : 0.08f;
    opt_.cacheWidth = or_default(o.cacheWidth, 80u);
    opt_.cacheHeight = or_default(o.cacheHeight, 60u);
    BF_REQUIRE(opt_.maxFrames > 0, BF_ERR_ARG, "maxFrames");
    const uint32_t S = opt_.submapSize;
    // a full result ring (RING submaps in flight) hands the oldest result over early, so a lag beyond
    // RING submaps could not be kept exactly
    BF_REQUIRE(opt_.resultLag <= RING * S, BF_ERR_ARG, "resultLag exceeds the result ring (8 submaps)");
    const uint32_t maxSubmaps = (opt_.maxFrames + S - 1) / S;
    opt_.maxKeyframes = std::max(or_default(o.maxKeyframes, maxSubmaps + 1), 2u);
    opt_.maxLocalCorr = or_default(o.maxLocalCorr, (S + 1) * S / 2 * 25u);
    opt_.maxGlobalCorr = or_default(o.maxGlobalCorr, opt_.maxKeyframes * 1000u);

    // bundling stream priority (BFReconOptions.bundlingPriority): normal (as the scene stream) by default since
    // the voxel pass runs in resident rounds (Scene::Scene); 1: high throughout; 2: round 4's policy keyed on each
    // solve's size (switchBundlingPriority). (The scene stream itself at the highest priority measured slower:
    // 1 517 -> 1 499-1 502 frames/s at the bench workload, config 4's stream 1 103 -> 1 055.)
    sharded_ = so && so->shardCount > 1;
    int prLeast = 0, prGreatest = 0;
    BF_HIP(hipDeviceGetStreamPriorityRange(&prLeast, &prGreatest));
    BF_HIP(hipStreamCreateWithFlags(&sceneStream_, hipStreamNonBlocking));
    BF_REQUIRE(o.bundlingPriority >= 0 && o.bundlingPriority <= 2, BF_ERR_ARG, "bundlingPriority 0..2");
    const bool keyed = o.bundlingPriority == 2;
    const bool forced = !keyed;
    if (forced) priorityPolicy_ = o.bundlingPriority;
    const bool needHigh = forced ? priorityPolicy_ == 1 : true;
    const bool needNormal = forced ? priorityPolicy_ == 0 : (!sharded_ && opt_.maxKeyframes > kHighPriorityMaxKeyframes);
    if (needHigh) {
        BF_HIP(hipStreamCreateWithPriority(&baStreamHi_, hipStreamNonBlocking, prGreatest));
        BF_HIP(hipStreamCreateWithPriority(&localStreamHi_, hipStreamNonBlocking, prGreatest));
    }
    if (needNormal) {  // normal priority, as the scene stream (ROCm's "least" priority is below normal)
        BF_HIP(hipStreamCreateWithFlags(&baStreamLo_, hipStreamNonBlocking));
        BF_HIP(hipStreamCreateWithFlags(&localStreamLo_, hipStreamNonBlocking));
    }
    baHigh_ = needHigh;
    baStream_ = baHigh_ ? baStreamHi_ : baStreamLo_;
    localStream_ = baHigh_ ? localStreamHi_ : localStreamLo_;
    for (int b = 0; b < 2; b++) {
        BF_HIP(hipEventCreateWithFlags(&localDone_[b], hipEventDisableTiming));
        BF_HIP(hipEventCreateWithFlags(&globalDone_[b], hipEventDisableTiming));
    }
    scene_.reset(new Scene(scene_config(hp, so), sceneStream_));
    scene_->enableErrorMirror();  // checkScene: the scene's error bits each frame without a synchronization
    tileStride_ = Scene::tileCount(cam_);
    framePixels_ = Scene::dcCount(cam_);
    // the cache costs 8 B per pixel per frame (12.3 GB for 5 000 VGA frames, next to the frame store
    // itself); beyond 32 GB each batch rebuilds its ops' images in the scene's scratch instead
    if (tileStride_ * opt_.maxFrames * sizeof(float2) <= (4ull << 30) &&
        framePixels_ * opt_.maxFrames * sizeof(uint2) <= (32ull << 30)) {
        frameTiles_.alloc(tileStride_ * opt_.maxFrames);
        frameDC_.alloc(framePixels_ * opt_.maxFrames);
    }
    local_.reset(new Solver(make_solver_config(S + 1, opt_.maxLocalCorr, &opt_.solver), localStream_));
    global_.reset(new Solver(make_solver_config(opt_.maxKeyframes, opt_.maxGlobalCorr, &opt_.solver), baStream_));
    tm_.reset(new TrajectoryManager(opt_.maxFrames, opt_.topNActive, opt_.minPoseDistSqrt));
    if (opt_.enableTiming) {
        scene_->integrateClock().enable(true);
        scene_->applyClock().enable(true);
        // one voxel-pass launch in four carries the timing events (every launch stamped cost the bench
        // ~0.9 % of its frame rate: 1 616 against 1 631 frames/s untimed); the mean is taken over those
        scene_->applyClock().setPeriod(4);
        local_->solveClock().enable(true);
        global_->solveClock().enable(true);
        global_->pcgClock().enable(true);
    }

    const uint32_t L = S + 1, K = opt_.maxKeyframes;
    frames_.resize(opt_.maxFrames);
    localCorr_.assign(maxSubmaps + 1, {nullptr, 0});
    localTraj_.resize(maxSubmaps + 1);
    localKnown_.assign(maxSubmaps + 1, 0);
    kf_.assign(K, identity());
    kfSolved_.assign(K, 0);
    globalT_.assign(K, identity());
    globalValid_.assign(K, 1);
    complete_.resize(opt_.maxFrames);

    for (LocalSet& b : ls_) {
        b.rot.alloc(6 * L + 1);
        b.trans = b.rot.p + 3 * L;
        b.gate = reinterpret_cast<int*>(b.rot.p + 6 * L);
        b.T.alloc(16 * L);
        b.valid.alloc(L);
        b.cache.alloc(L);
    }
    dGlobalCache_.alloc(K);
    dGlobalRot_.alloc(3 * K);
    dGlobalTrans_.alloc(3 * K);
    dGlobalT_.alloc(16 * K);
    dGlobalValid_.alloc(K);
    dSeedT_.alloc(16);
    dOne_.alloc(1);
    std::vector<int> ones(std::max(L, K), 1);
    for (LocalSet& b : ls_) {
        BF_HIP(hipMemcpyAsync(b.valid.p, ones.data(), 4 * L, hipMemcpyHostToDevice, baStream_));
        BF_HIP(hipMemcpyAsync(b.gate, ones.data(), 4, hipMemcpyHostToDevice, baStream_));
    }
    BF_HIP(hipMemcpyAsync(dGlobalValid_.p, ones.data(), 4 * K, hipMemcpyHostToDevice, baStream_));
    BF_HIP(hipMemcpyAsync(dOne_.p, ones.data(), 4, hipMemcpyHostToDevice, baStream_));
    BF_HIP(hipMemsetAsync(dGlobalRot_.p, 0, dGlobalRot_.bytes(), baStream_));
    BF_HIP(hipMemsetAsync(dGlobalTrans_.p, 0, dGlobalTrans_.bytes(), baStream_));
    BF_HIP(hipStreamSynchronize(baStream_));

    // asyncBundling 2: the solves are issued from a bundling thread (measured: no gain in the bench, the
    // scene stream stays fed either way)
    baThreaded_ = opt_.asyncBundling == 2;
    if (baThreaded_) baThread_ = std::thread([this] { baLoop(); });
    ring_.resize(RING);
    for (Pending& p : ring_) {
        BF_HIP(hipEventCreateWithFlags(&p.done, hipEventDisableTiming));
        p.localT = pinned<float>(16 * L);
        p.globalT = pinned<float>(16 * (size_t)K);
        p.valid = pinned<int>(K);
        p.ctrl = pinned<uint32_t>(2 * Solver::kResultWords);
        p.localInit = pinned<float>(16 * L);
        p.cacheTable = pinned<BFCachedFrame>(L);
        p.gate = pinned<int>(1);
        *p.gate = 1;
    }
}

Recon::~Recon() {
    if (baThread_.joinable()) {
        {
            std::lock_guard<std::mutex> lk(baMu_);
            baStop_ = true;
        }
        baCv_.notify_all();
        baThread_.join();
    }
    if (sceneStream_) (void)hipStreamSynchronize(sceneStream_);
    for (hipStream_t st : {baStreamHi_, baStreamLo_, localStreamHi_, localStreamLo_})
        if (st) (void)hipStreamSynchronize(st);
    for (int b = 0; b < 2; b++) {
        if (localDone_[b]) (void)hipEventDestroy(localDone_[b]);
        if (globalDone_[b]) (void)hipEventDestroy(globalDone_[b]);
    }
    for (hipEvent_t e : cacheEvF_)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : preEv_)
        if (e) (void)hipEventDestroy(e);
    for (Pending& p : ring_) {
        if (p.done) (void)hipEventDestroy(p.done);
        for (void* q : {(void*)p.localT, (void*)p.globalT, (void*)p.valid, (void*)p.ctrl, (void*)p.localInit,
                        (void*)p.cacheTable, (void*)p.gate})
            if (q) (void)hipHostFree(q);
    }
    scene_.reset();
    local_.reset();
    global_.reset();
    if (sceneStream_) (void)hipStreamDestroy(sceneStream_);
    for (hipStream_t st : {baStreamHi_, baStreamLo_, localStreamHi_, localStreamLo_})
        if (st) (void)hipStreamDestroy(st);
    if (copyStream_) (void)hipStreamDestroy(copyStream_);
}

void Recon::setFrame(uint32_t f, const float* depth, const uint8_t* color, const BFCachedFrame* cache, const BFMat4& Tinc) {
    BF_REQUIRE(f < opt_.maxFrames, BF_ERR_CAPACITY, "frame index beyond maxFrames");
    FrameRef& r = frames_[f];
    r.depth = depth;
    r.color = color;
    r.cache = cache ? *cache : BFCachedFrame{};
    r.Tinc = Tinc;
    r.set = true;
    r.tilesReady = false;
    r.pre = false;  // a new frame-store slot: its preprocessing (if any) is still to run
}

VoxelOp Recon::frameOp(uint32_t f, const BFMat4& T, bool deint) {
    FrameRef& fr = frames_[f];
    VoxelOp op{T, fr.depth, fr.color, deint};
    if (frameTiles_.p) {
        op.tiles = frameTiles_.p + tileStride_ * f;
        op.dc = frameDC_.p + framePixels_ * f;
        op.tilesReady = fr.tilesReady;
        fr.tilesReady = true;  // this batch computes them (before any op of a later batch reads them)
    }
    return op;
}

void Recon::setLocalCorrespondences(uint32_t submap, BFEntryJ* corr, uint32_t n) {
    BF_REQUIRE(submap < localCorr_.size(), BF_ERR_CAPACITY, "submap index");
    BF_REQUIRE(n <= opt_.maxLocalCorr, BF_ERR_CAPACITY, "local correspondences exceed maxLocalCorr");
    localCorr_[submap] = {corr, n};
}

void Recon::setGlobalCorrespondences(BFEntryJ* corr, uint32_t n, const uint32_t* prefix, uint32_t numKeyframes) {
    BF_REQUIRE(n <= opt_.maxGlobalCorr, BF_ERR_CAPACITY, "global correspondences exceed maxGlobalCorr");
    // the app appends each keyframe's correspondences to the same list: the pair bounds then extend
    // from the new entries alone (no drain of the bundling stream, no copy of the whole list)
    const bool extends = corr == globalCorr_ && n >= globalCorrN_ && numKeyframes >= globalPrefix_.size() &&
                         std::equal(globalPrefix_.begin(), globalPrefix_.end(), prefix);
    globalCorr_ = corr;
    globalCorrN_ = n;
    globalPrefix_.assign(prefix, prefix + numKeyframes);
    if (comm_) computePairBounds(extends);
}

void Recon::setComm(Comm* c) {
    BF_REQUIRE(numFrames_ == 0, BF_ERR_STATE, "set the communicator before the first frame");
    comm_ = c;
    global_->setShard(c ? (uint32_t)c->size() : 1u, c ? (uint32_t)c->rank() : 0u, c);
    if (comm_ && globalCorr_) computePairBounds(false);
}

// The sharded global solve all-reduces its pair blocks, so the host must know how many there are, the
// same count on every rank: the distinct image pairs of every keyframe prefix, counted from the entries
// as they were handed over (removals and the per-image cap only ever drop pairs, so these counts bound
// every later solve). append: the list only grew since the last count (the app's per-keyframe appends),
// so only the new entries are read, which no solve touches yet (a submap's issue captures the list
// length of its own frame); otherwise everything is recounted after the bundling work drains.
void Recon::computePairBounds(bool append) {
    if (!append) {
        baDrain();
        BF_HIP(hipStreamSynchronize(baStream_));
        pairSeen_.clear();
        pairCountedN_ = 0;
        pairBound_.clear();
    }
    const uint32_t from = std::min(pairCountedN_, globalCorrN_);
    std::vector<BFEntryJ> h(globalCorrN_ - from);
    if (!h.empty()) {  // on a stream of its own: no other stream's work (nor the null stream's device-wide order) waits
        if (!copyStream_) BF_HIP(hipStreamCreateWithFlags(&copyStream_, hipStreamNonBlocking));
        BF_HIP(hipMemcpyAsync(h.data(), globalCorr_ + from, sizeof(BFEntryJ) * h.size(), hipMemcpyDeviceToHost, copyStream_));
        BF_HIP(hipStreamSynchronize(copyStream_));
    }
    uint32_t e = from;
    for (size_t s = pairBound_.size(); s < globalPrefix_.size(); s++) {
        const uint32_t end = std::min(globalPrefix_[s], globalCorrN_);
        for (; e < end; e++) {
            const BFEntryJ& c = h[e - from];
            const uint32_t i = c.imgIdx_i, j = c.imgIdx_j;
            if (i == BF_INVALID_IMAGE || i == j) continue;
            pairSeen_.insert(((uint64_t)std::min(i, j) << 32) | std::max(i, j));
        }
        pairBound_.push_back((uint32_t)pairSeen_.size());
    }
    pairCountedN_ = e;
}

void Recon::setInitialPose(const BFMat4& T0) {
    kf_[0] = T0;
    kfSolved_[0] = 1;
    globalT_[0] = T0;
    baDrain();
    BF_HIP(hipMemcpyAsync(dSeedT_.p, T0.m, 64, hipMemcpyHostToDevice, baStream_));
    matrices_to_poses(dSeedT_.p, 1, dGlobalRot_.p, dGlobalTrans_.p, dOne_.p, baStream_);
    BF_HIP(hipStreamSynchronize(baStream_));
}

void Recon::checkScene(bool exact) {
    const uint32_t e = exact ? scene_->errorFlags() : scene_->mirroredErrorFlags();
    if (e == 0) return;
    std::string why;
    if (e & 1u) why += " alloc candidate buffer overflow (raise BFSceneOptions.candidateCapacity);";
    if (e & 2u) why += " SDF block heap exhausted (raise s_hashNumSDFBlocks);";
    if (e & 4u) why += " alloc candidate dedup set congested (raise BFSceneOptions.candidateCapacity);";
    throw Error(BF_ERR_CAPACITY, "scene capacity exceeded, blocks were dropped (BFSceneCapacity.errorFlags = " +
                                     std::to_string(e) + "):" + why);
}

void Recon::captureGlobalSolve(uint32_t s) {
    BF_REQUIRE(numFrames_ <= s * opt_.submapSize, BF_ERR_STATE, "capture a submap's global solve before it is issued");
    const size_t K = opt_.maxKeyframes;
    capCorrIn_.alloc(opt_.maxGlobalCorr);
    capCorrOut_.alloc(opt_.maxGlobalCorr);
    capPoseIn_.alloc(6 * K);
    capPoseOut_.alloc(6 * K);
    capValid_.alloc(K);
    capSubmap_ = s;
    capDone_ = false;
}

void Recon::capturedGlobalSolve(BFEntryJ* corrIn, BFEntryJ* corrOut, uint32_t cap, uint32_t* nCorr, float* poseIn,
                                float* poseOut, int32_t* valid, uint32_t capImages, uint32_t* nImages) {
    synchronize();
    BF_REQUIRE(capDone_, BF_ERR_STATE, "the captured submap's global solve has not run");
    const size_t K = opt_.maxKeyframes;
    const uint32_t n = std::min(cap, capN_), k = std::min(capImages, capK_);
    if (corrIn && n) BF_HIP(hipMemcpy(corrIn, capCorrIn_.p, sizeof(BFEntryJ) * n, hipMemcpyDeviceToHost));
    if (corrOut && n) BF_HIP(hipMemcpy(corrOut, capCorrOut_.p, sizeof(BFEntryJ) * n, hipMemcpyDeviceToHost));
    for (int which = 0; which < 2; which++) {  // [rot 3k | trans 3k] per output
        float* dst = which ? poseOut : poseIn;
        const float* src = which ? capPoseOut_.p : capPoseIn_.p;
        if (!dst || !k) continue;
        BF_HIP(hipMemcpy(dst, src, 12 * (size_t)k, hipMemcpyDeviceToHost));
        BF_HIP(hipMemcpy(dst + 3 * (size_t)k, src + 3 * K, 12 * (size_t)k, hipMemcpyDeviceToHost));
    }
    if (valid && k) BF_HIP(hipMemcpy(valid, capValid_.p, 4 * (size_t)k, hipMemcpyDeviceToHost));
    if (nCorr) *nCorr = capN_;
    if (nImages) *nImages = capK_;
}

void Recon::setRender(const BFRayCastParams* rp) {
    render_ = rp != nullptr;
    if (!rp) return;
    BF_REQUIRE(rp->width > 0 && rp->height > 0, BF_ERR_ARG, "render size");
    renderParams_ = *rp;
    const size_t P = (size_t)rp->width * rp->height;
    if (rDepth_.n < P) {
        BF_HIP(hipStreamSynchronize(sceneStream_));  // an earlier render may still write the old images
        rDepth_.alloc(P);
        rDepth4_.alloc(P);
        rNormals_.alloc(P);
        rColors_.alloc(P);
    }
}

void Recon::renderOutput(const float** depth, const float** depth4, const float** normals, const float** colors) const {
    if (depth) *depth = rDepth_.p;
    if (depth4) *depth4 = reinterpret_cast<const float*>(rDepth4_.p);
    if (normals) *normals = reinterpret_cast<const float*>(rNormals_.p);
    if (colors) *colors = reinterpret_cast<const float*>(rColors_.p);
}

void Recon::logOp(int kind, uint32_t frame, const BFMat4* T) {
    if (!opt_.recordOps) return;
    BFFixOp e{};
    e.kind = kind;
    e.frame = frame;
    if (T) std::memcpy(kind == 1 ? e.oldT : e.newT, T->m, 64);
    log_.push_back(e);
}

// frame f's images were produced on stream s (preprocessing): the scene stream waits for that in the batch
// that first reads them (awaitPreproc)
void Recon::recordInputs(uint32_t f, hipStream_t s) {
    hipEvent_t& e = preEv_[f % kPreSlots];
    if (!e) BF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    BF_HIP(hipEventRecord(e, s));
    prePending_[f % kPreSlots] = true;
    preFrame_[f % kPreSlots] = f;
}

void Recon::inputsProduced(uint32_t f, hipStream_t s) {
    BF_REQUIRE(f < opt_.maxFrames, BF_ERR_CAPACITY, "frame index beyond maxFrames");
    recordInputs(f, s);
}

void Recon::awaitPreproc(uint32_t f) {
    if (!prePending_[f % kPreSlots]) return;
    BF_HIP(hipStreamWaitEvent(sceneStream_, preEv_[f % kPreSlots], 0));
    prePending_[f % kPreSlots] = false;
}

// reintegrate() (DepthSensing.cpp:854-902). The frame's fixes are applied as one op batch
// (Scene::applyOps: voxel results equal the sequential deIntegrate / integrate calls).
void Recon::runReintegrate() {
    // the batch integrates the previous frame (pendingOp_): it reads that frame's preprocessed images
    if (pendingInt_ && numFrames_ > 0) awaitPreproc(numFrames_ - 1);
    {
        BF_HOST_T(HS_QUEUE);
        tm_->nextFixes(opt_.maxFrameFixes, ops_);
    }
    traceQueue(2, 0, (uint32_t)ops_.size(), nullptr, &ops_);
    std::vector<VoxelOp>& batch = batch_;
    batch.clear();
    if (pendingInt_) {  // the previous frame's integration, in its place in the call sequence
        batch.push_back(pendingOp_);
        pendingInt_ = false;
    }
    for (const FixOp& op : ops_) {
        const FrameRef& fr = frames_[op.frame];
        BF_REQUIRE(fr.set, BF_ERR_STATE, "re-integration of a frame that is not in the frame store");
        if (op.kind == FixKind::ReIntegrate) {  // deIntegrate(old) + integrate(new)
            batch.push_back(frameOp(op.frame, op.oldT, true));
            batch.push_back(frameOp(op.frame, op.newT, false));
            logOp(1, op.frame, &op.oldT);
            logOp(2, op.frame, &op.newT);
            st_.deintegrations++;
            st_.integrations++;
        } else if (op.kind == FixKind::DeIntegrate) {
            batch.push_back(frameOp(op.frame, op.oldT, true));
            logOp(1, op.frame, &op.oldT);
            st_.deintegrations++;
        } else if (op.kind == FixKind::Integrate) {
            batch.push_back(frameOp(op.frame, op.newT, false));
            logOp(2, op.frame, &op.newT);
            st_.integrations++;
        }
        st_.fixOps++;
    }
    {
        BF_HOST_T(HS_SCENE);
        for (size_t k = 0; k < batch.size(); k += Scene::kMaxOps)
            scene_->applyOps(batch.data() + k, (uint32_t)std::min<size_t>(Scene::kMaxOps, batch.size() - k), cam_);
    }
    {
        BF_HOST_T(HS_GC);
        scene_->garbageCollect();
    }
    logOp(4, 0, nullptr);
}

void Recon::processFrame(uint32_t f) {
    const auto tStart = std::chrono::steady_clock::now();
    BF_REQUIRE(f == numFrames_, BF_ERR_STATE, "frames must be processed in order");
    checkScene(false);  // a block dropped by an earlier frame's batch fails the loop (no silent holes)
    BF_REQUIRE(f < opt_.maxFrames && frames_[f].set, BF_ERR_STATE, "frame not in the frame store");
    const uint32_t S = opt_.submapSize;
    const uint32_t s = f / S;
    // CUDAImageManager::process (DepthSensing.cpp:986 -> CUDAImageManager.cpp:22-158): the raw sensor
    // frame into its frame-store slot; the scene stream (which integrates it with the next frame's batch)
    // and the cache (which reads the raw depth) are ordered after it by an event
#ifdef BF_HOST_PROFILE
    HostTimer allT(HS_ALL);
    g_hostFrames++;
#endif
    if (preproc_ && frames_[f].rawDepth && !frames_[f].pre) {
        BF_HOST_T(HS_PRE);
        preprocessFrame(f);
    }
    // processInput -> storeCachedFrame before anything reads the frame's cache (the submap ending at
    // this frame includes it as its overlap frame)
    if (cache_) {
        BF_HOST_T(HS_CACHE);
        storeCacheFrame(f);
    }
    // the next frame's preprocessing, issued now rather than when the loop reaches it: the host may block
    // below on a bundling result, and the scene stream would then reach the batch that reads frame f + 1
    // (frame f + 2's) before its input work had even been queued (the frame store slot and the raw buffer
    // of parity f + 1 are free: frame f - 1's cache store is ordered before it, preprocessFrame)
    if (preproc_ && f + 1 < opt_.maxFrames && frames_[f + 1].rawDepth && frames_[f + 1].set && !frames_[f + 1].pre) {
        BF_HOST_T(HS_PRE);
        preprocessFrame(f + 1);
    }
    {
        BF_HOST_T(HS_PENDING);
        applyPending(false);
    }
    FrameRef& fr = frames_[f];
    if (f % S == 0 && f > 0) {
        BF_HOST_T(HS_SUBMAP);
        endSubmap(s - 1, S + 1);
        if (!opt_.asyncBundling) applyPending(true);
        if (!kfSolved_[s]) {  // solver result not back yet: dead-reckon the new keyframe
            BF_REQUIRE(s < kf_.size(), BF_ERR_CAPACITY, "keyframes exceed maxKeyframes");
            kf_[s] = mat4_mul(kf_[s - 1], mat4_mul(frames_[f - 1].Tlocal, fr.Tinc));
        }
    }
    const bool renderNow = render_ && pendingInt_;  // this frame's batch integrates frame f - 1 at pendingOp_.T
    const BFMat4 renderT = pendingOp_.T;
    runReintegrate();
    if (renderNow) {  // visualizeFrame (DepthSensing.cpp:790-793) of the frame the batch integrated
        BF_HOST_T(HS_SCENE);
        scene_->raycast(renderT, cam_, renderParams_, rDepth_.p, rDepth4_.p, rNormals_.p, rColors_.p, nullptr, nullptr);
        st_.renders++;
    }
    fr.Tlocal = (f % S == 0) ? identity() : mat4_mul(frames_[f - 1].Tlocal, fr.Tinc);
    const BFMat4 T = mat4_mul(kf_[s], fr.Tlocal);  // getCurrentIntegrationFrame
    pendingOp_ = frameOp(f, T, false);
    pendingInt_ = true;
    logOp(2, f, &T);
    st_.integrations++;
    tm_->addFrame(FrameType::Integrated, T, f);
    traceQueue(0, f, 1, &T, nullptr);
    numFrames_++;
    st_.frames++;
    st_.hostMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tStart).count();
}

void Recon::reintegrate() {
    checkScene(false);
    applyPending(false);
    runReintegrate();
}

void Recon::flushIntegrate() {
    if (!pendingInt_) return;
    if (numFrames_ > 0) awaitPreproc(numFrames_ - 1);
    pendingInt_ = false;
    scene_->applyOps(&pendingOp_, 1, cam_);  // = integrate(); also fills the frame's tile cache
}

void Recon::finish() {
    const uint32_t S = opt_.submapSize;
    if (numFrames_ == 0) return;
    const uint32_t s = (numFrames_ - 1) / S, n = numFrames_ - s * S;
    // a last submap of one frame is only the previous submap's overlap frame, solved with it
    // (isLastLocalFrame skips prepareLocalSolve for it, OnlineBundler.cpp:170-172, OnlineBundler.h:42)
    if (s != lastSubmapEnqueued_ && n >= 2) endSubmap(s, n);
    synchronize();
}

// end of submap s: optimizeLocal -> processGlobal/optimizeGlobal -> initNextGlobalTransform, all
// enqueued on the BA stream; the poses come back through pinned memory and an event
void Recon::endSubmap(uint32_t s, uint32_t n) {
    const uint32_t S = opt_.submapSize;
    const uint32_t base = s * S;
    if (inflight_.size() == RING) {  // ring full: wait for the oldest result
        Pending& old = ring_[inflight_.front()];
        const auto tw = std::chrono::steady_clock::now();
        baWaitFor(old.job);
        BF_HIP(hipEventSynchronize(old.done));
        st_.hostWaitMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
        apply(old);
        inflight_.pop_front();
    }
    const uint32_t slot = ringNext_;
    ringNext_ = (ringNext_ + 1) % RING;
    Pending& P = ring_[slot];
    P.submap = s;
    P.numLocal = n;
    P.localSolved = P.globalSolved = false;
    P.endSolve = false;
    P.issueFrame = numFrames_;

    // ---- local solve over frames base .. base+n-1 (first frame fixed) ----------------------
    bool haveCache = opt_.useLocalDense != 0;
    for (uint32_t i = 0; i < n; i++) {
        const FrameRef& fr = frames_[base + i];
        BF_REQUIRE(fr.set, BF_ERR_STATE, "local solve over a frame not in the frame store");
        // the submap's last local frame is the next submap's first: chain it from frame S-1
        const BFMat4 Tl = (i < S) ? fr.Tlocal : mat4_mul(frames_[base + S - 1].Tlocal, fr.Tinc);
        std::memcpy(P.localInit + 16 * i, Tl.m, 64);
        P.cacheTable[i] = fr.cache;
        if (!fr.cache.depth) haveCache = false;
    }
    const uint32_t nk = s + 1;
    BF_REQUIRE(nk + 1 <= opt_.maxKeyframes, BF_ERR_CAPACITY, "keyframes exceed maxKeyframes");
    switchBundlingPriority(nk);
    P.numKeyframes = nk;
    const std::pair<BFEntryJ*, uint32_t> lc = localCorr_[s];
    // everything below only issues work on baStream_ from state fixed at this point: the bundling
    // thread runs it while the frame loop goes on enqueuing scene work
    const hipEvent_t cev = cacheEv_;  // the submap's last cache store (the frame thread re-points cacheEv_)
    // the global list as of this frame: the frame thread may append keyframes' correspondences (the app)
    // while a bundling thread issues this submap, so the issue works from these values, not the members
    GlobalView gv{globalCorr_, globalCorrN_, (s < globalPrefix_.size()) ? globalPrefix_[s] : globalCorrN_,
                  (comm_ && s < pairBound_.size()) ? std::max(pairBound_[s], 1u) : 0u};
    baPost([this, s, n, S, slot, haveCache, lc, nk, cev, gv]() { issueSubmap(s, n, S, slot, haveCache, lc, nk, cev, gv); });
    P.job = lastJob_;
    inflight_.push_back(slot);
    lastSubmapEnqueued_ = s;
    // m_totalNumOptLocalFrames (OnlineBundler.cpp:268): the frames the complete trajectory covers
    optimizedFrames_ = S * s + std::min(n, S);
}

// Round 5: with the voxel pass in four resident rounds (a slot frees every ~120 us instead of once per pass),
// the bundling streams run at normal priority by default: the bench stream 1 446-1 458 (high) -> 1 470-1 474
// frames/s, the G = 8 rehearsal 3 707-3 732 -> 3 812-3 825 (profiles/r10_ba_priority_ab.txt). The keyed
// policy below (BF_BA_HIGH_PRIORITY=keyed) was round 4's, measured with one resident round:
// Bundling streams at the highest queue priority take CU slots ahead of the scene stream's next workgroups
// (priority orders dispatch; it never preempts a running workgroup):
// - sharded, each GPU has a fraction of the voxel work and the (replicated) bundling is co-critical: +7 % at
//   G = 4, +11 % at G = 8 (one rank's share on one GPU, profiles/r3n_late_experiments.txt);
// - unsharded, while the global solve's persistent grid (about N / 4 workgroups of the 512 slots at 2 per
//   CU) leaves the scene stream a quarter of the device: the bench stream (K = 500) 1 300 -> 1 362-1 367
//   frames/s, config 5's stream (K = 1 000) 181.6 -> 183.7. At normal priority each of a solve's dependent
//   launches waits for slots behind the voxel pass, the submap's result misses its hand-off frame and the
//   frame loop blocks with less work queued (profiles/r8u_*, r8v_*, r9b_*);
// - solves above kHighPriorityMaxKeyframes keyframes (config 4's 2 000), whose grid needs nearly every
//   slot, starve the scene stream at high priority instead (981 -> 921 frames/s): they run at normal priority.
// Keyed on the solve being issued (nk keyframes), not on the run's capacity: a run sized for 2 000
// keyframes bundles at high priority until its solves pass the bound. The switch (once per run: K only
// grows) orders the new streams after the old ones' work and moves both solvers onto them.
void Recon::switchBundlingPriority(uint32_t nk) {
    if (priorityPolicy_ >= 0) return;  // fixed by BF_BA_HIGH_PRIORITY
    const bool high = sharded_ || nk <= kHighPriorityMaxKeyframes;
    if (high == baHigh_) return;
    hipStream_t ba = high ? baStreamHi_ : baStreamLo_, loc = high ? localStreamHi_ : localStreamLo_;
    if (!ba || !loc) return;  // that priority was not created for this run
    baDrain();                // a bundling thread has issued everything queued on the old streams
    hipEvent_t e[2];
    for (hipEvent_t& x : e) BF_HIP(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    BF_HIP(hipEventRecord(e[0], baStream_));
    BF_HIP(hipEventRecord(e[1], localStream_));
    for (hipStream_t st : {ba, loc})
        for (hipEvent_t x : e) BF_HIP(hipStreamWaitEvent(st, x, 0));
    for (hipEvent_t x : e) BF_HIP(hipEventDestroy(x));
    baStream_ = ba;
    localStream_ = loc;
    global_->setStream(ba);
    local_->setStream(loc);
    baHigh_ = high;
}

void Recon::issueSubmap(uint32_t s, uint32_t n, uint32_t S, uint32_t slot, bool haveCache,
                        std::pair<BFEntryJ*, uint32_t> lc, uint32_t nk, hipEvent_t cev, GlobalView gv) {
    Pending& P = ring_[slot];
    const uint32_t L = S + 1;
    const int bi = (int)(s & 1u);
    LocalSet& B = ls_[bi];
    // ---- local solve over frames base .. base+n-1 (first frame fixed), on the local stream ----------
    // set bi was last read by global solve s - 2
    BF_HIP(hipStreamWaitEvent(localStream_, globalDone_[bi], 0));
    if (cev) BF_HIP(hipStreamWaitEvent(localStream_, cev, 0));  // the submap's cache frames
    BF_HIP(hipMemcpyAsync(B.T.p, P.localInit, 64 * n, hipMemcpyHostToDevice, localStream_));
    matrices_to_poses(B.T.p, n, B.rot.p, B.trans, B.valid.p, localStream_);
    // multi-GPU: submap s's local solve runs on rank s % R only (the submaps are independent units,
    // SURVEY.md §8(e)2); its poses and verification outcome are then broadcast so that every rank
    // continues identically. The broadcast goes on the BA stream (the communicator's one order on
    // every rank), after the owner's solve; the solve itself overlaps the previous global solve.
    const bool shardLocal = comm_ && comm_->size() > 1;
    const int localOwner = shardLocal ? (int)(s % (uint32_t)comm_->size()) : 0;
    const bool solveHere = !shardLocal || localOwner == comm_->rank();
    const bool verify = opt_.disableLocalVerify == 0;
    const size_t bcast = 6 * (size_t)L + 1;  // [rot | trans | gate]
    const bool haveLocal = n >= 2 && lc.first && lc.second > 0;
    if (haveLocal && solveHere) {
        if (haveCache)
            BF_HIP(hipMemcpyAsync(B.cache.p, P.cacheTable, sizeof(BFCachedFrame) * n, hipMemcpyHostToDevice, localStream_));
        std::vector<float> ws(opt_.localNonLin, 1.0f), wd(opt_.localNonLin), wc(opt_.localNonLin, 0.0f);
        for (uint32_t i = 0; i < opt_.localNonLin; i++) wd[i] = haveCache ? (float)(i + 1) : 0.0f;  // SBA.cpp:28-31
        SolveArgs a{};
        a.corr = lc.first;
        a.numCorr = lc.second;
        a.valid = B.valid.p;
        a.numImages = n;
        a.nNonLin = opt_.localNonLin;
        a.nLin = opt_.localLin;
        a.wSparse = ws.data();
        a.wDenseDepth = wd.data();
        a.wDenseColor = wc.data();
        a.cache = haveCache ? B.cache.p : nullptr;
        a.cacheW = opt_.cacheWidth;
        a.cacheH = opt_.cacheHeight;
        std::memcpy(a.intrinsics, opt_.cacheIntrinsics, sizeof(a.intrinsics));
        a.rot = B.rot.p;
        a.trans = B.trans;
        a.rebuildJT = true;
        // optimizeLocal removes no max residual (OnlineBundler.cpp:255-256); the residual analysis
        // only counts the high residuals useVerification asks for
        a.findMaxResidual = verify;
        local_->solve(a);
        poses_to_matrices(B.rot.p, B.trans, n, B.T.p, B.valid.p, localStream_);
        // SBA::align :106-109 -> Bundler::optimize :259-274 (needs the submap's cache frames)
        const bool check = verify && haveCache;
        if (check) {
            VerifyParams vp = verify_params(&opt_.verify);
            vp.T = B.T.p;
            vp.valid = B.valid.p;
            vp.numImages = n;
            vp.cache = B.cache.p;
            vp.cacheW = opt_.cacheWidth;
            vp.cacheH = opt_.cacheHeight;
            std::memcpy(vp.intrinsics, opt_.cacheIntrinsics, sizeof(vp.intrinsics));
            vp.numCorr = lc.second;
            local_->verify(vp);
        }
        set_gate(B.gate, check ? local_->verifyFlag() : nullptr, localStream_);
        local_->resultAsync(P.ctrl);
        P.localSolved = true;
    } else if (!haveLocal) {
        set_gate(B.gate, nullptr, localStream_);
        std::memcpy(P.localT, P.localInit, 64 * n);
    }
    BF_HIP(hipEventRecord(localDone_[bi], localStream_));
    BF_HIP(hipStreamWaitEvent(baStream_, localDone_[bi], 0));
    if (haveLocal) {
        if (shardLocal) {
            comm_->broadcast(B.rot.p, bcast, localOwner, baStream_);
            if (!solveHere) poses_to_matrices(B.rot.p, B.trans, n, B.T.p, B.valid.p, baStream_);
        }
        BF_HIP(hipMemcpyAsync(P.localT, B.T.p, 64 * n, hipMemcpyDeviceToHost, baStream_));
    }
    // ---- global solve over keyframes 0..s ---------------------------------------------------
    // an invalid local submap (gate 0) becomes an invalid keyframe without correspondences and its
    // global solve is skipped (processGlobal / optimizeGlobal INVALIDATE, OnlineBundler.cpp:351-360,
    // 399-405). Keyframe 0 is never invalidated (the reference exits on an invalid first chunk,
    // Bundler.cpp:377-384).
    const int* gate = (verify && s > 0) ? B.gate : nullptr;
    if (gate && gv.corr) invalidate_local(gate, s, dGlobalValid_.p, gv.corr, gv.n, baStream_);
    const uint32_t ncorr = gv.ncorr;
    if (nk >= 2 && gv.corr && ncorr > 0) {
        std::vector<float> ws(opt_.globalNonLin, 1.0f), wz(opt_.globalNonLin, 0.0f);  // SBA.cpp:34-39, dense off
        SolveArgs a{};
        a.corr = gv.corr;
        a.numCorr = ncorr;
        a.valid = dGlobalValid_.p;
        a.numImages = nk;
        a.nNonLin = opt_.globalNonLin;
        a.nLin = opt_.globalLin;
        a.wSparse = ws.data();
        a.wDenseDepth = wz.data();
        a.wDenseColor = wz.data();
        a.rot = dGlobalRot_.p;
        a.trans = dGlobalTrans_.p;
        a.rebuildJT = true;
        a.findMaxResidual = true;
        a.gate = gate;
        if (gv.pairBound) a.pairBound = gv.pairBound;
        const bool capture = s == capSubmap_;
        if (capture) {  // test hook: the solve's inputs, as it sees them (after invalidate_local)
            const size_t K = opt_.maxKeyframes;
            BF_HIP(hipMemcpyAsync(capCorrIn_.p, gv.corr, sizeof(BFEntryJ) * ncorr, hipMemcpyDeviceToDevice, baStream_));
            BF_HIP(hipMemcpyAsync(capPoseIn_.p, dGlobalRot_.p, 12 * (size_t)nk, hipMemcpyDeviceToDevice, baStream_));
            BF_HIP(hipMemcpyAsync(capPoseIn_.p + 3 * K, dGlobalTrans_.p, 12 * (size_t)nk, hipMemcpyDeviceToDevice, baStream_));
            BF_HIP(hipMemcpyAsync(capValid_.p, dGlobalValid_.p, 4 * (size_t)nk, hipMemcpyDeviceToDevice, baStream_));
        }
        global_->solve(a);
        if (capture) {  // ... and its outcome, before the max-residual removal
            const size_t K = opt_.maxKeyframes;
            BF_HIP(hipMemcpyAsync(capCorrOut_.p, gv.corr, sizeof(BFEntryJ) * ncorr, hipMemcpyDeviceToDevice, baStream_));
            BF_HIP(hipMemcpyAsync(capPoseOut_.p, dGlobalRot_.p, 12 * (size_t)nk, hipMemcpyDeviceToDevice, baStream_));
            BF_HIP(hipMemcpyAsync(capPoseOut_.p + 3 * K, dGlobalTrans_.p, 12 * (size_t)nk, hipMemcpyDeviceToDevice, baStream_));
            capN_ = ncorr;
            capK_ = nk;
            capDone_ = true;
        }
        // removeMaxResidualCUDA with getMaxResidual's (0, <10) exemption, on the device
        global_->removeMaxResidualAsync(gv.corr, ncorr, dGlobalValid_.p, nk, opt_.maxResidualThresh);
        global_->resultAsync(P.ctrl + Solver::kResultWords);
        P.globalSolved = true;
    }
    poses_to_matrices(dGlobalRot_.p, dGlobalTrans_.p, nk, dGlobalT_.p, dGlobalValid_.p, baStream_);
    BF_HIP(hipMemcpyAsync(P.globalT, dGlobalT_.p, 64 * nk, hipMemcpyDeviceToHost, baStream_));
    BF_HIP(hipMemcpyAsync(P.valid, dGlobalValid_.p, 4 * nk, hipMemcpyDeviceToHost, baStream_));
    BF_HIP(hipMemcpyAsync(P.gate, B.gate, 4, hipMemcpyDeviceToHost, baStream_));
    // ---- initNextGlobalTransformCU (OnlineBundler.cu:112-140): keyframe s+1 from the last local
    if (n == S + 1) seed_keyframe(B.rot.p, B.trans, S, dGlobalRot_.p, dGlobalTrans_.p, s, baStream_, gate);
    BF_HIP(hipEventRecord(globalDone_[bi], baStream_));
    BF_HIP(hipEventRecord(P.done, baStream_));
}

// One end-of-sequence global solve (OnlineBundler.cpp:171-197 + optimizeGlobal with isSequenceDone,
// :373-398): every keyframe and correspondence, max-residual removal, optionally the dense depth term
// of USE_GLOBAL_DENSE_AT_END (:177-189) over the keyframes' cache frames.
void Recon::issueEndSolve(uint32_t slot, uint32_t nk, uint32_t ncorr, float wDense, hipEvent_t t0, hipEvent_t t1) {
    Pending& P = ring_[slot];
    std::vector<float> ws(opt_.globalNonLin, 1.0f), wd(opt_.globalNonLin, wDense), wc(opt_.globalNonLin, 0.0f);
    SolveArgs a{};
    a.corr = globalCorr_;
    a.numCorr = ncorr;
    a.valid = dGlobalValid_.p;
    a.numImages = nk;
    a.nNonLin = opt_.globalNonLin;
    a.nLin = opt_.globalLin;
    a.wSparse = ws.data();
    a.wDenseDepth = wd.data();
    a.wDenseColor = wc.data();
    a.cache = wDense > 0.0f ? dGlobalCache_.p : nullptr;
    a.cacheW = opt_.cacheWidth;
    a.cacheH = opt_.cacheHeight;
    std::memcpy(a.intrinsics, opt_.cacheIntrinsics, sizeof(a.intrinsics));
    a.rot = dGlobalRot_.p;
    a.trans = dGlobalTrans_.p;
    a.rebuildJT = true;
    a.findMaxResidual = true;
    if (cacheEv_ && wDense > 0.0f) BF_HIP(hipStreamWaitEvent(baStream_, cacheEv_, 0));
    const uint32_t last = nk - 1;
    if (comm_ && last < pairBound_.size()) a.pairBound = std::max(pairBound_[last], 1u);
    BF_HIP(hipEventRecord(t0, baStream_));
    global_->solve(a);
    BF_HIP(hipEventRecord(t1, baStream_));
    global_->removeMaxResidualAsync(globalCorr_, ncorr, dGlobalValid_.p, nk, opt_.maxResidualThresh);
    global_->resultAsync(P.ctrl + Solver::kResultWords);
    P.globalSolved = true;
    poses_to_matrices(dGlobalRot_.p, dGlobalTrans_.p, nk, dGlobalT_.p, dGlobalValid_.p, baStream_);
    BF_HIP(hipMemcpyAsync(P.globalT, dGlobalT_.p, 64 * nk, hipMemcpyDeviceToHost, baStream_));
    BF_HIP(hipMemcpyAsync(P.valid, dGlobalValid_.p, 4 * nk, hipMemcpyDeviceToHost, baStream_));
    BF_HIP(hipEventRecord(P.done, baStream_));
}

SolveResult Recon::endSolve(float wDense, float* ms) {
    synchronize();  // every submap result applied: the ring is empty
    const uint32_t S = opt_.submapSize;
    BF_REQUIRE(numFrames_ > 0, BF_ERR_STATE, "end solve before the first frame");
    // the global problem holds one keyframe per solved submap (fuseToGlobal, OnlineBundler.cpp:298)
    if (lastSubmapEnqueued_ == 0xFFFFFFFFu) {
        SolveResult none{};
        none.skipped = 1;
        if (ms) *ms = 0.0f;
        return none;
    }
    const uint32_t last = lastSubmapEnqueued_, nk = last + 1;
    const uint32_t ncorr = (last < globalPrefix_.size()) ? globalPrefix_[last] : globalCorrN_;
    SolveResult res{};
    res.skipped = 1;
    if (ms) *ms = 0.0f;
    if (nk < 2 || !globalCorr_ || ncorr == 0) return res;
    if (wDense > 0.0f) {
        std::vector<BFCachedFrame> tab(nk);
        for (uint32_t k = 0; k < nk; k++) {
            tab[k] = frames_[k * S].cache;  // Bundler::fuseToGlobal keeps the submap's first frame
            BF_REQUIRE(tab[k].depth, BF_ERR_STATE, "dense end solve: a keyframe has no cache frame");
        }
        BF_HIP(hipMemcpyAsync(dGlobalCache_.p, tab.data(), sizeof(BFCachedFrame) * nk, hipMemcpyHostToDevice, baStream_));
        BF_HIP(hipStreamSynchronize(baStream_));
    }
    const uint32_t slot = ringNext_;
    ringNext_ = (ringNext_ + 1) % RING;
    Pending& P = ring_[slot];
    P.submap = last;
    P.numLocal = 0;
    P.numKeyframes = nk;
    P.localSolved = P.globalSolved = false;
    P.endSolve = true;
    *P.gate = 1;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    BF_HIP(hipEventCreate(&t0));
    BF_HIP(hipEventCreate(&t1));
    try {
        baPost([this, slot, nk, ncorr, wDense, t0, t1]() { issueEndSolve(slot, nk, ncorr, wDense, t0, t1); });
        P.job = lastJob_;
        baWaitFor(P.job);
        BF_HIP(hipEventSynchronize(P.done));
        if (ms) BF_HIP(hipEventElapsedTime(ms, t0, t1));
    } catch (...) {
        (void)hipEventDestroy(t0);
        (void)hipEventDestroy(t1);
        throw;
    }
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    apply(P);
    st_.endSolves++;
    return Solver::decodeResult(P.ctrl + Solver::kResultWords);
}

void Recon::submapPoses(uint32_t s, float* local, float* global, int32_t* valid, uint32_t* numLocal, uint32_t* numKeyframes,
                        int32_t* localValid) const {
    BF_REQUIRE(opt_.recordOps, BF_ERR_STATE, "submap history needs recordOps");
    BF_REQUIRE(s < history_.size() && !history_[s].local.empty(), BF_ERR_ARG, "no record of this submap");
    const SubmapRecord& r = history_[s];
    if (local) std::memcpy(local, r.local.data(), 64 * r.local.size());
    if (global) std::memcpy(global, r.global.data(), 64 * r.global.size());
    if (valid) std::memcpy(valid, r.valid.data(), 4 * r.valid.size());
    if (numLocal) *numLocal = (uint32_t)r.local.size();
    if (numKeyframes) *numKeyframes = (uint32_t)r.global.size();
    if (localValid) *localValid = r.localOk;
}

void Recon::baPost(std::function<void()> job) {
    ++lastJob_;
    if (!baThreaded_) {
        job();
        baDone_.store(lastJob_, std::memory_order_release);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(baMu_);
        baJobs_.push_back(std::move(job));
    }
    baCv_.notify_one();
}

void Recon::baLoop() {
    for (;;) {
        std::function<void()> job;
        {
            std::unique_lock<std::mutex> lk(baMu_);
            baCv_.wait(lk, [this] { return baStop_ || !baJobs_.empty(); });
            if (baJobs_.empty()) return;  // stop requested and nothing left
            job = std::move(baJobs_.front());
            baJobs_.pop_front();
        }
        try {
            job();
        } catch (...) {
            std::lock_guard<std::mutex> lk(baMu_);
            if (!baErr_) baErr_ = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> lk(baMu_);
            baDone_.fetch_add(1, std::memory_order_release);
        }
        baDoneCv_.notify_all();
    }
}

void Recon::baWaitFor(uint64_t job) {
    if (baDone_.load(std::memory_order_acquire) < job) {
        std::unique_lock<std::mutex> lk(baMu_);
        baDoneCv_.wait(lk, [this, job] { return baDone_.load(std::memory_order_acquire) >= job; });
    }
    std::exception_ptr e;
    {
        std::lock_guard<std::mutex> lk(baMu_);
        e = baErr_;
        baErr_ = nullptr;
    }
    if (e) std::rethrow_exception(e);
}

void Recon::baDrain() { baWaitFor(lastJob_); }

void Recon::applyPending(bool block) {
    if (!block && opt_.asyncBundling && opt_.resultLag) {
        // repeatable hand-off: submap results are applied exactly resultLag frames after their issue
        while (!inflight_.empty()) {
            Pending& P = ring_[inflight_.front()];
            if (numFrames_ < P.issueFrame + opt_.resultLag) break;
            const auto tw = std::chrono::steady_clock::now();
            baWaitFor(P.job);
            BF_HIP(hipEventSynchronize(P.done));
            st_.hostWaitMs += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count();
            apply(P);
            inflight_.pop_front();
        }
        return;
    }
    while (!inflight_.empty()) {
        Pending& P = ring_[inflight_.front()];
        if (!block && baDone_.load(std::memory_order_acquire) < P.job) break;  // not issued yet
        baWaitFor(P.job);
        if (block) {
            BF_HIP(hipEventSynchronize(P.done));
        } else {
            const hipError_t q = hipEventQuery(P.done);
            if (q == hipErrorNotReady) break;
            BF_HIP(q);
        }
        apply(P);
        inflight_.pop_front();
    }
}

// updateTrajectoryCU (OnlineBundler.cu:73-110) + TrajectoryManager::updateOptimizedTransform
void Recon::apply(Pending& P) {
    const uint32_t S = opt_.submapSize, s = P.submap, n = P.numLocal, nk = P.numKeyframes;
    // the submap's solves are done (its event): a collective among them (the local-pose broadcast, the pair-
    // statistics all-reduces) that failed leaves poses no rank may use
    if (comm_) comm_->checkError();
    // a solve whose result is not a valid solve is never consumed: the loop fails instead (a timed-out
    // persistent PCG launch is redone on the device and flagged BF_SOLVE_PCG_RECOVERED, which is valid)
    for (int which = 0; which < 2; which++) {
        if (!(which ? P.globalSolved : P.localSolved)) continue;
        const SolveResult r = Solver::decodeResult(P.ctrl + (which ? Solver::kResultWords : 0));
        BF_REQUIRE(!(r.error & BF_SOLVE_ERR_FATAL), BF_ERR_INTERNAL,
                   which ? "global solve failed (BFSolveResult.error has a BF_SOLVE_ERR_FATAL bit)"
                         : "local solve failed (BFSolveResult.error has a BF_SOLVE_ERR_FATAL bit)");
        if (r.error & BF_SOLVE_PCG_RECOVERED) st_.pcgRecoveries++;
    }
    const bool localOk = *P.gate != 0;
    std::vector<BFMat4>& traj = localTraj_[s];
    if (!P.endSolve) {
        traj.resize(n);
        std::memcpy(traj.data(), P.localT, 64 * n);
        localKnown_[s] = 1;
    }
    std::memcpy(globalValid_.data(), P.valid, 4 * nk);
    for (uint32_t k = 0; k < nk; k++) {
        if (!globalValid_[k]) continue;
        std::memcpy(globalT_[k].m, P.globalT + 16 * k, 64);
        kf_[k] = globalT_[k];
        kfSolved_[k] = 1;
    }
    // keyframe s+1 from the solver's seed; after an invalid local the reference copies keyframe s
    // (initializeNextTransformUnknown), which the front end's dead reckoning here improves on
    if (!P.endSolve && n == S + 1 && globalValid_[s] && localOk) {
        kf_[s + 1] = mat4_mul(globalT_[s], traj[S]);
        kfSolved_[s + 1] = 1;
    }
    if (P.localSolved) {
        const SolveResult r = Solver::decodeResult(P.ctrl);
        st_.localSolves++;
        st_.localGnIterations += r.gnIterations;
        st_.localPcgIterations += r.pcgIterations;
        if (r.verifyUsed) st_.localVerifications++;
    }
    if (!P.endSolve && !localOk) st_.invalidLocals++;
    if (P.globalSolved) {
        const SolveResult r = Solver::decodeResult(P.ctrl + Solver::kResultWords);
        lastGlobalResult_ = r;
        if (!r.skipped) {
            st_.globalSolves++;
            st_.globalGnIterations += r.gnIterations;
            st_.globalPcgIterations += r.pcgIterations;
            if (r.removedI != BF_INVALID_IMAGE) st_.removedPairs++;
        }
    }
    if (opt_.recordOps && !P.endSolve) {
        if (history_.size() <= s) history_.resize(s + 1);
        SubmapRecord& rec = history_[s];
        rec.local = traj;
        rec.global.resize(nk);
        std::memcpy(rec.global.data(), P.globalT, 64 * nk);
        rec.valid.assign(P.valid, P.valid + nk);
        rec.localOk = localOk ? 1 : 0;
    }
    // frames of invalid keyframes (and of invalidated local submaps) get -inf transforms: the queue
    // de-integrates them (invalidateImages + updateTrajectoryCU, OnlineBundler.cpp:317-320, 387-394)
    const uint32_t optimized = P.endSolve ? std::min(optimizedFrames_, numFrames_) : std::min(S * s + std::min(n, S), numFrames_);
    HostPool::get().parallel_for(optimized, [this, S](size_t b, size_t e) {  // independent per frame
        for (size_t g = b; g < e; g++) {
            const size_t k = g / S;
            complete_[g] = (globalValid_[k] && localKnown_[k]) ? mat4_mul(globalT_[k], localTraj_[k][g % S]) : ninf_mat();
        }
    }, 1024);
    tm_->updateOptimizedTransforms(complete_.data(), optimized);
    traceQueue(1, 0, optimized, complete_.data(), nullptr);
}

void Recon::synchronize() {
    flushIntegrate();
    baDrain();
    BF_HIP(hipStreamSynchronize(sceneStream_));
    BF_HIP(hipStreamSynchronize(localStream_));
    BF_HIP(hipStreamSynchronize(baStream_));
    if (comm_) comm_->checkError();
    checkScene(true);
    applyPending(true);
}

BFReconStats Recon::stats() {
#ifdef BF_HOST_PROFILE
    if (g_hostFrames) {
        fprintf(stderr, "host us per frame (since the last resetStats) over %llu frames:", (unsigned long long)g_hostFrames);
        for (int k = 0; k < HS_N; k++) fprintf(stderr, " %s %.1f", kHostSecName[k], g_hostSec[k] / (double)g_hostFrames);
        fprintf(stderr, "\n");
    }
#endif
    synchronize();
    BFReconStats s = st_;
    if (opt_.enableTiming) {
        s.integrateKernelMs = scene_->integrateClock().totalMs();
        s.integrateLaunches = scene_->integrateClock().launches();
        s.reintegrateKernelMs = scene_->applyClock().totalMs();
        s.reintegrateLaunches = scene_->applyClock().launches();
        s.localSolveMs = local_->solveClock().totalMs();
        s.globalSolveMs = global_->solveClock().totalMs();
        s.globalPcgKernelMs = global_->pcgClock().totalMs();
        s.globalPcgLaunches = global_->pcgClock().launches();
    }
    return s;
}

void Recon::resetStats() {
    synchronize();
    st_ = BFReconStats{};
#ifdef BF_HOST_PROFILE
    for (double& v : g_hostSec) v = 0.0;
    g_hostFrames = 0;
#endif
    scene_->resetStats();
    scene_->integrateClock().reset();
    scene_->applyClock().reset();
    local_->solveClock().reset();
    global_->solveClock().reset();
    global_->pcgClock().reset();
}

void Recon::attachCache(Cache* c) {
    BF_REQUIRE(numFrames_ == 0, BF_ERR_STATE, "attach the cache before the first frame");
    BF_REQUIRE(!c || c->config().width == opt_.cacheWidth && c->config().height == opt_.cacheHeight, BF_ERR_ARG,
               "cache size differs from the loop's cacheWidth x cacheHeight");
    BF_REQUIRE(!c || !preproc_ || (preproc_->depthWidth() == c->config().inputWidth && preproc_->depthHeight() == c->config().inputHeight),
               BF_ERR_ARG, "the cache's input size differs from the attached preprocessing's sensor depth size");
    cache_ = c;
    for (hipEvent_t& e : cacheEvF_)
        if (c && !e) BF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

void Recon::setFrameSource(uint32_t f, const float* depth, const uint8_t* color, uint32_t colorW, uint32_t colorH) {
    BF_REQUIRE(f < opt_.maxFrames, BF_ERR_CAPACITY, "frame index beyond maxFrames");
    FrameRef& r = frames_[f];
    r.srcDepth = depth;
    r.srcColor = color;
    r.srcW = colorW;
    r.srcH = colorH;
}

void Recon::attachPreproc(Preproc* p) {
    BF_REQUIRE(numFrames_ == 0, BF_ERR_STATE, "attach the preprocessing before the first frame");
    BF_REQUIRE(!p || (p->integrationWidth() == cam_.imageWidth && p->integrationHeight() == cam_.imageHeight), BF_ERR_ARG,
               "preprocessing output size differs from the integration size");
    // the cache reads the preprocessing's sensor-size raw depth (k_cache_geometry: inputWidth x inputHeight)
    BF_REQUIRE(!p || !cache_ || (p->depthWidth() == cache_->config().inputWidth && p->depthHeight() == cache_->config().inputHeight),
               BF_ERR_ARG, "the attached cache's input size differs from the preprocessing's sensor depth size");
    preproc_ = p;
    for (hipEvent_t& e : preEv_)
        if (p && !e) BF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

void Recon::setFrameRaw(uint32_t f, const uint16_t* depthU16, const uint8_t* rgbx) {
    BF_REQUIRE(f < opt_.maxFrames, BF_ERR_CAPACITY, "frame index beyond maxFrames");
    frames_[f].rawDepth = depthU16;
    frames_[f].rawColor = rgbx;
    frames_[f].pre = false;
}

void Recon::preprocessFrame(uint32_t f) {
    FrameRef& fr = frames_[f];
    BF_REQUIRE(fr.depth && fr.color, BF_ERR_STATE, "preprocessing needs the frame's frame-store slot (bf_recon_set_frame)");
    const hipStream_t ps = preproc_->stream();
    // the raw sensor-depth buffer this run ends in (slot f & 1) was last read by frame f - 2's cache store;
    // frame f - 1's may still be running (its buffer is the other one)
    if (cacheEvF_[f & 1] && cache_ && cache_->stream() != ps) BF_HIP(hipStreamWaitEvent(ps, cacheEvF_[f & 1], 0));
    // colour at the integration size already: the loop reads the raw colour itself (no copy); the raw
    // images stay registered for as long as the frame store's
    const bool colorAsIs = preproc_->colorWidth() == cam_.imageWidth && preproc_->colorHeight() == cam_.imageHeight;
    preproc_->run(fr.rawDepth, fr.rawColor, const_cast<float*>(fr.depth), colorAsIs ? nullptr : const_cast<uint8_t*>(fr.color),
                  (int)(f & 1));
    if (colorAsIs) fr.color = fr.rawColor;
    // the scene stream first reads frame f in the batch of frame f + 1 (its integration is deferred,
    // pendingOp_), so it waits there (awaitPreproc), not here: frame f's preprocessing overlaps the
    // voxel pass of frame f's batch
    recordInputs(f, ps);
    fr.pre = true;
#ifdef BF_PRE_EARLY_WAIT  // A/B build: the scene stream waits right away (the first form)
    awaitPreproc(f);
#endif
    // copyToBundling: the cache takes the sensor-size raw depth and colour (as the FriedLiver app does)
    fr.srcDepth = preproc_->rawDepth();
    fr.srcColor = fr.rawColor;
    fr.srcW = preproc_->colorWidth();
    fr.srcH = preproc_->colorHeight();
}

// Bundler::storeCachedFrame (Bundler.cpp:278-281) for frame f, on the cache's stream
void Recon::storeCacheFrame(uint32_t f) {
    FrameRef& fr = frames_[f];
    // the frame's inputs were produced on another stream (the loop's preprocessing, or the caller's own work
    // announced by bf_recon_frame_ready): the cache reads them only after that work (its own stream waits)
    if (preFrame_[f % kPreSlots] == f) BF_HIP(hipStreamWaitEvent(cache_->stream(), preEv_[f % kPreSlots], 0));
    BF_REQUIRE(cache_->numFrames() == f, BF_ERR_STATE, "attached cache must hold exactly the frames before this one");
    // multi-GPU: a rank solves only its own local submaps (round-robin, issueSubmap), so it builds the cache
    // frames of those and the keyframes (the dense end solve runs on every rank); other slots stay empty
    const uint32_t S = opt_.submapSize;
    if (comm_ && comm_->size() > 1 && f % S != 0 && (f / S) % (uint32_t)comm_->size() != (uint32_t)comm_->rank()) {
        cache_->increment();
        fr.cache = BFCachedFrame{};
        return;
    }
    const float* d = fr.srcDepth ? fr.srcDepth : fr.depth;
    const uint8_t* c = fr.srcDepth ? fr.srcColor : fr.color;
    const uint32_t w = fr.srcDepth ? fr.srcW : cam_.imageWidth, h = fr.srcDepth ? fr.srcH : cam_.imageHeight;
    // k_cache_geometry reads the depth as the cache's input size: without a frame source the frame
    // store's integration-size depth must be that size
    BF_REQUIRE(fr.srcDepth || (cache_->config().inputWidth == cam_.imageWidth && cache_->config().inputHeight == cam_.imageHeight),
               BF_ERR_ARG, "the attached cache's input size differs from the integration size: set a frame source (bf_recon_set_frame_source)");
    cache_->storeFrame(d, c, w, h);
    fr.cache = cache_->frame(f);
    cacheEv_ = cacheEvF_[f & 1];
    BF_HIP(hipEventRecord(cacheEv_, cache_->stream()));
}

BFEndSequenceResult Recon::endSequence(const BFEndSequenceOptions& o) {
    BFEndSequenceResult res{};
    synchronize();
    if (numFrames_ == 0) return res;
    const int32_t N = o.numSolveFramesBeforeExit;
    const uint32_t cap = o.maxPastEndFrames ? o.maxPastEndFrames : 100000u;
    const uint32_t denseLimit = o.denseFrameLimit ? o.denseFrameLimit : 10000u;
    const float wDense = o.denseDepthWeight > 0.0f ? o.denseDepthWeight : 15.0f;
    const uint32_t S = opt_.submapSize, last = (numFrames_ - 1) / S, n = numFrames_ - last * S;
    auto keyframeCaches = [&]() {
        if (lastSubmapEnqueued_ == 0xFFFFFFFFu) return false;
        for (uint32_t k = 0; k <= lastSubmapEnqueued_; k++)
            if (!frames_[k * S].cache.depth) return false;
        return true;
    };
    for (uint32_t p = 0; p < cap; p++) {
        res.pastEndFrames = p + 1;
        if (N < 0 || (int64_t)p <= (int64_t)N) {
            if (p == 0 && last != lastSubmapEnqueued_ && n >= 2) {
                // prepareLocalSolve(curFrame, true) at the first past-the-end processInput, then process():
                // the partial submap's local solve, fuseToGlobal and the global solve
                const uint64_t before = st_.globalSolves;
                endSubmap(last, n);
                synchronize();
                res.localSolved = 1;
                res.globalSolves += (uint32_t)(st_.globalSolves - before);
                res.last = to_abi(lastGlobalResult_);
            } else {
                // setSolveWeights(sparse 1, dense depth 15, colour 0) at numFramesPastEnd == N (:177-189)
                const bool dense = N >= 0 && (int64_t)p == (int64_t)N && !o.disableDenseAtEnd &&
                                   numFrames_ - 1 < denseLimit && keyframeCaches();
                float ms = 0.0f;
                const SolveResult r = endSolve(dense ? wDense : 0.0f, &ms);
                if (!r.skipped) res.globalSolves++;
                if (dense) {
                    res.denseSolve = 1;
                    res.denseSolveMs = ms;
                }
                res.last = to_abi(r);
            }
        }
        reintegrate();
        // exit check (DepthSensing.cpp:1116-1123) once the solves are done
        if (N >= 0 && (int64_t)p >= (int64_t)N) {  // N < 0 (the reference's -1) never exits: maxPastEndFrames bounds it
            tm_->generateUpdateLists();
            const uint32_t active = tm_->numActiveOperations();
            traceQueue(3, 0, active, nullptr, nullptr);
            if (active == 0) {
                res.queueDrained = 1;
                break;
            }
        }
    }
    synchronize();
    return res;
}

uint32_t Recon::optimizedTrajectory(BFMat4* out, uint32_t cap) const {
    const uint32_t n = std::min(tm_->numAddedFrames(), tm_->numOptimizedFrames());
    for (uint32_t i = 0; i < n && i < cap; i++)
        out[i] = tm_->type(i) == FrameType::Invalid ? ninf_mat() : tm_->optimized(i);
    return n;
}

void Recon::traceQueue(int32_t kind, uint32_t frame, uint32_t count, const BFMat4* T, const std::vector<FixOp>* fixes) {
    if (!opt_.recordOps) return;
    BFQueueEvent e{};
    e.kind = kind;
    e.frame = frame;
    e.count = count;
    if (kind == 0 || kind == 1) {
        e.offset = (uint32_t)qT_.size();
        qT_.insert(qT_.end(), T, T + count);
    } else if (kind == 2) {
        e.offset = (uint32_t)qFixes_.size();
        for (const FixOp& op : *fixes) {
            BFFixOp b{};
            b.kind = (int32_t)op.kind;
            b.frame = op.frame;
            std::memcpy(b.oldT, op.oldT.m, 64);
            std::memcpy(b.newT, op.newT.m, 64);
            qFixes_.push_back(b);
        }
    }
    qEvents_.push_back(e);
}

void Recon::trajectory(BFMat4* out, uint32_t n) const {
    for (uint32_t i = 0; i < n && i < opt_.maxFrames; i++) {
        const bool integrated = i < tm_->numAddedFrames() &&
                                (tm_->type(i) == FrameType::Integrated || tm_->type(i) == FrameType::ReIntegration);
        out[i] = integrated ? tm_->integrated(i) : ninf_mat();
    }
}

}  // namespace bf
