// recon.h — the per-frame reconstruction loop with on-the-fly re-integration and the
// hierarchical (local submap -> global keyframe) bundle adjustment, i.e. the parts of
// DepthSensing.cpp's frame loop (Source/DepthSensing/DepthSensing.cpp:1003-1056, reintegrate
// :854-902) and OnlineBundler (Source/OnlineBundler.cpp:242-416, OnlineBundler.cu:6-140) that sit
// on the north-star path. Correspondence *production* (SiftGPU) is out of scope: EntryJ lists
// are inputs, as if the matcher had filled SIFTImageManager's global correspondence array.
//
// Ordering per frame f (submap size S, s = f / S):
//   0. pick up finished bundling results (async mode): poses -> trajectory -> TrajectoryManager
//   1. if f is the first frame of submap s > 0: enqueue the end of submap s-1 on the BA stream —
//      local solve over its S+1 frames (dense term on the 80x60 cache), global solve over
//      keyframes 0..s-1, device-side max residual removal (SBA.cpp:164-203), seed of keyframe s
//      = global[s-1] * local[s-1][S] (initNextGlobalTransformCU), async copies of the poses
//   2. reintegrate(): up to maxFrameFixes de-/re-/integrate ops from the TrajectoryManager, then GC
//   3. integrate frame f with kf[s] * L[f] and addFrame(Integrated), where L chains the front end's
//      frame-to-frame estimates Tinc inside the submap (L = I at its first frame) and kf[s] is the
//      keyframe pose — from the solver when its result has arrived, else dead-reckoned
// In async mode the TSDF never waits for the solver, as the reference's reconstruction thread
// never waits for its bundling thread; in sync mode step 1 waits, which makes runs repeatable.
#pragma once
#include <array>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/bf/bf.h"
#include "ba.h"
#include "cache.h"
#include "frames.h"
#include "trajectory.h"
#include "tsdf.h"

namespace bf {

class Recon {
public:
    Recon(const BFHashParams& hp, const BFSceneOptions* so, const BFDepthCameraParams& cam, const BFReconOptions& opt);
    ~Recon();

    void setFrame(uint32_t f, const float* depth, const uint8_t* color, const BFCachedFrame* cache, const BFMat4& Tinc);
    void setLocalCorrespondences(uint32_t submap, BFEntryJ* corr, uint32_t n);
    // global EntryJ list ordered by max(i, j); prefix[k] = #entries with max(i, j) <= k
    void setGlobalCorrespondences(BFEntryJ* corr, uint32_t n, const uint32_t* prefix, uint32_t numKeyframes);
    void setInitialPose(const BFMat4& T0);
    void setComm(Comm* c);  // shard the global solve's normal equations over c's ranks
    void processFrame(uint32_t f);
    void finish();       // end of sequence: solve the last (partial) submap and wait for all results
    void reintegrate();  // one render-loop iteration without a new frame: apply results, fix ops, GC
    void synchronize();  // drain both streams and apply every pending bundling result
    // one end-of-sequence global solve over every keyframe (dense depth weight wDense when > 0); waits
    SolveResult endSolve(float wDense, float* ms);
    // the render loop past the last frame (bf_recon_end_sequence: OnlineBundler.cpp:167-196, 373-408,
    // DepthSensing.cpp:1114-1126)
    BFEndSequenceResult endSequence(const BFEndSequenceOptions& o);
    // per-frame CUDACache::storeFrame inside processFrame (OnlineBundler.cpp:199-204); c is borrowed
    void attachCache(Cache* c);
    void setFrameSource(uint32_t f, const float* depth, const uint8_t* color, uint32_t colorW, uint32_t colorH);
    // frame f's frame-store images are being produced on stream s (the FriedLiver app's input stream): the
    // scene stream waits for that before the batch that first reads them
    void inputsProduced(uint32_t f, hipStream_t s);
    // CUDAImageManager::process inside the loop: frame f's raw sensor images are preprocessed into its
    // frame-store slot when it is processed (the cache then reads the raw sensor depth and colour)
    void attachPreproc(Preproc* p);
    void setFrameRaw(uint32_t f, const uint16_t* depthU16, const uint8_t* rgbx);
    // TrajectoryManager::getOptimizedTransforms (TrajectoryManager.h:50-68)
    uint32_t optimizedTrajectory(BFMat4* out, uint32_t cap) const;
    // recordOps: the TrajectoryManager call sequence (bf_recon_queue_trace)
    const std::vector<BFQueueEvent>& queueEvents() const { return qEvents_; }
    const std::vector<BFMat4>& queueTransforms() const { return qT_; }
    const std::vector<BFFixOp>& queueFixes() const { return qFixes_; }
    // recordOps history: submap s's local trajectory and the keyframe poses after its global solve
    void submapPoses(uint32_t s, float* local, float* global, int32_t* valid, uint32_t* numLocal, uint32_t* numKeyframes,
                     int32_t* localValid) const;

    BFReconStats stats();
    void resetStats();
    void trajectory(BFMat4* out, uint32_t n) const;   // integrated transform per frame (-inf if none)
    Scene& scene() {  // external access sees every frame integrated so far
        flushIntegrate();
        return *scene_;
    }
    BFSceneCapacity sceneCapacity() { return scene().capacity(); }
    // test hook (bf_recon_capture_global_solve): keep the inputs and the outcome of submap s's in-loop global solve
    void captureGlobalSolve(uint32_t s);
    void capturedGlobalSolve(BFEntryJ* corrIn, BFEntryJ* corrOut, uint32_t cap, uint32_t* nCorr, float* poseIn,
                             float* poseOut, int32_t* valid, uint32_t capImages, uint32_t* nImages);
    // visualizeFrame's render after every frame's integration (bf_recon_set_render); nullptr stops
    void setRender(const BFRayCastParams* rp);
    void renderOutput(const float** depth, const float** depth4, const float** normals, const float** colors) const;
    const BFDepthCameraParams& camera() const { return cam_; }
    const std::vector<BFFixOp>& opLog() const { return log_; }

private:
    struct Pending {  // one submap's bundling results in flight
        uint32_t submap = 0, numLocal = 0, numKeyframes = 0;
        uint32_t issueFrame = 0;    // the frame whose processing issued it (resultLag)
        uint64_t job = 0;  // bundling-thread job that enqueues this submap's work (see baPost)
        bool localSolved = false, globalSolved = false;
        bool endSolve = false;      // an end-of-sequence global solve (no local part)
        hipEvent_t done = nullptr;
        int* gate = nullptr;        // pinned: the submap's verification outcome (1 valid)
        float* localT = nullptr;    // pinned [S+1][16]
        float* globalT = nullptr;   // pinned [maxKeyframes][16]
        int* valid = nullptr;       // pinned [maxKeyframes]
        uint32_t* ctrl = nullptr;   // pinned [2][kResultWords]: local, global solver words
        float* localInit = nullptr;          // pinned staging [S+1][16] (H2D of the initial local poses)
        BFCachedFrame* cacheTable = nullptr; // pinned staging [S+1] (H2D of the local cache table)
    };
    void endSubmap(uint32_t s, uint32_t numFrames);
    struct GlobalView {  // the global correspondence list as a submap's issue sees it
        BFEntryJ* corr;
        uint32_t n, ncorr, pairBound;
    };
    void issueSubmap(uint32_t s, uint32_t n, uint32_t S, uint32_t slot, bool haveCache, std::pair<BFEntryJ*, uint32_t> lc,
                     uint32_t nk, hipEvent_t cacheEv, GlobalView gv);
    void issueEndSolve(uint32_t slot, uint32_t nk, uint32_t ncorr, float wDense, hipEvent_t t0, hipEvent_t t1);
    void applyPending(bool block);
    void apply(Pending& p);
    void runReintegrate();
    void logOp(int kind, uint32_t frame, const BFMat4* T);
    // fail with BF_ERR_CAPACITY once the scene dropped a block (its sticky error bits): exact = read the device
    // word (after a synchronization), else the copy the last GC kernel mirrored to the host
    void checkScene(bool exact);
    uint32_t capSubmap_ = 0xFFFFFFFFu;  // captureGlobalSolve
    bool capDone_ = false;
    uint32_t capN_ = 0, capK_ = 0;
    DevBuf<BFEntryJ> capCorrIn_, capCorrOut_;
    DevBuf<float> capPoseIn_, capPoseOut_;  // [rot 3K | trans 3K]
    DevBuf<int> capValid_;
    bool render_ = false;  // setRender
    BFRayCastParams renderParams_{};
    DevBuf<float> rDepth_;
    DevBuf<float4> rDepth4_, rNormals_, rColors_;

    BFReconOptions opt_;
    BFDepthCameraParams cam_;
    // baStream_: global solves (and the multi-GPU exchanges, in one order on every rank); localStream_:
    // local solves, which depend only on their submap's frames, so submap s+1's local solve runs while
    // submap s's global solve is still in flight
    hipStream_t sceneStream_ = nullptr, baStream_ = nullptr, localStream_ = nullptr;
    hipStream_t copyStream_ = nullptr;  // host readbacks of inputs (computePairBounds), created on first use
    // bundling streams at the highest and at normal queue priority; baStream_ / localStream_ are the active
    // pair (switchBundlingPriority, keyed on the size of the solve being issued)
    hipStream_t baStreamHi_ = nullptr, baStreamLo_ = nullptr, localStreamHi_ = nullptr, localStreamLo_ = nullptr;
    static constexpr uint32_t kHighPriorityMaxKeyframes = 1537;  // persistent grid <= ~3/4 of the CU slots
    bool baHigh_ = true, sharded_ = false;
    int priorityPolicy_ = -1;  // -1: by solve size; 0 / 1: normal / high throughout (BFReconOptions.bundlingPriority)
    void switchBundlingPriority(uint32_t nk);
    std::unique_ptr<Scene> scene_;
    std::unique_ptr<Solver> local_, global_;
    std::unique_ptr<TrajectoryManager> tm_;

    struct FrameRef {
        const float* depth = nullptr;
        const uint8_t* color = nullptr;
        BFCachedFrame cache{};
        BFMat4 Tinc{};    // front-end estimate: camera f in camera f-1 coordinates
        BFMat4 Tlocal{};  // chained estimate relative to the submap's first frame
        const float* srcDepth = nullptr;   // cache source images (setFrameSource; null: the frame store's)
        const uint8_t* srcColor = nullptr;
        uint32_t srcW = 0, srcH = 0;
        const uint16_t* rawDepth = nullptr;  // sensor images preprocessed into depth / color (attachPreproc)
        bool pre = false;                    // preprocessed (the loop runs frame f + 1's ahead, at frame f)
        const uint8_t* rawColor = nullptr;
        bool set = false;
        bool tilesReady = false;  // its band-cull depth tiles and dc image are in frameTiles_ / frameDC_
    };
    // per-frame band-cull depth tiles (Scene::tileCount each) and interleaved {depth, colour} image
    // (W*H uint2): computed the first time a frame enters an op batch, reused by every later
    // (re-)integration of that frame
    DevBuf<float2> frameTiles_;
    size_t tileStride_ = 0;
    DevBuf<uint2> frameDC_;
    size_t framePixels_ = 0;
    VoxelOp frameOp(uint32_t f, const BFMat4& T, bool deint);
    std::vector<FrameRef> frames_;
    std::vector<std::pair<BFEntryJ*, uint32_t>> localCorr_;
    BFEntryJ* globalCorr_ = nullptr;
    uint32_t globalCorrN_ = 0;
    std::vector<uint32_t> globalPrefix_;
    Comm* comm_ = nullptr;
    std::vector<uint32_t> pairBound_;  // distinct image pairs among the entries of each keyframe prefix
    std::unordered_set<uint64_t> pairSeen_;  // the pairs counted so far (entries [0, pairCountedN_))
    uint32_t pairCountedN_ = 0;
    void computePairBounds(bool append);

    std::vector<BFMat4> kf_;            // keyframe poses used for integration (solver or dead reckoning)
    std::vector<char> kfSolved_;        // kf_[k] came from the solver
    std::vector<BFMat4> globalT_;       // last solver keyframe poses
    std::vector<int> globalValid_;
    std::vector<std::vector<BFMat4>> localTraj_;  // per submap, S+1 local poses
    std::vector<char> localKnown_;
    std::vector<BFMat4> complete_;
    std::vector<FixOp> ops_;
    std::vector<VoxelOp> batch_;
    // The integration of frame f is the scene call right before frame f+1's fixes (nothing touches
    // the scene in between), so it is deferred and runs as op 0 of that batch: one voxel pass less
    // per frame, same call sequence. Any other scene access flushes it first.
    bool pendingInt_ = false;
    VoxelOp pendingOp_{};
    void flushIntegrate();
    uint32_t lastSubmapEnqueued_ = 0xFFFFFFFFu;
    uint32_t optimizedFrames_ = 0;      // frames covered by the complete trajectory (m_totalNumOptLocalFrames)
    SolveResult lastGlobalResult_{};
    uint32_t numFrames_ = 0;

    std::vector<Pending> ring_;
    std::deque<uint32_t> inflight_;     // ring indices in submap order
    uint32_t ringNext_ = 0;

    // Bundling thread (the reference's bundling thread, OnlineBundler), asyncBundling = 2: a submap's
    // local + global solves are ~450 kernel launches; the frame loop posts them as one job and this
    // thread issues them on baStream_ in post order, so the loop never spends the launch time. Off by
    // default (jobs run inline): without a profiler the host issues them faster than the scene stream
    // drains its queue, and the bench showed no difference (949 vs 949 frames/s).
    void baPost(std::function<void()> job);  // returns the job's sequence number in lastJob_
    void baWaitFor(uint64_t job);            // until job `job` has been issued (rethrows its error)
    void baDrain();                          // until every posted job has been issued
    void baLoop();
    bool baThreaded_ = true;
    std::thread baThread_;
    std::mutex baMu_;
    std::condition_variable baCv_, baDoneCv_;
    std::deque<std::function<void()>> baJobs_;
    bool baStop_ = false;
    uint64_t lastJob_ = 0;           // jobs posted (frame-loop thread)
    std::atomic<uint64_t> baDone_{0};  // jobs issued
    std::exception_ptr baErr_;

    // per-submap local state, double-buffered by submap parity: set s & 1 is written by local solve s
    // and read by global solve s (gate, keyframe seed); local solve s + 2 waits for globalDone_[s & 1]
    struct LocalSet {
        DevBuf<float> rot, T;     // rot holds [rot 3L | trans 3L | gate] (one broadcast)
        float* trans = nullptr;
        int* gate = nullptr;      // the submap's verification outcome, read by the gated global solve
        DevBuf<int> valid;
        DevBuf<BFCachedFrame> cache;
    };
    LocalSet ls_[2];
    hipEvent_t localDone_[2] = {nullptr, nullptr}, globalDone_[2] = {nullptr, nullptr};
    DevBuf<BFCachedFrame> dGlobalCache_; // keyframe k's cache frame (frame k * S), for the end-of-sequence dense solve
    struct SubmapRecord {  // recordOps history
        std::vector<BFMat4> local, global;
        std::vector<int> valid;
        int localOk = 1;
    };
    std::vector<SubmapRecord> history_;
    DevBuf<float> dGlobalRot_, dGlobalTrans_, dGlobalT_;
    DevBuf<int> dGlobalValid_;
    DevBuf<float> dSeedT_;
    DevBuf<int> dOne_;

    BFReconStats st_{};
    std::vector<BFFixOp> log_;

    Cache* cache_ = nullptr;            // attached frame cache (borrowed)
    hipEvent_t cacheEv_ = nullptr;      // the last storeFrame on the cache's stream (one of cacheEvF_)
    hipEvent_t cacheEvF_[2] = {nullptr, nullptr};  // frame f's storeFrame: cacheEvF_[f & 1]
    Preproc* preproc_ = nullptr;        // attached input preprocessing (borrowed)
    // a frame's input production (preprocessing, or the app's input stream) on its stream, per frame f & 3: frame
    // f + 1 is preprocessed ahead while frame f - 1's record still awaits its batch
    static constexpr uint32_t kPreSlots = 4;
    hipEvent_t preEv_[kPreSlots] = {nullptr, nullptr, nullptr, nullptr};
    bool prePending_[kPreSlots] = {false, false, false, false};  // recorded and not yet awaited by the scene stream
    // the frame whose inputs preEv_[slot] marks (the cache store of that frame waits on it, whichever stream
    // produced the inputs: the loop's preprocessor or a caller's, bf_recon_frame_ready)
    uint32_t preFrame_[kPreSlots] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    void recordInputs(uint32_t f, hipStream_t s);
    void awaitPreproc(uint32_t f);               // the scene stream after frame f's preprocessing
    void storeCacheFrame(uint32_t f);
    void preprocessFrame(uint32_t f);

    // recordOps: TrajectoryManager call trace
    std::vector<BFQueueEvent> qEvents_;
    std::vector<BFMat4> qT_;
    std::vector<BFFixOp> qFixes_;
    void traceQueue(int32_t kind, uint32_t frame, uint32_t count, const BFMat4* T, const std::vector<FixOp>* fixes);
};

}  // namespace bf
