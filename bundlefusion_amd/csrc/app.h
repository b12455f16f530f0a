// app.h — FriedLiver's application loop over the north-star path (bf_app_*, include/bf/bf.h):
// main() (Source/FriedLiver.cpp:184-320) + OnD3D11FrameRender (Source/DepthSensing/DepthSensing.cpp:
// 966-1129) + StopScanningAndExit (:904-953), with the reference's threads replaced by: decode threads
// that read and decompress .sens frames ahead of the loop (SensorDataReader's RGBDFrameCacheRead),
// one HIP stream for input preprocessing and the dense-term cache, and the loop's own scene / bundling
// streams (recon.h). Parameters come from the two zParameters files exactly as GlobalAppState and
// GlobalBundlingState read them (two separate name spaces: both files define s_depthSigmaD etc.).
#pragma once
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bf/bf.h"
#include "cache.h"
#include "corr.h"
#include "frames.h"
#include "io.h"
#include "recon.h"

namespace bf {

// What bf_app_create derives from the two parameter files and the .sens header (host only)
struct AppConfig {
    BFAppInfo info{};
    BFReconOptions ro{};
    std::string sensPath, outDir;
    float mcThreshFactor = 10.0f;
    uint32_t mcMaxTriangles = 3000000;
    uint32_t S = 10, L = 11;
    uint32_t localMinPerPair = 5;
    std::vector<BFMat4> sensPose;  // the .sens trajectory
};
AppConfig load_app_config(const std::string& appParams, const std::string& bundlingParams, const BFAppOptions& o);

class App {
public:
    App(const std::string& appParams, const std::string& bundlingParams, const BFAppOptions& o);
    ~App();
    bool step();            // one input frame through the loop; false at the end of the input
    BFAppResult finish();   // end of sequence + exit outputs
    BFAppResult run();
    Recon& recon() { return *recon_; }
    const BFAppInfo& info() const { return info_; }
    BFMat4 frontEndPose(uint32_t f) const;
    BFAppTiming timing() const;

private:
    struct Slot {  // one decoded frame (pinned host memory)
        uint16_t* depth = nullptr;
        uint8_t* rgbx = nullptr;
        int64_t frame = -1;  // frame held, -1 free
        int64_t expect = 0;  // the next frame this slot takes (slot index, + numSlots per use)
        bool ready = false;
        std::string error;
    };
    void decodeLoop(uint32_t worker);
    Slot& waitFrame(uint32_t f);
    void releaseFrame(uint32_t f);
    void releaseUploaded();  // the last uploaded frame's pinned slot, once its copies ran
    void localCorrespondences(uint32_t s, uint32_t n);  // submap s's EntryJ (local indices)
    void keyframeCorrespondences(uint32_t k);           // keyframe k against keyframes 0..k-1
    void writeOutputs(BFAppResult& r);

    BFAppOptions opt_;
    BFAppInfo info_{};
    std::string sensPath_, outDir_;
    float mcThreshFactor_ = 10.0f;
    uint32_t mcMaxTriangles_ = 3000000;
    uint32_t S_ = 10, L_ = 11;
    uint32_t localMinPerPair_ = 5;
    uint32_t shardCount_ = 1, shardIndex_ = 0;  // this rank's TSDF shard (BFAppOptions)
    std::vector<BFMat4> sensPose_;      // the .sens trajectory (front end + EntryJ stand-in)
    std::vector<BFMat4> tinc_;

    // decode threads
    uint32_t numSlots_ = 16, numWorkers_ = 4;
    std::vector<Slot> slots_;
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;

    // device
    hipStream_t pre_ = nullptr;         // preprocessing + cache stream
    hipEvent_t uploadEv_ = nullptr;     // after the last frame's H2D copies
    int64_t uploaded_ = -1;             // that frame (its pinned slot not yet released), or -1
    std::unique_ptr<Preproc> preproc_;
    std::unique_ptr<Cache> cache_;
    std::unique_ptr<Recon> recon_;
    DevBuf<uint16_t> dDepthU16_;
    DevBuf<uint8_t> dRgbx_;
    DevBuf<float> frameDepth_;          // frame store: integration-size depth per frame
    DevBuf<uint8_t> frameColor_;        // ... and colour (uchar4)
    DevBuf<float> localDepth_;          // sensor-size filtered depth of the last L frames (ring)
    DevBuf<float> kfDepth_;             // ... of every keyframe
    DevBuf<float> localT_, localTinv_, kfT_, kfTinv_;
    DevBuf<const float*> depthPtrs_;    // pointer table handed to the EntryJ producer
    DevBuf<BFEntryJ> localCorr_, globalCorr_;
    CorrScratch corrScratch_;           // the EntryJ producer's buffers (no per-call allocation)
    std::vector<uint32_t> globalPrefix_;
    uint32_t globalN_ = 0;
    uint32_t next_ = 0;                 // next input frame
    bool finished_ = false;
    double loopSeconds_ = 0.0;
    BFAppTiming tm_{};                  // host time per section (bf_app_timing)
    double decodeSeconds_ = 0.0;        // summed over the workers (under mu_)
};

}  // namespace bf
