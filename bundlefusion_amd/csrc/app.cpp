// app.cpp — see app.h.
#include "app.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <fstream>
#include <limits>

#include "frontend.h"

namespace bf {

BFMat4 mat4_inverse(const BFMat4& M);  // api.cpp (cuda_SimpleMatrixUtil.h getInverse)

namespace {

// GlobalAppState / GlobalBundlingState: a key missing from the file keeps the default of the reference's
// own zParameters*Default.txt (the reference warns and default-constructs, GlobalAppState.h:129-131)
double num(const ParamFile& f, const char* key, double def) { return f.has(key) ? f.number(key) : def; }
float flt(const ParamFile& f, const char* key, float def) { return f.has(key) ? f.floats(key).at(0) : def; }
bool flag(const ParamFile& f, const char* key, bool def) { return f.has(key) ? f.boolean(key) : def; }

std::string dir_of(const std::string& p) {
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}
std::string stem_of(const std::string& p) {  // util::removeExtensions(util::fileNameFromPath(p))
    const size_t k = p.find_last_of('/');
    std::string n = k == std::string::npos ? p : p.substr(k + 1);
    const size_t d = n.find('.');
    return d == std::string::npos ? n : n.substr(0, d);
}
bool finite_pose(const BFMat4& T) {
    for (float v : T.m)
        if (!std::isfinite(v)) return false;
    return true;
}
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// The parameter half of bf_app_create (FriedLiver.cpp:228-250 + the .sens header): everything the app derives
// from the two zParameters files and the sensor file, without touching the device (bf_app_resolve).
AppConfig load_app_config(const std::string& appParams, const std::string& bundlingParams, const BFAppOptions& o) {
    AppConfig c;
    ParamFile ap, bp;  // FriedLiver.cpp:228-250: two files, two name spaces
    ap.load(appParams);
    bp.load(bundlingParams);
    c.sensPath = (o.sensFile && *o.sensFile) ? std::string(o.sensFile) : ap.str("s_binaryDumpSensorFile");
    c.outDir = (o.outputDir && *o.outputDir) ? std::string(o.outputDir) : dir_of(c.sensPath);

    // ---- SensorDataReader::createFirstConnected (SensorDataReader.cpp:38-79) ----------------------------
    SensReader reader(c.sensPath);
    const BFSensInfo si = reader.info();
    BF_REQUIRE(si.depthWidth >= 2 && si.depthHeight >= 2, BF_ERR_IO, "no depth stream in " + c.sensPath);
    BF_REQUIRE(si.colorCompression >= 0 && si.colorCompression <= 2 && si.colorWidth >= 2 && si.colorHeight >= 2, BF_ERR_ARG,
               "the path integrates colour: raw / PNG / JPEG colour stream required");
    c.S = (uint32_t)num(bp, "s_submapSize", 10);
    c.L = c.S + 1;
    const uint32_t maxNumImages = (uint32_t)num(bp, "s_maxNumImages", 1200);
    uint64_t frames = si.numFrames;
    if (o.maxFrames) frames = std::min<uint64_t>(frames, o.maxFrames);
    BF_REQUIRE(frames <= (uint64_t)maxNumImages * c.S, BF_ERR_CAPACITY,
               "sens file #frames = " + std::to_string(frames) + ", please change param file to accommodate");
    BF_REQUIRE(frames >= 1, BF_ERR_IO, "empty .sens file");
    c.info.numFrames = (uint32_t)frames;
    c.info.sensorDepthWidth = si.depthWidth;
    c.info.sensorDepthHeight = si.depthHeight;
    c.info.sensorColorWidth = si.colorWidth;
    c.info.sensorColorHeight = si.colorHeight;
    c.sensPose.resize(frames);
    for (uint64_t f = 0; f < frames; f++) reader.pose(f, c.sensPose[f].m);

    // ---- parameters ---------------------------------------------------------------------------------
    const uint32_t iw = (uint32_t)num(ap, "s_integrationWidth", 320), ih = (uint32_t)num(ap, "s_integrationHeight", 240);
    const float* K = si.depthIntrinsic;  // row-major mat4f: fx K[0], fy K[5], mx K[2], my K[6]
    BFDepthCameraParams cam{};           // CUDAImageManager.h:160-166 + DepthSensing.cpp:636-643
    cam.fx = K[0] * ((float)iw / (float)si.depthWidth);
    cam.fy = K[5] * ((float)ih / (float)si.depthHeight);
    cam.mx = K[2] * ((float)(iw - 1) / (float)(si.depthWidth - 1));
    cam.my = K[6] * ((float)(ih - 1) / (float)(si.depthHeight - 1));
    cam.imageWidth = iw;
    cam.imageHeight = ih;
    cam.sensorDepthWorldMin = flt(ap, "s_renderDepthMin", 0.1f);
    cam.sensorDepthWorldMax = flt(ap, "s_renderDepthMax", 4.0f);
    c.info.integrationCamera = cam;
    c.info.hashParams = hash_params_from(ap);
    c.info.preprocess = preprocess_options_from(bp, si.depthShift);
    c.mcThreshFactor = flt(ap, "s_SDFMarchingCubeThreshFactor", 10.0f);
    c.mcMaxTriangles = (uint32_t)num(ap, "s_marchingCubesMaxNumTriangles", 3000000);
    c.info.numSolveFramesBeforeExit = o.numSolveFramesBeforeExit ? o.numSolveFramesBeforeExit
                                                               : (int32_t)num(ap, "s_numSolveFramesBeforeExit", 30);

    // CUDACache (Bundler.cpp:33-38): sensor-size depth input, s_downsampledWidth x Height
    BFCacheOptions& co = c.info.cache;
    co.inputWidth = si.depthWidth;
    co.inputHeight = si.depthHeight;
    co.width = (uint32_t)num(bp, "s_downsampledWidth", 80);
    co.height = (uint32_t)num(bp, "s_downsampledHeight", 60);
    co.maxFrames = c.info.numFrames;
    std::memcpy(co.inputIntrinsics, si.depthIntrinsic, 64);
    co.colorSigma = flt(bp, "s_colorDownSigma", 2.5f);
    co.depthSigmaD = flt(bp, "s_depthDownSigmaD", 1.0f);
    co.depthSigmaR = flt(bp, "s_depthDownSigmaR", 0.05f);

    // the EntryJ producer (AddCurrToResidualsCU's siftIntrinsicsInv at the sensor depth size)
    BFCorrOptions& cr = c.info.corr;
    cr.intrinsics[0] = K[0];
    cr.intrinsics[1] = K[5];
    cr.intrinsics[2] = K[2];
    cr.intrinsics[3] = K[6];
    BFMat4 Km;
    std::memcpy(Km.m, si.depthIntrinsic, 64);
    const BFMat4 Kinv = mat4_inverse(Km);
    std::memcpy(cr.intrinsicsInv, Kinv.m, 64);
    cr.width = si.depthWidth;
    cr.height = si.depthHeight;
    cr.stride = o.corrStride ? o.corrStride : 16u;
    cr.maxPerPair = 25;  // MAX_MATCHES_PER_IMAGE_PAIR_FILTERED
    cr.minDepth = flt(ap, "s_sensorDepthMin", 0.1f);
    cr.maxDepth = flt(ap, "s_SDFMaxIntegrationDistance", 3.0f);
    cr.depthThresh = o.corrDepthThresh > 0.0f ? o.corrDepthThresh : 0.02f;

    const uint32_t numSubmaps = (c.info.numFrames + c.S - 1) / c.S;
    c.info.submapSize = c.S;
    c.info.maxKeyframes = numSubmaps + 1;
    c.info.maxLocalCorr = cr.maxPerPair * c.L * (c.L - 1) / 2;
    const uint64_t Kf = c.info.maxKeyframes;
    c.info.maxGlobalCorr = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1000, cr.maxPerPair * Kf * (Kf - 1) / 2), 0xFFFFFFFFull);

    c.ro.maxFrames = c.info.numFrames;
    c.ro.submapSize = c.S;
    c.ro.maxFrameFixes = (uint32_t)num(ap, "s_maxFrameFixes", 10);
    c.ro.topNActive = (uint32_t)num(ap, "s_topNActive", 30);
    c.ro.minPoseDistSqrt = flt(ap, "s_minPoseDistSqrt", 0.0f);
    c.ro.localNonLin = (uint32_t)num(bp, "s_numLocalNonLinIterations", 2);
    c.ro.localLin = (uint32_t)num(bp, "s_numLocalLinIterations", 100);
    c.ro.globalNonLin = (uint32_t)num(bp, "s_numGlobalNonLinIterations", 3);
    c.ro.globalLin = (uint32_t)num(bp, "s_numGlobalLinIterations", 150);
    c.ro.maxKeyframes = c.info.maxKeyframes;
    c.ro.maxLocalCorr = c.info.maxLocalCorr;
    c.ro.maxGlobalCorr = c.info.maxGlobalCorr;
    c.ro.maxResidualThresh = flt(bp, "s_optMaxResThresh", 0.08f);
    c.ro.useLocalDense = flag(bp, "s_useLocalDense", true) ? 1 : 0;
    c.ro.cacheWidth = co.width;
    c.ro.cacheHeight = co.height;
    // CUDACache::m_intrinsics: the input intrinsics scaled to the cache size (CUDACache.cpp:14-21)
    c.info.cacheIntrinsics[0] = K[0] * ((float)co.width / (float)co.inputWidth);
    c.info.cacheIntrinsics[1] = K[5] * ((float)co.height / (float)co.inputHeight);
    c.info.cacheIntrinsics[2] = K[2] * ((float)(co.width - 1) / (float)(co.inputWidth - 1));
    c.info.cacheIntrinsics[3] = K[6] * ((float)(co.height - 1) / (float)(co.inputHeight - 1));
    std::memcpy(c.ro.cacheIntrinsics, c.info.cacheIntrinsics, 16);
    c.ro.enableTiming = o.enableTiming;
    c.ro.recordOps = o.recordOps;
    c.ro.asyncBundling = o.asyncBundling;
    c.ro.resultLag = o.resultLag;
    c.ro.solver.denseDistThresh = flt(bp, "s_denseDistThresh", 0.15f);
    c.ro.solver.denseNormalThresh = flt(bp, "s_denseNormalThresh", 0.97f);
    c.ro.solver.denseColorThresh = flt(bp, "s_denseColorThresh", 0.1f);
    c.ro.solver.denseColorGradientMin = flt(bp, "s_denseColorGradientMin", 0.005f);
    c.ro.solver.denseDepthMin = flt(bp, "s_denseDepthMin", 0.5f);
    c.ro.solver.denseDepthMax = flt(bp, "s_denseDepthMax", 4.0f);
    c.ro.solver.denseOverlapSubsample = (uint32_t)num(bp, "s_denseOverlapCheckSubsampleFactor", 4);
    c.ro.disableLocalVerify = flag(bp, "s_useLocalVerify", true) ? 0 : 1;
    c.ro.verify.projCorrDistThresh = flt(bp, "s_projCorrDistThres", 0.15f);
    c.ro.verify.projCorrNormalThresh = flt(bp, "s_projCorrNormalThres", 0.97f);
    c.ro.verify.verifyOptErrThresh = flt(bp, "s_verifyOptErrThresh", 0.05f);
    c.ro.verify.verifyOptCorrThresh = flt(bp, "s_verifyOptCorrThresh", 0.001f);
    // the matcher's s_minNumMatchesLocal / Global filter on a pair (5)
    const uint32_t minLocal = (uint32_t)num(bp, "s_minNumMatchesLocal", 5), minGlobal = (uint32_t)num(bp, "s_minNumMatchesGlobal", 5);
    cr.minPerPair = minGlobal;
    c.localMinPerPair = minLocal;

    return c;
}

App::App(const std::string& appParams, const std::string& bundlingParams, const BFAppOptions& o) : opt_(o) {
    AppConfig c = load_app_config(appParams, bundlingParams, o);
    info_ = c.info;
    sensPath_ = c.sensPath;
    outDir_ = c.outDir;
    sensPose_ = std::move(c.sensPose);
    S_ = c.S;
    L_ = c.L;
    mcThreshFactor_ = c.mcThreshFactor;
    mcMaxTriangles_ = c.mcMaxTriangles;
    localMinPerPair_ = c.localMinPerPair;
    BFReconOptions ro = c.ro;
    const BFCacheOptions& co = info_.cache;
    const uint32_t iw = info_.integrationCamera.imageWidth, ih = info_.integrationCamera.imageHeight;
    const BFDepthCameraParams cam = info_.integrationCamera;
    const uint32_t numSubmaps = (info_.numFrames + S_ - 1) / S_;
    BFSensInfo si{};
    si.depthWidth = info_.sensorDepthWidth;
    si.depthHeight = info_.sensorDepthHeight;
    si.colorWidth = info_.sensorColorWidth;
    si.colorHeight = info_.sensorColorHeight;

    // ---- front end (frontend.h) ----------------------------------------------------------------------
    const float dr = o.noFrontEndDrift ? 0.0f : (o.frontEndDriftRad > 0.0f ? o.frontEndDriftRad : 0.05f * 3.14159265f / 180.0f);
    const float dm = o.noFrontEndDrift ? 0.0f : (o.frontEndDriftM > 0.0f ? o.frontEndDriftM : 0.002f);
    const uint32_t seed = o.frontEndSeed ? o.frontEndSeed : 1u;
    tinc_.resize(info_.numFrames);
    tinc_[0] = BFMat4{};
    tinc_[0].m[0] = tinc_[0].m[5] = tinc_[0].m[10] = tinc_[0].m[15] = 1.0f;
    for (uint32_t f = 1; f < info_.numFrames; f++)
        tinc_[f] = front_end_tinc(sensPose_[f - 1].m, sensPose_[f].m, f, seed, dr, dm);

    // ---- device state ----------------------------------------------------------------------------------
    {   // the input stream (upload, preprocessing, cache, EntryJ) feeds the loop's next batch: highest priority
        int prLeast = 0, prGreatest = 0;
        BF_HIP(hipDeviceGetStreamPriorityRange(&prLeast, &prGreatest));
        BF_HIP(hipStreamCreateWithPriority(&pre_, hipStreamNonBlocking, prGreatest));
    }
    BF_HIP(hipEventCreateWithFlags(&uploadEv_, hipEventDisableTiming));
    preproc_.reset(new Preproc(si.depthWidth, si.depthHeight, si.colorWidth, si.colorHeight, iw, ih, info_.preprocess, pre_));
    CacheConfig cc{};
    cc.inputWidth = co.inputWidth;
    cc.inputHeight = co.inputHeight;
    cc.width = co.width;
    cc.height = co.height;
    cc.maxFrames = co.maxFrames;
    std::memcpy(cc.inputIntrinsics, co.inputIntrinsics, 64);
    cc.colorSigma = co.colorSigma;
    cc.depthSigmaD = co.depthSigmaD;
    cc.depthSigmaR = co.depthSigmaR;
    cache_.reset(new Cache(cc, pre_));  // on the preprocessing stream: it reads that stream's buffers
    BFSceneOptions so{};  // multi-GPU: this rank's TSDF chunk-ownership shard
    so.shardCount = std::max(1u, o.shardCount);
    so.shardIndex = o.shardIndex;
    so.shardChunk = o.shardChunk;
    BF_REQUIRE(so.shardIndex < so.shardCount, BF_ERR_ARG, "shardIndex >= shardCount");
    shardCount_ = so.shardCount;
    shardIndex_ = so.shardIndex;
    recon_.reset(new Recon(info_.hashParams, &so, cam, ro));
    recon_->attachCache(cache_.get());
    const size_t ip = (size_t)iw * ih, dp = (size_t)si.depthWidth * si.depthHeight;
    dDepthU16_.alloc(dp);
    dRgbx_.alloc((size_t)si.colorWidth * si.colorHeight * 4);
    frameDepth_.alloc(ip * info_.numFrames);
    frameColor_.alloc(ip * 4 * info_.numFrames);
    localDepth_.alloc(dp * L_);
    kfDepth_.alloc(dp * info_.maxKeyframes);
    localT_.alloc(16 * L_);
    localTinv_.alloc(16 * L_);
    kfT_.alloc(16 * (size_t)info_.maxKeyframes);
    kfTinv_.alloc(16 * (size_t)info_.maxKeyframes);
    depthPtrs_.alloc(std::max(L_, info_.maxKeyframes));
    localCorr_.alloc((size_t)info_.maxLocalCorr * (numSubmaps + 1));
    globalCorr_.alloc(info_.maxGlobalCorr);
    globalPrefix_.reserve(info_.maxKeyframes);
    recon_->setInitialPose(finite_pose(sensPose_[0]) ? sensPose_[0] : tinc_[0]);

    // ---- decode threads (SensorDataReader's RGBDFrameCacheRead, SensorDataReader.cpp:76-77) ---------------
    numSlots_ = std::max(2u, o.prefetchFrames ? o.prefetchFrames : 16u);
    // decoding (zlib + JPEG at 640x480: ~3 ms per frame and thread) sets the pace below ~8 threads
    numWorkers_ = std::max(1u, std::min(numSlots_, o.decodeThreads ? o.decodeThreads : 8u));
    slots_.resize(numSlots_);
    for (uint32_t k = 0; k < numSlots_; k++) slots_[k].expect = k;
    for (Slot& s : slots_) {
        BF_HIP(hipHostMalloc((void**)&s.depth, dp * 2, hipHostMallocDefault));
        BF_HIP(hipHostMalloc((void**)&s.rgbx, (size_t)si.colorWidth * si.colorHeight * 4, hipHostMallocDefault));
    }
    for (uint32_t w = 0; w < numWorkers_; w++) workers_.emplace_back([this, w] { decodeLoop(w); });
}

App::~App() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : workers_)
        if (t.joinable()) t.join();
    if (pre_) (void)hipStreamSynchronize(pre_);  // no copy out of a pinned slot still in flight
    recon_.reset();
    cache_.reset();
    preproc_.reset();
    for (Slot& s : slots_) {
        if (s.depth) (void)hipHostFree(s.depth);
        if (s.rgbx) (void)hipHostFree(s.rgbx);
    }
    if (uploadEv_) (void)hipEventDestroy(uploadEv_);
    if (pre_) (void)hipStreamDestroy(pre_);
}

// worker w decodes frames w, w + W, ... into slot f % numSlots once the slot is free
void App::decodeLoop(uint32_t w) {
    std::unique_ptr<SensReader> r;
    std::string err;
    try {
        r.reset(new SensReader(sensPath_));
    } catch (const std::exception& e) {
        err = e.what();
    }
    for (uint32_t f = w; f < info_.numFrames; f += numWorkers_) {
        Slot& s = slots_[f % numSlots_];
        {
            std::unique_lock<std::mutex> lk(mu_);
            // in frame order per slot: frame f + numSlots waits until frame f has been consumed
            cv_.wait(lk, [&] { return stop_ || (s.frame < 0 && s.expect == (int64_t)f); });
            if (stop_) return;
            s.frame = f;
            s.ready = false;
        }
        std::string e = err;
        const double t0 = now_s();
        if (e.empty()) {
            try {
                r->depthU16(f, s.depth);
                r->colorRGBX(f, s.rgbx);
            } catch (const std::exception& ex) {
                e = ex.what();
            }
        }
        const double dt = now_s() - t0;
        {
            std::lock_guard<std::mutex> lk(mu_);
            decodeSeconds_ += dt;
            s.error = e;
            s.ready = true;
        }
        cv_.notify_all();
    }
}

void App::releaseUploaded() {
    if (uploaded_ < 0) return;
    BF_HIP(hipEventSynchronize(uploadEv_));
    releaseFrame((uint32_t)uploaded_);
    uploaded_ = -1;
}

App::Slot& App::waitFrame(uint32_t f) {
    Slot& s = slots_[f % numSlots_];
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return s.frame == (int64_t)f && s.ready; });
    if (!s.error.empty()) throw Error(BF_ERR_IO, "frame " + std::to_string(f) + ": " + s.error);
    return s;
}

void App::releaseFrame(uint32_t f) {
    {
        std::lock_guard<std::mutex> lk(mu_);
        Slot& s = slots_[f % numSlots_];
        s.frame = -1;
        s.ready = false;
        s.expect += numSlots_;
    }
    cv_.notify_all();
}

BFAppTiming App::timing() const {
    BFAppTiming t = tm_;
    t.decodeThreads = numWorkers_;
    {
        std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(mu_));
        t.decodeSeconds = decodeSeconds_;
    }
    return t;
}

BFMat4 App::frontEndPose(uint32_t f) const {
    BF_REQUIRE(f < tinc_.size(), BF_ERR_ARG, "frame index out of range");
    return tinc_[f];
}

// submap s = frames s*S .. s*S + n - 1: EntryJ of every pair (i, cur), cur = 1 .. n-1, local indices,
// matched with the .sens poses (AddCurrToResidualsCU as each frame arrives, SIFTImageManager.cu:610-686)
void App::localCorrespondences(uint32_t s, uint32_t n) {
    const uint32_t base = s * S_;
    const size_t dp = (size_t)info_.sensorDepthWidth * info_.sensorDepthHeight;
    std::vector<const float*> ptrs(n);
    std::vector<BFMat4> T(n), Ti(n);
    for (uint32_t i = 0; i < n; i++) {
        ptrs[i] = localDepth_.p + dp * ((base + i) % L_);
        T[i] = sensPose_[base + i];
        Ti[i] = mat4_inverse(T[i]);
    }
    BF_HIP(hipMemcpyAsync(depthPtrs_.p, ptrs.data(), sizeof(float*) * n, hipMemcpyHostToDevice, pre_));
    BF_HIP(hipMemcpyAsync(localT_.p, T.data(), 64 * n, hipMemcpyHostToDevice, pre_));
    BF_HIP(hipMemcpyAsync(localTinv_.p, Ti.data(), 64 * n, hipMemcpyHostToDevice, pre_));
    BFCorrOptions o = info_.corr;
    o.minPerPair = localMinPerPair_;
    BFEntryJ* out = localCorr_.p + (size_t)info_.maxLocalCorr * s;
    // every pair (i, cur), cur = 1 .. n-1, i < cur, in the order AddCurrToResidualsCU appends them as each
    // frame arrives: one launch for the submap on the input stream
    std::vector<uint2> list;
    for (uint32_t cur = 1; cur < n; cur++)
        for (uint32_t i = 0; i < cur; i++) list.push_back(make_uint2(i, cur));
    const uint32_t total = corr_from_pairs(depthPtrs_.p, localT_.p, localTinv_.p, list.data(), (uint32_t)list.size(), o, out,
                                           info_.maxLocalCorr, nullptr, pre_, corrScratch_);
    if (total) recon_->setLocalCorrespondences(s, out, total);
}

// keyframe k (frame k*S): EntryJ against every earlier keyframe, appended to the global list (ordered by
// max(i, j) = k); prefix[k] = its length
void App::keyframeCorrespondences(uint32_t k) {
    const size_t dp = (size_t)info_.sensorDepthWidth * info_.sensorDepthHeight;
    const BFMat4 T = sensPose_[(size_t)k * S_], Ti = mat4_inverse(T);
    BF_HIP(hipMemcpyAsync(kfT_.p + 16 * (size_t)k, T.m, 64, hipMemcpyHostToDevice, pre_));
    BF_HIP(hipMemcpyAsync(kfTinv_.p + 16 * (size_t)k, Ti.m, 64, hipMemcpyHostToDevice, pre_));
    if (k > 0) {
        std::vector<const float*> ptrs(k + 1);
        for (uint32_t i = 0; i <= k; i++) ptrs[i] = kfDepth_.p + dp * i;
        BF_HIP(hipMemcpyAsync(depthPtrs_.p, ptrs.data(), sizeof(float*) * (k + 1), hipMemcpyHostToDevice, pre_));
        std::vector<uint2> list(k);
        for (uint32_t i = 0; i < k; i++) list[i] = make_uint2(i, k);
        globalN_ += corr_from_pairs(depthPtrs_.p, kfT_.p, kfTinv_.p, list.data(), k, info_.corr, globalCorr_.p + globalN_,
                                    info_.maxGlobalCorr - globalN_, nullptr, pre_, corrScratch_);
    }
    globalPrefix_.push_back(globalN_);
    recon_->setGlobalCorrespondences(globalCorr_.p, globalN_, globalPrefix_.data(), (uint32_t)globalPrefix_.size());
}

bool App::step() {
    BF_REQUIRE(!finished_, BF_ERR_STATE, "the sequence has ended");
    if (next_ >= info_.numFrames) return false;
    const double t0 = now_s();
    const uint32_t f = next_;
    const BFDepthCameraParams& cam = info_.integrationCamera;
    const size_t ip = (size_t)cam.imageWidth * cam.imageHeight;
    const size_t dp = (size_t)info_.sensorDepthWidth * info_.sensorDepthHeight;
    // ---- CUDAImageManager::process ---------------------------------------------------------------------
    // the previous frame's pinned slot goes back to the decoders once its copies have run (a frame ago)
    releaseUploaded();
    Slot& sl = waitFrame(f);
    const double t1 = now_s();
    tm_.decodeWaitSeconds += t1 - t0;
    BF_HIP(hipMemcpyAsync(dDepthU16_.p, sl.depth, dp * 2, hipMemcpyHostToDevice, pre_));
    BF_HIP(hipMemcpyAsync(dRgbx_.p, sl.rgbx, dRgbx_.n, hipMemcpyHostToDevice, pre_));
    float* depth = frameDepth_.p + ip * f;
    uint8_t* color = frameColor_.p + ip * 4 * f;
    preproc_->run(dDepthU16_.p, dRgbx_.p, depth, color);
    // the bundler's copies (copyToBundling): filtered depth for the EntryJ producer (submap ring, keyframes)
    BF_HIP(hipMemcpyAsync(localDepth_.p + dp * (f % L_), preproc_->filteredDepth(), dp * 4, hipMemcpyDeviceToDevice, pre_));
    if (f % S_ == 0)
        BF_HIP(hipMemcpyAsync(kfDepth_.p + dp * (f / S_), preproc_->filteredDepth(), dp * 4, hipMemcpyDeviceToDevice, pre_));
    // no host wait: every later reader of the staging buffers (this frame's cache store, the next frame's
    // copies) is queued on pre_ behind them; the pinned slot is released at the next step
    BF_HIP(hipEventRecord(uploadEv_, pre_));
    uploaded_ = (int64_t)f;
    // the frame-store images are written on pre_: the loop's scene stream waits for them
    recon_->inputsProduced(f, pre_);
    const double t2 = now_s();
    tm_.uploadSeconds += t2 - t1;
    tm_.uploadBytes += (double)(dp * 2 + dRgbx_.n);
    // ---- processInput: cache source (stored by the loop on this stream), correspondences ------------
    recon_->setFrame(f, depth, color, nullptr, tinc_[f]);
    recon_->setFrameSource(f, preproc_->rawDepth(), dRgbx_.p, info_.sensorColorWidth, info_.sensorColorHeight);
    if (f % S_ == 0 && f > 0) {  // frame f closes submap s-1 (its overlap frame): the loop solves it now
        const uint32_t s = f / S_ - 1;
        localCorrespondences(s, L_);
        keyframeCorrespondences(s);
    }
    const double t3 = now_s();
    tm_.corrSeconds += t3 - t2;
    // ---- OnD3D11FrameRender: reintegrate + integrate (+ the submap's solves) -----------------------------
    recon_->processFrame(f);
    next_++;
    const double t4 = now_s();
    tm_.loopSeconds += t4 - t3;
    tm_.stepSeconds += t4 - t0;
    tm_.frames++;
    loopSeconds_ += t4 - t0;
    return true;
}

BFAppResult App::finish() {
    BF_REQUIRE(!finished_, BF_ERR_STATE, "finish called twice");
    releaseUploaded();
    BFAppResult r{};
    r.frames = next_;
    if (next_ > 0) {
        // the last (partial) submap: its EntryJ and keyframe before the end-of-sequence phase solves it
        const uint32_t last = (next_ - 1) / S_, n = next_ - last * S_;
        const double t0 = now_s();
        if (n >= 2 && globalPrefix_.size() == last) {
            localCorrespondences(last, n);
            keyframeCorrespondences(last);
        }
        if (info_.numSolveFramesBeforeExit != -2) {
            BFEndSequenceOptions eo{};
            eo.numSolveFramesBeforeExit = info_.numSolveFramesBeforeExit;
            r.end = recon_->endSequence(eo);
        } else {
            recon_->finish();
        }
        r.endSeconds = now_s() - t0;
    }
    r.loopSeconds = loopSeconds_;
    writeOutputs(r);
    finished_ = true;
    return r;
}

// StopScanningAndExit (DepthSensing.cpp:904-953)
void App::writeOutputs(BFAppResult& r) {
    Scene& scene = recon_->scene();
    recon_->synchronize();
    r.heapFreeCount = scene.heapFreeCount();
    std::vector<BFMat4> traj(info_.numFrames);
    r.numTransforms = recon_->optimizedTrajectory(traj.data(), (uint32_t)traj.size());
    traj.resize(r.numTransforms);
    for (const BFMat4& T : traj)
        if (T.m[0] != -std::numeric_limits<float>::infinity()) r.numValidTransforms++;
    r.valid = (r.heapFreeCount >= 800 && r.numValidTransforms >= (uint32_t)std::lround(0.5f * (float)r.numTransforms)) ? 1 : 0;
    // marching cubes (StopScanningAndExtractIsoSurfaceMC, :335-365) — counted even without outputs
    BFMarchingCubesParams mp{};
    mp.threshMarchingCubes = mp.threshMarchingCubes2 = mcThreshFactor_ * info_.hashParams.virtualVoxelSize;
    mp.maxNumTriangles = mcMaxTriangles_;
    DevBuf<BFMcTriangle> dt(mcMaxTriangles_);
    const uint32_t nt = scene.extractMesh(mp, dt.p, mcMaxTriangles_, nullptr);
    r.meshTriangles = nt;
    if (opt_.skipOutputs) return;
    std::vector<BFMcTriangle> tris(nt);
    if (nt) BF_HIP(hipMemcpy(tris.data(), dt.p, sizeof(BFMcTriangle) * nt, hipMemcpyDeviceToHost));
    const std::string stem = stem_of(sensPath_);
    const Mesh m = mesh_from_triangles(tris.data(), nt, nullptr);
    // a TSDF shard meshes its own blocks: one .ply per rank, the trajectory outputs (identical on every
    // rank) from shard 0 only
    const std::string part = shardCount_ > 1 ? ".shard" + std::to_string(shardIndex_) + "of" + std::to_string(shardCount_) : "";
    mesh_save_ply(outDir_ + "/" + stem + part + ".ply", m);
    r.meshVertices = (uint32_t)(m.vertices.size() / 3);
    r.meshFaces = (uint32_t)(m.faces.size() / 3);
    if (shardIndex_ != 0) return;
    const std::string sensOut = opt_.overwriteSens ? sensPath_ : outDir_ + "/" + stem + ".optimized.sens";
    sens_save_with_trajectory(sensPath_, sensOut, traj.data(), traj.size());
    std::ofstream s(outDir_ + "/processed.txt");
    BF_REQUIRE(s.good(), BF_ERR_IO, "cannot write " + outDir_ + "/processed.txt");
    s << (r.valid ? "valid = true" : "valid = false") << "\n";
    s << "heapFreeCount = " << r.heapFreeCount << "\n";
    s << "numValidOptTransforms = " << r.numValidTransforms << "\n";
    s << "numTransforms = " << r.numTransforms << "\n";
}

BFAppResult App::run() {
    while (step()) {
    }
    return finish();
}

}  // namespace bf
