// oracle/recon.cpp — TEST INFRASTRUCTURE (CPU oracle, see oracle.h header).
//
// Serial restatement of the bundling side of the reconstruction loop, in the order the product's
// synchronous mode (BFReconOptions.asyncBundling = 0) runs it, with every solve done by the oracle
// solver (ba.cpp) and the re-integration queue by the oracle TrajectoryManager (traj.cpp):
//   OnlineBundler::optimizeLocal      (Source/OnlineBundler.cpp:242-271)   local solve, no removal
//   SBA::align verification           (Source/SBA.cpp:106-109, Bundler.cpp:259-274,
//                                      Solver/CUDASolverBundling.cpp:454-476, SIFTImageManager.cu:1036-1159)
//   processGlobal / optimizeGlobal    (Source/OnlineBundler.cpp:280-408)   global solve + max-residual
//                                      removal (SBA.cpp:164-203), INVALIDATE path for a failed local
//   initNextGlobalTransformCU         (Source/OnlineBundler.cu:112-140), initializeNextTransformUnknown
//                                      (Source/Bundler.h:75-79)
//   updateTrajectoryCU                (Source/OnlineBundler.cu:73-110) -> TrajectoryManager
//   reintegrate()                     (Source/DepthSensing/DepthSensing.cpp:854-902), the op log only:
//                                      the TSDF does not feed back into the poses.
// The front end (SiftGPU tracking, computeSiftTransformCU) is replaced as in the product by the
// frames' frame-to-frame estimates Tinc chained inside a submap from the keyframe pose.
#include "oracle.h"
#include "or_lie.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

using namespace orc;

namespace {

const float NEG_INF = -std::numeric_limits<float>::infinity();

m4 identity() {
    m4 m{};
    for (int i = 0; i < 16; i++) m.e[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    return m;
}
m4 ninf() {
    m4 m;
    for (float& v : m.e) v = NEG_INF;
    return m;
}
m4 ld(const float* p) {
    m4 m;
    std::memcpy(m.e, p, 64);
    return m;
}

struct Rec {
    std::vector<m4> local, global;
    std::vector<int> valid;
    int localOk = 1;
};

struct Recon {
    ORReconParams P;
    uint32_t S = 10, L = 11, maxSubmaps = 0, K = 0;
    std::vector<m4> Tinc, Tlocal;
    std::vector<BFCachedFrame> cache;
    std::vector<char> frameSet;
    std::vector<std::vector<BFEntryJ>> localCorr;
    std::vector<BFEntryJ> globalCorr;
    std::vector<uint32_t> prefix;
    std::vector<m4> kf, globalT, complete;
    std::vector<char> kfSolved, localKnown;
    std::vector<int> globalValid;
    std::vector<std::vector<m4>> localTraj;
    std::vector<f3> gRot, gTrans, lRot, lTrans;  // the solver state (device arrays in the product)
    std::vector<m4> gMat;                        // dGlobalT_: matrices of the valid keyframes
    void* tm = nullptr;
    uint32_t numFrames = 0, lastSubmapEnqueued = 0xFFFFFFFFu;
    uint32_t optimizedFrames = 0;  // m_totalNumOptLocalFrames (OnlineBundler.cpp:268)
    std::vector<BFFixOp> log;
    std::vector<Rec> history;
    ORReconStats st{};

    void logOp(int kind, uint32_t frame, const m4* T) {
        BFFixOp e{};
        e.kind = kind;
        e.frame = frame;
        if (T) std::memcpy(kind == 1 ? e.oldT : e.newT, T->e, 64);
        log.push_back(e);
    }

    ORSolveParams solveParams(uint32_t n, uint32_t ncorr, uint32_t nNonLin, uint32_t nLin, uint32_t capPerImage,
                              const float* ws, const float* wd, const float* wc, const BFCachedFrame* cf) const {
        ORSolveParams sp{};
        sp.numImages = n;
        sp.numCorr = ncorr;
        sp.nNonLin = nNonLin;
        sp.nLin = nLin;
        sp.maxCorrPerImage = capPerImage;
        sp.weightsSparse = ws;
        sp.weightsDenseDepth = wd;
        sp.weightsDenseColor = wc;
        sp.cache = cf;
        sp.cacheW = P.cacheWidth;
        sp.cacheH = P.cacheHeight;
        std::memcpy(sp.intrinsics, P.cacheIntrinsics, 16);
        sp.denseDistThresh = 0.15f;
        sp.denseNormalThresh = 0.97f;
        sp.denseColorThresh = 0.1f;
        sp.denseColorGradientMin = 0.005f;
        sp.denseDepthMin = 0.5f;
        sp.denseDepthMax = 4.0f;
        sp.denseOverlapSubsample = 4;
        sp.disableEarlyOut = P.disableEarlyOut;
        return sp;
    }

    // global solve over nk keyframes and the first ncorr correspondences + removeMaxResidualCUDA
    // (SBA.cpp:164-203 with getMaxResidual's (0, <10) exemption, CUDASolverBundling.cpp:429-452) and
    // CheckForInvalidFramesSimpleCU (SIFTImageManager.cu:725-745) over the solve's table counts
    void globalSolve(uint32_t nk, uint32_t ncorr, float wDense) {
        std::vector<int> numEntries(nk, 0);
        for (uint32_t c = 0; c < ncorr; c++) {
            const BFEntryJ& e = globalCorr[c];
            if (e.imgIdx_i == BF_INVALID_IMAGE) continue;
            numEntries[e.imgIdx_i]++;
            numEntries[e.imgIdx_j]++;
        }
        std::vector<float> ws(P.globalNonLin, 1.0f), wd(P.globalNonLin, wDense), wc(P.globalNonLin, 0.0f);
        std::vector<BFCachedFrame> kc;
        if (wDense > 0.0f)
            for (uint32_t k = 0; k < nk; k++) kc.push_back(cache[k * S]);  // Bundler::fuseToGlobal's keyframe
        const ORSolveParams sp = solveParams(nk, ncorr, P.globalNonLin, P.globalLin, P.maxCorrPerImageGlobal, ws.data(),
                                             wd.data(), wc.data(), wDense > 0.0f ? kc.data() : nullptr);
        std::vector<float> rot(3 * nk), trans(3 * nk);
        for (uint32_t k = 0; k < nk; k++) {
            rot[3 * k] = gRot[k].x; rot[3 * k + 1] = gRot[k].y; rot[3 * k + 2] = gRot[k].z;
            trans[3 * k] = gTrans[k].x; trans[3 * k + 1] = gTrans[k].y; trans[3 * k + 2] = gTrans[k].z;
        }
        ORSolveResult r{};
        or_ba_solve(globalCorr.data(), globalValid.data(), &sp, rot.data(), trans.data(), &r);
        for (uint32_t k = 0; k < nk; k++) {
            gRot[k] = {rot[3 * k], rot[3 * k + 1], rot[3 * k + 2]};
            gTrans[k] = {trans[3 * k], trans[3 * k + 1], trans[3 * k + 2]};
        }
        st.globalSolves++;
        st.globalPcgIterations += r.pcgIterations;
        if (r.maxResidual > P.maxResidualThresh) {
            const BFEntryJ e = globalCorr[r.maxResidualIndex];
            if (e.imgIdx_i != BF_INVALID_IMAGE && !(e.imgIdx_i == 0 && e.imgIdx_j < 10)) {
                for (uint32_t c = 0; c < ncorr; c++)  // InvalidateImageToImageCU (SIFTImageManager.cu:692-719)
                    if (globalCorr[c].imgIdx_i == e.imgIdx_i && globalCorr[c].imgIdx_j == e.imgIdx_j)
                        globalCorr[c].imgIdx_i = globalCorr[c].imgIdx_j = BF_INVALID_IMAGE;
                for (uint32_t k = 0; k < nk; k++)
                    if (numEntries[k] == 0) globalValid[k] = 0;
                st.removedPairs++;
            }
        }
    }
    void globalToMatrices(uint32_t nk) {  // convertPosesToMatricesCU for valid images (SBA.cu:100-119)
        for (uint32_t k = 0; k < nk; k++)
            if (globalValid[k]) gMat[k] = poseToMatrix(gRot[k], gTrans[k]);
    }

    void endSubmap(uint32_t s, uint32_t n) {
        const uint32_t base = s * S;
        std::vector<m4> init(n);
        bool haveCache = P.useLocalDense != 0;
        for (uint32_t i = 0; i < n; i++) {
            init[i] = (i < S) ? Tlocal[base + i] : matmul(Tlocal[base + S - 1], Tinc[base + i]);
            if (!cache[base + i].depth) haveCache = false;
        }
        const uint32_t nk = s + 1;
        // ---- optimizeLocal (OnlineBundler.cpp:242-271) --------------------------------------------
        const bool verify = P.disableLocalVerify == 0;
        std::vector<m4> traj = init;
        int ok = 1;
        const std::vector<BFEntryJ>& lc0 = localCorr[s];
        if (n >= 2 && !lc0.empty()) {
            std::vector<BFEntryJ> lc = lc0;
            for (uint32_t i = 0; i < n; i++) matrixToPose(init[i], lRot[i], lTrans[i]);
            std::vector<float> rot(3 * n), trans(3 * n);
            for (uint32_t i = 0; i < n; i++) {
                rot[3 * i] = lRot[i].x; rot[3 * i + 1] = lRot[i].y; rot[3 * i + 2] = lRot[i].z;
                trans[3 * i] = lTrans[i].x; trans[3 * i + 1] = lTrans[i].y; trans[3 * i + 2] = lTrans[i].z;
            }
            std::vector<float> ws(P.localNonLin, 1.0f), wd(P.localNonLin), wc(P.localNonLin, 0.0f);
            for (uint32_t i = 0; i < P.localNonLin; i++) wd[i] = haveCache ? (float)(i + 1) : 0.0f;  // SBA.cpp:28-31
            const ORSolveParams sp = solveParams(n, (uint32_t)lc.size(), P.localNonLin, P.localLin, P.maxCorrPerImageLocal,
                                                 ws.data(), wd.data(), wc.data(), haveCache ? &cache[base] : nullptr);
            std::vector<int> lv(n, 1);
            ORSolveResult r{};
            or_ba_solve(lc.data(), lv.data(), &sp, rot.data(), trans.data(), &r);
            st.localSolves++;
            st.localPcgIterations += r.pcgIterations;
            for (uint32_t i = 0; i < n; i++) {
                lRot[i] = {rot[3 * i], rot[3 * i + 1], rot[3 * i + 2]};
                lTrans[i] = {trans[3 * i], trans[3 * i + 1], trans[3 * i + 2]};
                traj[i] = poseToMatrix(lRot[i], lTrans[i]);
            }
            if (verify && haveCache) {
                // useVerification with the local sparse weight (the reference passes an uninitialised
                // SolverParameters::weightSparse, CUDASolverBundling.cpp:456-472)
                const uint32_t high = or_ba_count_high_residuals(lc.data(), (uint32_t)lc.size(), rot.data(), trans.data(),
                                                                 ws.back(), P.verifyOptDistThresh);
                if ((float)high / (float)lc.size() >= P.verifyOptPercentThresh) {
                    st.localVerifications++;
                    std::vector<float> Tm(16 * (size_t)n);
                    for (uint32_t i = 0; i < n; i++) std::memcpy(&Tm[16 * i], traj[i].e, 64);
                    ORVerifyParams vp{};
                    vp.numImages = n;
                    vp.width = P.cacheWidth;
                    vp.height = P.cacheHeight;
                    std::memcpy(vp.intrinsics, P.cacheIntrinsics, 16);
                    vp.distThresh = P.projCorrDistThresh;
                    vp.normalThresh = P.projCorrNormalThresh;
                    vp.errThresh = P.verifyOptErrThresh;
                    vp.corrThresh = P.verifyOptCorrThresh;
                    vp.depthMin = 0.1f;
                    vp.depthMax = 3.0f;
                    ok = or_verify_trajectory(lv.data(), Tm.data(), &cache[base], &vp, nullptr);
                }
            }
        }
        // ---- processGlobal / optimizeGlobal (OnlineBundler.cpp:280-408) ---------------------------
        const bool gated = verify && s > 0 && !ok;
        if (gated) {
            globalValid[s] = 0;
            for (BFEntryJ& e : globalCorr)
                if (e.imgIdx_i == s || e.imgIdx_j == s) e.imgIdx_i = e.imgIdx_j = BF_INVALID_IMAGE;
        }
        const uint32_t ncorr = (s < prefix.size()) ? prefix[s] : (uint32_t)globalCorr.size();
        if (nk >= 2 && !globalCorr.empty() && ncorr > 0 && !gated) globalSolve(nk, ncorr, 0.0f);
        globalToMatrices(nk);
        Rec rec;
        rec.global.assign(gMat.begin(), gMat.begin() + nk);
        rec.valid.assign(globalValid.begin(), globalValid.begin() + nk);
        // ---- initNextGlobalTransformCU / initializeNextTransformUnknown ---------------------------
        if (n == S + 1) {
            if (gated) {
                gRot[s + 1] = gRot[s];
                gTrans[s + 1] = gTrans[s];
            } else {
                const m4 G = poseToMatrix(gRot[s], gTrans[s]);
                const m4 Lm = poseToMatrix(lRot[S], lTrans[S]);
                matrixToPose(matmul(G, Lm), gRot[s + 1], gTrans[s + 1]);
            }
        }
        lastSubmapEnqueued = s;
        optimizedFrames = S * s + std::min(n, S);
        // ---- the loop picks the results up (Recon::apply) -----------------------------------------
        localTraj[s] = traj;
        localKnown[s] = 1;
        for (uint32_t k = 0; k < nk; k++) {
            if (!globalValid[k]) continue;
            globalT[k] = gMat[k];
            kf[k] = globalT[k];
            kfSolved[k] = 1;
        }
        if (n == S + 1 && globalValid[s] && ok) {
            kf[s + 1] = matmul(globalT[s], traj[S]);
            kfSolved[s + 1] = 1;
        }
        if (!ok) st.invalidLocals++;
        rec.local = traj;
        rec.localOk = ok;
        if (history.size() <= s) history.resize(s + 1);
        history[s] = rec;
        updateTrajectory(std::min(S * s + std::min(n, S), numFrames));
    }

    void updateTrajectory(uint32_t optimized) {  // updateTrajectoryCU (OnlineBundler.cu:73-110)
        for (uint32_t g = 0; g < optimized; g++) {
            const uint32_t k = g / S;
            complete[g] = (globalValid[k] && localKnown[k]) ? matmul(globalT[k], localTraj[k][g % S]) : ninf();
        }
        std::vector<float> flat(16 * (size_t)optimized);
        for (uint32_t g = 0; g < optimized; g++) std::memcpy(&flat[16 * g], complete[g].e, 64);
        or_traj_update_optimized(tm, flat.data(), optimized);
    }

    void runReintegrate() {  // reintegrate(), DepthSensing.cpp:854-902
        const uint32_t cap = P.maxFrameFixes;
        std::vector<int> kinds(cap);
        std::vector<unsigned> fr(cap);
        std::vector<float> oT(16 * (size_t)cap), nT(16 * (size_t)cap);
        const unsigned n = or_traj_next_fixes(tm, cap, kinds.data(), fr.data(), oT.data(), nT.data());
        for (unsigned i = 0; i < n; i++) {
            const m4 o = ld(&oT[16 * i]), w = ld(&nT[16 * i]);
            if (kinds[i] == 3) {
                logOp(1, fr[i], &o);
                logOp(2, fr[i], &w);
            } else if (kinds[i] == 1) {
                logOp(1, fr[i], &o);
            } else if (kinds[i] == 2) {
                logOp(2, fr[i], &w);
            }
        }
        logOp(4, 0, nullptr);
    }

    void processFrame(uint32_t f) {
        const uint32_t s = f / S;
        if (f % S == 0 && f > 0) {
            endSubmap(s - 1, S + 1);
            if (!kfSolved[s]) kf[s] = matmul(kf[s - 1], matmul(Tlocal[f - 1], Tinc[f]));
        }
        runReintegrate();
        Tlocal[f] = (f % S == 0) ? identity() : matmul(Tlocal[f - 1], Tinc[f]);
        const m4 T = matmul(kf[s], Tlocal[f]);
        logOp(2, f, &T);
        or_traj_add_frame(tm, 0, T.e, f);
        numFrames++;
    }
};

}  // namespace

extern "C" {

ORRecon* or_recon_create(const ORReconParams* p, const float T0[16]) {
    Recon* r = new Recon();
    r->P = *p;
    r->S = p->submapSize ? p->submapSize : 10u;
    r->L = r->S + 1;
    r->maxSubmaps = (p->maxFrames + r->S - 1) / r->S;
    r->K = std::max(p->maxKeyframes ? p->maxKeyframes : r->maxSubmaps + 1, 2u);
    const uint32_t F = p->maxFrames;
    r->Tinc.assign(F, identity());
    r->Tlocal.assign(F, identity());
    r->cache.assign(F, BFCachedFrame{});
    r->localCorr.assign(r->maxSubmaps + 1, {});
    r->kf.assign(r->K, identity());
    r->kfSolved.assign(r->K, 0);
    r->globalT.assign(r->K, identity());
    r->globalValid.assign(r->K, 1);
    r->gMat.assign(r->K, identity());
    r->gRot.assign(r->K, f3{0, 0, 0});
    r->gTrans.assign(r->K, f3{0, 0, 0});
    r->lRot.assign(r->L, f3{0, 0, 0});
    r->lTrans.assign(r->L, f3{0, 0, 0});
    r->localTraj.assign(r->maxSubmaps + 1, {});
    r->localKnown.assign(r->maxSubmaps + 1, 0);
    r->complete.assign(F, identity());
    r->tm = or_traj_create(F, p->topNActive ? p->topNActive : 30u, p->minPoseDistSqrt);
    // setInitialPose
    const m4 T = ld(T0);
    r->kf[0] = T;
    r->kfSolved[0] = 1;
    r->globalT[0] = T;
    matrixToPose(T, r->gRot[0], r->gTrans[0]);
    return reinterpret_cast<ORRecon*>(r);
}

void or_recon_destroy(ORRecon* h) {
    Recon* r = reinterpret_cast<Recon*>(h);
    if (!r) return;
    or_traj_destroy(r->tm);
    delete r;
}

void or_recon_set_frame(ORRecon* h, uint32_t f, const float Tinc[16], const BFCachedFrame* cache) {
    Recon* r = reinterpret_cast<Recon*>(h);
    r->Tinc[f] = ld(Tinc);
    r->cache[f] = cache ? *cache : BFCachedFrame{};
}

void or_recon_set_local_corr(ORRecon* h, uint32_t s, const BFEntryJ* corr, uint32_t n) {
    Recon* r = reinterpret_cast<Recon*>(h);
    r->localCorr[s].assign(corr, corr + n);
}

void or_recon_set_global_corr(ORRecon* h, const BFEntryJ* corr, uint32_t n, const uint32_t* prefix, uint32_t numKeyframes) {
    Recon* r = reinterpret_cast<Recon*>(h);
    r->globalCorr.assign(corr, corr + n);
    r->prefix.assign(prefix, prefix + numKeyframes);
}

// the app's incremental form: keyframe k's correspondences appended (earlier entries keep the in-place
// invalidations of the solves so far), prefix[k] = the new length
void or_recon_append_global_corr(ORRecon* h, const BFEntryJ* corr, uint32_t n) {
    Recon* r = reinterpret_cast<Recon*>(h);
    r->globalCorr.insert(r->globalCorr.end(), corr, corr + n);
    r->prefix.push_back((uint32_t)r->globalCorr.size());
}

void or_recon_process_frame(ORRecon* h, uint32_t f) { reinterpret_cast<Recon*>(h)->processFrame(f); }

void or_recon_finish(ORRecon* h) {
    Recon* r = reinterpret_cast<Recon*>(h);
    if (r->numFrames == 0) return;
    const uint32_t s = (r->numFrames - 1) / r->S, n = r->numFrames - s * r->S;
    // a one-frame last submap is the previous submap's overlap frame (isLastLocalFrame, OnlineBundler.h:42)
    if (s != r->lastSubmapEnqueued && n >= 2) r->endSubmap(s, n);
}

void or_recon_reintegrate(ORRecon* h) { reinterpret_cast<Recon*>(h)->runReintegrate(); }

// one past-the-end global solve over the keyframes of the solved submaps (fuseToGlobal adds one per
// submap, OnlineBundler.cpp:298); returns 1 if it ran
static int end_solve(Recon* r, float denseDepthWeight) {
    if (r->numFrames == 0 || r->lastSubmapEnqueued == 0xFFFFFFFFu) return 0;
    const uint32_t last = r->lastSubmapEnqueued, nk = last + 1;
    const uint32_t ncorr = (last < r->prefix.size()) ? r->prefix[last] : (uint32_t)r->globalCorr.size();
    if (nk < 2 || r->globalCorr.empty() || ncorr == 0) return 0;
    r->globalSolve(nk, ncorr, denseDepthWeight);
    r->globalToMatrices(nk);
    for (uint32_t k = 0; k < nk; k++) {
        if (!r->globalValid[k]) continue;
        r->globalT[k] = r->gMat[k];
        r->kf[k] = r->globalT[k];
        r->kfSolved[k] = 1;
    }
    r->updateTrajectory(std::min(r->optimizedFrames, r->numFrames));
    r->st.endSolves++;
    return 1;
}

void or_recon_end_solve(ORRecon* h, float denseDepthWeight) { end_solve(reinterpret_cast<Recon*>(h), denseDepthWeight); }

// The render loop past the last frame, the product's Recon::endSequence (bf_recon_end_sequence):
// OnlineBundler::processInput's past-the-end branch (OnlineBundler.cpp:167-196), optimizeGlobal with
// isSequenceDone (:373-408), the exit check of OnD3D11FrameRender (DepthSensing.cpp:1114-1126).
// out[5] = {pastEndFrames, globalSolves, localSolved, denseSolve, queueDrained}.
void or_recon_end_sequence(ORRecon* h, int32_t N, int32_t disableDense, uint32_t denseLimit, float wDense, uint32_t cap,
                           uint32_t* out) {
    Recon* r = reinterpret_cast<Recon*>(h);
    for (int i = 0; i < 5; i++) out[i] = 0;
    if (r->numFrames == 0) return;
    const uint32_t S = r->S, last = (r->numFrames - 1) / S, n = r->numFrames - last * S;
    if (!cap) cap = 100000u;
    if (!denseLimit) denseLimit = 10000u;
    if (!(wDense > 0.0f)) wDense = 15.0f;
    for (uint32_t p = 0; p < cap; p++) {
        out[0] = p + 1;
        if (N < 0 || (int64_t)p <= (int64_t)N) {
            if (p == 0 && last != r->lastSubmapEnqueued && n >= 2) {
                const uint64_t before = r->st.globalSolves;
                r->endSubmap(last, n);
                out[1] += (uint32_t)(r->st.globalSolves - before);
                out[2] = 1;
            } else {
                bool caches = r->lastSubmapEnqueued != 0xFFFFFFFFu;
                for (uint32_t k = 0; caches && k <= r->lastSubmapEnqueued; k++)
                    if (!r->cache[k * S].depth) caches = false;
                const bool dense = N >= 0 && (int64_t)p == (int64_t)N && !disableDense && r->numFrames - 1 < denseLimit && caches;
                out[1] += (uint32_t)end_solve(r, dense ? wDense : 0.0f);
                if (dense) out[3] = 1;
            }
        }
        r->runReintegrate();
        if (N >= 0 && (int64_t)p >= (int64_t)N) {  // N < 0 (the reference's -1) never exits: maxPastEndFrames bounds it
            if (or_traj_generate_and_count(r->tm) == 0) {
                out[4] = 1;
                break;
            }
        }
    }
}

uint32_t or_recon_op_log(const ORRecon* h, BFFixOp* out, uint32_t cap) {
    const Recon* r = reinterpret_cast<const Recon*>(h);
    for (uint32_t i = 0; i < cap && i < r->log.size(); i++) out[i] = r->log[i];
    return (uint32_t)r->log.size();
}

int or_recon_submap_poses(const ORRecon* h, uint32_t s, float* local, float* global, int32_t* valid, uint32_t* numLocal,
                          uint32_t* numKeyframes, int32_t* localValid) {
    const Recon* r = reinterpret_cast<const Recon*>(h);
    if (s >= r->history.size() || r->history[s].local.empty()) return -1;
    const Rec& rec = r->history[s];
    for (size_t i = 0; i < rec.local.size(); i++) std::memcpy(local + 16 * i, rec.local[i].e, 64);
    for (size_t i = 0; i < rec.global.size(); i++) std::memcpy(global + 16 * i, rec.global[i].e, 64);
    for (size_t i = 0; i < rec.valid.size(); i++) valid[i] = rec.valid[i];
    *numLocal = (uint32_t)rec.local.size();
    *numKeyframes = (uint32_t)rec.global.size();
    *localValid = rec.localOk;
    return 0;
}

// integrated camera -> world transform per frame (-inf when not integrated), Recon::trajectory
void or_recon_trajectory(const ORRecon* h, float* T, uint32_t n) {
    const Recon* r = reinterpret_cast<const Recon*>(h);
    for (uint32_t i = 0; i < n; i++) {
        int type = 0;
        float d = 0;
        or_traj_frame_info(r->tm, i, &type, &d);
        const bool integrated = i < r->numFrames && (type == 0 || type == 4);
        if (!integrated) {
            for (int k = 0; k < 16; k++) T[16 * i + k] = NEG_INF;
            continue;
        }
        or_traj_integrated(r->tm, i, T + 16 * i);
    }
}

void or_recon_stats(const ORRecon* h, ORReconStats* out) { *out = reinterpret_cast<const Recon*>(h)->st; }

}  // extern "C"
