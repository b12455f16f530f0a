// trajectory.h — re-integration queue (replaces TrajectoryManager, Source/TrajectoryManager.h:6-118,
// Source/TrajectoryManager.cpp:8-200) and the per-frame fix loop of reintegrate()
// (Source/DepthSensing/DepthSensing.cpp:854-902).
//
// Host-side state, as in the reference: a frame table with integrated / optimized camera-to-world
// transforms, three FIFO lists (de-integrate, integrate, re-integrate) and a sort by pose distance.
// The only change of behaviour is a deterministic tie-break: the reference's std::sort leaves the
// order of equal keys unspecified; here equal keys keep ascending frame index (stable sort over
// the frame-added order), so every shard of a multi-GPU run derives the identical op list.
#pragma once
#include <cstddef>
#include <cstdint>
#include <deque>
#include <vector>

#include "../../include/bf/types.h"

namespace bf {

enum class FrameType : int32_t {
    Integrated = 0,
    NotIntegrated_NoTransform = 1,
    NotIntegrated_WithTransform = 2,
    Invalid = 3,
    ReIntegration = 4,
};

enum class FixKind : int32_t { None = 0, DeIntegrate = 1, Integrate = 2, ReIntegrate = 3 };

struct FixOp {
    FixKind kind;
    uint32_t frame;
    BFMat4 oldT;  // de-integrate / re-integrate: the transform the frame was integrated with
    BFMat4 newT;  // integrate / re-integrate: the optimized transform
};

// PoseHelper::MatrixToPose in USE_LIE_SPACE mode (Source/PoseHelper.h:332-362): [u (3) | omega (3)]
void pose_helper_matrix_to_pose(const BFMat4& T, float out[6]);

class TrajectoryManager {
public:
    // s_topNActive (30), s_minPoseDistSqrt (0.0), featureRescaleRotToTrans 2 (TrajectoryManager.cpp:20-22)
    TrajectoryManager(uint32_t maxFrames, uint32_t topNActive = 30, float minPoseDistSqrt = 0.0f);

    void addFrame(FrameType what, const BFMat4& T, uint32_t idx);
    // updateOptimizedTransform (:32-42): host copy of the optimized trajectory [numFrames]
    void updateOptimizedTransforms(const BFMat4* T, uint32_t numFrames);
    void generateUpdateLists();                    // :44-109
    void confirmIntegration(uint32_t frameIdx);    // :111-115
    bool topReIntegrate(BFMat4& oldT, BFMat4& newT, uint32_t& frame);  // :117-138
    bool topIntegrate(BFMat4& T, uint32_t& frame);                     // :140-157
    bool topDeIntegrate(BFMat4& T, uint32_t& frame);                   // :159-170
    uint32_t numActiveOperations() const;
    uint32_t numAddedFrames() const { return numAdded_; }
    uint32_t numOptimizedFrames() const { return numOptimized_; }

    // reintegrate() (DepthSensing.cpp:854-902) minus the scene calls: regenerate the lists when
    // fewer than maxFixes ops are pending, then pop up to maxFixes ops in the reference's priority
    // (de-integrate, integrate, re-integrate). Integrate / re-integrate ops are confirmed here,
    // as the reference confirms them right after issuing the scene calls.
    uint32_t nextFixes(uint32_t maxFixes, std::vector<FixOp>& ops);

    FrameType type(uint32_t i) const { return frames_[i].type; }
    float dist(uint32_t i) const { return frames_[i].dist; }
    const BFMat4& integrated(uint32_t i) const { return frames_[i].integrated; }
    const BFMat4& optimized(uint32_t i) const { return optimized_[i]; }

private:
    struct Frame {
        FrameType type;
        uint32_t frameIdx;
        BFMat4 integrated;
        float dist;
    };
    void invalidateFrame(uint32_t i);
    void setIntegrated(uint32_t i, const BFMat4& T);
    void setOptimized(uint32_t i, const BFMat4& T);
    void sortFrames(uint32_t numFrames);

    std::vector<BFMat4> optimized_;
    std::vector<Frame> frames_;
    std::vector<uint32_t> sortOrder_;  // m_framesSort (frame indices in added order)
    uint32_t numAdded_ = 0, numOptimized_ = 0;
    std::deque<uint32_t> deint_, integ_, reint_;
    // generateUpdateLists' two MatrixToPose per frame, cached until the transform changes (the
    // loop calls it every few frames over every frame so far: at 5 000 frames it was most of the
    // host time per frame); the values are the same calls on the same matrices
    struct PoseCache {
        float p[6];
        bool valid = false;
        bool fresh = false;  // (integrated entry) a pose of the frame was converted since its distance was computed
    };
    std::vector<PoseCache> integratedPose_, optimizedPose_;
    size_t stalePoses_ = 0;  // caches invalidated since the last generateUpdateLists
    std::vector<uint64_t> sortKeys_, sortKeys2_;
    std::vector<uint32_t> sortTmp_;
    uint32_t topN_;
    float minDist_;
    float rescale_ = 2.0f;
};

}  // namespace bf
