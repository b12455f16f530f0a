// trajectory.cpp — see trajectory.h. Host code (the reference's TrajectoryManager is host C++).
#include "trajectory.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace bf {

namespace {

const float NEG_INF = -std::numeric_limits<float>::infinity();

struct V3 {
    float x, y, z;
};
inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float length(V3 a) { return std::sqrt(dot(a, a)); }

struct M3 {
    float m[9];
    float operator()(int r, int c) const { return m[r * 3 + c]; }
    float& operator()(int r, int c) { return m[r * 3 + c]; }
};
inline V3 mul(const M3& R, V3 v) {
    return {R(0, 0) * v.x + R(0, 1) * v.y + R(0, 2) * v.z, R(1, 0) * v.x + R(1, 1) * v.y + R(1, 2) * v.z,
            R(2, 0) * v.x + R(2, 1) * v.y + R(2, 2) * v.z};
}

// PoseHelper::rodrigues_so3_exp (Source/PoseHelper.h:213-243)
M3 rodrigues_so3_exp(V3 w, float A, float B) {
    M3 R;
    const float wx2 = w.x * w.x, wy2 = w.y * w.y, wz2 = w.z * w.z;
    R(0, 0) = 1.0f - B * (wy2 + wz2);
    R(1, 1) = 1.0f - B * (wx2 + wz2);
    R(2, 2) = 1.0f - B * (wx2 + wy2);
    {
        const float a = A * w.z, b = B * (w.x * w.y);
        R(0, 1) = b - a;
        R(1, 0) = b + a;
    }
    {
        const float a = A * w.y, b = B * (w.x * w.z);
        R(0, 2) = b + a;
        R(2, 0) = b - a;
    }
    {
        const float a = A * w.x, b = B * (w.y * w.z);
        R(1, 2) = b - a;
        R(2, 1) = b + a;
    }
    return R;
}

// PoseHelper::exp_rotation (:245-271)
M3 exp_rotation(V3 w) {
    const float one_6th = 1.0f / 6.0f, one_20th = 1.0f / 20.0f;
    const float theta_sq = dot(w, w);
    const float theta = std::sqrt(theta_sq);
    float A, B;
    if (theta_sq < 1e-8f) {
        A = 1.0f - one_6th * theta_sq;
        B = 0.5f;
    } else if (theta_sq < 1e-6f) {
        B = 0.5f - 0.25f * one_6th * theta_sq;
        A = 1.0f - theta_sq * one_6th * (1.0f - one_20th * theta_sq);
    } else {
        const float inv_theta = 1.0f / theta;
        A = std::sin(theta) * inv_theta;
        B = (1 - std::cos(theta)) * (inv_theta * inv_theta);
    }
    return rodrigues_so3_exp(w, A, B);
}

// PoseHelper::ln_rotation (:272-330)
V3 ln_rotation(const M3& R) {
    const float cos_angle = (R(0, 0) + R(1, 1) + R(2, 2) - 1.0f) * 0.5f;
    V3 result{(R(2, 1) - R(1, 2)) * 0.5f, (R(0, 2) - R(2, 0)) * 0.5f, (R(1, 0) - R(0, 1)) * 0.5f};
    const float sin_angle_abs = length(result);
    if (cos_angle > 0.70710678118654752440f) {
        if (sin_angle_abs > 0) result = result * (std::asin(sin_angle_abs) / sin_angle_abs);
    } else if (cos_angle > -0.70710678118654752440f) {
        const float angle = std::acos(cos_angle);
        result = result * (angle / sin_angle_abs);
    } else {
        const float angle = 3.14159265358979323846f - std::asin(sin_angle_abs);
        const float d0 = R(0, 0) - cos_angle, d1 = R(1, 1) - cos_angle, d2 = R(2, 2) - cos_angle;
        V3 r2;
        if (std::fabs(d0) > std::fabs(d1) && std::fabs(d0) > std::fabs(d2)) {
            r2 = {d0, (R(1, 0) + R(0, 1)) * 0.5f, (R(0, 2) + R(2, 0)) * 0.5f};
        } else if (std::fabs(d1) > std::fabs(d2)) {
            r2 = {(R(1, 0) + R(0, 1)) * 0.5f, d1, (R(2, 1) + R(1, 2)) * 0.5f};
        } else {
            r2 = {(R(0, 2) + R(2, 0)) * 0.5f, (R(2, 1) + R(1, 2)) * 0.5f, d2};
        }
        if (dot(r2, result) < 0) r2 = r2 * -1.0f;
        result = r2;
        result = result * (angle / length(r2));
    }
    return result;
}

}  // namespace

void pose_helper_matrix_to_pose(const BFMat4& T, float out[6]) {
    M3 R;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R(r, c) = T.m[r * 4 + c];
    const V3 t{T.m[3], T.m[7], T.m[11]};
    const V3 rot = ln_rotation(R);
    const float theta = length(rot);
    float shtot = 0.5f;
    if (theta > 0.00001f) shtot = std::sin(theta * 0.5f) / theta;
    const V3 rot_half = rot * -0.5f;
    const M3 halfrotator = exp_rotation(rot_half);
    V3 rottrans = mul(halfrotator, t);
    if (theta > 0.001f)
        rottrans = rottrans - rot * (dot(t, rot) * (1 - 2 * shtot) / dot(rot, rot));
    else
        rottrans = rottrans - rot * (dot(t, rot) / 24);
    rottrans = rottrans * (1.0f / (2 * shtot));
    out[0] = rottrans.x; out[1] = rottrans.y; out[2] = rottrans.z;
    out[3] = rot.x; out[4] = rot.y; out[5] = rot.z;
}

TrajectoryManager::TrajectoryManager(uint32_t maxFrames, uint32_t topNActive, float minPoseDistSqrt)
    : topN_(topNActive), minDist_(minPoseDistSqrt) {
    BFMat4 ninf;
    for (float& v : ninf.m) v = NEG_INF;
    optimized_.assign(maxFrames, ninf);
    frames_.assign(maxFrames, Frame{FrameType::NotIntegrated_NoTransform, 0xFFFFFFFFu, ninf, 0.0f});
    sortOrder_.reserve(maxFrames);
}

void TrajectoryManager::addFrame(FrameType what, const BFMat4& T, uint32_t idx) {
    Frame& f = frames_.at(idx);
    f.type = what;
    f.frameIdx = idx;
    f.integrated = T;
    optimized_[idx] = T;
    sortOrder_.push_back(idx);
    numAdded_++;
}

void TrajectoryManager::updateOptimizedTransforms(const BFMat4* T, uint32_t numFrames) {
    numOptimized_ = numFrames;
    numFrames = std::min(numFrames, numAdded_);
    for (uint32_t i = 0; i < numFrames; i++) optimized_[i] = T[i];
}

void TrajectoryManager::invalidateFrame(uint32_t i) {
    if (frames_[i].type == FrameType::Invalid) return;
    const FrameType before = frames_[i].type;
    frames_[i].type = FrameType::Invalid;
    if (before == FrameType::Integrated) deint_.push_back(i);
}

void TrajectoryManager::generateUpdateLists() {
    const uint32_t numFrames = std::min(numOptimized_, numAdded_);
    for (uint32_t i = 0; i < numFrames; i++) {
        Frame& f = frames_[i];
        if (optimized_[i].m[0] == NEG_INF) {
            invalidateFrame(i);
            continue;
        }
        if (f.type == FrameType::NotIntegrated_NoTransform || f.type == FrameType::Invalid) {
            f.type = FrameType::NotIntegrated_WithTransform;
            integ_.push_back(i);
        }
        float po[6], pi[6];
        pose_helper_matrix_to_pose(optimized_[i], po);
        pose_helper_matrix_to_pose(f.integrated, pi);
        for (int k = 0; k < 3; k++) {
            po[k] *= rescale_;
            pi[k] *= rescale_;
        }
        float d = 0.0f;  // vec6f operator| (dot), summed in index order
        for (int k = 0; k < 6; k++) d += (pi[k] - po[k]) * (pi[k] - po[k]);
        f.dist = d;
    }
    auto less = [this](uint32_t a, uint32_t b) {
        const Frame& l = frames_[a];
        const Frame& r = frames_[b];
        if (l.type == FrameType::Integrated && r.type != FrameType::Integrated) return true;
        if (l.type != FrameType::Integrated) return false;
        if (r.type != FrameType::Integrated) return false;
        return l.dist > r.dist;
    };
    std::stable_sort(sortOrder_.begin(), sortOrder_.begin() + numFrames, less);
    for (uint32_t i = (uint32_t)reint_.size(); i < topN_ && i < numFrames; i++) {
        Frame& f = frames_[sortOrder_[i]];
        if (f.dist > minDist_ && f.type == FrameType::Integrated) {
            f.type = FrameType::ReIntegration;
            reint_.push_back(sortOrder_[i]);
        } else {
            break;
        }
    }
}

void TrajectoryManager::confirmIntegration(uint32_t frameIdx) { frames_[frameIdx].type = FrameType::Integrated; }

bool TrajectoryManager::topReIntegrate(BFMat4& oldT, BFMat4& newT, uint32_t& frame) {
    if (reint_.empty()) return false;
    while (!reint_.empty()) {  // some may have been invalidated since (TrajectoryManager.cpp:122-134)
        const uint32_t i = reint_.front();
        newT = optimized_[i];
        frame = i;
        oldT = frames_[i].integrated;
        reint_.pop_front();
        if (newT.m[0] != NEG_INF) {
            frames_[i].integrated = newT;
            break;
        }
    }
    return true;
}

bool TrajectoryManager::topIntegrate(BFMat4& T, uint32_t& frame) {
    if (integ_.empty()) return false;
    const uint32_t i = integ_.front();
    T = optimized_[i];
    frame = i;
    frames_[i].integrated = T;
    integ_.pop_front();
    return true;
}

bool TrajectoryManager::topDeIntegrate(BFMat4& T, uint32_t& frame) {
    if (deint_.empty()) return false;
    const uint32_t i = deint_.front();
    T = frames_[i].integrated;
    frame = i;
    deint_.pop_front();
    return true;
}

uint32_t TrajectoryManager::numActiveOperations() const {
    return (uint32_t)(deint_.size() + integ_.size() + reint_.size());
}

uint32_t TrajectoryManager::nextFixes(uint32_t maxFixes, std::vector<FixOp>& ops) {
    ops.clear();
    if (numActiveOperations() < maxFixes) generateUpdateLists();
    for (uint32_t fixes = 0; fixes < maxFixes; fixes++) {
        FixOp op{};
        if (topDeIntegrate(op.oldT, op.frame)) {
            op.kind = FixKind::DeIntegrate;
            ops.push_back(op);
            continue;
        }
        if (topIntegrate(op.newT, op.frame)) {
            op.kind = FixKind::Integrate;
            ops.push_back(op);
            confirmIntegration(op.frame);
            continue;
        }
        if (topReIntegrate(op.oldT, op.newT, op.frame)) {
            // an all-invalid pop still consumes the fix slot, as in the reference loop
            if (op.newT.m[0] != NEG_INF) {
                op.kind = FixKind::ReIntegrate;
                ops.push_back(op);
                confirmIntegration(op.frame);
            }
            continue;
        }
        break;
    }
    return (uint32_t)ops.size();
}

}  // namespace bf
