// trajectory.cpp — see trajectory.h. Host code (the reference's TrajectoryManager is host C++).
#include "trajectory.h"

#include "host_pool.h"

#include <algorithm>
#include <cmath>
#include <cstring>
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
    integratedPose_.assign(maxFrames, PoseCache{});
    optimizedPose_.assign(maxFrames, PoseCache{});
    sortOrder_.reserve(maxFrames);
}

void TrajectoryManager::setIntegrated(uint32_t i, const BFMat4& T) {
    if (std::memcmp(frames_[i].integrated.m, T.m, sizeof(T.m)) != 0 && integratedPose_[i].valid) {
        integratedPose_[i].valid = false;
        stalePoses_++;
    }
    frames_[i].integrated = T;
}

void TrajectoryManager::setOptimized(uint32_t i, const BFMat4& T) {
    if (std::memcmp(optimized_[i].m, T.m, sizeof(T.m)) != 0 && optimizedPose_[i].valid) {
        optimizedPose_[i].valid = false;
        stalePoses_++;
    }
    optimized_[i] = T;
}

void TrajectoryManager::addFrame(FrameType what, const BFMat4& T, uint32_t idx) {
    Frame& f = frames_.at(idx);
    f.type = what;
    f.frameIdx = idx;
    setIntegrated(idx, T);
    setOptimized(idx, T);
    sortOrder_.push_back(idx);
    numAdded_++;
}

void TrajectoryManager::updateOptimizedTransforms(const BFMat4* T, uint32_t numFrames) {
    numOptimized_ = numFrames;
    numFrames = std::min(numFrames, numAdded_);
    for (uint32_t i = 0; i < numFrames; i++) setOptimized(i, T[i]);
}

void TrajectoryManager::invalidateFrame(uint32_t i) {
    if (frames_[i].type == FrameType::Invalid) return;
    const FrameType before = frames_[i].type;
    frames_[i].type = FrameType::Invalid;
    if (before == FrameType::Integrated) deint_.push_back(i);
}

void TrajectoryManager::generateUpdateLists() {
    const uint32_t numFrames = std::min(numOptimized_, numAdded_);
    // the MatrixToPose conversions of the transforms that changed (after a solve: every frame's
    // optimized one) are independent per frame: on the host pool when there are many, before the
    // serial pass (new frames' caches start invalid and are converted here too)
    const size_t minPer = stalePoses_ >= 1024 ? 256 : ~(size_t)0;
    stalePoses_ = 0;
    HostPool::get().parallel_for(numFrames, [this](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
            if (optimized_[i].m[0] == NEG_INF) continue;
            PoseCache& co = optimizedPose_[i];
            PoseCache& ci = integratedPose_[i];
            if (!co.valid) {
                pose_helper_matrix_to_pose(optimized_[i], co.p);
                co.valid = true;
                ci.fresh = true;  // the distance must be recomputed below
            }
            if (!ci.valid) {
                pose_helper_matrix_to_pose(frames_[i].integrated, ci.p);
                ci.valid = true;
                ci.fresh = true;
            }
        }
    }, minPer);
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
        // the distance changes only with one of the two poses, i.e. when a cache was invalidated
        PoseCache& co = optimizedPose_[i];
        PoseCache& ci = integratedPose_[i];
        if (!ci.fresh) continue;
        ci.fresh = false;
        float po[6], pi[6];
        std::memcpy(po, co.p, sizeof(po));
        std::memcpy(pi, ci.p, sizeof(pi));
        for (int k = 0; k < 3; k++) {
            po[k] *= rescale_;
            pi[k] *= rescale_;
        }
        float d = 0.0f;  // vec6f operator| (dot), summed in index order
        for (int k = 0; k < 6; k++) d += (pi[k] - po[k]) * (pi[k] - po[k]);
        f.dist = d;
    }
    sortFrames(numFrames);
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

// m_framesSort's sort (TrajectoryManager.cpp:87-100): integrated frames first by decreasing distance,
// everything else after them; equal keys keep their order (see trajectory.h). The same permutation
// as std::stable_sort with that comparator, from a radix sort of unique 64-bit keys
// {not integrated, ~distance bits, position}: the distances are sums of squares, so for the
// integrated frames (the only ones whose distance is compared) the float order is the bit order
// unless one is NaN, which takes the comparator sort itself.
void TrajectoryManager::sortFrames(uint32_t numFrames) {
    auto less = [this](uint32_t a, uint32_t b) {
        const Frame& l = frames_[a];
        const Frame& r = frames_[b];
        if (l.type == FrameType::Integrated && r.type != FrameType::Integrated) return true;
        if (l.type != FrameType::Integrated) return false;
        if (r.type != FrameType::Integrated) return false;
        return l.dist > r.dist;
    };
    if (numFrames == 0) return;
    bool keyed = numFrames < (1u << 20);
    sortKeys_.resize(numFrames);
    for (uint32_t p = 0; p < numFrames && keyed; p++) {
        const Frame& f = frames_[sortOrder_[p]];
        uint64_t k = 1ull << 52;
        if (f.type == FrameType::Integrated) {
            uint32_t bits;
            std::memcpy(&bits, &f.dist, 4);
            if (f.dist != f.dist || (bits >> 31)) keyed = false;  // NaN / negative: not a plain bit order
            k = (uint64_t)(~bits) << 20;
        }
        sortKeys_[p] = k | p;
    }
    if (!keyed) {
        std::stable_sort(sortOrder_.begin(), sortOrder_.begin() + numFrames, less);
        return;
    }
    // LSD radix sort on the 33 bits above the position, 11 bits per pass: each pass is stable and the
    // keys enter in position order, so equal {class, distance} keep it
    sortKeys2_.resize(numFrames);
    uint64_t* a = sortKeys_.data();
    uint64_t* b = sortKeys2_.data();
    for (int shift = 20; shift < 53; shift += 11) {
        uint32_t count[2048 + 1] = {0};
        for (uint32_t p = 0; p < numFrames; p++) count[((a[p] >> shift) & 2047u) + 1]++;
        if (count[((a[0] >> shift) & 2047u) + 1] == numFrames) continue;  // one digit value: the order stands
        for (int d = 0; d < 2048; d++) count[d + 1] += count[d];
        for (uint32_t p = 0; p < numFrames; p++) b[count[(a[p] >> shift) & 2047u]++] = a[p];
        std::swap(a, b);
    }
    sortTmp_.assign(sortOrder_.begin(), sortOrder_.begin() + numFrames);
    for (uint32_t p = 0; p < numFrames; p++) sortOrder_[p] = sortTmp_[a[p] & 0xFFFFFu];
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
            setIntegrated(i, newT);
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
    setIntegrated(i, T);
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
