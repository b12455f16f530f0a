// oracle/traj.cpp — TEST INFRASTRUCTURE (CPU oracle, see oracle.h header).
//
// Restatement of TrajectoryManager (Source/TrajectoryManager.cpp:8-200), of the list logic of
// reintegrate() (Source/DepthSensing/DepthSensing.cpp:854-902) and of PoseHelper::MatrixToPose
// in USE_LIE_SPACE mode (Source/PoseHelper.h:245-362), written as a literal transcription of the
// reference's pointer lists. Deviation kept identical to the product: std::sort's unspecified
// order of equal keys is replaced by a stable sort over the persistent m_framesSort order.
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <list>
#include <vector>

namespace {

const float kNegInf = -std::numeric_limits<float>::infinity();

// PoseHelper.h:213-243 / :245-271 / :272-330, on float[9] row-major
void so3_exp(const float w[3], float R[9]) {
    const float theta_sq = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    const float theta = std::sqrt(theta_sq);
    float A, B;
    if (theta_sq < 1e-8f) {
        A = 1.0f - (1.0f / 6.0f) * theta_sq;
        B = 0.5f;
    } else if (theta_sq < 1e-6f) {
        B = 0.5f - 0.25f * (1.0f / 6.0f) * theta_sq;
        A = 1.0f - theta_sq * (1.0f / 6.0f) * (1.0f - (1.0f / 20.0f) * theta_sq);
    } else {
        const float inv = 1.0f / theta;
        A = std::sin(theta) * inv;
        B = (1 - std::cos(theta)) * (inv * inv);
    }
    R[0] = 1.0f - B * (w[1] * w[1] + w[2] * w[2]);
    R[4] = 1.0f - B * (w[0] * w[0] + w[2] * w[2]);
    R[8] = 1.0f - B * (w[0] * w[0] + w[1] * w[1]);
    float a = A * w[2], b = B * (w[0] * w[1]);
    R[1] = b - a;
    R[3] = b + a;
    a = A * w[1];
    b = B * (w[0] * w[2]);
    R[2] = b + a;
    R[6] = b - a;
    a = A * w[0];
    b = B * (w[1] * w[2]);
    R[5] = b - a;
    R[7] = b + a;
}

void so3_ln(const float R[9], float out[3]) {
    const float c = (R[0] + R[4] + R[8] - 1.0f) * 0.5f;
    float r[3] = {(R[7] - R[5]) * 0.5f, (R[2] - R[6]) * 0.5f, (R[3] - R[1]) * 0.5f};
    const float s = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (c > 0.70710678118654752440f) {
        if (s > 0) {
            const float k = std::asin(s) / s;
            for (float& v : r) v *= k;
        }
    } else if (c > -0.70710678118654752440f) {
        const float k = std::acos(c) / s;
        for (float& v : r) v *= k;
    } else {
        const float angle = 3.14159265358979323846f - std::asin(s);
        const float d0 = R[0] - c, d1 = R[4] - c, d2 = R[8] - c;
        float r2[3];
        if (std::fabs(d0) > std::fabs(d1) && std::fabs(d0) > std::fabs(d2)) {
            r2[0] = d0; r2[1] = (R[3] + R[1]) * 0.5f; r2[2] = (R[2] + R[6]) * 0.5f;
        } else if (std::fabs(d1) > std::fabs(d2)) {
            r2[0] = (R[3] + R[1]) * 0.5f; r2[1] = d1; r2[2] = (R[7] + R[5]) * 0.5f;
        } else {
            r2[0] = (R[2] + R[6]) * 0.5f; r2[1] = (R[7] + R[5]) * 0.5f; r2[2] = d2;
        }
        if (r2[0] * r[0] + r2[1] * r[1] + r2[2] * r[2] < 0) for (float& v : r2) v *= -1.0f;
        const float len = std::sqrt(r2[0] * r2[0] + r2[1] * r2[1] + r2[2] * r2[2]);
        for (int i = 0; i < 3; i++) r[i] = r2[i] * (angle / len);
    }
    out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
}

struct TF {  // TrajectoryManager::TrajectoryFrame
    int type;
    unsigned frameIdx;
    float integrated[16];
    float* optimized;  // reference into the optimized array
    float dist;
};

struct TM {
    std::vector<float> opt;  // [maxFrames][16]
    std::vector<TF> frames;
    std::vector<TF*> sorted;
    unsigned numAdded = 0, numOptimized = 0;
    std::list<TF*> deint, integ, reint;
    unsigned topN;
    float minDist;
};

enum { Integrated = 0, NoTransform = 1, WithTransform = 2, Invalid = 3, ReIntegration = 4 };

}  // namespace

extern "C" {

void or_pose_helper_matrix_to_pose(const float* T, float out[6]) {
    const float R[9] = {T[0], T[1], T[2], T[4], T[5], T[6], T[8], T[9], T[10]};
    const float t[3] = {T[3], T[7], T[11]};
    float rot[3];
    so3_ln(R, rot);
    const float theta = std::sqrt(rot[0] * rot[0] + rot[1] * rot[1] + rot[2] * rot[2]);
    float shtot = 0.5f;
    if (theta > 0.00001f) shtot = std::sin(theta * 0.5f) / theta;
    const float half[3] = {rot[0] * -0.5f, rot[1] * -0.5f, rot[2] * -0.5f};
    float H[9];
    so3_exp(half, H);
    float rt[3] = {H[0] * t[0] + H[1] * t[1] + H[2] * t[2], H[3] * t[0] + H[4] * t[1] + H[5] * t[2],
                   H[6] * t[0] + H[7] * t[1] + H[8] * t[2]};
    const float tr = t[0] * rot[0] + t[1] * rot[1] + t[2] * rot[2];
    if (theta > 0.001f) {
        const float k = tr * (1 - 2 * shtot) / (rot[0] * rot[0] + rot[1] * rot[1] + rot[2] * rot[2]);
        for (int i = 0; i < 3; i++) rt[i] -= rot[i] * k;
    } else {
        const float k = tr / 24;
        for (int i = 0; i < 3; i++) rt[i] -= rot[i] * k;
    }
    for (int i = 0; i < 3; i++) rt[i] *= 1.0f / (2 * shtot);
    out[0] = rt[0]; out[1] = rt[1]; out[2] = rt[2];
    out[3] = rot[0]; out[4] = rot[1]; out[5] = rot[2];
}

void* or_traj_create(unsigned maxFrames, unsigned topN, float minDist) {
    TM* tm = new TM();
    tm->opt.assign((size_t)maxFrames * 16, kNegInf);
    tm->frames.resize(maxFrames);
    for (unsigned i = 0; i < maxFrames; i++) {
        TF& f = tm->frames[i];
        f.type = NoTransform;
        f.frameIdx = (unsigned)-1;
        for (float& v : f.integrated) v = kNegInf;
        f.optimized = &tm->opt[(size_t)i * 16];
        f.dist = 0.0f;
    }
    tm->topN = topN;
    tm->minDist = minDist;
    return tm;
}

void or_traj_destroy(void* h) { delete static_cast<TM*>(h); }

void or_traj_add_frame(void* h, int type, const float* T, unsigned idx) {  // addFrame (:24-32)
    TM* tm = static_cast<TM*>(h);
    TF& f = tm->frames[idx];
    f.type = type;
    f.frameIdx = idx;
    float m[16];
    for (int k = 0; k < 16; k++) m[k] = (type == NoTransform) ? kNegInf : T[k];
    std::memcpy(f.integrated, m, 64);
    std::memcpy(f.optimized, m, 64);
    tm->sorted.push_back(&f);
    tm->numAdded++;
}

void or_traj_update_optimized(void* h, const float* T, unsigned numFrames) {  // :34-43
    TM* tm = static_cast<TM*>(h);
    tm->numOptimized = numFrames;
    numFrames = std::min(numFrames, tm->numAdded);
    std::memcpy(tm->opt.data(), T, (size_t)numFrames * 64);
}

static void invalidate(TM* tm, unsigned i) {  // invalidateFrame (:190-200)
    TF& f = tm->frames[i];
    if (f.type == Invalid) return;
    const int before = f.type;
    f.type = Invalid;
    if (before == Integrated) tm->deint.push_back(&f);
}

static void generate(TM* tm) {  // generateUpdateLists (:45-109)
    const unsigned numFrames = std::min(tm->numOptimized, tm->numAdded);
    for (unsigned i = 0; i < numFrames; i++) {
        TF& f = tm->frames[i];
        if (f.optimized[0] == kNegInf) {
            invalidate(tm, i);
        } else {
            if (f.type == NoTransform || f.type == Invalid) {
                f.type = WithTransform;
                tm->integ.push_back(&f);
            }
            float po[6], pi[6];
            or_pose_helper_matrix_to_pose(f.optimized, po);
            or_pose_helper_matrix_to_pose(f.integrated, pi);
            for (int k = 0; k < 3; k++) {
                po[k] *= 2.0f;
                pi[k] *= 2.0f;
            }
            float d = 0.0f;
            for (int k = 0; k < 6; k++) d += (pi[k] - po[k]) * (pi[k] - po[k]);
            f.dist = d;
        }
    }
    std::stable_sort(tm->sorted.begin(), tm->sorted.begin() + numFrames, [](const TF* l, const TF* r) {
        if (l->type == Integrated && r->type != Integrated) return true;
        if (l->type != Integrated) return false;
        return l->type == Integrated && r->type == Integrated && l->dist > r->dist;
    });
    for (unsigned i = (unsigned)tm->reint.size(); i < tm->topN && i < numFrames; i++) {
        TF* f = tm->sorted[i];
        if (f->dist > tm->minDist && f->type == Integrated) {
            f->type = ReIntegration;
            tm->reint.push_back(f);
        } else {
            break;
        }
    }
}

// reintegrate() list logic (DepthSensing.cpp:854-902); writes up to maxFixes ops as
// {kind, frame, oldT[16], newT[16]} (34 floats/ints per op: int kind, uint frame, 32 floats)
unsigned or_traj_next_fixes(void* h, unsigned maxFixes, int* kinds, unsigned* framesOut, float* oldT, float* newT) {
    TM* tm = static_cast<TM*>(h);
    if (tm->deint.size() + tm->integ.size() + tm->reint.size() < maxFixes) generate(tm);
    unsigned n = 0;
    for (unsigned fixes = 0; fixes < maxFixes; fixes++) {
        if (!tm->deint.empty()) {  // getTopFromDeIntegrateList (:159-170)
            TF* f = tm->deint.front();
            tm->deint.pop_front();
            kinds[n] = 1;
            framesOut[n] = f->frameIdx;
            std::memcpy(oldT + 16 * n, f->integrated, 64);
            n++;
            continue;
        }
        if (!tm->integ.empty()) {  // getTopFromIntegrateList (:140-157) + confirmIntegration
            TF* f = tm->integ.front();
            tm->integ.pop_front();
            std::memcpy(f->integrated, f->optimized, 64);
            kinds[n] = 2;
            framesOut[n] = f->frameIdx;
            std::memcpy(newT + 16 * n, f->optimized, 64);
            f->type = Integrated;
            n++;
            continue;
        }
        if (!tm->reint.empty()) {  // getTopFromReIntegrateList (:117-138)
            TF* f = nullptr;
            float o[16], nw[16];
            while (!tm->reint.empty()) {
                f = tm->reint.front();
                std::memcpy(nw, f->optimized, 64);
                std::memcpy(o, f->integrated, 64);
                tm->reint.pop_front();
                if (nw[0] != kNegInf) {
                    std::memcpy(f->integrated, nw, 64);
                    break;
                }
            }
            if (nw[0] != kNegInf) {
                kinds[n] = 3;
                framesOut[n] = f->frameIdx;
                std::memcpy(oldT + 16 * n, o, 64);
                std::memcpy(newT + 16 * n, nw, 64);
                f->type = Integrated;
                n++;
            }
            continue;
        }
        break;
    }
    return n;
}

// the exit check of the render loop past the end (DepthSensing.cpp:1116-1123): generateUpdateLists,
// then getNumActiveOperations
unsigned or_traj_generate_and_count(void* h) {
    TM* tm = static_cast<TM*>(h);
    generate(tm);
    return (unsigned)(tm->deint.size() + tm->integ.size() + tm->reint.size());
}

void or_traj_integrated(void* h, unsigned idx, float* T) {
    std::memcpy(T, static_cast<TM*>(h)->frames[idx].integrated, 64);
}

void or_traj_frame_info(void* h, unsigned idx, int* type, float* dist) {
    TM* tm = static_cast<TM*>(h);
    *type = tm->frames[idx].type;
    *dist = tm->frames[idx].dist;
}

}  // extern "C"
