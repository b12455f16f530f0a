// oracle/or_lie.h — TEST INFRASTRUCTURE (CPU oracle, see oracle.h header).
// se(3) maps and Jacobians restated from Source/Solver/LieDerivUtil.h (line cites below)
// and the matrix helpers of Source/SiftGPU/cuda_SimpleMatrixUtil.h.
#pragma once
#include "or_math.h"

namespace orc {

struct m3 { float e[9]; };  // row-major float3x3
inline float& at(m3& m, int r, int c) { return m.e[r * 3 + c]; }
inline float at(const m3& m, int r, int c) { return m.e[r * 3 + c]; }
inline f3 mul(const m3& m, f3 v) {  // float3x3 * float3 (cuda_SimpleMatrixUtil.h:517-523)
    return {m.e[0] * v.x + m.e[1] * v.y + m.e[2] * v.z, m.e[3] * v.x + m.e[4] * v.y + m.e[5] * v.z,
            m.e[6] * v.x + m.e[7] * v.y + m.e[8] * v.z};
}
inline m3 mul(const m3& a, const m3& b) {  // float3x3 * float3x3 (:487-501)
    m3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.e[i * 3 + j] = a.e[i * 3 + 0] * b.e[0 * 3 + j] + a.e[i * 3 + 1] * b.e[1 * 3 + j] + a.e[i * 3 + 2] * b.e[2 * 3 + j];
    return r;
}
inline m3 scale(const m3& a, float t) { m3 r; for (int i = 0; i < 9; i++) r.e[i] = a.e[i] * t; return r; }
inline m3 rot3(const m4& m) { m3 r; for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) r.e[i * 3 + j] = m.e[i * 4 + j]; return r; }
inline f3 trans3(const m4& m) { return {m.e[3], m.e[7], m.e[11]}; }
// float4x4 * float4x4 (:1164-1187)
inline m4 mul(const m4& a, const m4& b) {
    m4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.e[i * 4 + j] = a.e[i * 4 + 0] * b.e[0 * 4 + j] + a.e[i * 4 + 1] * b.e[1 * 4 + j] + a.e[i * 4 + 2] * b.e[2 * 4 + j] +
                             a.e[i * 4 + 3] * b.e[3 * 4 + j];
    return r;
}

const float ONE_TWENTIETH = 0.05f, ONE_SIXTH = 0.16666667f;

// rodrigues_so3_exp, LieDerivUtil.h:19-47
inline m3 rodrigues(f3 w, float A, float B) {
    m3 R;
    const float wx2 = w.x * w.x, wy2 = w.y * w.y, wz2 = w.z * w.z;
    at(R, 0, 0) = 1.0f - B * (wy2 + wz2);
    at(R, 1, 1) = 1.0f - B * (wx2 + wz2);
    at(R, 2, 2) = 1.0f - B * (wx2 + wy2);
    { const float a = A * w.z, b = B * (w.x * w.y); at(R, 0, 1) = b - a; at(R, 1, 0) = b + a; }
    { const float a = A * w.y, b = B * (w.x * w.z); at(R, 0, 2) = b + a; at(R, 2, 0) = b - a; }
    { const float a = A * w.x, b = B * (w.y * w.z); at(R, 1, 2) = b - a; at(R, 2, 1) = b + a; }
    return R;
}

// exp_rotation, :50-76
inline m3 exp_rotation(f3 w) {
    const float theta_sq = dot(w, w);
    const float theta = std::sqrt(theta_sq);
    float A, B;
    if (theta_sq < 1e-8f) { A = 1.0f - ONE_SIXTH * theta_sq; B = 0.5f; }
    else if (theta_sq < 1e-6f) { B = 0.5f - 0.25f * ONE_SIXTH * theta_sq; A = 1.0f - theta_sq * ONE_SIXTH * (1.0f - ONE_TWENTIETH * theta_sq); }
    else { const float inv = 1.0f / theta; A = std::sin(theta) * inv; B = (1 - std::cos(theta)) * (inv * inv); }
    return rodrigues(w, A, B);
}

// ln_rotation, :79-133
inline f3 ln_rotation(const m3& R) {
    f3 r;
    const float cos_angle = (at(R, 0, 0) + at(R, 1, 1) + at(R, 2, 2) - 1.0f) * 0.5f;
    r.x = (at(R, 2, 1) - at(R, 1, 2)) * 0.5f;
    r.y = (at(R, 0, 2) - at(R, 2, 0)) * 0.5f;
    r.z = (at(R, 1, 0) - at(R, 0, 1)) * 0.5f;
    float sin_angle_abs = length(r);
    if (cos_angle > (float)0.70710678118654752440) {
        if (sin_angle_abs > 0) r = r * (std::asin(sin_angle_abs) / sin_angle_abs);
    } else if (cos_angle > -(float)0.70710678118654752440) {
        float angle = std::acos(cos_angle);
        r = r * (angle / sin_angle_abs);
    } else {
        const float angle = 3.141592654f - std::asin(sin_angle_abs);
        const float d0 = at(R, 0, 0) - cos_angle, d1 = at(R, 1, 1) - cos_angle, d2 = at(R, 2, 2) - cos_angle;
        f3 r2;
        if (std::fabs(d0) > std::fabs(d1) && std::fabs(d0) > std::fabs(d2)) {
            r2 = {d0, (at(R, 1, 0) + at(R, 0, 1)) * 0.5f, (at(R, 0, 2) + at(R, 2, 0)) * 0.5f};
        } else if (std::fabs(d1) > std::fabs(d2)) {
            r2 = {(at(R, 1, 0) + at(R, 0, 1)) * 0.5f, d1, (at(R, 2, 1) + at(R, 1, 2)) * 0.5f};
        } else {
            r2 = {(at(R, 0, 2) + at(R, 2, 0)) * 0.5f, (at(R, 2, 1) + at(R, 1, 2)) * 0.5f, d2};
        }
        if (dot(r2, r) < 0) r2 = r2 * -1.0f;
        r = r2 * (angle / length(r2));
    }
    return r;
}

// matrixToPose, :135-158
inline void matrixToPose(const m4& M, f3& rot, f3& trans) {
    const m3 R = rot3(M);
    const f3 t = trans3(M);
    rot = ln_rotation(R);
    const float theta = length(rot);
    float shtot = 0.5f;
    if (theta > 0.00001f) shtot = std::sin(theta * 0.5f) / theta;
    f3 rot_half = rot * -0.5f;
    const m3 half = exp_rotation(rot_half);
    trans = mul(half, t);
    if (theta > 0.001f) trans = trans - rot * (dot(t, rot) * (1 - 2 * shtot) / dot(rot, rot));
    else trans = trans - rot * (dot(t, rot) / 24);
    trans = trans * (1.0f / (2 * shtot));
}

// poseToMatrix, :160-207
inline m4 poseToMatrix(f3 rot, f3 trans) {
    m4 M = {{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}};
    const float theta_sq = dot(rot, rot);
    const float theta = std::sqrt(theta_sq);
    float A, B;
    f3 cr = cross(rot, trans);
    f3 translation;
    if (theta_sq < 1e-8f) {
        A = 1.0f - ONE_SIXTH * theta_sq;
        B = 0.5f;
        translation = trans + cr * 0.5f;
    } else {
        float C;
        if (theta_sq < 1e-6f) {
            C = ONE_SIXTH * (1.0f - ONE_TWENTIETH * theta_sq);
            A = 1.0f - theta_sq * C;
            B = 0.5f - 0.25f * ONE_SIXTH * theta_sq;
        } else {
            const float inv = 1.0f / theta;
            A = std::sin(theta) * inv;
            B = (1 - std::cos(theta)) * (inv * inv);
            C = (1 - A) * (inv * inv);
        }
        f3 w_cross = cross(rot, cr);
        translation = trans + cr * B + w_cross * C;
    }
    m3 R = rodrigues(rot, A, B);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) M.e[i * 4 + j] = R.e[i * 3 + j];
    M.e[3] = translation.x; M.e[7] = translation.y; M.e[11] = translation.z;
    return M;
}

// evalLie_dAlpha/dBeta/dGamma, :231-242
inline f3 dAlpha(f3 p) { return {0.0f, -p.z, p.y}; }
inline f3 dBeta(f3 p) { return {p.z, 0.0f, -p.x}; }
inline f3 dGamma(f3 p) { return {-p.y, p.x, 0.0f}; }

struct m36 { float e[18]; };  // 3x6 row-major
inline float& at(m36& m, int r, int c) { return m.e[r * 6 + c]; }
inline float at(const m36& m, int r, int c) { return m.e[r * 6 + c]; }

inline m3 skew(f3 v) {  // VectorToSkewSymmetricMatrix, :216-225
    m3 r = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    at(r, 1, 0) = v.z; at(r, 2, 0) = -v.y; at(r, 2, 1) = v.x;
    at(r, 0, 1) = -v.z; at(r, 0, 2) = v.y; at(r, 1, 2) = -v.x;
    return r;
}

// evalLie_derivI, :247-272 — deriv of (A e^e D)^-1 p, A = Tj^-1, D = Ti
inline m36 derivI(const m4& A, const m4& D, f3 p) {
    float j0[3][12] = {{0}}, j1[12][6] = {{0}};
    const m4 T = mul(A, D);
    f3 pt = p - trans3(T);
    j0[0][0] = pt.x; j0[0][1] = pt.y; j0[0][2] = pt.z;
    j0[1][3] = pt.x; j0[1][4] = pt.y; j0[1][5] = pt.z;
    j0[2][6] = pt.x; j0[2][7] = pt.y; j0[2][8] = pt.z;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            j0[r][c + 9] = -T.e[c * 4 + r];
            j1[r + 9][c] = A.e[r * 4 + c];
        }
    const m3 RA = rot3(A);
    for (int k = 0; k < 4; k++) {
        m3 m = scale(mul(RA, skew({D.e[0 * 4 + k], D.e[1 * 4 + k], D.e[2 * 4 + k]})), -1.0f);
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) j1[3 * k + r][3 + c] = at(m, r, c);
    }
    m36 out;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 6; j++) {
            float s = 0.0f;
            for (int k = 0; k < 12; k++) s += j0[i][k] * j1[k][j];
            at(out, i, j) = s;
        }
    return out;
}

// evalLie_derivJ, :277-295 — deriv of (A e^e D) p, A = Ti^-1, D = Tj
inline m36 derivJ(const m4& A, const m4& D, f3 p) {
    f3 dr1 = {D.e[0], D.e[1], D.e[2]}, dr2 = {D.e[4], D.e[5], D.e[6]}, dr3 = {D.e[8], D.e[9], D.e[10]};
    float dtx = D.e[3], dty = D.e[7], dtz = D.e[11];
    m36 jac;
    at(jac, 0, 0) = 1.0f; at(jac, 0, 1) = 0.0f; at(jac, 0, 2) = 0.0f;
    at(jac, 1, 0) = 0.0f; at(jac, 1, 1) = 1.0f; at(jac, 1, 2) = 0.0f;
    at(jac, 2, 0) = 0.0f; at(jac, 2, 1) = 0.0f; at(jac, 2, 2) = 1.0f;
    at(jac, 0, 3) = 0.0f; at(jac, 0, 4) = dot(p, dr3) + dtz; at(jac, 0, 5) = -(dot(p, dr2) + dty);
    at(jac, 1, 3) = -(dot(p, dr3) + dtz); at(jac, 1, 4) = 0.0f; at(jac, 1, 5) = dot(p, dr1) + dtx;
    at(jac, 2, 3) = dot(p, dr2) + dty; at(jac, 2, 4) = -(dot(p, dr1) + dtx); at(jac, 2, 5) = 0.0f;
    const m3 RA = rot3(A);
    m36 out;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 6; j++) {
            float s = 0.0f;
            for (int k = 0; k < 3; k++) s += at(RA, i, k) * at(jac, k, j);
            at(out, i, j) = s;
        }
    return out;
}

// computeLieUpdate, :301-307
inline void lieUpdate(f3 dW, f3 dT, f3 curW, f3 curT, f3& newW, f3& newT) {
    const m4 upd = poseToMatrix(dW, dT);
    const m4 cur = poseToMatrix(curW, curT);
    matrixToPose(mul(upd, cur), newW, newT);
}

}  // namespace orc
