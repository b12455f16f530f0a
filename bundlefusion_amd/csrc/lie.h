// lie.h — se(3) exponential / logarithm and the dense-term Jacobians for the gfx950 solver
// (restated from Source/Solver/LieDerivUtil.h; line cites below).
#pragma once
#include "bf_math.h"

namespace bf {

struct m3 { float e[9]; };
BF_HD float& at3(m3& m, int r, int c) { return m.e[r * 3 + c]; }
BF_HD float at3(const m3& m, int r, int c) { return m.e[r * 3 + c]; }
BF_HD f3 mul3v(const m3& m, f3 v) {
    return mk3(m.e[0] * v.x + m.e[1] * v.y + m.e[2] * v.z, m.e[3] * v.x + m.e[4] * v.y + m.e[5] * v.z,
               m.e[6] * v.x + m.e[7] * v.y + m.e[8] * v.z);
}
BF_HD m3 mul33(const m3& a, const m3& b) {
    m3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.e[i * 3 + j] = a.e[i * 3 + 0] * b.e[0 * 3 + j] + a.e[i * 3 + 1] * b.e[1 * 3 + j] + a.e[i * 3 + 2] * b.e[2 * 3 + j];
    return r;
}
BF_HD m3 rot_of(const m4& m) {
    m3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.e[i * 3 + j] = m.e[i * 4 + j];
    return r;
}
BF_HD f3 trans_of(const m4& m) { return mk3(m.e[3], m.e[7], m.e[11]); }
BF_HD m4 mul44(const m4& a, const m4& b) {  // cuda_SimpleMatrixUtil.h:1164-1187
    m4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.e[i * 4 + j] = a.e[i * 4 + 0] * b.e[0 * 4 + j] + a.e[i * 4 + 1] * b.e[1 * 4 + j] + a.e[i * 4 + 2] * b.e[2 * 4 + j] +
                             a.e[i * 4 + 3] * b.e[3 * 4 + j];
    return r;
}
BF_HD f3 xf(const m4& m, f3 v) {
    const float* e = m.e;
    return mk3(e[0] * v.x + e[1] * v.y + e[2] * v.z + e[3] * 1.0f, e[4] * v.x + e[5] * v.y + e[6] * v.z + e[7] * 1.0f,
               e[8] * v.x + e[9] * v.y + e[10] * v.z + e[11] * 1.0f);
}

// general inverse (cuda_SimpleMatrixUtil.h:980-1090)
BF_HD m4 inverse44(const m4& M) {
    const float* e = M.e;
    float inv[16];
    inv[0] = e[5] * e[10] * e[15] - e[5] * e[11] * e[14] - e[9] * e[6] * e[15] + e[9] * e[7] * e[14] + e[13] * e[6] * e[11] - e[13] * e[7] * e[10];
    inv[4] = -e[4] * e[10] * e[15] + e[4] * e[11] * e[14] + e[8] * e[6] * e[15] - e[8] * e[7] * e[14] - e[12] * e[6] * e[11] + e[12] * e[7] * e[10];
    inv[8] = e[4] * e[9] * e[15] - e[4] * e[11] * e[13] - e[8] * e[5] * e[15] + e[8] * e[7] * e[13] + e[12] * e[5] * e[11] - e[12] * e[7] * e[9];
    inv[12] = -e[4] * e[9] * e[14] + e[4] * e[10] * e[13] + e[8] * e[5] * e[14] - e[8] * e[6] * e[13] - e[12] * e[5] * e[10] + e[12] * e[6] * e[9];
    inv[1] = -e[1] * e[10] * e[15] + e[1] * e[11] * e[14] + e[9] * e[2] * e[15] - e[9] * e[3] * e[14] - e[13] * e[2] * e[11] + e[13] * e[3] * e[10];
    inv[5] = e[0] * e[10] * e[15] - e[0] * e[11] * e[14] - e[8] * e[2] * e[15] + e[8] * e[3] * e[14] + e[12] * e[2] * e[11] - e[12] * e[3] * e[10];
    inv[9] = -e[0] * e[9] * e[15] + e[0] * e[11] * e[13] + e[8] * e[1] * e[15] - e[8] * e[3] * e[13] - e[12] * e[1] * e[11] + e[12] * e[3] * e[9];
    inv[13] = e[0] * e[9] * e[14] - e[0] * e[10] * e[13] - e[8] * e[1] * e[14] + e[8] * e[2] * e[13] + e[12] * e[1] * e[10] - e[12] * e[2] * e[9];
    inv[2] = e[1] * e[6] * e[15] - e[1] * e[7] * e[14] - e[5] * e[2] * e[15] + e[5] * e[3] * e[14] + e[13] * e[2] * e[7] - e[13] * e[3] * e[6];
    inv[6] = -e[0] * e[6] * e[15] + e[0] * e[7] * e[14] + e[4] * e[2] * e[15] - e[4] * e[3] * e[14] - e[12] * e[2] * e[7] + e[12] * e[3] * e[6];
    inv[10] = e[0] * e[5] * e[15] - e[0] * e[7] * e[13] - e[4] * e[1] * e[15] + e[4] * e[3] * e[13] + e[12] * e[1] * e[7] - e[12] * e[3] * e[5];
    inv[14] = -e[0] * e[5] * e[14] + e[0] * e[6] * e[13] + e[4] * e[1] * e[14] - e[4] * e[2] * e[13] - e[12] * e[1] * e[6] + e[12] * e[2] * e[5];
    inv[3] = -e[1] * e[6] * e[11] + e[1] * e[7] * e[10] + e[5] * e[2] * e[11] - e[5] * e[3] * e[10] - e[9] * e[2] * e[7] + e[9] * e[3] * e[6];
    inv[7] = e[0] * e[6] * e[11] - e[0] * e[7] * e[10] - e[4] * e[2] * e[11] + e[4] * e[3] * e[10] + e[8] * e[2] * e[7] - e[8] * e[3] * e[6];
    inv[11] = -e[0] * e[5] * e[11] + e[0] * e[7] * e[9] + e[4] * e[1] * e[11] - e[4] * e[3] * e[9] - e[8] * e[1] * e[7] + e[8] * e[3] * e[5];
    inv[15] = e[0] * e[5] * e[10] - e[0] * e[6] * e[9] - e[4] * e[1] * e[10] + e[4] * e[2] * e[9] + e[8] * e[1] * e[6] - e[8] * e[2] * e[5];
    const float det = e[0] * inv[0] + e[1] * inv[4] + e[2] * inv[8] + e[3] * inv[12];
    const float detr = 1.0f / det;
    m4 r;
    for (int i = 0; i < 16; i++) r.e[i] = inv[i] * detr;
    return r;
}

constexpr float ONE_TWENTIETH = 0.05f, ONE_SIXTH = 0.16666667f;

// rodrigues_so3_exp, LieDerivUtil.h:19-47
BF_HD m3 rodrigues(f3 w, float A, float B) {
    m3 R;
    const float wx2 = w.x * w.x, wy2 = w.y * w.y, wz2 = w.z * w.z;
    at3(R, 0, 0) = 1.0f - B * (wy2 + wz2);
    at3(R, 1, 1) = 1.0f - B * (wx2 + wz2);
    at3(R, 2, 2) = 1.0f - B * (wx2 + wy2);
    { const float a = A * w.z, b = B * (w.x * w.y); at3(R, 0, 1) = b - a; at3(R, 1, 0) = b + a; }
    { const float a = A * w.y, b = B * (w.x * w.z); at3(R, 0, 2) = b + a; at3(R, 2, 0) = b - a; }
    { const float a = A * w.x, b = B * (w.y * w.z); at3(R, 1, 2) = b - a; at3(R, 2, 1) = b + a; }
    return R;
}
// exp_rotation, :50-76
BF_HD m3 exp_rotation(f3 w) {
    const float theta_sq = dot3(w, w);
    const float theta = sqrtf(theta_sq);
    float A, B;
    if (theta_sq < 1e-8f) { A = 1.0f - ONE_SIXTH * theta_sq; B = 0.5f; }
    else if (theta_sq < 1e-6f) { B = 0.5f - 0.25f * ONE_SIXTH * theta_sq; A = 1.0f - theta_sq * ONE_SIXTH * (1.0f - ONE_TWENTIETH * theta_sq); }
    else { const float inv = 1.0f / theta; A = sinf(theta) * inv; B = (1 - cosf(theta)) * (inv * inv); }
    return rodrigues(w, A, B);
}
// ln_rotation, :79-133
BF_HD f3 ln_rotation(const m3& R) {
    f3 r;
    const float cos_angle = (at3(R, 0, 0) + at3(R, 1, 1) + at3(R, 2, 2) - 1.0f) * 0.5f;
    r.x = (at3(R, 2, 1) - at3(R, 1, 2)) * 0.5f;
    r.y = (at3(R, 0, 2) - at3(R, 2, 0)) * 0.5f;
    r.z = (at3(R, 1, 0) - at3(R, 0, 1)) * 0.5f;
    const float s = length3(r);
    if (cos_angle > (float)0.70710678118654752440) {
        if (s > 0) r = r * (asinf(s) / s);
    } else if (cos_angle > -(float)0.70710678118654752440) {
        const float angle = acosf(cos_angle);
        r = r * (angle / s);
    } else {
        const float angle = 3.141592654f - asinf(s);
        const float d0 = at3(R, 0, 0) - cos_angle, d1 = at3(R, 1, 1) - cos_angle, d2 = at3(R, 2, 2) - cos_angle;
        f3 r2;
        if (fabsf(d0) > fabsf(d1) && fabsf(d0) > fabsf(d2)) r2 = mk3(d0, (at3(R, 1, 0) + at3(R, 0, 1)) * 0.5f, (at3(R, 0, 2) + at3(R, 2, 0)) * 0.5f);
        else if (fabsf(d1) > fabsf(d2)) r2 = mk3((at3(R, 1, 0) + at3(R, 0, 1)) * 0.5f, d1, (at3(R, 2, 1) + at3(R, 1, 2)) * 0.5f);
        else r2 = mk3((at3(R, 0, 2) + at3(R, 2, 0)) * 0.5f, (at3(R, 2, 1) + at3(R, 1, 2)) * 0.5f, d2);
        if (dot3(r2, r) < 0) r2 = r2 * -1.0f;
        r = r2 * (angle / length3(r2));
    }
    return r;
}
// matrixToPose, :135-158
BF_HD void matrix_to_pose(const m4& M, f3& rot, f3& trans) {
    const m3 R = rot_of(M);
    const f3 t = trans_of(M);
    rot = ln_rotation(R);
    const float theta = length3(rot);
    float shtot = 0.5f;
    if (theta > 0.00001f) shtot = sinf(theta * 0.5f) / theta;
    const m3 half = exp_rotation(rot * -0.5f);
    trans = mul3v(half, t);
    if (theta > 0.001f) trans = trans - rot * (dot3(t, rot) * (1 - 2 * shtot) / dot3(rot, rot));
    else trans = trans - rot * (dot3(t, rot) / 24);
    trans = trans * (1.0f / (2 * shtot));
}
// poseToMatrix, :160-207
BF_HD m4 pose_to_matrix(f3 rot, f3 trans) {
    m4 M;
    for (int i = 0; i < 16; i++) M.e[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    const float theta_sq = dot3(rot, rot);
    const float theta = sqrtf(theta_sq);
    float A, B;
    const f3 cr = cross3(rot, trans);
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
            A = sinf(theta) * inv;
            B = (1 - cosf(theta)) * (inv * inv);
            C = (1 - A) * (inv * inv);
        }
        const f3 wc = cross3(rot, cr);
        translation = trans + cr * B + wc * C;
    }
    const m3 R = rodrigues(rot, A, B);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) M.e[i * 4 + j] = R.e[i * 3 + j];
    M.e[3] = translation.x; M.e[7] = translation.y; M.e[11] = translation.z;
    return M;
}
// computeLieUpdate, :301-307
BF_HD void lie_update(f3 dW, f3 dT, f3 curW, f3 curT, f3& newW, f3& newT) {
    matrix_to_pose(mul44(pose_to_matrix(dW, dT), pose_to_matrix(curW, curT)), newW, newT);
}

struct m36 { float e[18]; };
BF_HD m3 skew(f3 v) {  // :216-225
    m3 r;
    for (int i = 0; i < 9; i++) r.e[i] = 0.0f;
    at3(r, 1, 0) = v.z; at3(r, 2, 0) = -v.y; at3(r, 2, 1) = v.x;
    at3(r, 0, 1) = -v.z; at3(r, 0, 2) = v.y; at3(r, 1, 2) = -v.x;
    return r;
}
// evalLie_derivI, :247-272 (the 3x12 * 12x6 product, skipping its structural zeros)
BF_HD m36 deriv_i(const m4& A, const m4& D, f3 p) {
    const m4 T = mul44(A, D);
    const f3 pt = p - trans_of(T);
    float j1[12][6];
    for (int r = 0; r < 12; r++)
        for (int c = 0; c < 6; c++) j1[r][c] = 0.0f;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) j1[r + 9][c] = A.e[r * 4 + c];
    const m3 RA = rot_of(A);
    for (int k = 0; k < 4; k++) {
        const m3 m = mul33(RA, skew(mk3(D.e[0 * 4 + k], D.e[1 * 4 + k], D.e[2 * 4 + k])));
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) j1[3 * k + r][3 + c] = m.e[r * 3 + c] * -1.0f;
    }
    float j0[3][12];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 12; c++) j0[r][c] = 0.0f;
    j0[0][0] = pt.x; j0[0][1] = pt.y; j0[0][2] = pt.z;
    j0[1][3] = pt.x; j0[1][4] = pt.y; j0[1][5] = pt.z;
    j0[2][6] = pt.x; j0[2][7] = pt.y; j0[2][8] = pt.z;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) j0[r][c + 9] = -T.e[c * 4 + r];
    m36 out;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 6; j++) {
            float s = 0.0f;
            for (int k = 0; k < 12; k++) s += j0[i][k] * j1[k][j];
            out.e[i * 6 + j] = s;
        }
    return out;
}
// evalLie_derivJ, :277-295
BF_HD m36 deriv_j(const m4& A, const m4& D, f3 p) {
    const f3 dr1 = mk3(D.e[0], D.e[1], D.e[2]), dr2 = mk3(D.e[4], D.e[5], D.e[6]), dr3 = mk3(D.e[8], D.e[9], D.e[10]);
    const float dtx = D.e[3], dty = D.e[7], dtz = D.e[11];
    float jac[3][6] = {{1.0f, 0.0f, 0.0f, 0.0f, dot3(p, dr3) + dtz, -(dot3(p, dr2) + dty)},
                       {0.0f, 1.0f, 0.0f, -(dot3(p, dr3) + dtz), 0.0f, dot3(p, dr1) + dtx},
                       {0.0f, 0.0f, 1.0f, dot3(p, dr2) + dty, -(dot3(p, dr1) + dtx), 0.0f}};
    m36 out;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 6; j++) {
            float s = 0.0f;
            for (int k = 0; k < 3; k++) s += A.e[i * 4 + k] * jac[k][j];
            out.e[i * 6 + j] = s;
        }
    return out;
}

}  // namespace bf
