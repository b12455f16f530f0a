// oracle/ba.cpp — TEST INFRASTRUCTURE (CPU oracle, see oracle.h header).
//
// Serial restatement of CUDASolverBundling::solve (Source/Solver/CUDASolverBundling.cpp:187-284)
// -> solveBundlingStub (Source/Solver/SolverBundling.cu:1137-1220): Lie-space Gauss-Newton with
// a Jacobi-preconditioned CG inner loop over the sparse point-to-point term (EntryJ) and the
// optional dense depth/colour term. Every kernel is executed as a serial loop; float atomics of
// the reference become sums in index order (the reference's order is undefined).
#include "oracle.h"
#include "or_lie.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

using namespace orc;

namespace {

const float MINF = -std::numeric_limits<float>::infinity();
const float FLOAT_EPSILON = 0.000001f;  // Source/SolverUtil.h:9

inline f3 ld3(const float* p) { return {p[0], p[1], p[2]}; }
inline f3 ld3(const BFFloat3& p) { return {p.x, p.y, p.z}; }
inline f3 fabs3(f3 a) { return {std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)}; }

struct Frame {  // host view of a BFCachedFrame
    const float* depth;
    const float* campos;   // float4
    const float* normals;  // float4
    const uint8_t* normalsU8;
    const float* intensity;
    const float* intensityDeriv;  // float2
};

struct Solver {
    const ORSolveParams& P;
    BFEntryJ* corr;
    const int* valid;
    uint32_t N, Nc;
    std::vector<f3> xRot, xTrans, dRot, dTrans, rRot, rTrans, zRot, zTrans, pRot, pTrans, apRot, apTrans, mRot, mTrans;
    std::vector<float> rDotzOld;
    float scanAlpha[2];
    std::vector<m4> T, Tinv;
    std::vector<int> table;  // [N][maxCorrPerImage], -1 = hole
    std::vector<int> numEntries;
    std::vector<float> jtj, jtr;
    double denseEnergy = 0.0;  // sum w r^2 of the dense rows (d_sumResidual analogue), for gradient checks
    uint32_t densePairs = 0;
    float wSparse = 0, wDepth = 0, wColor = 0;
    bool useDense = false;
    uint32_t pcgIters = 0;

    Solver(const ORSolveParams& p, BFEntryJ* c, const int* v) : P(p), corr(c), valid(v), N(p.numImages), Nc(p.numCorr) {
        auto z = f3{0, 0, 0};
        for (auto* vec : {&xRot, &xTrans, &dRot, &dTrans, &rRot, &rTrans, &zRot, &zTrans, &pRot, &pTrans, &apRot, &apTrans, &mRot, &mTrans})
            vec->assign(N, z);
        rDotzOld.assign(N, 0.0f);
        T.resize(N);
        Tinv.resize(N);
    }

    bool corrValid(const BFEntryJ& e) const { return e.imgIdx_i != BF_INVALID_IMAGE; }

    // buildVariablesToCorrespondencesTable (CUDASolverBundling.cpp:286-292) ->
    // BuildVariablesToCorrespondencesTableDevice (SolverBundling.cu:1226-1248), serial in corr order
    void buildTable() {
        const uint32_t cap = P.maxCorrPerImage;
        table.assign((size_t)N * cap, -1);
        numEntries.assign(N, 0);
        for (uint32_t x = 0; x < Nc; x++) {
            BFEntryJ& c = corr[x];
            if (!corrValid(c)) continue;
            int o0 = numEntries[c.imgIdx_i]++;
            int o1 = numEntries[c.imgIdx_j]++;
            if ((uint32_t)o0 < cap && (uint32_t)o1 < cap) {
                table[(size_t)c.imgIdx_i * cap + o0] = (int)x;
                table[(size_t)c.imgIdx_j * cap + o1] = (int)x;
            } else {
                c.imgIdx_i = c.imgIdx_j = BF_INVALID_IMAGE;  // setInvalid
            }
        }
    }

    // convertLiePosesToMatricesCU (SolverBundling.cu:1114-1130)
    void posesToMatrices() {
        for (uint32_t i = 0; i < N; i++) {
            T[i] = poseToMatrix(xRot[i], xTrans[i]);
            Tinv[i] = inverse(T[i]);
        }
    }

    // ---- dense term (SolverBundling.cu:29-471, SolverBundlingDenseUtil.h) ----------------
    Frame frame(uint32_t i) const {
        const BFCachedFrame& f = P.cache[i];
        return {f.depth, f.campos, f.normals, f.normalsU8, f.intensity, f.intensityDeriv};
    }
    f3 depthToCamera(int x, int y, float depth) const {  // CUDACameraUtil.h:15-19
        const float xx = ((float)x - P.intrinsics[2]) / P.intrinsics[0];
        const float yy = ((float)y - P.intrinsics[3]) / P.intrinsics[1];
        return {depth * xx, depth * yy, depth};
    }
    void cameraToDepth(f3 p, float& u, float& v) const {  // CUDACameraUtil.h:9-14
        u = p.x * P.intrinsics[0] / p.z + P.intrinsics[2];
        v = p.y * P.intrinsics[1] / p.z + P.intrinsics[3];
    }
    // bilinearInterpolationFloat{,4} (ICPUtil.h:56-111); comp = number of floats per texel
    void bilinear(float x, float y, const float* img, int comp, float* out) const {
        const int W = (int)P.cacheW, H = (int)P.cacheH;
        const int px = (int)std::floor(x), py = (int)std::floor(y);
        const float alpha = x - (float)px, beta = y - (float)py;
        float s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0}, w0 = 0, w1 = 0;
        auto tap = [&](int qx, int qy, float wt, float* s, float& w) {
            if ((unsigned)qx < (unsigned)W && (unsigned)qy < (unsigned)H) {
                const float* v = img + ((size_t)qy * W + qx) * comp;
                if (v[0] != MINF) {
                    for (int k = 0; k < comp; k++) s[k] += wt * v[k];
                    w += wt;
                }
            }
        };
        tap(px, py, 1.0f - alpha, s0, w0);
        tap(px + 1, py, alpha, s0, w0);
        tap(px, py + 1, 1.0f - alpha, s1, w1);
        tap(px + 1, py + 1, alpha, s1, w1);
        float ss[4] = {0, 0, 0, 0}, ww = 0;
        if (w0 > 0.0f) { for (int k = 0; k < comp; k++) ss[k] += (1.0f - beta) * (s0[k] / w0); ww += (1.0f - beta); }
        if (w1 > 0.0f) { for (int k = 0; k < comp; k++) ss[k] += beta * (s1[k] / w1); ww += beta; }
        for (int k = 0; k < comp; k++) out[k] = (ww > 0.0f) ? ss[k] / ww : MINF;
    }
    // computeAngleDiff (SolverBundlingDenseUtil.h:416-424)
    bool angleOk(const m4& t, float thresh) const {
        f3 x = normalize(f3{1.0f, 1.0f, 1.0f});
        f3 v = mul(rot3(t), x);
        float a = std::acos(std::max(-1.0f, std::min(dot(x, v), 1.0f)));
        return std::fabs(a) < thresh;
    }
    // findDenseCorr depth-only (:22-42)
    bool corrDepthOnly(uint32_t idx, const m4& t, const float* tgtDepth, const float* srcDepth) const {
        const uint32_t W = P.cacheW, H = P.cacheH;
        const int x = (int)(idx % W), y = (int)(idx / W);
        const f3 cposj = depthToCamera(x, y, srcDepth[idx]);
        if (!(cposj.z > P.denseDepthMin && cposj.z < P.denseDepthMax)) return false;
        f3 s2t = xform(t, cposj);
        float u, v;
        cameraToDepth(s2t, u, v);
        const int tx = (int)std::round(u), ty = (int)std::round(v);
        if (!(tx >= 0 && ty >= 0 && tx < (int)W && ty < (int)H)) return false;
        f3 cpt = depthToCamera(tx, ty, tgtDepth[ty * W + tx]);
        if (!(cpt.z > P.denseDepthMin && cpt.z < P.denseDepthMax)) return false;
        return length(s2t - cpt) <= P.denseDistThresh;
    }
    // findDenseCorr depth + uchar4 normals (:152-184)
    bool corrU8(uint32_t idx, const m4& t, const Frame& tgt, const Frame& src) const {
        const uint32_t W = P.cacheW, H = P.cacheH;
        const int x = (int)(idx % W), y = (int)(idx / W);
        const f3 cposj = depthToCamera(x, y, src.depth[idx]);
        if (!(cposj.z > P.denseDepthMin && cposj.z < P.denseDepthMax)) return false;
        const uint8_t* nj = src.normalsU8 + 4 * idx;
        uint32_t njw;
        std::memcpy(&njw, nj, 4);
        if (njw == 0) return false;
        f3 nrmj = f3{(float)nj[0], (float)nj[1], (float)nj[2]} / 255.0f * 2.0f - f3{1.0f, 1.0f, 1.0f};
        nrmj = mul(rot3(t), nrmj);
        f3 s2t = xform(t, cposj);
        float u, v;
        cameraToDepth(s2t, u, v);
        const int tx = (int)std::round(u), ty = (int)std::round(v);
        if (!(tx >= 0 && ty >= 0 && tx < (int)W && ty < (int)H)) return false;
        f3 cpt = depthToCamera(tx, ty, tgt.depth[ty * W + tx]);
        if (!(cpt.z > P.denseDepthMin && cpt.z < P.denseDepthMax)) return false;
        const uint8_t* ni = tgt.normalsU8 + 4 * (ty * W + tx);
        uint32_t niw;
        std::memcpy(&niw, ni, 4);
        if (niw == 0) return false;
        f3 nrmi = f3{(float)ni[0], (float)ni[1], (float)ni[2]} / 255.0f * 2.0f - f3{1.0f, 1.0f, 1.0f};
        float dist = length(s2t - cpt);
        float dn = dot(nrmj, nrmi);
        return dn >= P.denseNormalThresh && dist <= P.denseDistThresh;
    }
    // findDenseCorr camera positions + float4 normals (:79-113)
    bool corrCamPos(uint32_t idx, const m4& t, const Frame& tgt, const Frame& src, f3& camPosSrc, f3& s2t, float& u,
                    float& v, f3& camPosTgt, f3& normalTgt) const {
        const uint32_t W = P.cacheW, H = P.cacheH;
        const float* cp = src.campos + 4 * idx;
        if (!(cp[2] > P.denseDepthMin && cp[2] < P.denseDepthMax)) return false;
        camPosSrc = {cp[0], cp[1], cp[2]};
        const float* nj = src.normals + 4 * idx;
        if (nj[0] == MINF) return false;
        f3 nrmj = xform4(t, f3{nj[0], nj[1], nj[2]}, nj[3]);
        const float nrmjw = t.e[12] * nj[0] + t.e[13] * nj[1] + t.e[14] * nj[2] + t.e[15] * nj[3];
        s2t = xform(t, camPosSrc);
        cameraToDepth(s2t, u, v);
        const int tx = (int)std::round(u), ty = (int)std::round(v);
        if (!(tx >= 0 && ty >= 0 && tx < (int)W && ty < (int)H)) return false;
        float cposi[4];
        bilinear(u, v, tgt.campos, 4, cposi);
        if (!(cposi[2] > P.denseDepthMin && cposi[2] < P.denseDepthMax)) return false;
        camPosTgt = {cposi[0], cposi[1], cposi[2]};
        float nrmi[4];
        bilinear(u, v, tgt.normals, 4, nrmi);
        if (nrmi[0] == MINF) return false;
        normalTgt = {nrmi[0], nrmi[1], nrmi[2]};
        float dist = length(s2t - camPosTgt);
        float dn = nrmj.x * nrmi[0] + nrmj.y * nrmi[1] + nrmj.z * nrmi[2] + nrmjw * nrmi[3];  // float4 dot
        return dn >= P.denseNormalThresh && dist <= P.denseDistThresh;
    }

    // addToLocalSystem (SolverBundlingDenseUtil.h:229-288), serial
    void addToLocal(const float Ji[6], const float Jj[6], uint32_t vi, uint32_t vj, float res, float w) {
        const uint32_t dim = 6 * N;
        denseEnergy += (double)w * res * res;
        for (int i = 0; i < 6; i++) {
            for (int j = i; j < 6; j++) {
                float dii = 0, djj = 0, dij = 0, dji = 0;
                if (vi > 0) dii = Ji[i] * Ji[j] * w;
                if (vj > 0) djj = Jj[i] * Jj[j] * w;
                if (vi > 0 && vj > 0) {
                    dij = Ji[i] * Jj[j] * w;
                    if (i != j) dji = Ji[j] * Jj[i] * w;
                }
                jtj[(size_t)(vi * 6 + j) * dim + (vi * 6 + i)] += dii;
                jtj[(size_t)(vj * 6 + j) * dim + (vj * 6 + i)] += djj;
                jtj[(size_t)(vj * 6 + j) * dim + (vi * 6 + i)] += dij;
                jtj[(size_t)(vj * 6 + i) * dim + (vi * 6 + j)] += dji;
            }
            float jtri = 0, jtrj = 0;
            if (vi > 0) jtri = Ji[i] * res * w;
            if (vj > 0) jtrj = Jj[i] * res * w;
            jtr[vi * 6 + i] += jtri;
            jtr[vj * 6 + i] += jtrj;
        }
    }

    // BuildDenseSystem (SolverBundling.cu:308-471)
    bool buildDense() {
        const uint32_t dim = 6 * N;
        const uint32_t W = P.cacheW, H = P.cacheH, npix = W * H;
        jtj.assign((size_t)dim * dim, 0.0f);
        jtr.assign(dim, 0.0f);
        denseEnergy = 0.0;
        densePairs = 0;
        std::vector<std::pair<uint32_t, uint32_t>> pairs;
        // FindImageImageCorr_Kernel<true> (:29-79)
        const uint32_t sub = P.denseOverlapSubsample, subW = W / sub;
        for (uint32_t i = 0; i < N; i++)
            for (uint32_t j = i + 1; j < N; j++) {
                if (valid[i] == 0 || valid[j] == 0) continue;
                const m4 t = mul(Tinv[i], T[j]);
                if (!angleOk(t, 0.52f)) continue;
                int found = 0;
                for (uint32_t tid = 0; tid < 512; tid++) {
                    const uint32_t x = (tid % subW) * sub, y = (tid / subW) * sub, idx = y * W + x;
                    if (idx < npix && corrDepthOnly(idx, t, P.cache[i].depth, P.cache[j].depth)) found++;
                }
                if (found > 10) pairs.push_back({i, j});
            }
        densePairs = (uint32_t)pairs.size();
        if (pairs.empty()) return false;
        // FindDenseCorrespondences_Kernel (:92-160) + WeightDenseCorrespondences_Kernel (:162-180)
        std::vector<float> pw(pairs.size());
        for (size_t k = 0; k < pairs.size(); k++) {
            const uint32_t i = pairs[k].first, j = pairs[k].second;
            const m4 t = mul(Tinv[i], T[j]);
            const Frame fi = frame(i), fj = frame(j);
            int count = 0;
            for (uint32_t idx = 0; idx < npix; idx++)
                if (corrU8(idx, t, fi, fj)) count++;
            float x = (float)count;
            if (x > 0) x = (x < 800) ? 0.0f : 1.0f / std::min(std::log(x), 9.0f);
            pw[k] = x;
        }
        // BuildDenseSystem_Kernel<depth, color> (:182-306)
        const bool useDepth = wDepth > 0.0f;
        const bool useColor = !useDepth || wColor > 0.0f;
        const float fx = P.intrinsics[0], fy = P.intrinsics[1];
        for (size_t k = 0; k < pairs.size(); k++) {
            if (pw[k] == 0.0f) continue;
            const uint32_t i = pairs[k].first, j = pairs[k].second;
            const m4& Ti = T[i];
            const m4& Tj = T[j];
            const m4& Tiinv = Tinv[i];
            const m4& Tjinv = Tinv[j];
            const m4 t = mul(Tiinv, Tj);
            const Frame fi = frame(i), fj = frame(j);
            for (uint32_t src = 0; src < npix; src++) {
                f3 camPosSrc{0, 0, 0}, s2t{0, 0, 0}, camPosTgt{0, 0, 0}, nT{0, 0, 0};
                float u = 0, v = 0;
                bool found = corrCamPos(src, t, fi, fj, camPosSrc, s2t, u, v, camPosTgt, nT);
                if (useDepth && found) {
                    float Ji[6] = {0}, Jj[6] = {0};
                    f3 diff = camPosTgt - s2t;
                    float res = dot(diff, nT);
                    float base = std::max(0.0f, 1.0f - camPosTgt.z / 2.0f);
                    float w = wDepth * pw[k] * std::pow(base, 2.5f);
                    if (i > 0) {  // computeJacobianBlockRow_i (SolverBundlingEquationsLie.h:234-241)
                        m36 jac = derivI(Tjinv, Ti, camPosSrc);
                        for (int c = 0; c < 6; c++) Ji[c] = -dot(f3{at(jac, 0, c), at(jac, 1, c), at(jac, 2, c)}, nT);
                    }
                    if (j > 0) {
                        m36 jac = derivJ(Tiinv, Tj, camPosSrc);
                        for (int c = 0; c < 6; c++) Jj[c] = -dot(f3{at(jac, 0, c), at(jac, 1, c), at(jac, 2, c)}, nT);
                    }
                    addToLocal(Ji, Jj, i, j, res, w);
                }
                if (useColor && found) {
                    float dI[2], It;
                    bilinear(u, v, fi.intensityDeriv, 2, dI);
                    bilinear(u, v, fi.intensity, 1, &It);
                    float colorRes = It - fj.intensity[src];
                    bool ok = dI[0] != MINF && std::fabs(colorRes) < P.denseColorThresh &&
                              std::sqrt(dI[0] * dI[0] + dI[1] * dI[1]) > P.denseColorGradientMin;
                    if (ok) {
                        float Ji[6] = {0}, Jj[6] = {0};
                        // dCameraToScreen (ICPUtil.h:14-25)
                        const float wSq = s2t.z * s2t.z;
                        const float d00 = fx / s2t.z, d11 = fy / s2t.z, d02 = -fx * s2t.x / wSq, d12 = -fy * s2t.y / wSq;
                        auto row = [&](const m36& jac, float* out) {
                            for (int c = 0; c < 6; c++) {
                                // dProj * jac (2x3 * 3x6), then dColorB * that (1x2 * 2x6)
                                float r0 = d00 * at(jac, 0, c) + 0.0f * at(jac, 1, c) + d02 * at(jac, 2, c);
                                float r1 = 0.0f * at(jac, 0, c) + d11 * at(jac, 1, c) + d12 * at(jac, 2, c);
                                out[c] = dI[0] * r0 + dI[1] * r1;
                            }
                        };
                        if (i > 0) row(derivI(Tjinv, Ti, camPosSrc), Ji);
                        if (j > 0) row(derivJ(Tiinv, Tj, camPosSrc), Jj);
                        float w = wColor * pw[k] * std::max(0.0f, 1.0f - std::fabs(colorRes) / (1.15f * P.denseColorThresh));
                        addToLocal(Ji, Jj, i, j, colorRes, w);
                    }
                }
            }
        }
        // FlipJtJ_Kernel (:81-91)
        for (uint32_t y = 0; y < dim; y++)
            for (uint32_t x = y + 1; x < dim; x++) jtj[(size_t)y * dim + x] = jtj[(size_t)x * dim + y];
        return true;
    }

    // evalMinusJTFDevice (SolverBundlingEquationsLie.h:63-148) + PCGInit_Kernel1 (SolverBundling.cu:755-787)
    // OpenMP over images / correspondences: every per-image sum keeps its serial order and every
    // cross-image reduction is summed afterwards in image order, so the result equals the serial run's
    void init() {
        scanAlpha[0] = 0.0f;
        const uint32_t cap = P.maxCorrPerImage;
        std::vector<float> part(N, 0.0f);
#pragma omp parallel for schedule(dynamic, 8)
        for (long xl = 1; xl < (long)N; xl++) {
            const uint32_t x = (uint32_t)xl;
            f3 rR{0, 0, 0}, rT{0, 0, 0}, pR{0, 0, 0}, pT{0, 0, 0};
            dRot[x] = dTrans[x] = {0, 0, 0};
            const int n = std::min(numEntries[x], (int)cap);
            for (int k = 0; k < n; k++) {
                const int ci = table[(size_t)x * cap + k];
                if (ci < 0) continue;
                const BFEntryJ& c = corr[ci];
                if (!corrValid(c)) continue;
                const m4& TI = T[c.imgIdx_i];
                const m4& TJ = T[c.imgIdx_j];
                float sign = 1.0f;
                f3 wp;
                if (x != c.imgIdx_i) { sign = -1.0f; wp = xform(TJ, ld3(c.pos_j)); }
                else wp = xform(TI, ld3(c.pos_i));
                const f3 da = dAlpha(wp), db = dBeta(wp), dc = dGamma(wp);
                const f3 r = xform(TI, ld3(c.pos_i)) - xform(TJ, ld3(c.pos_j));
                rR = rR + sign * f3{dot(da, r), dot(db, r), dot(dc, r)};
                rT = rT + sign * r;
                pR = pR + f3{dot(da, da), dot(db, db), dot(dc, dc)};
                pT = pT + f3{1.0f, 1.0f, 1.0f};
            }
            f3 resR = (-wSparse) * rR, resT = (-wSparse) * rT;
            if (useDense) {
                resR = resR - f3{jtr[x * 6 + 3], jtr[x * 6 + 4], jtr[x * 6 + 5]};
                resT = resT - f3{jtr[x * 6 + 0], jtr[x * 6 + 1], jtr[x * 6 + 2]};
            }
            auto inv = [](float v) { return v > FLOAT_EPSILON ? 1.0f / v : 1.0f; };
            mRot[x] = {inv(pR.x), inv(pR.y), inv(pR.z)};
            mTrans[x] = {inv(pT.x), inv(pT.y), inv(pT.z)};
            rRot[x] = resR;
            rTrans[x] = resT;
            pRot[x] = orc::mul(mRot[x], resR);
            pTrans[x] = orc::mul(mTrans[x], resT);
            part[x] = dot(resR, pRot[x]) + dot(resT, pTrans[x]);
            apRot[x] = apTrans[x] = {0, 0, 0};
        }
        for (uint32_t x = 1; x < N; x++) scanAlpha[0] += part[x];
        for (uint32_t x = 1; x < N; x++) rDotzOld[x] = scanAlpha[0];  // PCGInit_Kernel2 (:789-794)
    }

    // applyJDevice (SolverBundlingEquationsLie.h:195-228)
    f3 applyJ(const BFEntryJ& c) const {
        f3 b{0, 0, 0};
        if (!corrValid(c)) return b;
        if (c.imgIdx_i > 0) {
            const f3 wp = xform(T[c.imgIdx_i], ld3(c.pos_i));
            const f3 pp = pRot[c.imgIdx_i];
            b = b + (dAlpha(wp) * pp.x + dBeta(wp) * pp.y + dGamma(wp) * pp.z + pTrans[c.imgIdx_i]);
        }
        if (c.imgIdx_j > 0) {
            const f3 wp = xform(T[c.imgIdx_j], ld3(c.pos_j));
            const f3 pp = pRot[c.imgIdx_j];
            b = b - (dAlpha(wp) * pp.x + dBeta(wp) * pp.y + dGamma(wp) * pp.z + pTrans[c.imgIdx_j]);
        }
        return b * wSparse;
    }

    // PCGIteration (SolverBundling.cu:1024-1108); returns true on the exiting iteration
    bool pcgIteration(bool useSparse, bool last) {
        scanAlpha[0] = scanAlpha[1] = 0.0f;
        const uint32_t cap = P.maxCorrPerImage;
        if (useSparse) {
            std::vector<f3> Jp(Nc);
#pragma omp parallel for schedule(static)
            for (long c = 0; c < (long)Nc; c++) Jp[c] = applyJ(corr[c]);  // PCGStep_Kernel0
#pragma omp parallel for schedule(dynamic, 8)
            for (long xl = 1; xl < (long)N; xl++) {                      // PCGStep_Kernel1a / applyJTDevice
                const uint32_t x = (uint32_t)xl;
                f3 oR{0, 0, 0}, oT{0, 0, 0};
                const int n = std::min(numEntries[x], (int)cap);
                for (int k = 0; k < n; k++) {
                    const int ci = table[(size_t)x * cap + k];
                    if (ci < 0) continue;
                    const BFEntryJ& c = corr[ci];
                    if (!corrValid(c)) continue;
                    float sign = 1.0f;
                    f3 wp;
                    if (x != c.imgIdx_i) { sign = -1.0f; wp = xform(T[c.imgIdx_j], ld3(c.pos_j)); }
                    else wp = xform(T[c.imgIdx_i], ld3(c.pos_i));
                    const f3 j = Jp[ci];
                    oR = oR + sign * f3{dot(dAlpha(wp), j), dot(dBeta(wp), j), dot(dGamma(wp), j)};
                    oT = oT + sign * j;
                }
                apRot[x] = apRot[x] + oR;
                apTrans[x] = apTrans[x] + oT;
            }
        }
        if (useDense) {  // PCGStep_Kernel_Dense / applyJTJDenseDevice (SolverBundlingDenseUtil.h:371-411)
            const uint32_t dim = 6 * N;
#pragma omp parallel for schedule(dynamic, 8)
            for (long xl = 1; xl < (long)N; xl++) {
                const uint32_t x = (uint32_t)xl;
                f3 oR{0, 0, 0}, oT{0, 0, 0};
                const uint32_t bv = x * 6;
                for (uint32_t i = 1; i < N; i++) {
                    const uint32_t bi = 6 * i;
                    auto blk = [&](uint32_t r0, uint32_t c0, f3 v) {
                        const float* row0 = &jtj[(size_t)(bv + r0 + 0) * dim + bi + c0];
                        const float* row1 = &jtj[(size_t)(bv + r0 + 1) * dim + bi + c0];
                        const float* row2 = &jtj[(size_t)(bv + r0 + 2) * dim + bi + c0];
                        return f3{row0[0] * v.x + row0[1] * v.y + row0[2] * v.z, row1[0] * v.x + row1[1] * v.y + row1[2] * v.z,
                                  row2[0] * v.x + row2[1] * v.y + row2[2] * v.z};
                    };
                    oT = oT + (blk(0, 0, pTrans[i]) + blk(0, 3, pRot[i]));
                    oR = oR + (blk(3, 0, pTrans[i]) + blk(3, 3, pRot[i]));
                }
                apRot[x] = apRot[x] + oR;
                apTrans[x] = apTrans[x] + oT;
            }
        }
        for (uint32_t x = 1; x < N; x++) scanAlpha[0] += dot(pRot[x], apRot[x]) + dot(pTrans[x], apTrans[x]);  // Kernel1b
        const float dotProduct = scanAlpha[0];
        for (uint32_t x = 1; x < N; x++) {  // Kernel2
            float alpha = 0.0f;
            if (dotProduct > FLOAT_EPSILON) alpha = rDotzOld[x] / dotProduct;
            dRot[x] = dRot[x] + alpha * pRot[x];
            dTrans[x] = dTrans[x] + alpha * pTrans[x];
            rRot[x] = rRot[x] - alpha * apRot[x];
            rTrans[x] = rTrans[x] - alpha * apTrans[x];
            zRot[x] = orc::mul(mRot[x], rRot[x]);
            zTrans[x] = orc::mul(mTrans[x], rTrans[x]);
            scanAlpha[1] += dot(zRot[x], rRot[x]) + dot(zTrans[x], rTrans[x]);
        }  // (N-long: serial)
        if (!P.disableEarlyOut && std::fabs(scanAlpha[0]) < 5e-7) last = true;  // ENABLE_EARLY_OUT (:1088-1093)
        for (uint32_t x = 1; x < N; x++) {  // Kernel3
            const float rDotzNew = scanAlpha[1];
            float beta = 0.0f;
            if (rDotzOld[x] > FLOAT_EPSILON) beta = rDotzNew / rDotzOld[x];
            rDotzOld[x] = rDotzNew;
            pRot[x] = zRot[x] + beta * pRot[x];
            pTrans[x] = zTrans[x] + beta * pTrans[x];
            apRot[x] = apTrans[x] = {0, 0, 0};
            if (last) {
                f3 nr, nt;
                lieUpdate(dRot[x], dTrans[x], xRot[x], xTrans[x], nr, nt);
                xRot[x] = nr;
                xTrans[x] = nt;
            }
        }
        pcgIters++;
        return last;
    }

    float gnConvergence() const {  // EvalGNConvergence (:694-749)
        float m = 0.0f;
        for (uint32_t x = 1; x < N; x++) {
            if (valid[x] == 0) continue;
            f3 a = fabs3(dRot[x]), b = fabs3(dTrans[x]);
            f3 r3{std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)};
            float r = std::fmax(r3.x, std::fmax(r3.y, r3.z));
            m = std::max(m, r);
        }
        return m;
    }

    // evalAbsMaxResidualDevice (SolverBundlingEquationsLie.h:27-40) / EvalMaxResidual + host max
    void maxResidual(float& mr, int& mi) const {
        mr = 0.0f;
        mi = 0;
        if (!(wSparse > 0.0f)) return;
        std::vector<m4> Tm(N);
        for (uint32_t i = 0; i < N; i++) Tm[i] = poseToMatrix(xRot[i], xTrans[i]);
        // per chunk: the first maximum; chunks combined in order (strict >: the lowest index wins ties)
        const uint32_t chunk = 1u << 16, nChunks = (Nc + chunk - 1) / chunk;
        std::vector<float> cm(nChunks, 0.0f);
        std::vector<int> ci(nChunks, 0);
#pragma omp parallel for schedule(dynamic, 1)
        for (long k = 0; k < (long)nChunks; k++) {
            float m = 0.0f;
            int idx = 0;
            const uint32_t lo = (uint32_t)k * chunk, hi = std::min(Nc, lo + chunk);
            for (uint32_t c = lo; c < hi; c++) {
                const BFEntryJ& e = corr[c];
                float r = 0.0f;
                if (corrValid(e)) {
                    f3 d = wSparse * fabs3(xform(Tm[e.imgIdx_i], ld3(e.pos_i)) - xform(Tm[e.imgIdx_j], ld3(e.pos_j)));
                    r = std::max(d.z, std::max(d.x, d.y));
                }
                if (m < r) { m = r; idx = (int)c; }
            }
            cm[k] = m;
            ci[k] = idx;
        }
        for (uint32_t k = 0; k < nChunks; k++)
            if (mr < cm[k]) { mr = cm[k]; mi = ci[k]; }
    }

    float energy() const {  // EvalResidual (:570-614): sum of w * |r|^2 (serial float sum, as before)
        std::vector<m4> Tm(N);
        for (uint32_t i = 0; i < N; i++) Tm[i] = poseToMatrix(xRot[i], xTrans[i]);
        std::vector<float> term(Nc, 0.0f);
#pragma omp parallel for schedule(static)
        for (long c = 0; c < (long)Nc; c++) {
            const BFEntryJ& e = corr[c];
            if (!corrValid(e)) continue;
            f3 r = xform(Tm[e.imgIdx_i], ld3(e.pos_i)) - xform(Tm[e.imgIdx_j], ld3(e.pos_j));
            term[c] = wSparse * dot(r, r);
        }
        float s = 0.0f;
        for (uint32_t c = 0; c < Nc; c++) {
            if (!corrValid(corr[c])) continue;
            s += term[c];
        }
        return s;
    }
};

}  // namespace

extern "C" {

void or_pose_to_matrix(const float rot[3], const float trans[3], float M[16]) {
    m4 m = poseToMatrix(f3{rot[0], rot[1], rot[2]}, f3{trans[0], trans[1], trans[2]});
    std::memcpy(M, m.e, 64);
}

void or_matrix_to_pose(const float M[16], float rot[3], float trans[3]) {
    m4 m;
    std::memcpy(m.e, M, 64);
    f3 r, t;
    matrixToPose(m, r, t);
    rot[0] = r.x; rot[1] = r.y; rot[2] = r.z;
    trans[0] = t.x; trans[1] = t.y; trans[2] = t.z;
}

// CUDASolverBundling::solve (CUDASolverBundling.cpp:187-284) with rebuildJT = true and
// findMaxResidual = true; solveBundlingStub (SolverBundling.cu:1137-1220).
void or_ba_solve(BFEntryJ* corr, const int* validImages, const ORSolveParams* p, float* rot, float* trans,
                 ORSolveResult* res) {
    Solver S(*p, corr, validImages);
    for (uint32_t i = 0; i < S.N; i++) {
        S.xRot[i] = {rot[3 * i], rot[3 * i + 1], rot[3 * i + 2]};
        S.xTrans[i] = {trans[3 * i], trans[3 * i + 1], trans[3 * i + 2]};
    }
    S.buildTable();
    uint32_t gn = 0;
    for (uint32_t it = 0; it < p->nNonLin; it++) {
        gn++;
        S.wSparse = p->weightsSparse[it];
        S.wDepth = p->weightsDenseDepth ? p->weightsDenseDepth[it] : 0.0f;
        S.wColor = p->weightsDenseColor ? p->weightsDenseColor[it] : 0.0f;
        S.useDense = (S.wDepth > 0 || S.wColor > 0) && p->cache != nullptr;
        S.posesToMatrices();
        if (S.useDense) S.useDense = S.buildDense();
        S.init();
        const bool sparse = S.wSparse > 0.0f;
        for (uint32_t li = 0; li < p->nLin; li++)
            if (S.pcgIteration(sparse, li == p->nLin - 1)) break;
        if (it < p->nNonLin - 1 && S.gnConvergence() < 0.005f && !p->disableEarlyOut) break;  // ENABLE_EARLY_OUT (:1204-1210)
    }
    for (uint32_t i = 0; i < S.N; i++) {
        rot[3 * i] = S.xRot[i].x; rot[3 * i + 1] = S.xRot[i].y; rot[3 * i + 2] = S.xRot[i].z;
        trans[3 * i] = S.xTrans[i].x; trans[3 * i + 1] = S.xTrans[i].y; trans[3 * i + 2] = S.xTrans[i].z;
    }
    if (res) {
        res->gnIterations = gn;
        res->pcgIterations = S.pcgIters;
        S.maxResidual(res->maxResidual, res->maxResidualIndex);
        res->finalEnergy = S.energy();
    }
}

// Test hook: the dense system (JtJ [6N x 6N], Jtr [6N], energy, #pairs) at the given poses with
// weightsDenseDepth[0] / weightsDenseColor[0]; used for finite-difference gradient checks.
void or_ba_dense_system(const int* validImages, const ORSolveParams* p, const float* rot, const float* trans,
                        float* jtjOut, float* jtrOut, double* energyOut, uint32_t* pairsOut) {
    Solver S(*p, nullptr, validImages);
    for (uint32_t i = 0; i < S.N; i++) {
        S.xRot[i] = {rot[3 * i], rot[3 * i + 1], rot[3 * i + 2]};
        S.xTrans[i] = {trans[3 * i], trans[3 * i + 1], trans[3 * i + 2]};
    }
    S.wDepth = p->weightsDenseDepth ? p->weightsDenseDepth[0] : 0.0f;
    S.wColor = p->weightsDenseColor ? p->weightsDenseColor[0] : 0.0f;
    S.posesToMatrices();
    const bool ok = S.buildDense();
    const size_t dim = 6 * (size_t)S.N;
    if (jtjOut) for (size_t k = 0; k < dim * dim; k++) jtjOut[k] = ok ? S.jtj[k] : 0.0f;
    if (jtrOut) for (size_t k = 0; k < dim; k++) jtrOut[k] = ok ? S.jtr[k] : 0.0f;
    if (energyOut) *energyOut = ok ? S.denseEnergy : 0.0;
    if (pairsOut) *pairsOut = S.densePairs;
}

uint32_t or_ba_count_high_residuals(const BFEntryJ* corr, uint32_t n, const float* rot, const float* trans, float w,
                                    float thresh) {
    uint32_t cnt = 0;
    for (uint32_t c = 0; c < n; c++) {
        const BFEntryJ& e = corr[c];
        if (e.imgIdx_i == BF_INVALID_IMAGE) continue;
        const m4 TI = poseToMatrix(ld3(rot + 3 * e.imgIdx_i), ld3(trans + 3 * e.imgIdx_i));
        const m4 TJ = poseToMatrix(ld3(rot + 3 * e.imgIdx_j), ld3(trans + 3 * e.imgIdx_j));
        const f3 d = w * fabs3(xform(TI, ld3(e.pos_i)) - xform(TJ, ld3(e.pos_j)));
        if (std::max(d.z, std::max(d.x, d.y)) > thresh) cnt++;
    }
    return cnt;
}

// VerifyTrajectoryCU_Kernel (SiftGPU/SIFTImageManager.cu:1036-1127) / computeProjError (:418-487)
int or_verify_trajectory(const int* valid, const float* Tall, const BFCachedFrame* cache, const ORVerifyParams* p,
                         float* pairStats) {
    const uint32_t N = p->numImages, W = p->width, H = p->height;
    if (N < 2) return 0;  // VerifyTrajectoryCU: numImages < 2 -> 0
    m4 K{};
    for (float& x : K.e) x = 0.0f;
    K.e[0] = p->intrinsics[0]; K.e[2] = p->intrinsics[2]; K.e[5] = p->intrinsics[1]; K.e[6] = p->intrinsics[3];
    K.e[10] = 1.0f; K.e[15] = 1.0f;
    auto mv4 = [](const m4& m, const float* v, float* o) {  // float4x4 * float4 (cuda_SimpleMatrixUtil.h:925-933)
        const float* e = m.e;
        for (int r = 0; r < 4; r++) o[r] = e[4 * r] * v[0] + e[4 * r + 1] * v[1] + e[4 * r + 2] * v[2] + e[4 * r + 3] * v[3];
    };
    auto projErr = [&](uint32_t idx, const m4& tr, const BFCachedFrame& in, const BFCachedFrame& model, float out[3]) {
        out[0] = out[1] = out[2] = 0.0f;
        const float* pIn = in.campos + 4 * (size_t)idx;
        float nIn[4] = {in.normals[4 * idx], in.normals[4 * idx + 1], in.normals[4 * idx + 2], 0.0f};
        const float dIn = in.depth[idx];
        if (!(pIn[0] != MINF && nIn[0] != MINF && dIn >= p->depthMin && dIn <= p->depthMax)) return;
        float pT[4], nT[4];
        mv4(tr, pIn, pT);
        mv4(tr, nIn, nT);
        const f3 q = xform(K, f3{pT[0], pT[1], pT[2]});
        const int sx = f2i(std::round(q.x / q.z)), sy = f2i(std::round(q.y / q.z));
        if (!(sx >= 0 && sy >= 0 && sx < (int)W && sy < (int)H)) return;
        const size_t t = (size_t)sy * W + (size_t)sx;
        const float* pTg = model.campos + 4 * t;
        const float* nTg = model.normals + 4 * t;
        if (!(pTg[0] != MINF && nTg[0] != MINF)) return;
        const float dx = pT[0] - pTg[0], dy = pT[1] - pTg[1], dz = pT[2] - pTg[2], dw = pT[3] - pTg[3];
        const float d = std::sqrt(dx * dx + dy * dy + dz * dz + dw * dw);
        const float dN = nT[0] * nTg[0] + nT[1] * nTg[1] + nT[2] * nTg[2];
        const float tgtDepth = model.depth[t];
        if (!(tgtDepth >= p->depthMin && tgtDepth <= p->depthMax)) return;
        const bool bad = (tgtDepth != MINF && pT[2] < tgtDepth) && d > p->distThresh;
        if (!((dN >= p->normalThresh && d <= p->distThresh) || bad)) return;
        const float camZ = (pT[2] - p->depthMin) / (p->depthMax - p->depthMin);
        out[0] = d;
        out[1] = std::max(0.0f, 0.5f * ((1.0f - d / p->distThresh) + (1.0f - camZ)));
        out[2] = 1.0f;
    };
    int ok = 1;
    constexpr uint32_t WGS = 256;
    std::vector<float> part(3 * WGS);
    for (uint32_t i = 0; i < N; i++)
        for (uint32_t j = i + 1; j < N; j++) {
            if (valid[i] == 0 || valid[j] == 0) continue;
            m4 Ti, Tj;
            std::memcpy(Ti.e, Tall + 16 * (size_t)i, 64);
            std::memcpy(Tj.e, Tall + 16 * (size_t)j, 64);
            const m4 tr = matmul(inverse(Tj), Ti);  // d_trajectory[img1].getInverse() * d_trajectory[img0]
            const m4 trInv = inverse(tr);
            for (uint32_t t = 0; t < WGS; t++) {
                float sr = 0, sw = 0, sn = 0;
                for (uint32_t idx = t; idx < W * H; idx += WGS) {
                    float a[3], b[3];
                    projErr(idx, tr, cache[i], cache[j], a);
                    projErr(idx, trInv, cache[j], cache[i], b);
                    sr += a[0] + b[0];
                    sw += a[1] + b[1];
                    sn += a[2] + b[2];
                }
                part[3 * t] = sr; part[3 * t + 1] = sw; part[3 * t + 2] = sn;
            }
            float s[3];
            for (int q = 0; q < 3; q++) {
                float wv[4];
                for (uint32_t w = 0; w < 4; w++) {  // shfl_down tree: lane 0 of each wave
                    float v[64];
                    for (int l = 0; l < 64; l++) v[l] = part[3 * (64 * w + l) + q];
                    for (int off = 32; off > 0; off >>= 1)
                        for (int l = 0; l < off; l++) v[l] += v[l + off];
                    wv[w] = v[0];
                }
                s[q] = ((wv[0] + wv[1]) + wv[2]) + wv[3];
            }
            if (pairStats)
                for (int q = 0; q < 3; q++) pairStats[((size_t)i * N + j) * 3 + q] = s[q];
            const float err = s[0] / s[1];
            const float corr = 0.5f * s[2] / (float)(W * H);
            if (corr < p->corrThresh || err > p->errThresh || std::isnan(err)) ok = 0;
        }
    return ok;
}

}  // extern "C"
