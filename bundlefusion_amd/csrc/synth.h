// synth.h — seeded analytic RGB-D scene (SURVEY.md §8(d) "concrete synthetic inputs"):
// a 6x5x3 m box room with boxes and spheres, a 0.25 m checker colour per object, a smooth
// Lissajous camera loop at 1.5 m height, and the structured-light depth noise model
// sigma(d) = 0.0012 + 0.0019 (d - 0.4)^2 quantised to 1 mm (the .sens ushort/1000
// convention, SensorDataReader.cpp:104-107). World frame: y points down (floor y = 0),
// cameras look along +z with x right / y down, as the Kinect convention of the reference.
// Shared by the GPU renderer (bench/tests) and its host twin.
#pragma once
#include "bf_math.h"
#include "../../include/bf/bf.h"

namespace bf {

BF_HD uint32_t pcg_hash(uint32_t v) {
    uint32_t state = v * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
BF_HD float u01(uint32_t h) { return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f); }

// ray o + t*d (d has camera z = 1 after rotation, so t is the camera depth)
BF_HD bool synth_trace(const BFSynthScene& sc, f3 o, f3 d, float& tHit, f3& pHit, f3& nHit, int& obj) {
    float best = 1e30f;
    int bestObj = -1;
    f3 bestN = mk3(0, 0, 0);
    // room interior: exit face of the AABB
    {
        float tx0 = (sc.roomMin[0] - o.x) / d.x, tx1 = (sc.roomMax[0] - o.x) / d.x;
        float ty0 = (sc.roomMin[1] - o.y) / d.y, ty1 = (sc.roomMax[1] - o.y) / d.y;
        float tz0 = (sc.roomMin[2] - o.z) / d.z, tz1 = (sc.roomMax[2] - o.z) / d.z;
        float ex = fmaxf(tx0, tx1), ey = fmaxf(ty0, ty1), ez = fmaxf(tz0, tz1);
        float t = fminf(ex, fminf(ey, ez));
        if (t > 0.0f && t < best) {
            best = t;
            if (t == ex) { bestObj = (tx1 > tx0) ? 1 : 0; bestN = mk3(tx1 > tx0 ? -1.0f : 1.0f, 0, 0); }
            else if (t == ey) { bestObj = (ty1 > ty0) ? 3 : 2; bestN = mk3(0, ty1 > ty0 ? -1.0f : 1.0f, 0); }
            else { bestObj = (tz1 > tz0) ? 5 : 4; bestN = mk3(0, 0, tz1 > tz0 ? -1.0f : 1.0f); }
        }
    }
    for (uint32_t k = 0; k < sc.numPrimitives && k < 64; k++) {
        const float* P = sc.prims[k];
        f3 c = mk3(P[1], P[2], P[3]);
        if (P[0] < 0.5f) {  // axis-aligned box, hit the entry face
            f3 lo = c - mk3(P[4], P[5], P[6]), hi = c + mk3(P[4], P[5], P[6]);
            float tx0 = (lo.x - o.x) / d.x, tx1 = (hi.x - o.x) / d.x;
            float ty0 = (lo.y - o.y) / d.y, ty1 = (hi.y - o.y) / d.y;
            float tz0 = (lo.z - o.z) / d.z, tz1 = (hi.z - o.z) / d.z;
            float nx = fminf(tx0, tx1), ny = fminf(ty0, ty1), nz = fminf(tz0, tz1);
            float tn = fmaxf(nx, fmaxf(ny, nz));
            float tf = fminf(fmaxf(tx0, tx1), fminf(fmaxf(ty0, ty1), fmaxf(tz0, tz1)));
            if (tn > 0.0f && tn <= tf && tn < best) {
                best = tn;
                bestObj = 6 + (int)k;
                if (tn == nx) bestN = mk3(d.x > 0 ? -1.0f : 1.0f, 0, 0);
                else if (tn == ny) bestN = mk3(0, d.y > 0 ? -1.0f : 1.0f, 0);
                else bestN = mk3(0, 0, d.z > 0 ? -1.0f : 1.0f);
            }
        } else {  // sphere
            f3 oc = o - c;
            float a = dot3(d, d), b = 2.0f * dot3(d, oc), cc = dot3(oc, oc) - P[4] * P[4];
            float disc = b * b - 4.0f * a * cc;
            if (disc >= 0.0f) {
                float t = (-b - sqrtf(disc)) / (2.0f * a);
                if (t > 0.0f && t < best) {
                    best = t;
                    bestObj = 6 + (int)k;
                    bestN = normalize3(o + d * t - c);
                }
            }
        }
    }
    if (bestObj < 0) return false;
    tHit = best;
    pHit = o + d * best;
    nHit = bestN;
    obj = bestObj;
    return true;
}

BF_HD void synth_color(const BFSynthScene& sc, int obj, f3 p, uint8_t rgb[3]) {
    float hue = obj < 6 ? (float)obj / 6.0f : sc.prims[obj - 6][7];
    int cx = (int)floorf(p.x / 0.25f), cy = (int)floorf(p.y / 0.25f), cz = (int)floorf(p.z / 0.25f);
    float v = ((cx + cy + cz) & 1) ? 1.0f : 0.55f;
    float s = 0.6f;
    float h6 = (hue - floorf(hue)) * 6.0f;
    int hi = (int)h6;
    float f = h6 - (float)hi;
    float pp = v * (1 - s), q = v * (1 - s * f), t = v * (1 - s * (1 - f));
    float r, g, b;
    switch (hi % 6) {
        case 0: r = v; g = t; b = pp; break;
        case 1: r = q; g = v; b = pp; break;
        case 2: r = pp; g = v; b = t; break;
        case 3: r = pp; g = q; b = v; break;
        case 4: r = t; g = pp; b = v; break;
        default: r = v; g = pp; b = q; break;
    }
    rgb[0] = (uint8_t)(r * 254.0f);
    rgb[1] = (uint8_t)(g * 254.0f);
    rgb[2] = (uint8_t)(b * 254.0f);
}

// sigma(d) = 0.0012 + 0.0019 (d - 0.4)^2, Box-Muller from a counter hash; 1 mm quantisation.
BF_HD float synth_noisy_depth(float d, uint32_t noiseSeed, uint32_t frame, uint32_t pix) {
    if (noiseSeed == 0) return d;
    uint32_t h1 = pcg_hash(noiseSeed * 0x9E3779B9u ^ pcg_hash(frame * 0x85EBCA6Bu ^ pcg_hash(pix)));
    uint32_t h2 = pcg_hash(h1 ^ 0x68E31DA4u);
    float u1 = u01(h1), u2 = u01(h2);
    float n = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
    float sigma = 0.0012f + 0.0019f * (d - 0.4f) * (d - 0.4f);
    float dn = d + sigma * n;
    return floorf(dn * 1000.0f + 0.5f) / 1000.0f;
}

BF_HD void synth_pixel(const BFSynthScene& sc, const BFMat4& T, const BFDepthCameraParams& cam, uint32_t noiseSeed, uint32_t frame,
                       uint32_t x, uint32_t y, float& depthOut, uint32_t& colorOut) {
    f3 dc = mk3(((float)x - cam.mx) / cam.fx, ((float)y - cam.my) / cam.fy, 1.0f);
    f3 o = mk3(T.m[3], T.m[7], T.m[11]);
    f3 d = xform4(T, dc, 0.0f);
    float t;
    f3 p, n;
    int obj;
    depthOut = -INFINITY;
    colorOut = 0xFF000000u;
    if (!synth_trace(sc, o, d, t, p, n, obj)) return;
    uint8_t rgb[3];
    synth_color(sc, obj, p, rgb);
    colorOut = (uint32_t)rgb[0] | ((uint32_t)rgb[1] << 8) | ((uint32_t)rgb[2] << 16) | 0xFF000000u;
    float dn = synth_noisy_depth(t, noiseSeed, frame, y * cam.imageWidth + x);
    if (dn < 0.1f || dn > 4.0f) return;
    depthOut = dn;
}

// camera->world pose of frame f: Lissajous loop, period 1000 frames (<= 2 cm, < 1 deg per frame)
inline void synth_pose(uint32_t frame, float T[16]) {
    const double th = 2.0 * 3.14159265358979323846 * (double)frame / 1000.0;
    const double px = 1.5 * sin(th), py = -1.5 + 0.15 * sin(3.0 * th), pz = 1.2 * sin(2.0 * th);
    const double yaw = th + 0.35 * sin(5.0 * th);
    const double pitch = 0.1 * sin(3.0 * th);
    const double cy = cos(yaw), sy = sin(yaw), cp = cos(pitch), sp = sin(pitch);
    // R = Ry(yaw) * Rx(pitch)
    const double R[9] = {cy, sy * sp, sy * cp, 0.0, cp, -sp, -sy, cy * sp, cy * cp};
    T[0] = (float)R[0]; T[1] = (float)R[1]; T[2] = (float)R[2]; T[3] = (float)px;
    T[4] = (float)R[3]; T[5] = (float)R[4]; T[6] = (float)R[5]; T[7] = (float)py;
    T[8] = (float)R[6]; T[9] = (float)R[7]; T[10] = (float)R[8]; T[11] = (float)pz;
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}

}  // namespace bf
