// image_codec.cpp — JPEG / PNG decoders of the `.sens` colour stream (see image_codec.h).
#include "image_codec.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "bf_runtime.h"

namespace bf {

namespace {

// ================================ JPEG (ITU-T T.81) ================================================
// zig-zag index -> natural (row-major) index (T.81 Figure A.6); 16 extra entries absorb a corrupt
// run that overshoots coefficient 63, as the IJG table does
const uint8_t kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

[[noreturn]] void corrupt(const char* what) { throw Error(BF_ERR_IO, std::string("JPEG: ") + what); }

// Canonical Huffman table (T.81 Annex C / F.2.2.3) with a 9-bit direct lookup for short codes.
struct Huff {
    bool defined = false;
    int32_t mincode[17], maxcode[17], valptr[17];
    uint8_t vals[256];
    uint16_t fast[512];  // (length << 8) | value for codes of <= 9 bits, 0 otherwise
    void build(const uint8_t bits[17], const uint8_t* huffval, int nvals) {
        std::memcpy(vals, huffval, (size_t)nvals);
        std::memset(fast, 0, sizeof(fast));
        int32_t code = 0;
        int k = 0;
        for (int l = 1; l <= 16; l++) {
            valptr[l] = k;
            mincode[l] = code;
            for (int i = 0; i < bits[l]; i++, k++, code++) {
                if (code >= (1 << l)) corrupt("bad Huffman table");
                if (l <= 9) {
                    const int shift = 9 - l;
                    for (int s = 0; s < (1 << shift); s++) fast[(code << shift) | s] = (uint16_t)((l << 8) | vals[k]);
                }
            }
            maxcode[l] = bits[l] ? code - 1 : -1;
            code <<= 1;
        }
        defined = true;
    }
};

// Entropy-coded segment reader: MSB-aligned 32-bit accumulator, 0xFF00 unstuffing; at a marker or
// the end of the data it feeds zero bytes (lookahead), and a segment whose decode consumed any of
// them is corrupt (the IJG decoder warns "premature end of data segment" and continues on zeros;
// a .sens frame that short is refused instead).
struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint32_t acc = 0;
    int n = 0;
    bool atMarker = false;
    int pad = 0;  // zero bytes fed past the segment's data
    bool overran() const { return pad * 8 > n; }
    void fill() {
        while (n <= 24) {
            uint32_t b = 0;
            if (atMarker || p >= end) {
                pad++;
            } else {
                b = *p;
                if (b == 0xFF) {
                    const uint32_t nx = (p + 1 < end) ? p[1] : 0xD9;
                    if (nx == 0x00) {
                        p += 2;
                    } else {
                        atMarker = true;
                        b = 0;
                        pad++;
                    }
                } else {
                    p++;
                }
            }
            acc |= b << (24 - n);
            n += 8;
        }
    }
    void skip(int k) {
        acc <<= k;
        n -= k;
    }
    int decode(const Huff& h) {
        fill();
        const uint16_t f = h.fast[acc >> 23];
        if (f) {
            skip(f >> 8);
            return f & 0xFF;
        }
        for (int l = 10; l <= 16; l++) {
            const int32_t code = (int32_t)(acc >> (32 - l));
            if (h.maxcode[l] >= 0 && code <= h.maxcode[l] && code >= h.mincode[l]) {
                skip(l);
                return h.vals[h.valptr[l] + code - h.mincode[l]];
            }
        }
        corrupt("invalid Huffman code");
    }
    // RECEIVE + EXTEND (T.81 F.2.2.1, Figure F.12)
    int extend(int s) {
        if (s == 0) return 0;
        fill();
        int v = (int)(acc >> (32 - s));
        skip(s);
        if (v < (1 << (s - 1))) v -= (1 << s) - 1;
        return v;
    }
    // restart: drop the padding bits, consume the RSTn marker
    void restart() {
        if (overran()) corrupt("premature end of an entropy-coded segment");
        acc = 0;
        n = 0;
        pad = 0;
        atMarker = false;
        while (p + 1 < end) {
            if (p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7) {
                p += 2;
                return;
            }
            if (p[0] == 0xFF && p[1] != 0x00 && p[1] != 0xFF) return;  // another marker: leave it
            p++;
        }
    }
};

// IJG sample range limiting after the IDCT (jdmaster.c prepare_range_limit_table, used with
// RANGE_MASK 1023 by jidctint.c): x = value - 128 taken mod 1024
inline uint8_t idct_limit(int32_t x) {
    const int32_t i = x & 1023;
    if (i < 128) return (uint8_t)(i + 128);
    if (i < 512) return 255;
    if (i < 896) return 0;
    return (uint8_t)(i - 896);
}

// jidctint.c (IJG libjpeg 6b) jpeg_idct_islow: separable 8-point integer IDCT, CONST_BITS 13,
// PASS1_BITS 2, dequantization folded in; writes 8x8 samples at out (row stride `stride`)
constexpr int CONST_BITS = 13, PASS1_BITS = 2;
constexpr int32_t F_0_298631336 = 2446, F_0_390180644 = 3196, F_0_541196100 = 4433, F_0_765366865 = 6270,
                  F_0_899976223 = 7373, F_1_175875602 = 9633, F_1_501321110 = 12299, F_1_847759065 = 15137,
                  F_1_961570560 = 16069, F_2_053119869 = 16819, F_2_562915447 = 20995, F_3_072711026 = 25172;
inline int64_t descale(int64_t x, int n) { return (x + ((int64_t)1 << (n - 1))) >> n; }

void idct_islow(const int16_t* coef, const uint16_t* q, uint8_t* out, size_t stride) {
    int64_t ws[64];
    for (int c = 0; c < 8; c++) {
        const int16_t* in = coef + c;
        const uint16_t* qq = q + c;
        int64_t* w = ws + c;
        if (in[8] == 0 && in[16] == 0 && in[24] == 0 && in[32] == 0 && in[40] == 0 && in[48] == 0 && in[56] == 0) {
            const int64_t dc = ((int64_t)in[0] * qq[0]) * (1 << PASS1_BITS);
            for (int r = 0; r < 8; r++) w[8 * r] = dc;
            continue;
        }
        int64_t z2 = (int64_t)in[16] * qq[16], z3 = (int64_t)in[48] * qq[48];
        int64_t z1 = (z2 + z3) * F_0_541196100;
        int64_t tmp2 = z1 + z3 * (-F_1_847759065);
        int64_t tmp3 = z1 + z2 * F_0_765366865;
        z2 = (int64_t)in[0] * qq[0];
        z3 = (int64_t)in[32] * qq[32];
        int64_t tmp0 = (z2 + z3) * (1 << CONST_BITS);
        int64_t tmp1 = (z2 - z3) * (1 << CONST_BITS);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = (int64_t)in[56] * qq[56];
        tmp1 = (int64_t)in[40] * qq[40];
        tmp2 = (int64_t)in[24] * qq[24];
        tmp3 = (int64_t)in[8] * qq[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F_1_175875602;
        tmp0 *= F_0_298631336;
        tmp1 *= F_2_053119869;
        tmp2 *= F_3_072711026;
        tmp3 *= F_1_501321110;
        z1 *= -F_0_899976223;
        z2 *= -F_2_562915447;
        z3 *= -F_1_961570560;
        z4 *= -F_0_390180644;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        constexpr int S = CONST_BITS - PASS1_BITS;
        w[0] = descale(tmp10 + tmp3, S);
        w[56] = descale(tmp10 - tmp3, S);
        w[8] = descale(tmp11 + tmp2, S);
        w[48] = descale(tmp11 - tmp2, S);
        w[16] = descale(tmp12 + tmp1, S);
        w[40] = descale(tmp12 - tmp1, S);
        w[24] = descale(tmp13 + tmp0, S);
        w[32] = descale(tmp13 - tmp0, S);
    }
    for (int r = 0; r < 8; r++) {
        const int64_t* w = ws + 8 * r;
        uint8_t* o = out + (size_t)r * stride;
        constexpr int S = CONST_BITS + PASS1_BITS + 3;
        if (w[1] == 0 && w[2] == 0 && w[3] == 0 && w[4] == 0 && w[5] == 0 && w[6] == 0 && w[7] == 0) {
            const uint8_t v = idct_limit((int32_t)descale(w[0], PASS1_BITS + 3));
            for (int c = 0; c < 8; c++) o[c] = v;
            continue;
        }
        int64_t z2 = w[2], z3 = w[6];
        int64_t z1 = (z2 + z3) * F_0_541196100;
        int64_t tmp2 = z1 + z3 * (-F_1_847759065);
        int64_t tmp3 = z1 + z2 * F_0_765366865;
        int64_t tmp0 = (w[0] + w[4]) * (1 << CONST_BITS);
        int64_t tmp1 = (w[0] - w[4]) * (1 << CONST_BITS);
        const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = w[7];
        tmp1 = w[5];
        tmp2 = w[3];
        tmp3 = w[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        int64_t z4 = tmp1 + tmp3;
        const int64_t z5 = (z3 + z4) * F_1_175875602;
        tmp0 *= F_0_298631336;
        tmp1 *= F_2_053119869;
        tmp2 *= F_3_072711026;
        tmp3 *= F_1_501321110;
        z1 *= -F_0_899976223;
        z2 *= -F_2_562915447;
        z3 *= -F_1_961570560;
        z4 *= -F_0_390180644;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        o[0] = idct_limit((int32_t)descale(tmp10 + tmp3, S));
        o[7] = idct_limit((int32_t)descale(tmp10 - tmp3, S));
        o[1] = idct_limit((int32_t)descale(tmp11 + tmp2, S));
        o[6] = idct_limit((int32_t)descale(tmp11 - tmp2, S));
        o[2] = idct_limit((int32_t)descale(tmp12 + tmp1, S));
        o[5] = idct_limit((int32_t)descale(tmp12 - tmp1, S));
        o[3] = idct_limit((int32_t)descale(tmp13 + tmp0, S));
        o[4] = idct_limit((int32_t)descale(tmp13 - tmp0, S));
    }
}

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;     // Huffman table selectors of the current scan
    int pred = 0;           // DC predictor
    uint32_t dw = 0, dh = 0;        // downsampled size ceil(W h / Hmax) x ceil(H v / Vmax)
    uint32_t pw = 0, ph = 0;        // plane size (whole MCUs)
    std::vector<uint8_t> plane;     // reconstructed samples
};

inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
inline uint32_t div_ceil(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// Upsampled component row y of width 2*dw (or dw) -> full-resolution samples, as jdsample.c
// (h2v1_fancy_upsample, h1v2_fancy_upsample, h2v2_fancy_upsample, int_upsample); the context rows
// above the first / below the last downsampled row are copies of that row (jdmainct.c
// set_bottom_pointers / the xbuffer wraparound at the image top).
void upsample_row(const Component& c, int Hmax, int Vmax, uint32_t y, uint8_t* out) {
    const int hf = Hmax / c.h, vf = Vmax / c.v;
    const uint32_t dw = c.dw;
    auto row = [&](int64_t r) -> const uint8_t* {
        r = std::max<int64_t>(0, std::min<int64_t>(r, (int64_t)c.dh - 1));
        return c.plane.data() + (size_t)r * c.pw;
    };
    if (hf == 1 && vf == 1) {
        std::memcpy(out, row(y), dw);
    } else if (hf == 2 && vf == 1) {
        const uint8_t* in = row(y);
        if (dw <= 2) {
            for (uint32_t x = 0; x < dw; x++) out[2 * x] = out[2 * x + 1] = in[x];
            return;
        }
        int v = in[0];
        out[0] = (uint8_t)v;
        out[1] = (uint8_t)((v * 3 + in[1] + 2) >> 2);
        for (uint32_t x = 1; x + 1 < dw; x++) {
            v = in[x] * 3;
            out[2 * x] = (uint8_t)((v + in[x - 1] + 1) >> 2);
            out[2 * x + 1] = (uint8_t)((v + in[x + 1] + 2) >> 2);
        }
        v = in[dw - 1];
        out[2 * (dw - 1)] = (uint8_t)((v * 3 + in[dw - 2] + 1) >> 2);
        out[2 * (dw - 1) + 1] = (uint8_t)v;
    } else if (hf == 1 && vf == 2) {
        const uint32_t r = y / 2;
        const bool below = (y & 1) != 0;
        const uint8_t* in0 = row(r);
        const uint8_t* in1 = row(below ? (int64_t)r + 1 : (int64_t)r - 1);
        const int bias = below ? 2 : 1;
        for (uint32_t x = 0; x < dw; x++) out[x] = (uint8_t)((in0[x] * 3 + in1[x] + bias) >> 2);
    } else if (hf == 2 && vf == 2) {
        const uint32_t r = y / 2;
        const bool below = (y & 1) != 0;
        const uint8_t* in0 = row(r);
        const uint8_t* in1 = row(below ? (int64_t)r + 1 : (int64_t)r - 1);
        if (dw <= 2) {
            for (uint32_t x = 0; x < dw; x++) out[2 * x] = out[2 * x + 1] = in0[x];
            return;
        }
        int thiscol = in0[0] * 3 + in1[0];
        int nextcol = in0[1] * 3 + in1[1];
        out[0] = (uint8_t)((thiscol * 4 + 8) >> 4);
        out[1] = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
        int lastcol = thiscol;
        thiscol = nextcol;
        for (uint32_t x = 1; x + 1 < dw; x++) {
            nextcol = in0[x + 1] * 3 + in1[x + 1];
            out[2 * x] = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
            out[2 * x + 1] = (uint8_t)((thiscol * 3 + nextcol + 7) >> 4);
            lastcol = thiscol;
            thiscol = nextcol;
        }
        out[2 * (dw - 1)] = (uint8_t)((thiscol * 3 + lastcol + 8) >> 4);
        out[2 * (dw - 1) + 1] = (uint8_t)((thiscol * 4 + 7) >> 4);
    } else {  // integral factors: replication (int_upsample)
        const uint8_t* in = row(y / (uint32_t)vf);
        for (uint32_t x = 0; x < dw; x++)
            for (int k = 0; k < hf; k++) out[x * hf + k] = in[x];
    }
}

// jdcolor.c build_ycc_rgb_table (SCALEBITS 16): R = Y + 1.402 Cr, G = Y - 0.34414 Cb - 0.71414 Cr,
// B = Y + 1.772 Cb in fixed point, clamped to [0, 255]
struct YccTables {
    int crR[256], cbB[256];
    int32_t crG[256], cbG[256];
    YccTables() {
        constexpr int SB = 16;
        constexpr int32_t HALF = 1 << (SB - 1);
        auto fix = [](double x) { return (int32_t)(x * (1 << SB) + 0.5); };
        for (int i = 0; i < 256; i++) {
            const int32_t x = i - 128;
            crR[i] = (int)((fix(1.40200) * x + HALF) >> SB);
            cbB[i] = (int)((fix(1.77200) * x + HALF) >> SB);
            crG[i] = -fix(0.71414) * x;
            cbG[i] = -fix(0.34414) * x + HALF;
        }
    }
};
inline uint8_t clamp255(int v) { return (uint8_t)std::min(255, std::max(0, v)); }

}  // namespace

DecodedImage jpeg_decode(const uint8_t* data, size_t n, uint32_t expectW, uint32_t expectH) {
    if (n < 4 || data[0] != 0xFF || data[1] != 0xD8) corrupt("missing SOI");
    uint16_t q[4][64];  // natural order
    bool qdef[4] = {false, false, false, false};
    Huff dcT[4], acT[4];
    std::vector<Component> comp;
    uint32_t W = 0, H = 0, restartInterval = 0;
    int Hmax = 1, Vmax = 1;
    bool frame = false, sawScan = false, adobeRGB = false;
    int adobeTransform = -1;
    size_t pos = 2;
    while (pos + 4 <= n) {
        if (data[pos] != 0xFF) corrupt("marker expected");
        const uint8_t m = data[pos + 1];
        if (m == 0xFF) {  // fill byte
            pos++;
            continue;
        }
        if (m == 0xD9) break;  // EOI
        if (m >= 0xD0 && m <= 0xD7) {
            pos += 2;
            continue;
        }
        const uint16_t len = be16(data + pos + 2);
        if (len < 2 || pos + 2 + len > n) corrupt("truncated segment");
        const uint8_t* s = data + pos + 4;
        const size_t slen = len - 2;
        if (m == 0xDB) {  // DQT
            size_t k = 0;
            while (k < slen) {
                const int pq = s[k] >> 4, tq = s[k] & 15;
                if (tq > 3) corrupt("bad DQT");
                k++;
                for (int i = 0; i < 64; i++) {
                    if (k + (pq ? 2 : 1) > slen) corrupt("truncated DQT");
                    q[tq][kNatural[i]] = pq ? be16(s + k) : s[k];
                    k += pq ? 2 : 1;
                }
                qdef[tq] = true;
            }
        } else if (m == 0xC4) {  // DHT
            size_t k = 0;
            while (k + 17 <= slen) {
                const int tc = s[k] >> 4, th = s[k] & 15;
                if (tc > 1 || th > 3) corrupt("bad DHT");
                uint8_t bits[17] = {0};
                int total = 0;
                for (int l = 1; l <= 16; l++) total += (bits[l] = s[k + l]);
                if (total > 256 || k + 17 + total > slen) corrupt("bad DHT counts");
                (tc == 0 ? dcT[th] : acT[th]).build(bits, s + k + 17, total);
                k += 17 + total;
            }
        } else if (m == 0xDD) {  // DRI
            if (slen < 2) corrupt("bad DRI");
            restartInterval = be16(s);
        } else if (m == 0xEE && slen >= 12 && std::memcmp(s, "Adobe", 5) == 0) {
            adobeTransform = s[11];
        } else if (m == 0xC0 || m == 0xC1) {  // SOF0 / SOF1: sequential Huffman
            if (frame) corrupt("second frame");
            if (slen < 6 || s[0] != 8) throw Error(BF_ERR_ARG, "JPEG: only 8-bit samples are supported");
            H = be16(s + 1);
            W = be16(s + 3);
            const int nc = s[5];
            if (W == 0 || H == 0) throw Error(BF_ERR_ARG, "JPEG: DNL-defined height is not supported");
            if ((uint64_t)W * H > kMaxImagePixels) throw Error(BF_ERR_ARG, "JPEG: image dimensions exceed the decoder's limit");
            if ((expectW && W != expectW) || (expectH && H != expectH)) corrupt("frame size differs from the container's");
            if ((nc != 1 && nc != 3) || slen < 6 + 3 * (size_t)nc) throw Error(BF_ERR_ARG, "JPEG: 1 or 3 components supported");
            comp.resize(nc);
            for (int c = 0; c < nc; c++) {
                comp[c].id = s[6 + 3 * c];
                comp[c].h = s[7 + 3 * c] >> 4;
                comp[c].v = s[7 + 3 * c] & 15;
                comp[c].tq = s[8 + 3 * c];
                if (comp[c].h < 1 || comp[c].h > 4 || comp[c].v < 1 || comp[c].v > 4 || comp[c].tq > 3)
                    corrupt("bad component");
                Hmax = std::max(Hmax, comp[c].h);
                Vmax = std::max(Vmax, comp[c].v);
            }
            for (Component& c : comp) {
                if (Hmax % c.h || Vmax % c.v) throw Error(BF_ERR_ARG, "JPEG: non-integral sampling ratios");
            }
            const uint32_t mx = div_ceil(W, 8u * Hmax), my = div_ceil(H, 8u * Vmax);
            for (Component& c : comp) {
                c.dw = div_ceil(W * c.h, Hmax);
                c.dh = div_ceil(H * c.v, Vmax);
                c.pw = mx * c.h * 8;
                c.ph = my * c.v * 8;
                c.plane.assign((size_t)c.pw * c.ph, 0);
            }
            frame = true;
        } else if ((m >= 0xC2 && m <= 0xC3) || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC)) {
            throw Error(BF_ERR_ARG, "JPEG: progressive / lossless / arithmetic-coded streams are not supported");
        } else if (m == 0xDA) {  // SOS + entropy-coded data
            if (!frame) corrupt("scan before frame");
            if (slen < 1) corrupt("bad SOS");
            const int ns = s[0];
            if (ns < 1 || ns > (int)comp.size() || slen < 1 + 2 * (size_t)ns + 3) corrupt("bad SOS");
            std::vector<Component*> sc;
            for (int i = 0; i < ns; i++) {
                Component* c = nullptr;
                for (Component& cc : comp)
                    if (cc.id == s[1 + 2 * i]) c = &cc;
                if (!c) corrupt("scan component not in frame");
                c->td = s[2 + 2 * i] >> 4;
                c->ta = s[2 + 2 * i] & 15;
                if (c->td > 3 || c->ta > 3 || !dcT[c->td].defined || !acT[c->ta].defined || !qdef[c->tq])
                    corrupt("scan references an undefined table");
                c->pred = 0;
                sc.push_back(c);
            }
            Bits br{data + pos + 2 + len, data + n};
            int16_t blk[64];
            auto decode_block = [&](Component& c, uint32_t bx, uint32_t by) {
                std::memset(blk, 0, sizeof(blk));
                const int t = br.decode(dcT[c.td]);
                if (t > 11) corrupt("bad DC category");
                c.pred += br.extend(t);
                blk[0] = (int16_t)c.pred;
                for (int k = 1; k < 64;) {
                    const int rs = br.decode(acT[c.ta]);
                    const int r = rs >> 4, sz = rs & 15;
                    if (sz) {
                        k += r;
                        blk[kNatural[k]] = (int16_t)br.extend(sz);
                        k++;
                    } else if (r == 15) {
                        k += 16;
                    } else {
                        break;
                    }
                }
                if (bx * 8 < c.pw && by * 8 < c.ph)
                    idct_islow(blk, q[c.tq], c.plane.data() + (size_t)by * 8 * c.pw + bx * 8, c.pw);
            };
            uint32_t units, unitsX;
            if (ns == 1) {  // non-interleaved: the data unit is one block of the component (T.81 A.2.2)
                unitsX = div_ceil(sc[0]->dw, 8);
                units = unitsX * div_ceil(sc[0]->dh, 8);
            } else {
                unitsX = div_ceil(W, 8u * Hmax);
                units = unitsX * div_ceil(H, 8u * Vmax);
            }
            for (uint32_t u = 0; u < units; u++) {
                if (restartInterval && u > 0 && u % restartInterval == 0) {
                    br.restart();
                    for (Component* c : sc) c->pred = 0;
                }
                const uint32_t ux = u % unitsX, uy = u / unitsX;
                if (ns == 1) {
                    decode_block(*sc[0], ux, uy);
                } else {
                    for (Component* c : sc)
                        for (int by = 0; by < c->v; by++)
                            for (int bx = 0; bx < c->h; bx++) decode_block(*c, ux * c->h + bx, uy * c->v + by);
                }
            }
            if (br.overran()) corrupt("premature end of the entropy-coded segment");
            // continue at the first marker after the entropy-coded segment
            size_t p = (size_t)(br.p - data);
            while (p + 1 < n && !(data[p] == 0xFF && data[p + 1] != 0x00 && !(data[p + 1] >= 0xD0 && data[p + 1] <= 0xD7)))
                p++;
            pos = p;
            sawScan = true;
            continue;
        }
        pos += 2 + len;
    }
    if (!frame || !sawScan) corrupt("no image data");
    (void)adobeRGB;
    DecodedImage img;
    img.width = W;
    img.height = H;
    img.rgbx.resize((size_t)W * H * 4);
    const uint32_t rowCap = (uint32_t)Hmax * (comp[0].pw + 8);
    std::vector<uint8_t> r0(rowCap), r1(rowCap), r2(rowCap);
    if (comp.size() == 1) {
        for (uint32_t y = 0; y < H; y++) {
            upsample_row(comp[0], Hmax, Vmax, y, r0.data());
            uint8_t* o = img.rgbx.data() + (size_t)y * W * 4;
            for (uint32_t x = 0; x < W; x++) {
                o[4 * x] = o[4 * x + 1] = o[4 * x + 2] = r0[x];
                o[4 * x + 3] = 255;
            }
        }
        return img;
    }
    // RGB when an Adobe marker says "no transform" or the component ids spell R, G, B (jdapimin.c
    // default_decompress_parms); YCbCr otherwise (JFIF)
    const bool rgb = adobeTransform == 0 || (adobeTransform < 0 && comp[0].id == 'R' && comp[1].id == 'G' && comp[2].id == 'B');
    static const YccTables T;
    for (uint32_t y = 0; y < H; y++) {
        upsample_row(comp[0], Hmax, Vmax, y, r0.data());
        upsample_row(comp[1], Hmax, Vmax, y, r1.data());
        upsample_row(comp[2], Hmax, Vmax, y, r2.data());
        uint8_t* o = img.rgbx.data() + (size_t)y * W * 4;
        for (uint32_t x = 0; x < W; x++) {
            if (rgb) {
                o[4 * x] = r0[x];
                o[4 * x + 1] = r1[x];
                o[4 * x + 2] = r2[x];
            } else {
                const int Y = r0[x], cb = r1[x], cr = r2[x];
                o[4 * x] = clamp255(Y + T.crR[cr]);
                o[4 * x + 1] = clamp255(Y + (int)((T.cbG[cb] + T.crG[cr]) >> 16));
                o[4 * x + 2] = clamp255(Y + T.cbB[cb]);
            }
            o[4 * x + 3] = 255;
        }
    }
    return img;
}

// ================================ PNG (ISO/IEC 15948) =============================================
namespace {
[[noreturn]] void png_corrupt(const char* what) { throw Error(BF_ERR_IO, std::string("PNG: ") + what); }
inline uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
inline uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return (uint8_t)(pb <= pc ? b : c);
}
}  // namespace

DecodedImage png_decode(const uint8_t* data, size_t n, uint32_t expectW, uint32_t expectH) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    if (n < 8 || std::memcmp(data, sig, 8) != 0) png_corrupt("bad signature");
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    size_t pos = 8;
    bool end = false;
    while (pos + 12 <= n && !end) {
        const uint32_t len = be32(data + pos);
        if (pos + 12 + (size_t)len > n) png_corrupt("truncated chunk");
        const uint8_t* type = data + pos + 4;
        const uint8_t* d = data + pos + 8;
        if (std::memcmp(type, "IHDR", 4) == 0) {
            if (len < 13) png_corrupt("bad IHDR");
            W = be32(d);
            H = be32(d + 4);
            depth = d[8];
            ctype = d[9];
            interlace = d[12];
            if (d[10] != 0 || d[11] != 0) png_corrupt("unknown compression / filter method");
        } else if (std::memcmp(type, "PLTE", 4) == 0) {
            plte.assign(d, d + len);
        } else if (std::memcmp(type, "IDAT", 4) == 0) {
            idat.insert(idat.end(), d, d + len);
        } else if (std::memcmp(type, "IEND", 4) == 0) {
            end = true;
        }
        pos += 12 + len;
    }
    if (W == 0 || H == 0 || ctype < 0) png_corrupt("missing IHDR");
    // ISO/IEC 15948 caps each dimension at 2^31 - 1; the pixel cap keeps (stride + 1) * H and the
    // RGBX size far from size_t overflow whatever the file claims
    if (W > 0x7FFFFFFFu || H > 0x7FFFFFFFu || (uint64_t)W * H > kMaxImagePixels)
        throw Error(BF_ERR_ARG, "PNG: image dimensions exceed the decoder's limit");
    if ((expectW && W != expectW) || (expectH && H != expectH)) png_corrupt("image size differs from the container's");
    if (depth != 8) throw Error(BF_ERR_ARG, "PNG: only 8-bit channels are supported");
    if (interlace != 0) throw Error(BF_ERR_ARG, "PNG: interlaced images are not supported");
    int ch = 0;
    switch (ctype) {
        case 0: ch = 1; break;  // grey
        case 2: ch = 3; break;  // RGB
        case 3: ch = 1; break;  // palette
        case 4: ch = 2; break;  // grey + alpha
        case 6: ch = 4; break;  // RGBA
        default: png_corrupt("bad colour type");
    }
    if (ctype == 3 && plte.size() < 3) png_corrupt("palette image without PLTE");
    const size_t stride = (size_t)W * ch;
    std::vector<uint8_t> raw((stride + 1) * H);
    uLongf rawLen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawLen, idat.data(), (uLong)idat.size()) != Z_OK || rawLen != raw.size())
        png_corrupt("zlib stream corrupt");
    std::vector<uint8_t> cur(stride), prev(stride, 0);
    DecodedImage img;
    img.width = W;
    img.height = H;
    img.rgbx.resize((size_t)W * H * 4);
    for (uint32_t y = 0; y < H; y++) {
        const uint8_t ft = raw[y * (stride + 1)];
        const uint8_t* in = raw.data() + y * (stride + 1) + 1;
        for (size_t i = 0; i < stride; i++) {
            const int a = i >= (size_t)ch ? cur[i - ch] : 0, b = prev[i], c = i >= (size_t)ch ? prev[i - ch] : 0;
            int v = in[i];
            switch (ft) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: png_corrupt("bad filter type");
            }
            cur[i] = (uint8_t)v;
        }
        uint8_t* o = img.rgbx.data() + (size_t)y * W * 4;
        for (uint32_t x = 0; x < W; x++) {
            const uint8_t* p = cur.data() + (size_t)x * ch;
            if (ctype == 3) {
                const size_t k = (size_t)p[0] * 3;
                if (k + 2 >= plte.size()) png_corrupt("palette index out of range");
                o[4 * x] = plte[k];
                o[4 * x + 1] = plte[k + 1];
                o[4 * x + 2] = plte[k + 2];
            } else if (ch <= 2) {
                o[4 * x] = o[4 * x + 1] = o[4 * x + 2] = p[0];
            } else {
                o[4 * x] = p[0];
                o[4 * x + 1] = p[1];
                o[4 * x + 2] = p[2];
            }
            o[4 * x + 3] = 255;
        }
        std::swap(cur, prev);
    }
    return img;
}

}  // namespace bf
