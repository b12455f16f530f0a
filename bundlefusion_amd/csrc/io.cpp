// io.cpp — `.sens` reader / writer and `zParameters*.txt` parser (see io.h).
#include "io.h"

#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <array>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <unordered_map>
#include <unordered_set>

#include "bf_runtime.h"
#include "image_codec.h"

namespace bf {

namespace {

template <class T>
void rd(FILE* f, T* v, size_t n = 1) {
    BF_REQUIRE(std::fread(v, sizeof(T), n, f) == n, BF_ERR_IO, "truncated .sens file");
}
template <class T>
void wr(FILE* f, const T* v, size_t n = 1) {
    BF_REQUIRE(std::fwrite(v, sizeof(T), n, f) == n, BF_ERR_IO, "write failed");
}

}  // namespace

// ---- reader: header, then a frame index (offsets only; payloads are read on demand) ----------
SensReader::SensReader(const std::string& path) {
    f_ = std::fopen(path.c_str(), "rb");
    BF_REQUIRE(f_ != nullptr, BF_ERR_IO, "cannot open " + path);
    BF_REQUIRE(fseeko(f_, 0, SEEK_END) == 0, BF_ERR_IO, "seek failed");
    const uint64_t fileSize = (uint64_t)ftello(f_);
    BF_REQUIRE(fseeko(f_, 0, SEEK_SET) == 0, BF_ERR_IO, "seek failed");
    rd(f_, &info_.version);
    BF_REQUIRE(info_.version == 4, BF_ERR_IO, "unsupported .sens version " + std::to_string(info_.version));
    uint64_t nameLen = 0;
    rd(f_, &nameLen);
    BF_REQUIRE(nameLen < (1u << 20), BF_ERR_IO, "corrupt sensor name length");
    std::string name(nameLen, '\0');
    if (nameLen) rd(f_, &name[0], nameLen);
    std::strncpy(info_.sensorName, name.c_str(), sizeof(info_.sensorName) - 1);
    rd(f_, info_.colorIntrinsic, 16);
    rd(f_, info_.colorExtrinsic, 16);
    rd(f_, info_.depthIntrinsic, 16);
    rd(f_, info_.depthExtrinsic, 16);
    rd(f_, &info_.colorCompression);
    rd(f_, &info_.depthCompression);
    rd(f_, &info_.colorWidth);
    rd(f_, &info_.colorHeight);
    rd(f_, &info_.depthWidth);
    rd(f_, &info_.depthHeight);
    rd(f_, &info_.depthShift);
    rd(f_, &info_.numFrames);
    BF_REQUIRE(info_.numFrames < (1ull << 32), BF_ERR_IO, "corrupt frame count");
    frames_.resize(info_.numFrames);
    for (uint64_t i = 0; i < info_.numFrames; i++) {
        Frame& fr = frames_[i];
        rd(f_, fr.camToWorld, 16);
        rd(f_, &fr.tsColor);
        rd(f_, &fr.tsDepth);
        rd(f_, &fr.colorBytes);
        rd(f_, &fr.depthBytes);
        fr.colorOffset = (uint64_t)ftello(f_);
        fr.depthOffset = fr.colorOffset + fr.colorBytes;
        BF_REQUIRE(fr.colorBytes <= fileSize && fr.depthBytes <= fileSize && fr.depthOffset + fr.depthBytes <= fileSize,
                   BF_ERR_IO, "truncated .sens file (frame " + std::to_string(i) + ")");
        BF_REQUIRE(fseeko(f_, (off_t)(fr.depthOffset + fr.depthBytes), SEEK_SET) == 0, BF_ERR_IO, "seek failed");
    }
}

SensReader::~SensReader() {
    if (f_) std::fclose(f_);
}

const SensReader::Frame& SensReader::frame(uint64_t i) const {
    BF_REQUIRE(i < frames_.size(), BF_ERR_ARG, "frame index out of range");
    return frames_[i];
}

void SensReader::pose(uint64_t i, float camToWorld[16]) const { std::memcpy(camToWorld, frame(i).camToWorld, 64); }

void SensReader::timestamps(uint64_t i, uint64_t* tsColor, uint64_t* tsDepth) const {
    if (tsColor) *tsColor = frame(i).tsColor;
    if (tsDepth) *tsDepth = frame(i).tsDepth;
}

void SensReader::depthU16(uint64_t i, uint16_t* out) {
    const Frame& fr = frame(i);
    const uint64_t n = (uint64_t)info_.depthWidth * info_.depthHeight;
    buf_.resize(fr.depthBytes);
    BF_REQUIRE(fseeko(f_, (off_t)fr.depthOffset, SEEK_SET) == 0, BF_ERR_IO, "seek failed");
    if (fr.depthBytes) rd(f_, buf_.data(), fr.depthBytes);
    if (info_.depthCompression == 0) {
        BF_REQUIRE(fr.depthBytes == 2 * n, BF_ERR_IO, "raw depth size mismatch");
        std::memcpy(out, buf_.data(), 2 * n);
    } else if (info_.depthCompression == 1) {
        uLongf len = (uLongf)(2 * n);
        const int z = uncompress(reinterpret_cast<Bytef*>(out), &len, buf_.data(), (uLong)fr.depthBytes);
        BF_REQUIRE(z == Z_OK && len == 2 * n, BF_ERR_IO, "zlib depth stream corrupt");
    } else {
        throw Error(BF_ERR_ARG, "unsupported depth compression " + std::to_string(info_.depthCompression) +
                                    " (occi needs the vendor codec)");
    }
}

// Colour frame -> RGBX (SensorDataReader.cpp:98-116: the reader decompresses the colour stream and
// widens it to 4 B per pixel, :111-113). Raw colour is RGB, 3 B per pixel; PNG (1) and JPEG (2)
// streams go through the decoders of image_codec.cpp. A decoded frame must have the header's size.
void SensReader::colorRGBX(uint64_t i, uint8_t* out) {
    const Frame& fr = frame(i);
    const uint64_t n = (uint64_t)info_.colorWidth * info_.colorHeight;
    buf_.resize(fr.colorBytes);
    BF_REQUIRE(fseeko(f_, (off_t)fr.colorOffset, SEEK_SET) == 0, BF_ERR_IO, "seek failed");
    if (fr.colorBytes) rd(f_, buf_.data(), fr.colorBytes);
    if (info_.colorCompression == 0) {
        BF_REQUIRE(fr.colorBytes == 3 * n, BF_ERR_IO, "raw colour size mismatch");
        for (uint64_t p = 0; p < n; p++) {
            out[4 * p + 0] = buf_[3 * p + 0];
            out[4 * p + 1] = buf_[3 * p + 1];
            out[4 * p + 2] = buf_[3 * p + 2];
            out[4 * p + 3] = 255;
        }
        return;
    }
    BF_REQUIRE(info_.colorCompression == 1 || info_.colorCompression == 2, BF_ERR_ARG,
               "unsupported colour compression " + std::to_string(info_.colorCompression));
    const uint32_t cw = info_.colorWidth, ch = info_.colorHeight;
    const DecodedImage img = info_.colorCompression == 2 ? jpeg_decode(buf_.data(), buf_.size(), cw, ch)
                                                         : png_decode(buf_.data(), buf_.size(), cw, ch);
    BF_REQUIRE(img.width == info_.colorWidth && img.height == info_.colorHeight, BF_ERR_IO,
               "decoded colour frame size differs from the header");
    std::memcpy(out, img.rgbx.data(), 4 * n);
}

// ---- writer ------------------------------------------------------------------------------------
SensWriter::SensWriter(const std::string& path, const BFSensInfo& info) : info_(info) {
    BF_REQUIRE(info.colorCompression >= 0 && info.colorCompression <= 2 && info.depthCompression >= 0 && info.depthCompression <= 2,
               BF_ERR_ARG, "unknown compression type");
    f_ = std::fopen(path.c_str(), "wb");
    BF_REQUIRE(f_ != nullptr, BF_ERR_IO, "cannot create " + path);
    const uint32_t version = 4;
    wr(f_, &version);
    const std::string name(info.sensorName, strnlen(info.sensorName, sizeof(info.sensorName)));
    const uint64_t nameLen = name.size();
    wr(f_, &nameLen);
    if (nameLen) wr(f_, name.data(), nameLen);
    wr(f_, info.colorIntrinsic, 16);
    wr(f_, info.colorExtrinsic, 16);
    wr(f_, info.depthIntrinsic, 16);
    wr(f_, info.depthExtrinsic, 16);
    wr(f_, &info.colorCompression);
    wr(f_, &info.depthCompression);
    wr(f_, &info.colorWidth);
    wr(f_, &info.colorHeight);
    wr(f_, &info.depthWidth);
    wr(f_, &info.depthHeight);
    wr(f_, &info.depthShift);
    numFramesPos_ = std::ftell(f_);
    const uint64_t zero = 0;
    wr(f_, &zero);
}

SensWriter::~SensWriter() {
    try {
        close();
    } catch (...) {
    }
}

void SensWriter::addCompressedFrame(const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth, const uint8_t* color,
                                    uint64_t colorBytes, const uint8_t* depth, uint64_t depthBytes) {
    BF_REQUIRE(f_ != nullptr, BF_ERR_STATE, "writer closed");
    BF_REQUIRE((color || colorBytes == 0) && (depth || depthBytes == 0), BF_ERR_ARG, "null frame payload");
    wr(f_, camToWorld, 16);
    wr(f_, &tsColor);
    wr(f_, &tsDepth);
    wr(f_, &colorBytes);
    wr(f_, &depthBytes);
    if (colorBytes) wr(f_, color, colorBytes);
    if (depthBytes) wr(f_, depth, depthBytes);
    numFrames_++;
}

void SensWriter::addFrame(const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth, const uint16_t* depth,
                          const uint8_t* rgbx) {
    BF_REQUIRE(f_ != nullptr, BF_ERR_STATE, "writer closed");
    BF_REQUIRE(info_.colorCompression == 0 && (info_.depthCompression == 0 || info_.depthCompression == 1), BF_ERR_ARG,
               "addFrame encodes raw colour and raw / zlib depth (add pre-compressed streams with addCompressedFrame)");
    const uint64_t nd = (uint64_t)info_.depthWidth * info_.depthHeight, nc = (uint64_t)info_.colorWidth * info_.colorHeight;
    std::vector<uint8_t> rgb(3 * nc);
    for (uint64_t p = 0; p < nc; p++) {
        rgb[3 * p] = rgbx ? rgbx[4 * p] : 0;
        rgb[3 * p + 1] = rgbx ? rgbx[4 * p + 1] : 0;
        rgb[3 * p + 2] = rgbx ? rgbx[4 * p + 2] : 0;
    }
    const uint8_t* dptr = reinterpret_cast<const uint8_t*>(depth);
    uint64_t depthBytes = 2 * nd;
    if (info_.depthCompression == 1) {
        uLongf len = compressBound((uLong)(2 * nd));
        buf_.resize(len);
        BF_REQUIRE(compress2(buf_.data(), &len, dptr, (uLong)(2 * nd), Z_DEFAULT_COMPRESSION) == Z_OK, BF_ERR_IO, "zlib failed");
        dptr = buf_.data();
        depthBytes = len;
    }
    const uint64_t colorBytes = rgb.size();
    wr(f_, camToWorld, 16);
    wr(f_, &tsColor);
    wr(f_, &tsDepth);
    wr(f_, &colorBytes);
    wr(f_, &depthBytes);
    if (colorBytes) wr(f_, rgb.data(), colorBytes);
    if (depthBytes) wr(f_, dptr, depthBytes);
    numFrames_++;
}

void SensWriter::close() {
    if (!f_) return;
    const uint64_t numIMU = 0;
    wr(f_, &numIMU);
    BF_REQUIRE(std::fseek(f_, numFramesPos_, SEEK_SET) == 0, BF_ERR_IO, "seek failed");
    wr(f_, &numFrames_);
    std::fclose(f_);
    f_ = nullptr;
}

void sens_save_with_trajectory(const std::string& in, const std::string& out, const BFMat4* T, uint64_t n) {
    std::vector<uint64_t> offsets;
    {
        SensReader r(in);
        offsets.resize(r.info().numFrames);
        for (uint64_t i = 0; i < offsets.size(); i++) offsets[i] = r.poseOffset(i);
    }
    // the same file under another spelling (./a.sens, a symlink, a hard link) is patched in place: a
    // copy would truncate the input before reading it
    struct stat si{}, so{};
    const bool same = out == in || (::stat(in.c_str(), &si) == 0 && ::stat(out.c_str(), &so) == 0 && si.st_dev == so.st_dev &&
                                    si.st_ino == so.st_ino);
    if (!same) {
        FILE* src = std::fopen(in.c_str(), "rb");
        BF_REQUIRE(src != nullptr, BF_ERR_IO, "cannot open " + in);
        FILE* dst = std::fopen(out.c_str(), "wb");
        if (!dst) {
            std::fclose(src);
            throw Error(BF_ERR_IO, "cannot create " + out);
        }
        std::vector<uint8_t> buf(1 << 24);
        bool ok = true;
        for (size_t k; ok && (k = std::fread(buf.data(), 1, buf.size(), src)) > 0;) ok = std::fwrite(buf.data(), 1, k, dst) == k;
        ok = ok && !std::ferror(src);
        std::fclose(src);
        ok = (std::fclose(dst) == 0) && ok;
        BF_REQUIRE(ok, BF_ERR_IO, "copy " + in + " -> " + out + " failed");
    }
    FILE* f = std::fopen(out.c_str(), "r+b");
    BF_REQUIRE(f != nullptr, BF_ERR_IO, "cannot open " + out);
    float ninf[16];
    for (float& v : ninf) v = -std::numeric_limits<float>::infinity();
    bool ok = true;
    for (uint64_t i = 0; ok && i < offsets.size(); i++) {
        ok = fseeko(f, (off_t)offsets[i], SEEK_SET) == 0 && std::fwrite(i < n ? T[i].m : ninf, 4, 16, f) == 16;
    }
    ok = (std::fclose(f) == 0) && ok;
    BF_REQUIRE(ok, BF_ERR_IO, "writing the trajectory into " + out + " failed");
}

// ---- zParameters: `name = value;`, `//` comments outside quotes, values up to ';' ------------
void ParamFile::load(const std::string& path) {
    std::ifstream in(path);
    BF_REQUIRE(in.good(), BF_ERR_IO, "cannot open " + path);
    std::string line;
    while (std::getline(in, line)) {
        std::string s;
        bool quoted = false;
        for (size_t i = 0; i < line.size(); i++) {  // drop the comment, keep "//" inside quotes
            if (line[i] == '"') quoted = !quoted;
            if (!quoted && line[i] == '/' && i + 1 < line.size() && line[i + 1] == '/') break;
            s += line[i];
        }
        const size_t eq = s.find('=');
        if (eq == std::string::npos) continue;
        auto trim = [](std::string t) {
            size_t a = 0, b = t.size();
            while (a < b && std::isspace((unsigned char)t[a])) a++;
            while (b > a && std::isspace((unsigned char)t[b - 1])) b--;
            return t.substr(a, b - a);
        };
        std::string key = trim(s.substr(0, eq)), val = s.substr(eq + 1);
        const size_t semi = val.rfind(';');
        if (semi != std::string::npos) val = val.substr(0, semi);
        val = trim(val);
        if (!key.empty()) kv_[key] = val;
    }
}

const std::string& ParamFile::raw(const std::string& key) const {
    auto it = kv_.find(key);
    BF_REQUIRE(it != kv_.end(), BF_ERR_ARG, "missing parameter " + key);
    return it->second;
}

std::vector<float> ParamFile::floats(const std::string& key) const {
    std::istringstream ss(raw(key));
    std::vector<float> out;
    std::string tok;
    while (ss >> tok) {
        if (!tok.empty() && (tok.back() == 'f' || tok.back() == 'F')) tok.pop_back();
        char* end = nullptr;
        const float v = std::strtof(tok.c_str(), &end);
        BF_REQUIRE(end && *end == '\0', BF_ERR_ARG, "parameter " + key + " is not numeric: " + tok);
        out.push_back(v);
    }
    return out;
}

double ParamFile::number(const std::string& key) const {
    std::string t = raw(key);
    if (!t.empty() && (t.back() == 'f' || t.back() == 'F')) t.pop_back();
    char* end = nullptr;
    const double v = std::strtod(t.c_str(), &end);
    BF_REQUIRE(end && *end == '\0', BF_ERR_ARG, "parameter " + key + " is not a number: " + t);
    return v;
}

bool ParamFile::boolean(const std::string& key) const {
    const std::string& t = raw(key);
    if (t == "true" || t == "1") return true;
    if (t == "false" || t == "0") return false;
    throw Error(BF_ERR_ARG, "parameter " + key + " is not a bool: " + t);
}

std::string ParamFile::str(const std::string& key) const {
    std::string t = raw(key);
    if (t.size() >= 2 && t.front() == '"' && t.back() == '"') t = t.substr(1, t.size() - 2);
    return t;
}

// ---- mesh output (CUDAMarchingCubesHashSDF::saveMesh, CUDAMarchingCubesHashSDF.cpp:48-105) --------
// MeshData::mergeCloseVertices / removeDuplicateFaces / applyTransform and MeshIOf::saveToFile are
// mLib (not vendored): restated from their documented behaviour, parity unpinned.
namespace {

struct Key3Hash {
    size_t operator()(const std::array<int, 3>& k) const {
        return ((size_t)(uint32_t)k[0] * 73856093u) ^ ((size_t)(uint32_t)k[1] * 19349669u) ^ ((size_t)(uint32_t)k[2] * 83492791u);
    }
};

// toVirtualVoxelPos(v, thresh): round half away from zero of v / thresh, truncated to int
int snap(float v, float t) {
    const float q = v / t;
    return (int)(q + (float)((0.0f < q) - (q < 0.0f)) * 0.5f);
}

}  // namespace

Mesh mesh_from_triangles(const BFMcTriangle* tris, uint32_t n, const float* transform) {
    const float eps = 0.00001f;  // mergeCloseVertices(0.00001f, true) (CUDAMarchingCubesHashSDF.cpp:87)
    Mesh m;
    std::unordered_map<std::array<int, 3>, uint32_t, Key3Hash> cell;
    cell.reserve((size_t)n * 2);
    std::vector<uint32_t> face;
    face.reserve((size_t)n * 3);
    for (uint32_t t = 0; t < n; t++)
        for (int k = 0; k < 3; k++) {  // copyTrianglesToCPU: vertex 3t+k, colour vec4f(c, 1)
            const BFMcVertex& v = tris[t].v[k];
            const std::array<int, 3> key = {snap(v.p[0], eps), snap(v.p[1], eps), snap(v.p[2], eps)};
            auto it = cell.find(key);
            if (it != cell.end()) {
                face.push_back(it->second);
                continue;
            }
            const uint32_t id = (uint32_t)(m.vertices.size() / 3);
            cell.emplace(key, id);
            m.vertices.insert(m.vertices.end(), {v.p[0], v.p[1], v.p[2]});
            m.colors.insert(m.colors.end(), {v.c[0], v.c[1], v.c[2], 1.0f});
            face.push_back(id);
        }
    // degenerate faces (two corners merged) go, then removeDuplicateFaces: first face of each vertex set
    std::unordered_set<std::array<int, 3>, Key3Hash> seen;
    seen.reserve((size_t)n * 2);
    for (uint32_t t = 0; t < n; t++) {
        const uint32_t a = face[3 * t], b = face[3 * t + 1], c = face[3 * t + 2];
        if (a == b || b == c || a == c) continue;
        std::array<int, 3> k = {(int)a, (int)b, (int)c};
        std::sort(k.begin(), k.end());
        if (!seen.insert(k).second) continue;
        m.faces.insert(m.faces.end(), {a, b, c});
    }
    if (transform) {  // applyTransform: affine point transform
        const float* e = transform;
        for (size_t i = 0; i < m.vertices.size(); i += 3) {
            const float x = m.vertices[i], y = m.vertices[i + 1], z = m.vertices[i + 2];
            m.vertices[i] = e[0] * x + e[1] * y + e[2] * z + e[3];
            m.vertices[i + 1] = e[4] * x + e[5] * y + e[6] * z + e[7];
            m.vertices[i + 2] = e[8] * x + e[9] * y + e[10] * z + e[11];
        }
    }
    return m;
}

void mesh_save_ply(const std::string& path, const Mesh& m) {
    FILE* f = std::fopen(path.c_str(), "wb");
    BF_REQUIRE(f != nullptr, BF_ERR_IO, "cannot open " + path + " for writing");
    const size_t nv = m.vertices.size() / 3, nf = m.faces.size() / 3;
    std::string hdr = "ply\nformat binary_little_endian 1.0\nelement vertex " + std::to_string(nv) +
                      "\nproperty float x\nproperty float y\nproperty float z\nproperty uchar red\nproperty uchar green\n"
                      "property uchar blue\nproperty uchar alpha\nelement face " + std::to_string(nf) +
                      "\nproperty list uchar int vertex_indices\nend_header\n";
    std::vector<uint8_t> buf;
    buf.reserve(hdr.size() + nv * 16 + nf * 13);
    buf.insert(buf.end(), hdr.begin(), hdr.end());
    auto put = [&](const void* p, size_t n) { buf.insert(buf.end(), (const uint8_t*)p, (const uint8_t*)p + n); };
    for (size_t i = 0; i < nv; i++) {
        put(&m.vertices[3 * i], 12);
        uint8_t c[4];
        for (int k = 0; k < 4; k++) c[k] = (uint8_t)std::lround(std::fmin(std::fmax(m.colors[4 * i + k], 0.0f), 1.0f) * 255.0f);
        put(c, 4);
    }
    for (size_t i = 0; i < nf; i++) {
        const uint8_t three = 3;
        put(&three, 1);
        const int32_t idx[3] = {(int32_t)m.faces[3 * i], (int32_t)m.faces[3 * i + 1], (int32_t)m.faces[3 * i + 2]};
        put(idx, 12);
    }
    const bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    std::fclose(f);
    BF_REQUIRE(ok, BF_ERR_IO, "short write to " + path);
}

// ---- EntryJ dump (Bundler::saveSparseCorrsToFile, Bundler.cpp:396-409) ---------------------------
void corr_save(const std::string& path, const BFEntryJ* corr, uint64_t n) {
    BF_REQUIRE(corr != nullptr || n == 0, BF_ERR_ARG, "null correspondences");
    FILE* f = std::fopen(path.c_str(), "wb");
    BF_REQUIRE(f != nullptr, BF_ERR_IO, "cannot open " + path + " for writing");
    bool ok = std::fwrite(&n, 8, 1, f) == 1;
    if (n) ok = ok && std::fwrite(corr, sizeof(BFEntryJ), n, f) == n;
    std::fclose(f);
    BF_REQUIRE(ok, BF_ERR_IO, "short write to " + path);
}

uint64_t corr_load(const std::string& path, BFEntryJ* corr, uint64_t cap) {
    FILE* f = std::fopen(path.c_str(), "rb");
    BF_REQUIRE(f != nullptr, BF_ERR_IO, "cannot open " + path);
    uint64_t n = 0;
    bool ok = std::fread(&n, 8, 1, f) == 1;
    const uint64_t m = std::min(n, cap);
    if (ok && m) {
        BF_REQUIRE(corr != nullptr, BF_ERR_ARG, "null output");
        ok = std::fread(corr, sizeof(BFEntryJ), m, f) == m;
    }
    std::fclose(f);
    BF_REQUIRE(ok, BF_ERR_IO, "truncated correspondence file " + path);
    return n;
}

// CUDASceneRepHashSDF::parametersFromGlobalAppState (CUDASceneRepHashSDF.h:39-59)
BFHashParams hash_params_from(const ParamFile& f) {
    BFHashParams out;
    BFHashParams* o = &out;
    std::memset(o, 0, sizeof(*o));
    for (int i = 0; i < 16; i += 5) { o->rigidTransform.m[i] = 1.0f; o->rigidTransformInverse.m[i] = 1.0f; }
    o->hashNumBuckets = (uint32_t)f.number("s_hashNumBuckets");
    o->hashBucketSize = BF_HASH_BUCKET_SIZE;
    o->hashMaxCollisionLinkedListSize = (uint32_t)f.number("s_hashMaxCollisionLinkedListSize");
    o->numSDFBlocks = (uint32_t)f.number("s_hashNumSDFBlocks");
    o->SDFBlockSize = BF_SDF_BLOCK_SIZE;
    o->virtualVoxelSize = (float)f.floats("s_SDFVoxelSize").at(0);
    o->maxIntegrationDistance = f.floats("s_SDFMaxIntegrationDistance").at(0);
    o->truncation = f.floats("s_SDFTruncation").at(0);
    o->truncScale = f.floats("s_SDFTruncationScale").at(0);
    o->integrationWeightSample = (uint32_t)f.number("s_SDFIntegrationWeightSample");
    o->integrationWeightMax = (uint32_t)f.number("s_SDFIntegrationWeightMax");
    const std::vector<float> ext = f.floats("s_streamingVoxelExtents"), dims = f.floats("s_streamingGridDimensions"),
                             minp = f.floats("s_streamingMinGridPos");
    BF_REQUIRE(ext.size() == 3 && dims.size() == 3 && minp.size() == 3, BF_ERR_ARG, "streaming vectors need 3 values");
    o->streamingVoxelExtents = BFFloat3{ext[0], ext[1], ext[2]};
    o->streamingGridDimensions = BFInt3{(int)dims[0], (int)dims[1], (int)dims[2]};
    o->streamingMinGridPos = BFInt3{(int)minp[0], (int)minp[1], (int)minp[2]};
    o->streamingInitialChunkListSize = (uint32_t)f.number("s_streamingInitialChunkListSize");
    return out;
}
// CUDARayCastSDF::parametersFromGlobalAppState (CUDARayCastSDF.h:24-51)
BFRayCastParams raycast_params_from(const ParamFile& f, float fx, float fy, float mx, float my) {
    BFRayCastParams out;
    BFRayCastParams* o = &out;
    const uint32_t rw = (uint32_t)f.number("s_rayCastWidth"), rh = (uint32_t)f.number("s_rayCastHeight");
    const uint32_t iw = (uint32_t)f.number("s_integrationWidth"), ih = (uint32_t)f.number("s_integrationHeight");
    if (rw != iw || rh != ih) {  // adapt intrinsics (CUDARayCastSDF.h:26-32)
        fx *= (float)rw / (float)iw;
        fy *= (float)rh / (float)ih;
        mx *= (float)(rw - 1) / (float)(iw - 1);
        my *= (float)(rh - 1) / (float)(ih - 1);
    }
    std::memset(o, 0, sizeof(*o));
    o->width = rw;
    o->height = rh;
    o->fx = fx; o->fy = fy; o->mx = mx; o->my = my;
    o->minDepth = f.floats("s_renderDepthMin").at(0);
    o->maxDepth = f.floats("s_renderDepthMax").at(0);
    o->rayIncrement = f.floats("s_SDFRayIncrementFactor").at(0) * f.floats("s_SDFTruncation").at(0);
    o->thresSampleDist = f.floats("s_SDFRayThresSampleDistFactor").at(0) * o->rayIncrement;
    o->thresDist = f.floats("s_SDFRayThresDistFactor").at(0) * o->rayIncrement;
    o->useGradients = f.boolean("s_SDFUseGradients") ? 1 : 0;
    o->maxNumVertices = (uint32_t)f.number("s_hashNumSDFBlocks") * 6;
    return out;
}
// CUDAImageManager::process options from the bundling parameters
BFPreprocessOptions preprocess_options_from(const ParamFile& f, float depthShift) {
    BFPreprocessOptions out{};
    BFPreprocessOptions* o = &out;
    o->erode = f.boolean("s_erodeSIFTdepth") ? 1 : 0;
    o->erodeStructureSize = 3;      // CUDAImageManager.cpp:95-103
    o->erodeDepthThresh = 0.05f;
    o->erodeFraction = 0.3f;
    o->depthFilter = f.boolean("s_depthFilter") ? 1 : 0;
    o->sigmaD = f.floats("s_depthSigmaD").at(0);
    o->sigmaR = f.floats("s_depthSigmaR").at(0);
    o->depthShift = depthShift;
    return out;
}

}  // namespace bf
