// io.h — the reference's input formats (both parsers live in the
// un-vendored mLib, so the format is restated here and pinned by round-trip tests):
//   * `.sens` (mLib SensorData, version 4, as read by SensorDataReader.cpp:38-116): header,
//     per-frame {camToWorld, timestamps, compressed colour, compressed depth}, IMU records.
//   * `zParameters*.txt` (mLib ParameterFile, read by GlobalAppState / GlobalBundlingState):
//     `name = value;` lines with `//` comments.
// Host-only C++ (zlib for the depth stream); frames are read on demand, never all at once.
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

#include "../../include/bf/bf.h"

namespace bf {

class SensReader {
public:
    explicit SensReader(const std::string& path);
    ~SensReader();
    const BFSensInfo& info() const { return info_; }
    void pose(uint64_t frame, float camToWorld[16]) const;
    void timestamps(uint64_t frame, uint64_t* tsColor, uint64_t* tsDepth) const;
    void depthU16(uint64_t frame, uint16_t* out);
    void colorRGBX(uint64_t frame, uint8_t* out);
    // file offset of frame i's camToWorld matrix (the 64 B before its timestamps and sizes)
    uint64_t poseOffset(uint64_t frame) const { return this->frame(frame).colorOffset - 32 - 64; }

private:
    struct Frame {
        float camToWorld[16];
        uint64_t tsColor, tsDepth, colorBytes, depthBytes;
        uint64_t colorOffset, depthOffset;
    };
    FILE* f_ = nullptr;
    BFSensInfo info_{};
    std::vector<Frame> frames_;
    std::vector<uint8_t> buf_;
    const Frame& frame(uint64_t i) const;
};

class SensWriter {
public:
    SensWriter(const std::string& path, const BFSensInfo& info);
    ~SensWriter();
    void addFrame(const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth, const uint16_t* depth, const uint8_t* rgbx);
    // streams already compressed as the header's colorCompression / depthCompression say (e.g. JPEG colour)
    void addCompressedFrame(const float camToWorld[16], uint64_t tsColor, uint64_t tsDepth, const uint8_t* color,
                            uint64_t colorBytes, const uint8_t* depth, uint64_t depthBytes);
    void close();

private:
    FILE* f_ = nullptr;
    BFSensInfo info_{};
    long numFramesPos_ = 0;
    uint64_t numFrames_ = 0;
    std::vector<uint8_t> buf_;
};

// SensorDataReader::saveToFile (SensorDataReader.cpp:153-166): the input file with frame i's camToWorld
// replaced by T[i] for i < n and by -inf for the rest; every other byte (compressed colour / depth, IMU
// records) as read. out == in patches the file in place (the reference overwrites its input).
void sens_save_with_trajectory(const std::string& in, const std::string& out, const BFMat4* T, uint64_t n);

// Indexed mesh of CUDAMarchingCubesHashSDF::saveMesh (CUDAMarchingCubesHashSDF.cpp:71-100)
struct Mesh {
    std::vector<float> vertices;  // 3 per vertex
    std::vector<float> colors;    // 4 per vertex (vec4f(colour, 1))
    std::vector<uint32_t> faces;  // 3 per face
};
Mesh mesh_from_triangles(const BFMcTriangle* tris, uint32_t n, const float* transform);
void mesh_save_ply(const std::string& path, const Mesh& m);

// Bundler::saveSparseCorrsToFile format: uint64 count + raw EntryJ records
void corr_save(const std::string& path, const BFEntryJ* corr, uint64_t n);
uint64_t corr_load(const std::string& path, BFEntryJ* corr, uint64_t cap);
// EntryJ producer from depth + poses (corr.hip); device inputs / output, synchronizes
uint32_t corr_from_depth(const float* const* depth, const float* T, const float* Tinv, uint32_t cur, uint32_t start,
                         const BFCorrOptions& o, BFEntryJ* out, uint32_t cap, uint32_t* total);

class ParamFile {
public:
    void load(const std::string& path);  // later files override earlier keys
    bool has(const std::string& key) const { return kv_.count(key) != 0; }
    const std::string& raw(const std::string& key) const;
    std::vector<float> floats(const std::string& key) const;
    double number(const std::string& key) const;
    bool boolean(const std::string& key) const;
    std::string str(const std::string& key) const;
    size_t size() const { return kv_.size(); }

private:
    std::map<std::string, std::string> kv_;
};

// zParameters -> the structs the path reads (the bf_params_* getters)
BFHashParams hash_params_from(const ParamFile& f);
BFRayCastParams raycast_params_from(const ParamFile& f, float fx, float fy, float mx, float my);
BFPreprocessOptions preprocess_options_from(const ParamFile& f, float depthShift);

}  // namespace bf
