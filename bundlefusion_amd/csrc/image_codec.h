// image_codec.h — colour-stream decoders of the `.sens` reader (colorCompression 1 = PNG,
// 2 = JPEG; SensorDataReader.cpp:98-116 calls mLib's RGBDFrameCacheRead / SensorData::
// decompressColorAlloc, which hands the bytes to an image library). The image library is not
// vendored in the reference, so the decoders are written here from the published formats:
//   * JPEG: ITU-T T.81 baseline / extended sequential Huffman (SOF0 / SOF1, 8-bit), restart
//     intervals, any sampling factors; sample reconstruction as the IJG library does it (libjpeg 6b
//     jidctint "islow" integer IDCT, jdsample "fancy" triangular chroma upsampling, jdcolor fixed-
//     point YCbCr -> RGB tables), so the output equals libjpeg's default decode byte for byte.
//     Progressive / arithmetic-coded / 12-bit streams are rejected (BF_ERR_ARG).
//   * PNG: zlib inflate + the five scanline filters, 8-bit grey / grey-alpha / RGB / RGBA /
//     palette, non-interlaced (interlaced streams are rejected).
// Output is RGBX (X = 255), the layout SensorDataReader widens colour frames to (:111-113).
// Host-only C++.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace bf {

struct DecodedImage {
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgbx;  // width * height * 4
};

// Largest image either decoder accepts (2^28 pixels = 1 GiB of RGBX; a VGA frame is 2^18.3): a
// header claiming more is refused before anything is allocated.
constexpr uint64_t kMaxImagePixels = 1ull << 28;

// Throws bf::Error (BF_ERR_IO for corrupt data, BF_ERR_ARG for unsupported variants). expectW /
// expectH (0 = any): the size the caller's container header states (the .sens colour size); a stream
// whose own header disagrees is refused before its planes are allocated.
DecodedImage jpeg_decode(const uint8_t* data, size_t n, uint32_t expectW = 0, uint32_t expectH = 0);
DecodedImage png_decode(const uint8_t* data, size_t n, uint32_t expectW = 0, uint32_t expectH = 0);

}  // namespace bf
