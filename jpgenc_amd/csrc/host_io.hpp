// Host-side I/O around the GPU path: the PPM front end (reference loadPPM,
// Image.cpp:326-538), the JFIF segment writer (JpegSegments.hpp:55-377 as used by
// Image.cpp:933-954), quality-scaled quantisation tables, and the deterministic
// synthetic frame generator used by tests and the bench.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "huffman.hpp"

namespace jpge {

// Status codes shared with the C ABI (include/jpge.h).
enum Status : int {
    kOk = 0,
    kErrArg = 1,
    kErrNoSpace = 2,
    kErrHip = 3,
    kErrNoDevice = 4,
    kErrFormat = 5,
    kErrIo = 6,
    kErrTruncated = 7,
    kErrRange = 8,
    kErrTimeout = 9,
    kErrRccl = 10,
    kErrInternal = 11,
};

struct PpmImage {
    uint32_t width = 0, height = 0;
    int maxval = 0;
    std::vector<uint8_t> rgb;  // width*height*3 samples, unscaled (0..maxval)
};

// Parses P3/P6 with the reference tokenizer semantics (PPMFileBuffer::read_word,
// Image.cpp:334-390: whitespace skipping, '#' comment lines, fast_atoi for P3
// samples).  Differences, all on inputs where the reference has undefined
// or assert-only behaviour: truncated P6 data -> kErrTruncated; samples above
// maxval or maxval outside 1..255 -> kErrRange.
int parse_ppm(const uint8_t* buf, size_t n, PpmImage& out);
int load_ppm_file(const std::string& path, PpmImage& out);
// The same parse without a copy: P6 -> offset of the samples in buf; P3 -> the
// samples written over the text at buf[0..) (offset 0).
int parse_ppm_inplace(uint8_t* buf, size_t n, uint32_t& width, uint32_t& height, int& maxval, size_t& offset);

// Annex K tables (Image.cpp:850-869) scaled for quality 1..100 with the IJG rule
// (50 == the reference's tables unchanged).
void quality_tables(int quality, uint8_t qy[64], uint8_t qc[64]);

// Natural (row-major) index of zig-zag position i (Coding.hpp:57-81).
extern const uint8_t kZigzagToNatural[64];

// SOI, APP0, DQT(luma), DQT(chroma), SOF0, DHT x4, SOS, in that order
// (Image.cpp:936-954).  tables: Y-DC, Y-AC, C-DC, C-AC.  restart_mcus > 0 adds a DRI
// segment before SOS, s444 declares Y 1x1 (both not in the reference).
std::vector<uint8_t> jfif_headers(uint32_t real_width, uint32_t real_height, const uint8_t qy[64],
                                  const uint8_t qc[64], const HuffTable* const tables[4], uint32_t restart_mcus = 0,
                                  uint8_t ysamp = 0x22);

// Deterministic synthetic RGB8 frame (integer-only, identical on every host):
// kind 0 = smooth gradients + texture + noise (photo-like), 1 = uniform random
// bytes (worst-case symbol statistics), 2 = flat colour.
void synth_rgb8(uint64_t seed, uint32_t width, uint32_t height, int kind, uint8_t* out, size_t stride);

}  // namespace jpge
