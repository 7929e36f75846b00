// Device-side interface of the jpge HIP kernels (gfx950).  Host code fills
// these parameter blocks; kernels.hip owns the launch geometry.
//
// Data layout in HBM (per frame):
//   rgb   : interleaved RGB8, row pitch `stride` (16-byte aligned pitch/base = fast path)
//   coef  : int16 [nmcu][6][64]  quantised coefficients, NATURAL order inside a block,
//           blocks in MCU-interleave order Y00 Y01 Y10 Y11 Cb Cr (= entropy order)
//   mask  : u64   [nmcu][6]      AC non-zero mask, bit p = zig-zag position p (1..63)
//   hist  : u32 cnt[kHistReplicas][4][256], u64 key[4][256] (~first-occurrence key)
#pragma once
#include <cstdint>

#include <hip/hip_runtime_api.h>

#if defined(__HIPCC__)
#define JPGE_HD __host__ __device__
#else
#define JPGE_HD
#endif

namespace jpge {

// Frame geometry (reference: Image.cpp:480-531 pads to 16, Image.cpp:311-312
// halves the chroma planes).  One MCU = 16x16 px = Y00 Y01 Y10 Y11 Cb Cr.
struct Geometry {
    uint32_t width = 0, height = 0;  // real size
    uint32_t mw = 0, mh = 0;         // MCUs per row / column
    JPGE_HD uint32_t nmcu() const { return mw * mh; }
    JPGE_HD uint32_t nblocks() const { return nmcu() * 6; }
};

constexpr int kHistReplicas = 8;          // spread of the global histogram atomics
constexpr int kStatsTile = 128;           // blocks per statistics workgroup (4 lanes each)
constexpr int kEntropyTile = 128;         // blocks per entropy workgroup (4 lanes each)
constexpr int kStageBytesPerBlock = 216;  // >= worst-case 1665 bits of one block
// global fallback staging slot of an entropy tile whose bits exceed the LDS stage
constexpr uint32_t kScratchWordsPerTile = kEntropyTile * kStageBytesPerBlock / 4 + 8;

// Tables: 0 Y-DC, 1 Y-AC, 2 C-DC, 3 C-AC.
struct HistPtrs {
    uint32_t* cnt;
    uint64_t* key;
};

struct FdctArgs {
    const uint8_t* rgb;
    uint64_t stride;
    Geometry g;
    int maxval;          // 255 -> exact integer colour path
    const double* qtab;  // [128]: luma then chroma, natural order
    int16_t* coef;
};

struct StatsArgs {
    const int16_t* coef;
    uint64_t* mask;
    Geometry g;
    HistPtrs hist;
};

struct EntropyArgs {
    const int16_t* coef;
    const uint64_t* mask;
    Geometry g;
    const uint32_t* tables;  // [4][256] (len << 16) | code
    uint8_t* out;            // whole .jpg (header already at [0, hdr_len))
    uint64_t hdr_len;
    uint64_t out_cap;
    uint32_t* ticket;        // zeroed per launch
    uint64_t* lb_bits;       // [ntiles] zeroed
    uint64_t* lb_ff;         // [ntiles] zeroed
    uint32_t* tails;         // [ntiles] zeroed
    uint64_t* result;        // [0] total .jpg bytes, [1] error bits
    uint32_t* scratch;       // [ntiles][kScratchWordsPerTile] fallback staging
    uint32_t stage_cap;      // LDS staging bytes to use (0 forces the fallback; tests)
};

inline uint32_t entropy_tiles(const Geometry& g) {
    return (g.nblocks() + kEntropyTile - 1) / kEntropyTile;
}

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s);
hipError_t launch_stats(const StatsArgs& a, hipStream_t s);
hipError_t launch_entropy(const EntropyArgs& a, hipStream_t s);

}  // namespace jpge
