// Device-side interface of the jpge HIP kernels (gfx950).  Host code fills
// these parameter blocks; fdct.hip / stats.hip / entropy.hip own the launch
// geometry.
//
// Data layout in HBM (per frame):
//   rgb   : interleaved RGB8, row pitch `stride` (16-byte aligned pitch/base = fast path)
//   coef  : int16 [nmcu][6][64]  quantised coefficients, NATURAL order inside a block,
//           blocks in MCU-interleave order Y00 Y01 Y10 Y11 Cb Cr (= entropy order)
//   hist  : u32 cnt[kHistReplicas][4][256], u64 key[4][256] (~first-occurrence key)
//   ubuf  : u8 [G][kEntropyRegionBytes] each entropy workgroup's bit stream before
//           byte alignment and 0xFF stuffing, written and re-read by that workgroup
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
constexpr int kStatsTile = 128;           // blocks per statistics tile (4 lanes each)
constexpr int kEntropyTile = 128;         // blocks per entropy tile (4 lanes each)
constexpr int kEntropyMaxTilesPerWg = 4;  // tiles a persistent entropy workgroup may own
constexpr int kStageBytesPerBlock = 216;  // >= worst-case 1665 bits of one block
constexpr int kStampSlots = 16;           // diagnostic stamp words per workgroup (JPGE_STAMPS builds)
constexpr int kEntropyRecordBytes = 48;   // per entropy workgroup: bits, edge bits, 0xFF counts

// Tables: 0 Y-DC, 1 Y-AC, 2 C-DC, 3 C-AC.
struct HistPtrs {
    uint32_t* cnt;
    uint64_t* key;
};

struct FdctArgs {
    const uint8_t* rgb;
    uint64_t stride;
    Geometry g;
    int maxval;      // 255 -> exact integer colour path
    uint8_t q[128];  // luma then chroma quantisers, natural order (bytes: a small kernarg block)
    int16_t* coef;
    uint32_t* zero;       // the frame's control block, zeroed by this kernel (it runs first)
    uint32_t zero_words;
    // carried duty: import another frame's tables + headers from mapped host memory
    // (workgroup 0; 0 units = none)
    const uint4* imp_src;
    uint4* imp_dst;
    uint32_t imp_n16;
    uint64_t* dbg;   // diagnostic phase stamps (JPGE_STAMPS builds), else unused
};

struct StatsArgs {
    const int16_t* coef;
    Geometry g;
    HistPtrs hist;
    uint64_t* dbg;
};

struct EntropyArgs {
    const int16_t* coef;
    Geometry g;
    const uint32_t* tables;  // [4][256] (len << 16) | code, followed by the header bytes
    uint8_t* out;            // whole .jpg; the kernel writes the header to [0, hdr_len)
    uint64_t hdr_len;
    uint64_t out_cap;
    uint8_t* ubuf;           // per-workgroup unstuffed regions (entropy_ubuf_bytes)
    uint8_t* rec;            // [entropy_grid][kEntropyRecordBytes] code -> pack kernel records
    uint64_t* host_result;   // mapped pinned host memory: [0] .jpg bytes, [1] no-space (4),
                             // [2] reserved (0), [3] = seq, written last
    uint64_t seq;            // the frame's sequence number
    // carried duty of the code kernel: export another frame's histograms to mapped
    // host memory (workgroup 0; exp_cnt == nullptr: none)
    HistPtrs exp_hist;
    uint32_t* exp_cnt;
    uint64_t* exp_key;
    uint64_t* exp_seq;
    uint64_t exp_seqv;
    uint32_t wgs;            // workgroup count override (0 = automatic; tests)
    uint32_t diag;           // diagnostic switches (JPGE_DIAG; 0 in production)
    uint64_t* dbg;
};

inline uint32_t entropy_tiles(const Geometry& g) {
    return (g.nblocks() + kEntropyTile - 1) / kEntropyTile;
}
// bytes of one entropy workgroup's private region: its bit stream (workgroup-
// local offsets, worst case) plus slack, a whole number of 128-byte lines
constexpr uint64_t kEntropyRegionBytes = (uint64_t)kEntropyMaxTilesPerWg * kEntropyTile * kStageBytesPerBlock + 128;

uint32_t fdct_grid(const Geometry& g);
uint32_t stats_grid(const Geometry& g);
uint32_t entropy_grid(const Geometry& g, uint32_t wgs_override);

inline uint64_t entropy_ubuf_bytes(const Geometry& g, uint32_t wgs_override) {
    return (uint64_t)entropy_grid(g, wgs_override) * kEntropyRegionBytes;
}

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s);
hipError_t launch_stats(const StatsArgs& a, hipStream_t s);
// [4][256] summed counts and keys into (mapped) host memory, then *host_seq = seq
hipError_t launch_hist_export(const HistPtrs& h, uint32_t* host_cnt, uint64_t* host_key, uint64_t* host_seq,
                              uint64_t seq, hipStream_t s);
hipError_t launch_entropy(const EntropyArgs& a, hipStream_t s);

}  // namespace jpge
