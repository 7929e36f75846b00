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
// An MCU is yh x yv Y blocks (row by row) + one Cb + one Cr block, bpm = yh*yv + 2:
//   4:2:0 (the reference's S420_m, and the S420 / S420_lm filters): 2x2, 16x16 px;
//   4:4:4: 1x1, 8x8 px;  4:2:2: 2x1, 16x8 px;  4:1:1: 4x1, 32x8 px.
// cfilt selects the 4:2:0 chroma filter of applySubsampling (Image.cpp:279-306).
constexpr uint32_t kFiltS420m = 0, kFiltS420lm = 1, kFiltS420 = 2;
struct Geometry {
    uint32_t width = 0, height = 0;  // real size
    uint32_t mw = 0, mh = 0;         // MCUs per row / column
    uint32_t bpm = 6;
    uint32_t yh = 2;                 // Y blocks across an MCU (1, 2, 4)
    uint32_t cfilt = kFiltS420m;
    JPGE_HD uint32_t nmcu() const { return mw * mh; }
    JPGE_HD uint32_t nblocks() const { return nmcu() * bpm; }
    JPGE_HD uint32_t yv() const { return (bpm - 2) / yh; }  // Y blocks down an MCU (1, 2)
    JPGE_HD bool s444() const { return bpm == 3; }
    JPGE_HD bool row8() const { return bpm - 2 == yh; }  // MCUs one block row high
    JPGE_HD uint32_t mcu_w() const { return 8 * yh; }   // MCU size in pixels
    JPGE_HD uint32_t mcu_h() const { return 8 * yv(); }
};
// component of MCU slot k: 0 = Y, 1 = Cb, 2 = Cr (the last two slots are the chroma)
JPGE_HD inline int block_comp(int k, uint32_t bpm) { return k < (int)bpm - 2 ? 0 : k - ((int)bpm - 3); }

constexpr int kHistReplicas = 8;  // spread of the global histogram atomics
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
    bool solo;       // the kernel has the GPU to itself: whole-CU workgroups (else 4-wave ones)
    uint32_t wgs;    // pipeline grid override (0: the default cap; experiments, JPGE_FDCT_WGS)
    // luma then chroma quantisers, natural order (bytes: a small kernarg block; 16-byte
    // aligned so the kernels fetch it with scalar loads, see fdct.hip q_entry)
    alignas(16) uint8_t q[128];
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

// Stripe context of a frame (a row stripe of a larger image); the
// defaults describe a whole frame.
struct DcSeed {
    int v[3] = {0, 0, 0};  // DC chain predecessors of the first Y / Cb / Cr block (Image.cpp:638-678)
};

// Restart intervals (DRI / RSTn; opt-in, not in the reference):
// every `mcus` MCUs the DC predictions restart at 0, and the entropy stream is
// 1-filled to a byte boundary and followed by an RSTn marker (n = interval - 1 mod 8).
// mcus = 0: off (the reference's single interval).  mcu0: the frame's first MCU in
// the image's numbering (a stripe starts at an interval boundary).
struct Restart {
    uint32_t mcus = 0;
    uint32_t mcu0 = 0;
};

// The entropy kernels' partition of a frame: segments (restart intervals; one
// segment when restart is off), each cut into tiles of <= kEntropyTile blocks
// (balanced: tile i of a segment of nb blocks in tps tiles is blocks
// [i*nb/tps, (i+1)*nb/tps)), each run of tiles owned by one workgroup.  A
// workgroup's stream never crosses a segment boundary, so every segment starts
// byte-aligned after its predecessor's fill.
struct SegLayout {
    uint32_t nseg = 1;                    // segments
    uint32_t sblk = 0, tps = 0, wps = 0;  // a full segment: blocks, tiles, workgroups
    uint32_t lblk = 0, ltps = 0, lwps = 0;  // the last segment (the frame's tail)
    JPGE_HD uint32_t grid() const { return (nseg - 1) * wps + lwps; }
};

// Workgroup w's tiles: tiles [t0, t0 + nt) of segment seg (blocks [b0, b0 + nb) of
// the frame, in tps tiles).
struct WgTiles {
    uint64_t b0;
    uint32_t nb, tps, t0, nt, seg;
    bool first, last;  // the segment's first / last workgroup
    JPGE_HD uint64_t tile_b0(uint32_t i) const { return b0 + (uint64_t)i * nb / tps; }
    JPGE_HD uint32_t tile_nb(uint32_t i) const {
        return (uint32_t)((uint64_t)(i + 1) * nb / tps - (uint64_t)i * nb / tps);
    }
};
JPGE_HD inline WgTiles wg_tiles(const SegLayout& L, uint32_t w) {
    WgTiles r;
    uint32_t j, wps;
    if (w < (L.nseg - 1) * L.wps) {
        r.seg = w / L.wps; j = w % L.wps; r.tps = L.tps; wps = L.wps; r.nb = L.sblk;
    } else {
        r.seg = L.nseg - 1; j = w - (L.nseg - 1) * L.wps; r.tps = L.ltps; wps = L.lwps; r.nb = L.lblk;
    }
    r.b0 = (uint64_t)r.seg * L.sblk;
    r.t0 = (uint32_t)((uint64_t)j * r.tps / wps);
    r.nt = (uint32_t)((uint64_t)(j + 1) * r.tps / wps) - r.t0;
    r.first = j == 0;
    r.last = j == wps - 1;
    return r;
}

// Symbol records (K2 -> K3): the entropy-coded symbols of a tile in stream order,
// 16 bits each (round 6; 32-bit records had been 38% of a 4K frame's HBM bytes):
//   table << 14 | run << 10 | size << 6 | x     (table 0 Y-DC, 1 Y-AC, 2 C-DC, 3 C-AC;
//   a DC symbol is its category with run 0; EOB run 0 size 0; ZRL run 15 size 0), x = the
//   top min(size, 6) of the symbol's extra bits;
//   continuation: the component's AC table << 14 | n << 10 | the n (1..5) low extra bits
//   the record before it could not hold (size >= 7); run n with size 0 is no JPEG symbol
//   (Coding.hpp:148-196 codes zero runs only as ZRL and EOB), so it never collides with one.
// The code kernel indexes one 64-bit LDS entry per record by record >> 6.  A block codes
// at most 64 symbols (DC + 63 AC, or DC + 62 AC + EOB; a zero run long enough for a ZRL
// removes a coefficient), each with at most one continuation, so a tile's records fit
// kTileRecords halfwords; tile t's sit at recs + t * kTileRecords.  Tiles are the entropy
// partition's (seg_layout), numbered segment by segment.
constexpr int kRecPerBlock = 128;
constexpr int kTileRecords = kEntropyTile * kRecPerBlock;
constexpr uint32_t kRecXBits = 6;  // extra bits a head record holds
// A tile's records are written as kRecSub sub-streams, one per wave of the
// statistics kernel: sub-stream j of a tile of nb blocks holds blocks
// [j*nb/kRecSub, (j+1)*nb/kRecSub) of the tile, at recs + t*kTileRecords +
// j*kSubRecords, its count at tcount[t*kRecSub + j].  The code kernel reads a
// tile's sub-streams in order, so they form the tile's one record stream.
constexpr int kRecSub = 4;
constexpr int kSubRecords = kTileRecords / kRecSub;
static_assert(kTileRecords % kRecSub == 0, "sub-streams divide a tile's records");

struct StatsArgs {
    const int16_t* coef;
    Geometry g;
    HistPtrs hist;
    DcSeed seed;
    Restart rst;
    // first-occurrence key bases in the whole image's texts (Image.cpp:888-906):
    // Y raster index of the stripe's first Y block, Cb raster index of its first
    // Cb block, and the image's Cb block count (every Cr key follows all Cb keys)
    uint64_t key_y0 = 0, key_c0 = 0, key_ncb = 0;
    SegLayout seg;       // the entropy partition: the tiles the records are written in
    uint16_t* recs;      // [tiles][kTileRecords] symbol records
    uint32_t* tcount;    // [tiles][kRecSub] records per sub-stream
    uint32_t wgs = 0;    // workgroup count (0 = 3 per CU; the pipeline passes its own, stats_grid)
    uint64_t* dbg;
    // Set (single frames): the last workgroup to finish exports the histograms into
    // mapped host memory (export_hist), in place of a hist_export_kernel launch.  `done`
    // counts finished workgroups (zeroed per frame by K1).
    uint32_t* done = nullptr;
    uint32_t* host_cnt = nullptr;
    uint64_t* host_key = nullptr;
    uint64_t* host_seq = nullptr;
    uint64_t seq = 0;
};

// Where each entropy workgroup's bytes go (entropy_scan_kernel -> pack kernel).
struct alignas(16) WgPlace {
    uint64_t P;       // global bit offset of the workgroup's stream
    uint64_t Q;       // 0x00 stuffing bytes before its first owned byte
    uint32_t ftotal;  // 0xFF bytes it owns (its stuffing count)
    uint32_t split;   // value of its first byte when shared with the predecessor (P & 7 != 0)
    uint32_t fill;    // its 1-filled final byte (the last workgroup of a restart interval / the image)
    uint32_t seg;     // restart mode: its segment; the RST markers before its bytes = seg + seg_markers0
};

// A stripe's entropy summary (entropy_scan_kernel, summary mode): enough for the
// stripes to place their bytes after one all-gather.
struct StripeSummary {
    uint64_t bits;   // length of the stripe's stream (restart intervals: its bytes, markers and fills included)
    uint32_t ff[8];  // ff[a]: 0xFF bytes wholly inside the stripe when it starts at bit a (mod 8),
                     // the byte shared with the previous stripe and the final fill byte excluded
    uint32_t head;   // its first 8 bits (MSB-first byte)
    uint32_t tail;   // its last 8 bits
    uint32_t restart;  // 1: restart-interval stripe (byte-aligned; bits = byte length)
    uint32_t pad;
};

constexpr uint32_t kStripeFirst = 1u;  // holds the image's first bit: writes the headers
constexpr uint32_t kStripeLast = 2u;   // holds the last bit: 1-fill and EOI
constexpr uint32_t kExtPlace = 4u;     // pack kernel reads WgPlace (entropy_scan_kernel) instead of scanning

struct EntropyArgs {
    const int16_t* coef;
    const uint16_t* recs;    // the statistics kernel's symbol records (kTileRecords per tile)
    const uint32_t* tcount;  // records per tile
    Geometry g;
    const uint32_t* tables;  // [4][256] (len << 16) | code, followed by the header bytes
    uint8_t* out;            // whole .jpg; the kernel writes the header to [0, hdr_len)
    uint64_t hdr_len;
    uint64_t out_cap;
    uint8_t* ubuf;           // per-workgroup unstuffed regions (entropy_ubuf_bytes)
    uint8_t* rec;            // [entropy_grid][kEntropyRecordBytes] code -> pack kernel records
    uint32_t* done = nullptr;  // (zeroed per frame) code workgroups finished: the last one places all
    // (zeroed per frame) pack workgroups finished, then the last workgroup's end offset
    // (u64 at [2]) and no-space flag ([4]): the last to finish hands the result over
    uint32_t* pack_done = nullptr;
    uint64_t* host_result;   // mapped pinned host memory: [0] .jpg bytes, [1] no-space (4),
                             // [2] reserved (0), [3] = seq, written last, once every
                             // workgroup's output stores have completed (pack_done)
    uint64_t seq;            // the frame's sequence number
    // carried duty of the code kernel: export another frame's histograms to mapped
    // host memory (workgroup 0; exp_cnt == nullptr: none)
    HistPtrs exp_hist;
    uint32_t* exp_cnt;
    uint64_t* exp_key;
    uint64_t* exp_seq;
    uint64_t exp_seqv;
    uint32_t wgs;            // workgroup count override (0 = automatic; tests)
    DcSeed seed;             // DC chain predecessors (stripes)
    // placement (stripes / large grids): stream starts at global bit p_ext with q_ext
    // stuffing bytes before it; head_split = its first byte when p_ext & 7 != 0
    uint64_t p_ext = 0, q_ext = 0;
    uint32_t head_split = 0;
    uint32_t flags = kStripeFirst | kStripeLast;
    WgPlace* place = nullptr;          // [seg.grid()] (kExtPlace)
    StripeSummary* summary = nullptr;  // summary mode output
    Restart rst;                       // restart intervals (rst.mcus = 0: none)
    SegLayout seg;                     // workgroup partition (host: seg_layout)
    uint32_t seg_markers0 = 0;         // RST markers in this output before the frame's first segment (stripes)
    uint32_t seg_index0 = 0;           // the image's interval index of the frame's first segment (stripes)
    uint64_t out_base = 0;             // restart stripes: bytes of earlier stripes after the header
    uint64_t* dbg;
};

// tiles of a partition, and tile gt's blocks (the global tile number of segment s's
// tile i is s * tps + i)
JPGE_HD inline uint32_t seg_tiles(const SegLayout& L) { return (L.nseg - 1) * L.tps + L.ltps; }
JPGE_HD inline void seg_tile(const SegLayout& L, uint32_t gt, uint64_t& b0, uint32_t& nb) {
    uint32_t seg, i, tps, nbs;
    if (gt < (L.nseg - 1) * L.tps) {
        seg = gt / L.tps; i = gt % L.tps; tps = L.tps; nbs = L.sblk;
    } else {
        seg = L.nseg - 1; i = gt - seg * L.tps; tps = L.ltps; nbs = L.lblk;
    }
    b0 = (uint64_t)seg * L.sblk + (uint64_t)i * nbs / tps;
    nb = (uint32_t)((uint64_t)(i + 1) * nbs / tps - (uint64_t)i * nbs / tps);
}
// record sub-stream s (tile s / kRecSub, part s % kRecSub) and its blocks
JPGE_HD inline void sub_tile(const SegLayout& L, uint32_t s, uint64_t& b0, uint32_t& nb) {
    uint64_t tb;
    uint32_t tn;
    seg_tile(L, s / kRecSub, tb, tn);
    const uint32_t j = s % kRecSub;
    b0 = tb + j * tn / kRecSub;
    nb = (j + 1) * tn / kRecSub - j * tn / kRecSub;
}

inline uint32_t entropy_tiles(const Geometry& g) {
    return (g.nblocks() + kEntropyTile - 1) / kEntropyTile;
}
// bytes of one entropy workgroup's private region: its bit stream (workgroup-
// local offsets, worst case) plus slack, a whole number of 128-byte lines
constexpr uint64_t kEntropyRegionBytes = (uint64_t)kEntropyMaxTilesPerWg * kEntropyTile * kStageBytesPerBlock + 128;

// Kernel timing (sampled frames only): when given, the launch goes through
// hipExtLaunchKernel with these events, which the runtime binds to the kernel's own
// dispatch (its start and end timestamps, the ones rocprofv3 reports), so their
// elapsed time is the kernel's execution without launch gaps or marker packets.
struct KTimer {
    hipEvent_t start = nullptr, stop = nullptr;
};

// Frames launched together (frame sets): member f of a set owns workgroups
// [wg0[f], wg0[f + 1]) of one launch and runs exactly as if launched alone with its
// own arguments and wg0[f + 1] - wg0[f] workgroups.  The members share a geometry
// (one kernel shape).  Small frames go in sets: a 1080p frame's kernels alone leave
// most of the GPU idle while their fixed latencies (launch, first loads, last
// workgroup) pass, so 4 frames per launch do 4 frames' work in about one frame's
// latency.  Every kernel takes a set; a lone frame is a set of one.
constexpr int kMaxSet = 4;
// (N: the kernel instance's capacity; lone frames launch the N = 1 instance, whose
// kernel arguments are a quarter the size: a launch copies them whole)
template <typename A, int N = kMaxSet>
struct FrameSet {
    A a[N];
    uint32_t wg0[N + 1];
    uint32_t n;
};
// the member that owns workgroup b (uniform: scalar code; a fixed trip count, so the
// N = 1 instance reduces to member 0)
// (K2 keeps the rolled form: with it the compiler gives the statistics kernel 62 VGPRs
// instead of 69-70, and the kernel runs 4% faster)
JPGE_HD inline uint32_t set_member_rolled(const uint32_t* wg0, uint32_t n, uint32_t b) {
    uint32_t f = 0;
    for (uint32_t i = 1; i < n; ++i) f += b >= wg0[i] ? 1u : 0u;
    return f;
}
template <int N>
JPGE_HD inline uint32_t set_member(const uint32_t* wg0, uint32_t n, uint32_t b) {
    uint32_t f = 0;
    for (int i = 1; i < N; ++i) f += (i < (int)n && b >= wg0[i]) ? 1u : 0u;
    return f;
}
template <int N = kMaxSet, typename A>
inline FrameSet<A, N> frame_set(const A* a, int n, uint32_t grid_each) {
    FrameSet<A, N> s{};
    s.n = (uint32_t)n;
    for (int f = 0; f < n; ++f) {
        s.a[f] = a[f];
        s.wg0[f] = (uint32_t)f * grid_each;
    }
    s.wg0[n] = (uint32_t)n * grid_each;
    return s;
}

uint32_t fdct_grid(const Geometry& g, bool solo, uint32_t override_wgs = 0);
// statistics workgroups: wgs (0: 3 per CU), within the tile-table bound and the tile count
uint32_t stats_grid(const SegLayout& L, uint32_t wgs = 0);
// entropy partition of a frame: restart_mcus = 0 -> one segment over 128-block tiles
// (2..kEntropyMaxTilesPerWg per workgroup, about 384 workgroups or wgs_override)
SegLayout seg_layout(const Geometry& g, uint32_t restart_mcus, uint32_t wgs_override);
inline uint32_t entropy_grid(const Geometry& g, uint32_t wgs_override) { return seg_layout(g, 0, wgs_override).grid(); }

inline uint64_t entropy_ubuf_bytes(const SegLayout& L) { return (uint64_t)L.grid() * kEntropyRegionBytes; }

// Segment concatenation (concat.hip): segment k's len[k] bytes from src[k] to dst + off[k];
// workgroups [chunk0[k], chunk0[k+1]) copy segment k (concat_chunks(len, dst + off) each)
constexpr uint32_t kConcatMax = 96;  // segments per launch (the arguments stay under 4 KB)
struct ConcatArgs {
    uint8_t* dst;
    uint32_t n;
    uint32_t chunk0[kConcatMax + 1];
    const uint8_t* src[kConcatMax];
    uint64_t off[kConcatMax];
    uint64_t len[kConcatMax];
};
uint32_t concat_chunks(uint64_t len, uintptr_t dst);
hipError_t launch_concat(const ConcatArgs& a, uint32_t nchunks, hipStream_t s);

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s, const KTimer* t = nullptr);
hipError_t launch_stats(const StatsArgs& a, hipStream_t s, const KTimer* t = nullptr);
// frame sets (kMaxSet frames of one geometry, one launch per kernel): the members'
// arguments as launch_fdct / launch_stats / launch_entropy take them
hipError_t launch_fdct_set(const FdctArgs* a, int n, hipStream_t s, const KTimer* t = nullptr);
hipError_t launch_stats_set(const StatsArgs* a, int n, hipStream_t s, const KTimer* t = nullptr);
// (every member placed by its code kernel's last workgroup: a.done set, no restart)
hipError_t launch_entropy_set(const EntropyArgs* a, int n, hipStream_t s, const KTimer* code = nullptr,
                              const KTimer* pack = nullptr);
// [4][256] summed counts and keys into (mapped) host memory, then *host_seq = seq
hipError_t launch_hist_export(const HistPtrs& h, uint32_t* host_cnt, uint64_t* host_key, uint64_t* host_seq,
                              uint64_t seq, hipStream_t s);
// code + pack kernels (with the placement scan between them when kExtPlace)
hipError_t launch_entropy(const EntropyArgs& a, hipStream_t s, const KTimer* code = nullptr,
                          const KTimer* pack = nullptr);
// its two halves: the code kernel does not read hdr_len, so it can be queued before the
// header is known (encoder.cpp, encode()'s gate); the pack kernel (and placement)
hipError_t launch_entropy_code(const EntropyArgs& a, hipStream_t s, const KTimer* code = nullptr);
// encode()'s gate: wait (one workgroup, at most timeout_ticks of the 100 MHz realtime
// counter, then *fail = 1 and no copy) until *gate == value (mapped host memory), then copy
// n16 16-byte units src -> dst (src: device view of mapped host memory)
hipError_t launch_gate_copy(const uint32_t* gate, uint32_t value, const void* src, void* dst, uint32_t n16,
                            uint64_t* fail, uint64_t timeout_ticks, hipStream_t s);
hipError_t launch_entropy_pack(const EntropyArgs& a, hipStream_t s, const KTimer* pack = nullptr);
// stripes: code kernel + summary scan; then placement scan + pack kernel
hipError_t launch_entropy_code_summary(const EntropyArgs& a, hipStream_t s);
hipError_t launch_entropy_place_pack(const EntropyArgs& a, hipStream_t s);
// grids above this many workgroups place by a separate scan (each pack workgroup
// scanning every record would read G^2 records)
constexpr uint32_t kInlineScanMaxWgs = 1024;
// Grids the last code workgroup places (entropy_code_kernel, EntropyArgs::done).
// Hardware assumption (gfx950), not the HIP memory model's letter: each workgroup
// publishes its 48-byte record with agent-scope relaxed atomic stores, which gfx950
// issues write-through (sc1) to the agent's coherence point, waits for their
// completion (s_waitcnt vmcnt(0)), and only then counts itself with a device atomic
// performed at that point; the workgroup completing the count takes an agent-scope
// acquire fence (buffer_inv sc1) before reading every record.  The formal alternative,
// a release fence per workgroup, writes back the whole L2 (measured 26% slower).
// Covered by the GPU tests that run multi-lane batches and compare every frame with
// the oracle (test_gpu_parity.py: placement in code at 1..G workgroups, batches).
constexpr uint32_t kPlaceInCodeMaxWgs = 4096;

}  // namespace jpge
