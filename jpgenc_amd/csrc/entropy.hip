// K3 entropy coding (gfx950): Huffman emission (Image.cpp:737-829) in MCU
// interleave order (Image.cpp:957-968), 1-fill and 0xFF00 stuffing
// (BitstreamGeneric.hpp:213-248), EOI (Image.cpp:972).  Two launches:
//
// entropy_code_kernel — G persistent workgroups; workgroup w owns the contiguous
//   tiles [w*T/G, (w+1)*T/G) of 128 blocks (2..kEntropyMaxTilesPerWg tiles).
//   Its tiles' symbol records (written by the statistics kernel, stream order) form
//   one stream, in rounds of 4 records per thread across tile boundaries — code bits
//   from the tables, a workgroup scan of the bit counts, each record ORed into a
//   big-endian word stage at its workgroup-LOCAL bit offset (the next round's records
//   load meanwhile) — and complete words go to the workgroup's private region R when
//   the stage could not take another round (the partial last word carries over).
//   Then the workgroup counts
//   the 0xFF bytes its stream would hold at each of the 8 byte alignments and
//   writes a record {bits, first 8 bits, last 8 bits, ff[8]}.
// entropy_pack_kernel — G workgroups; each scans all G records (L2-resident): bit
//   offset P of its stream, alignment b = P & 7, the stuffed-byte prefix (every
//   record's count at its own alignment plus the bytes split between neighbours,
//   rebuilt from their edge bits) — then copies R shifted right by b bits to the
//   output with a 0x00 after every 0xFF (LDS, aligned 4-byte stores).  A byte
//   belongs to the workgroup holding its last bit; the last one 1-fills and writes
//   EOI.  No workgroup ever waits for another: the kernel boundary is the only
//   synchronisation.
// Global traffic: the symbol records once; R written once, read twice (L2 /
// Infinity Cache, workgroup-private lines); the workgroup records; the output once.
#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

constexpr int kK3Groups = 2;  // code kernel: 4-record groups per thread and round (one scan and barrier per round)
// waves per SIMD: the target is 7, and with 16-bit records and each group's bits
// concatenated before the round's scan the kernel takes 60 VGPRs, so it runs at 8 (4
// workgroups per CU): the pipeline +1.0% at Q90 and +2.8% at Q100 over the 66-VGPR form
// (3 per CU), and over an LDS-padded form held at 3 per CU (-3.6%); three groups per
// round (72 VGPRs) -3.4%.
constexpr int kK3Wpe = 7;
constexpr int kK3Blocks = kEntropyTile;
constexpr int kK3Threads = kK3Blocks * kPartsPerBlock;  // 512
constexpr int kK3Waves = kK3Threads / 64;
constexpr int kMaxTiles = kEntropyMaxTilesPerWg;
constexpr int kTcntSlots = kMaxTiles * kRecSub;  // record sub-streams of a workgroup's tiles
constexpr int kStageWords = kK3Blocks * kStageBytesPerBlock / 4 + 4;  // worst-case tile + lead
constexpr int kWin = 32;                                              // output bytes per lane per round
constexpr int kWinWords = kWin / 4;
static_assert(kWinWords == 8 && kEntropyRegionBytes % 16 == 0, "pack loads a window as two aligned uint4");
constexpr int kPackStoreAux = 16;  // sc1: write-through output stores (single-frame launches, pack_done)
constexpr int kPackStoreNt = 2;    // nt: streaming output stores (the pipeline: write-through cost 1.3%)
constexpr int kChunk = kK3Threads * kWin;                             // output bytes per round (pre-stuffing)

// per-workgroup record handed from the code kernel to the pack kernel
struct alignas(16) WgRecord {
    uint32_t ff[8];  // ff[b]: 0xFF bytes wholly inside the stream when it starts at bit b (mod 8)
    uint32_t bits;   // length of the workgroup's stream
    uint32_t edge;   // first 8 bits | last 8 bits << 8 (each as an MSB-first byte)
    uint32_t pad[2];
};
constexpr int kRecBits = 8, kRecEdge = 9;  // u32 indices
static_assert(sizeof(WgRecord) == kEntropyRecordBytes, "record size");

struct K3Lds {
    // the tile's big-endian bit stream (offset 0 of the kernel's only __shared__ object,
    // so 16-byte aligned; an alignas(16) here made the compiler spill 8 VGPRs)
    uint32_t stage[kStageWords];
    uint2 tab[4 * 256];           // lds_tab_entry, indexed by a record's bits 6-15
    uint32_t tcnt[kTcntSlots];    // symbol records of each sub-stream of the workgroup's tiles
    uint32_t tcum[kTcntSlots + 2];  // their first padded stream indices, the total, then a sentinel
    alignas(8) uint32_t wsum[2][kK3Waves];  // the rounds' scans, alternating (no barrier between rounds); the placement's 64-bit scans
    uint32_t cnt8[8];
    uint32_t carry;
};

// 0x80 in every byte of the big-endian word y that is 0xFF
__device__ __forceinline__ uint32_t ff_bytes(uint32_t y) {
    const uint32_t x = ~y;
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
// 0x80 in bytes [lo, hi) (0 = most significant) of a big-endian word; 0 <= lo, hi <= 4
__device__ __forceinline__ uint32_t byte_range(int lo, int hi) {
    const uint32_t ge = lo >= 4 ? 0u : 0xFFFFFFFFu >> (8 * lo);
    const uint32_t lt = hi >= 4 ? 0xFFFFFFFFu : ~(0xFFFFFFFFu >> (8 * hi));
    return ge & lt & 0x80808080u;
}

// The code kernel's LDS table entry for record index i = record >> 6 (kernels.hpp):
// table t = i >> 8, symbol s = i & 255.  .x = the code shifted past the extra bits the
// record holds, .y = that count | (code length + count) << 8.  A continuation (an AC
// index of size 0 and run n in 1..14) is n raw bits.  Host entries are (len << 16) | code.
// (Code lengths and bit counts clamped: whatever the tables and records hold, a record
// codes at most 16 + 6 bits, the bound the stage and region sizes assume.)
__device__ __forceinline__ uint2 lds_tab_entry(const uint32_t* tables, uint32_t i) {
    const uint32_t s = i & 0xFF, size = (i & 0x100) ? s & 15 : s, run = s >> 4;
    const bool cont = (i & 0x100) && size == 0 && run - 1u < 14u;
    const uint32_t host = cont ? 0u : tables[i], nb = min(cont ? run : size, kRecXBits);
    const uint32_t len = min(host >> 16, 16u);
    return make_uint2((host & 0xFFFF & ((1u << len) - 1u)) << nb, nb | ((len + nb) << 8));
}
// The record in bits [off, off + 16) of w as code bits: the table's code, then the extra
// bits the record holds; returns the bit count (<= 16 + 6).  (A read, two bit-field
// extracts, an OR and a shift; v_bfe takes the width from the entry's low 5 bits.)
__device__ __forceinline__ uint32_t rec_bits(uint32_t w, uint32_t off, const uint2* tab, uint32_t& bits) {
    const uint2 e = tab[__builtin_amdgcn_ubfe(w, off + 6u, 10u)];
    bits = e.x | __builtin_amdgcn_ubfe(w, off, e.y);
    return e.y >> 8;
}

// every workgroup's WgPlace from the records (the placement scan), kK3Threads threads
__device__ void place_all(const EntropyArgs& a, uint32_t G, uint32_t* wsum, int tid);
__device__ void write_wg_record(const EntropyArgs& a, uint32_t wg, uint32_t G, uint32_t edge, uint32_t Lb,
                                const uint32_t* cnt8, uint32_t* flag, uint32_t* wsum, int tid);

template <int kN>
__global__ __launch_bounds__(kK3Threads) __attribute__((amdgpu_waves_per_eu(kK3Wpe))) void entropy_code_kernel(
    FrameSet<EntropyArgs, kN> fs) {
    __shared__ K3Lds L;
    const uint32_t set_f = set_member<kN>(fs.wg0, fs.n, blockIdx.x);  // (frame sets: kernels.hpp)
    const EntropyArgs& a = fs.a[set_f];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t wg = blockIdx.x - fs.wg0[set_f], G = fs.wg0[set_f + 1] - fs.wg0[set_f];
    JPGE_STAMP(0);
    if (a.exp_cnt && wg == 0)  // carried: a later frame's histograms to the host
        export_hist<kK3Threads>(a.exp_hist, a.exp_cnt, a.exp_key, a.exp_seq, a.exp_seqv, tid);
    if (tid == 0) L.carry = 0;
    if (tid < 8) L.cnt8[tid] = 0;
    for (int i = tid; i < 1024; i += kK3Threads) L.tab[i] = lds_tab_entry(a.tables, (uint32_t)i);
    // (the stage zeroed in 16-byte stores; with K2's: 185.8 vs 184.4 GPix/s over 3 pairs)
    static_assert(kStageWords % 4 == 0, "the stage zeroes in 16-byte stores");
    for (int i = tid; i < kStageWords / 4; i += kK3Threads) reinterpret_cast<uint4*>(L.stage)[i] = make_uint4(0, 0, 0, 0);
    const WgTiles wt = wg_tiles(a.seg, wg);  // 1..kMaxTiles tiles of one segment (seg_layout)
    const int ntl = (int)wt.nt * kRecSub;  // the tiles' record sub-streams (kernels.hpp)
    if (tid < 64) {  // (wave 0: ntl <= kTcntSlots <= 64) the counts, and their padded prefix
        static_assert(kTcntSlots <= 63, "one wave scans the sub-stream counts");
        const uint32_t c = tid < ntl ? a.tcount[(wt.seg * a.seg.tps + wt.t0) * kRecSub + tid] : 0u;
        if (tid < ntl) L.tcnt[tid] = c;
        const uint32_t inc = wave_scan_incl((c + 3u) & ~3u);
        if (tid < ntl) L.tcum[tid + 1] = inc;
        if (tid == 0) L.tcum[0] = 0;
        if (tid == ntl) L.tcum[ntl + 1] = ~0u;
    }
    uint8_t* R8 = a.ubuf + (uint64_t)wg * kEntropyRegionBytes;
    uint32_t* R32 = reinterpret_cast<uint32_t*>(R8);

    // ---- emit the workgroup's records at workgroup-local bit offsets into R ----
    // The symbol records (K2) in rounds of 4 per thread: code bits of each, a
    // workgroup scan of the thread totals, each thread's records ORed into the stage at
    // its offset (every record spans at most two words).
    uint32_t wl = 0;  // workgroup-local bit position of the stage's first word
    // 0xFF bytes of the stream at each byte alignment, counted on the stage words as
    // they are stored (see the note after the loop).  A word's count needs the next
    // word's first 7 bits: the last complete word of a flush waits (thread 0's `pend`)
    // until the next flush has completed the word after it.
    uint32_t c8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto count_word = [&](uint32_t x, uint32_t nx) {
        uint32_t y = x;  // bit 31-t: stream bits [32m+t, 32m+t+8) are all ones
#pragma unroll
        for (int k = 1; k < 8; ++k) y &= __builtin_amdgcn_alignbit(x, nx, 32 - k);
#pragma unroll
        for (int r = 0; r < 8; ++r) c8[(8 - r) & 7] += __builtin_popcount(y & (0x80808080u >> r));
    };
    uint32_t pend = 0;
    bool has_pend = false;
    uint32_t head = 0;  // (thread 0) the stream's first 8 bits, from its first complete word
    uint64_t tq = JPGE_NOW();
    // Records through a buffer descriptor over this workgroup's tiles: every round
    // issues its next load unconditionally (past the end: an out-of-range offset,
    // zeros), so no branch merges in-flight registers and the in-order wait for a
    // round's records never waits for the prefetch behind it.
    const uint32_t gt0 = wt.seg * a.seg.tps + wt.t0;  // global number of the first tile
    constexpr uint32_t slot = kSubRecords;  // records per sub-stream
    const __amdgpu_buffer_rsrc_t rec_rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(a.recs + (uint64_t)gt0 * kTileRecords), 0, ntl * slot * 2, 0x00020000);
    constexpr int kGroups = kK3Groups;            // groups of 4 records per thread and round
    constexpr uint32_t kRound = 4 * kGroups * kK3Threads;  // records per round
    // The workgroup's records are one stream over its tiles: tile t's count padded to a
    // multiple of 4 (so a thread's 4 records are in one tile; the padding is never
    // valid), rounds of kRound records run across tile boundaries, and the stage is
    // flushed to R only when the next round might not fit (usually once, at the end).
    lds_barrier();  // the tile counts
    const uint32_t total = __builtin_amdgcn_readfirstlane(L.tcum[ntl]);  // padded records of all the workgroup's tiles
    uint32_t cs = 0;  // this thread's sub-stream cursor
    // the thread's 4 records from stream index i (nvalid: how many are records); the
    // cursor walks the padded prefix (the sentinel past the total stops it at ntl)
    auto rec_load = [&](uint32_t i, uint32_t& nvalid) -> uint2 {
        while (i >= L.tcum[cs + 1]) ++cs;
        uint32_t off = 0xFFFFFFF0u;  // (past the end: out of range, zeros)
        nvalid = 0;
        if (cs < (uint32_t)ntl) {
            const uint32_t rel = i - L.tcum[cs], c = L.tcnt[cs];
            nvalid = c > rel ? min(c - rel, 4u) : 0u;
            off = (cs * slot + rel) * 2;
        }
        return as_u2(__builtin_amdgcn_raw_buffer_load_b64(rec_rs, off, 0, 0));
    };
    constexpr uint32_t kStageBits = (kStageWords - 2) * 32;
    constexpr uint32_t kRoundMaxBits = kRound * 22;  // (a record codes at most 16 + 6 bits)
    static_assert(kStageBits > kRoundMaxBits, "the stage holds a round");
    uint2 nxt[kGroups];
    uint32_t nvn[kGroups];
#pragma unroll
    for (int g = 0; g < kGroups; ++g) nxt[g] = rec_load(4 * (kGroups * tid + g), nvn[g]);
    uint32_t lead = 0, pos = 0;  // bit position in the stage (lead: the carried partial word's bits)
    uint32_t par = 0;            // scan buffer of this round
    for (uint32_t r0 = 0; r0 < total; r0 += kRound) {
        // per group: its records' bits concatenated (acc: exact when they total <= 64 bits)
        // and their count; the records themselves for the rare longer group
        uint64_t acc[kGroups];
        uint32_t gl[kGroups], tl = 0;
        uint2 rvs[kGroups];
        uint32_t nvs[kGroups];

#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
            rvs[g] = nxt[g];
            nvs[g] = nvn[g];
            nxt[g] = rec_load(r0 + kRound + 4 * (kGroups * tid + g), nvn[g]);  // the next round's (prefetch)
            const uint32_t rr[4] = {rvs[g].x, rvs[g].x, rvs[g].y, rvs[g].y};
            gl[g] = 0;
            acc[g] = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t cb;
                const uint32_t n = (uint32_t)q < nvs[g] ? rec_bits(rr[q], (uint32_t)(q & 1) * 16u, L.tab, cb) : 0u;
                acc[g] = (acc[g] << n) | (n ? (uint64_t)cb : 0ull);
                gl[g] += n;
            }
            tl += gl[g];
        }
        JPGE_ACC(3, tq);
        uint32_t T;
        // (the one barrier of a round: wsum alternates, so no wave can overwrite a total
        // another still reads, and the stage ORs of consecutive rounds commute)
        const uint32_t ex = block_scan<kK3Waves, uint32_t, uint32_t, true, false>(tl, L.wsum[par], lane, wv, T);
        par ^= 1u;
        JPGE_ACC(4, tq);
        uint32_t bp = pos + ex;
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
        // A group's 4 records are adjacent in the stream: concatenated in a 64-bit word
        // they touch at most three stage words, of which only the first and the last
        // can be shared with a neighbour (LDS OR); a middle word is the thread's alone
        // (plain store).  One to three LDS writes instead of one or two atomics per
        // record.  More than 64 bits (rare: four long codes) take the per-record path.
        const uint32_t tg = gl[g];
        if (tg && tg <= 64) {
            const uint64_t A = acc[g] << (64 - tg);  // MSB-aligned
            const uint32_t sh = bp & 31, w = bp >> 5, end = sh + tg;
            const uint32_t hi = (uint32_t)(A >> 32), lo = (uint32_t)A;
            atomicOr(&L.stage[w], hi >> sh);
            if (end > 32) {
                const uint32_t v1 = sh ? (hi << (32 - sh)) | (lo >> sh) : lo;
                if (end >= 64) L.stage[w + 1] = v1;
                else atomicOr(&L.stage[w + 1], v1);
                if (end > 64) atomicOr(&L.stage[w + 2], lo << (32 - sh));
            }
            bp += tg;
        } else if (tg) {
            const uint32_t rr[4] = {rvs[g].x, rvs[g].x, rvs[g].y, rvs[g].y};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // each record into the one or two stage words it spans (a branch per record:
            // a branch-free 64-bit form ran 6 us slower per 4K frame)
            uint32_t cb;
            const uint32_t n = (uint32_t)q < nvs[g] ? rec_bits(rr[q], (uint32_t)(q & 1) * 16u, L.tab, cb) : 0u;
            if (n) {
                const uint32_t sh = bp & 31;
                const uint32_t v = cb << (32 - n);  // MSB-aligned (n >= 1)
                atomicOr(&L.stage[bp >> 5], v >> sh);
                if (sh + n > 32) atomicOr(&L.stage[(bp >> 5) + 1], v << (32 - sh));
                bp += n;
            }
        }
        }
        }
        pos += T;
        JPGE_ACC(6, tq);
        if (r0 + kRound < total && pos + kRoundMaxBits <= kStageBits) continue;
        // ---- flush: complete words to R, the partial word carried ----
        lds_barrier();  // every record of the stage ORed in
        const uint32_t ncw = pos >> 5;  // complete words in the stage
        const uint32_t wbase = wl >> 5;
        for (uint32_t w = tid; w < ncw; w += kK3Threads) {
            uint32_t v = L.stage[w];
            if (w == 0) v |= L.carry;  // partial last word of the previous flush
            R32[wbase + w] = __builtin_bswap32(v);
            if (w + 1 < ncw) count_word(v, L.stage[w + 1]);
        }
        if (tid == 0) {  // (thread 0 consumed the old carry above)
            if (ncw) {
                const uint32_t w0 = L.stage[0] | L.carry;
                if (has_pend) count_word(pend, w0);
                else head = w0 >> 24;
                pend = ncw == 1 ? w0 : L.stage[ncw - 1];
                has_pend = true;
            }
            uint32_t v = L.stage[ncw];
            if (ncw == 0) v |= L.carry;
            L.carry = v;
        }
        // the stage words used back to zero once everyone has read them (the stage
        // starts zeroed, so the rounds OR records in without a zeroing barrier); after
        // the last round nothing reuses the stage (thread 0 alone reads its carry)
        const bool more = r0 + kRound < total;
        if (more) {
            lds_barrier();
            for (uint32_t w = tid; w <= ncw; w += kK3Threads) L.stage[w] = 0;
            lds_barrier();
        }
        wl += pos - lead;
        lead = wl & 31;
        pos = lead;
        JPGE_ACC(2, tq);
    }
    const uint32_t Lb = wl;  // this workgroup's bits (>= 6: every block codes >= 2 bits, >= 3 blocks)
    // (thread 0) the stream's first and last 8 bits for the record, from the last complete
    // word and the partial one in registers: nothing reads R back, so no wave waits here
    // for its region stores to complete (the pack kernel reads R after the launch boundary).
    // A stream shorter than a byte (a 4:4:4 restart interval of one MCU) is only ever
    // placed byte-aligned: its "last 8 bits" are its bits, right-aligned.
    uint32_t edge = 0;
    if (tid == 0) {
        const uint32_t r = Lb & 31, carry = L.carry;
        if (r) R32[Lb >> 5] = __builtin_bswap32(carry);
        if (!has_pend) head = carry >> 24;
        const uint32_t tail = ((has_pend ? pend << r : 0u) | (r ? carry >> (32 - r) : 0u)) & 0xFFu;
        edge = head | (tail << 8);
    }
    JPGE_STAMP(1);

    // ---- 0xFF bytes of the stream at each byte alignment b ----
    // Starting at global bit offset P (b = P & 7), output byte j of this workgroup
    // holds local bits [8j - b, 8j - b + 8): it is 0xFF iff 8 one-bits start at
    // s = 8j - b.  Every run start was marked (y) and counted by s = -b (mod 8) as
    // the words were stored; the last complete word and the final partial word are
    // counted here, against zero padding.  Starts s < 0 (the byte split with the
    // predecessor) do not exist and runs past Lb meet the zero padding, so ff[b]
    // counts exactly the bytes wholly inside.
    if (tid == 0) {
        const uint32_t tail = (Lb & 31) ? L.carry : 0u;
        if (has_pend) count_word(pend, tail);
        if (Lb & 31) count_word(tail, 0u);
    }
    {
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint32_t s = c8[b];
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
            if (lane == 0 && s) atomicAdd(&L.cnt8[b], s);
        }
    }
    __syncthreads();
    write_wg_record(a, wg, G, edge, Lb, L.cnt8, &L.carry, &L.wsum[0][0], tid);
    JPGE_STAMP(2);
}

// The workgroup's record {bits, edge bits, ff[8]} for the pack kernel, and (a.done)
// the placement of every workgroup by the last one to finish.  flag: a scratch LDS
// word; wsum: 16 LDS words, 8-byte aligned (place_all's 64-bit scans).
__device__ void write_wg_record(const EntropyArgs& a, uint32_t wg, uint32_t G, uint32_t edge, uint32_t Lb,
                                const uint32_t* cnt8, uint32_t* flag, uint32_t* wsum, int tid) {
    if (tid < 3) {
        uint32_t* rec = reinterpret_cast<uint32_t*>(a.rec + (uint64_t)wg * kEntropyRecordBytes);
        uint4 v;
        if (tid == 0) {
            v = make_uint4(Lb, edge, 0u, 0u);  // (thread 0's first 8 bits | last 8 bits << 8)
        } else {
            const int b0 = 4 * (tid - 1);  // ff[0..3], ff[4..7]
            v = make_uint4(cnt8[b0], cnt8[b0 + 1], cnt8[b0 + 2], cnt8[b0 + 3]);
        }
        uint32_t* dst = rec + (tid == 0 ? 8 : 4 * (tid - 1));
        if (a.done) {
            // device-coherent stores (through this XCD's L2), complete before the count
            // below; a release fence would write back the whole L2 (26% slower)
            __hip_atomic_store(dst + 0, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(dst + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(dst + 2, v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(dst + 3, v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            vm_drain();
        } else {
            *reinterpret_cast<uint4*>(dst) = v;
        }
    }
    if (a.done) {
        // Placement by the last workgroup to finish (no placement launch between this
        // kernel and the pack kernel): every workgroup counts itself after its record is
        // visible device-wide; the one that completes the count reads all records.
        __syncthreads();
        if (tid == 0) *flag = atomicAdd(a.done, 1u) == G - 1 ? 1u : 0u;
        __syncthreads();
        if (*flag) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the other workgroups' records)
            place_all(a, G, wsum, tid);
        }
    }
}

// ---- record scan: bit offsets, byte splits and 0xFF prefixes ----
// A byte belongs to the workgroup holding its last bit.  The byte split between
// records k-1 and k (alignment b_k = P_k & 7 != 0) is rebuilt from k-1's last b_k
// bits and k's first 8 - b_k bits and counted for k; for k == 0 it is the byte the
// stripe shares with the previous stripe (a.head_split).  The image's last record
// owns the 1-filled final byte.
struct RecView {
    const uint8_t* base;
    uint32_t G;
    __device__ __forceinline__ const uint32_t* operator()(uint32_t k) const {
        return reinterpret_cast<const uint32_t*>(base + (uint64_t)k * kEntropyRecordBytes);
    }
};

__device__ __forceinline__ uint32_t split_bits(uint32_t ptail, uint32_t head, uint32_t b) {  // 0 < b < 8
    return (((ptail & ((1u << b) - 1)) << (8 - b)) | ((head & 0xFF) >> b)) & 0xFF;
}
__device__ __forceinline__ uint32_t split_byte(const RecView& R, uint32_t k, uint32_t b, const EntropyArgs& a) {
    if (k == 0) return a.head_split;
    return split_bits((R(k - 1)[kRecEdge] >> 8) & 0xFF, R(k)[kRecEdge], b);
}
__device__ __forceinline__ uint32_t fill_byte(uint32_t eb, uint32_t edge) {  // Bitstream::fill, BitstreamGeneric.hpp:243-248
    return ((((edge >> 8) & ((1u << eb) - 1)) << (8 - eb)) | (0xFFu >> eb)) & 0xFF;
}
// 0xFF bytes owned by record k when its stream starts at global bit p
__device__ __forceinline__ uint32_t owned_ff(const RecView& R, uint32_t k, uint64_t p, const EntropyArgs& a) {
    const uint32_t* r = R(k);
    const uint32_t b = (uint32_t)(p & 7), edge = r[kRecEdge];
    uint32_t f = r[b];
    if (b) f += split_byte(R, k, b, a) == 0xFF;
    const uint32_t eb = (uint32_t)((p + r[kRecBits]) & 7);
    if (k == R.G - 1 && (a.flags & kStripeLast) && eb) f += fill_byte(eb, edge) == 0xFF;
    return f;
}

// Thread t takes records [t*per, (t+1)*per); fn(k, P, Q, owned) for each of them.
template <int kWaves, class F>
__device__ __forceinline__ void scan_records(const EntropyArgs& a, const RecView& R, uint32_t* wsum, int tid, F&& fn) {
    const int lane = tid & 63, wv = tid >> 6;
    const uint32_t per = (R.G + kWaves * 64 - 1) / (kWaves * 64);
    const uint32_t k0 = min(R.G, tid * per), k1 = min(R.G, k0 + per);
    uint64_t lsum = 0;
    for (uint32_t k = k0; k < k1; ++k) lsum += R(k)[kRecBits];
    uint64_t ltot;
    const uint64_t pbase = a.p_ext + block_scan<kWaves>(lsum, wsum, lane, wv, ltot);
    uint64_t fsum = 0;
    {
        uint64_t p = pbase;
        for (uint32_t k = k0; k < k1; ++k) {
            fsum += owned_ff(R, k, p, a);
            p += R(k)[kRecBits];
        }
    }
    uint64_t ftot;
    const uint64_t fbase = a.q_ext + block_scan<kWaves>(fsum, wsum, lane, wv, ftot);
    uint64_t p = pbase, q = fbase;
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t o = owned_ff(R, k, p, a);
        fn(k, p, q, o);
        q += o;
        p += R(k)[kRecBits];
    }
}

__device__ __forceinline__ WgPlace make_place(const RecView& R, uint32_t k, uint64_t p, uint64_t q, uint32_t owned,
                                              const EntropyArgs& a) {
    const uint32_t* r = R(k);
    const uint32_t b = (uint32_t)(p & 7), edge = r[kRecEdge];
    const uint32_t eb = (uint32_t)((p + r[kRecBits]) & 7);
    WgPlace w;
    w.P = p;
    w.Q = q;
    w.ftotal = owned;
    w.split = b ? split_byte(R, k, b, a) : 0u;
    w.fill = (k == R.G - 1 && (a.flags & kStripeLast) && eb) ? fill_byte(eb, edge) : 0u;
    w.seg = 0;
    return w;
}

constexpr int kScanThreads = 1024;

// Restart mode (a.rst.mcus != 0): segment-aligned placement.  Each segment (restart
// interval) starts on a byte boundary; its last workgroup owns the segment's
// 1-filled final byte; inside a segment the records split bytes as above.  Thread t
// takes whole segments [t*per, (t+1)*per).  P counts entropy bits (each segment
// rounded up to a whole byte), Q the 0x00 stuffing bytes before; the pack kernel
// adds 2 bytes per RST marker before the workgroup's segment.
__device__ void place_restart(const EntropyArgs& a, const RecView& R, uint32_t* wsum, int tid) {
    constexpr int kW = kScanThreads / 64;
    const int lane = tid & 63, wv = tid >> 6;
    const SegLayout& L = a.seg;
    const uint32_t per = (L.nseg + kScanThreads - 1) / kScanThreads;
    const uint32_t s0 = min(L.nseg, tid * per), s1 = min(L.nseg, s0 + per);
    auto rec0 = [&](uint32_t s) { return s * L.wps; };
    auto nrec = [&](uint32_t s) { return s + 1 < L.nseg ? L.wps : L.lwps; };
    uint64_t lsum = 0;
    for (uint32_t s = s0; s < s1; ++s) {
        uint64_t t = 0;
        for (uint32_t k = rec0(s); k < rec0(s) + nrec(s); ++k) t += R(k)[kRecBits];
        lsum += (t + 7) & ~7ull;
    }
    uint64_t ptot;
    const uint64_t pbase = block_scan<kW>(lsum, wsum, lane, wv, ptot);
    // 0xFF bytes record k owns when its stream starts at bit p: inside bytes at its
    // alignment, the byte split with its predecessor (b != 0: never a segment's first
    // record), the segment's 1-filled final byte
    auto owned = [&](uint32_t s, uint32_t k, uint64_t p, uint32_t& split, uint32_t& fill) -> uint32_t {
        const uint32_t* r = R(k);
        const uint32_t b = (uint32_t)(p & 7), eb = (uint32_t)((p + r[kRecBits]) & 7);
        uint32_t f = r[b];
        split = b ? split_bits((R(k - 1)[kRecEdge] >> 8) & 0xFF, r[kRecEdge], b) : 0u;
        fill = (k == rec0(s) + nrec(s) - 1 && eb) ? fill_byte(eb, r[kRecEdge]) : 0u;
        return f + (b && split == 0xFF) + (fill == 0xFF);
    };
    uint64_t fsum = 0;
    {
        uint64_t p = pbase;
        for (uint32_t s = s0; s < s1; ++s) {
            for (uint32_t k = rec0(s); k < rec0(s) + nrec(s); ++k) {
                uint32_t sp, fl;
                fsum += owned(s, k, p, sp, fl);
                p += R(k)[kRecBits];
            }
            p = (p + 7) & ~7ull;
        }
    }
    uint64_t ftot;
    const uint64_t fbase = a.q_ext + block_scan<kW>(fsum, wsum, lane, wv, ftot);
    uint64_t p = pbase, q = fbase;
    for (uint32_t s = s0; s < s1; ++s) {
        for (uint32_t k = rec0(s); k < rec0(s) + nrec(s); ++k) {
            WgPlace w;
            w.P = p;
            w.Q = q;
            w.ftotal = owned(s, k, p, w.split, w.fill);
            w.seg = s;
            a.place[k] = w;
            q += w.ftotal;
            p += R(k)[kRecBits];
        }
        p = (p + 7) & ~7ull;
    }
    if (a.summary && s0 < s1 && s1 == L.nseg) {  // the frame's (stripe's) entropy byte length
        StripeSummary sm{};
        sm.bits = (p >> 3) + (q - a.q_ext) + 2ull * (L.nseg - 1 + a.seg_markers0);
        sm.restart = 1;
        *a.summary = sm;
    }
}

// entropy_scan_kernel — one workgroup over all G records.  Place mode: every
// workgroup's WgPlace (large grids, stripes).  Summary mode: the stripe's bits,
// edge bytes and its internal 0xFF count at each of the 8 start alignments.
__global__ __launch_bounds__(kScanThreads) void entropy_scan_kernel(EntropyArgs a, uint32_t G, int summary) {
    __shared__ uint32_t wsum[2 * (kScanThreads / 64)];
    __shared__ uint32_t tot8[8];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const RecView R{a.rec, G};
    if (!summary && a.rst.mcus) {
        place_restart(a, R, wsum, tid);
        return;
    }
    if (!summary) {
        scan_records<kScanThreads / 64>(a, R, wsum, tid, [&](uint32_t k, uint64_t p, uint64_t q, uint32_t o) {
            a.place[k] = make_place(R, k, p, q, o, a);
        });
        return;
    }
    if (tid < 8) tot8[tid] = 0;
    const uint32_t per = (G + kScanThreads - 1) / kScanThreads;
    const uint32_t k0 = min(G, tid * per), k1 = min(G, k0 + per);
    uint64_t lsum = 0;
    for (uint32_t k = k0; k < k1; ++k) lsum += R(k)[kRecBits];
    uint64_t total;
    const uint64_t pbase = block_scan<kScanThreads / 64>(lsum, wsum, lane, wv, total);  // stripe-local
    uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // c[al]: stripe starting at bit al (mod 8)
    {
        uint64_t p = pbase;
        for (uint32_t k = k0; k < k1; ++k) {
            const uint32_t* r = R(k);
#pragma unroll
            for (int al = 0; al < 8; ++al) {
                const uint32_t b = (uint32_t)((p + al) & 7);
                c[al] += r[b];
                if (b && k > 0) c[al] += split_bits((R(k - 1)[kRecEdge] >> 8) & 0xFF, r[kRecEdge], b) == 0xFF;
            }
            p += r[kRecBits];
        }
    }
#pragma unroll
    for (int al = 0; al < 8; ++al) {
        uint32_t v = c[al];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
        if (lane == 0 && v) atomicAdd(&tot8[al], v);
    }
    __syncthreads();
    if (tid == 0) {
        StripeSummary sm{};
        sm.bits = total;
#pragma unroll
        for (int al = 0; al < 8; ++al) sm.ff[al] = tot8[al];
        sm.head = R(0)[kRecEdge] & 0xFF;
        sm.tail = (R(G - 1)[kRecEdge] >> 8) & 0xFF;
        *a.summary = sm;
    }
}

__device__ void place_all(const EntropyArgs& a, uint32_t G, uint32_t* wsum, int tid) {
    const RecView R{a.rec, G};
    scan_records<kK3Waves>(a, R, wsum, tid, [&](uint32_t k, uint64_t p, uint64_t q, uint32_t o) {
        a.place[k] = make_place(R, k, p, q, o, a);
    });
}

// entropy_place_kernel — the scan kernel's place mode in a smaller workgroup for
// grids up to kPlaceSmallMaxWgs (restart off): a 4-wave workgroup finds a CU beside
// the other lanes' kernels sooner than a 16-wave one, and the lane's stream waits on it.
constexpr int kPlaceThreads = 256;
constexpr uint32_t kPlaceSmallMaxWgs = 4096;
__global__ __launch_bounds__(kPlaceThreads) void entropy_place_kernel(EntropyArgs a, uint32_t G) {
    __shared__ uint32_t wsum[2 * (kPlaceThreads / 64)];
    const RecView R{a.rec, G};
    scan_records<kPlaceThreads / 64>(a, R, wsum, threadIdx.x, [&](uint32_t k, uint64_t p, uint64_t q, uint32_t o) {
        a.place[k] = make_place(R, k, p, q, o, a);
    });
}
// the place mode's launch: the small kernel where it applies, else the scan kernel
hipError_t launch_place(const EntropyArgs& b, uint32_t G, hipStream_t s) {
    if (!b.rst.mcus && G <= kPlaceSmallMaxWgs && kPlaceThreads < kScanThreads)
        hipLaunchKernelGGL(entropy_place_kernel, dim3(1), dim3(kPlaceThreads), 0, s, b, G);
    else
        hipLaunchKernelGGL(entropy_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, b, G, 0);
    return hipGetLastError();
}

struct PackLds {
    uint8_t ob[2 * kChunk + 8];  // stuffed output of one round
    uint32_t wsum[2 * kK3Waves];  // (room for 64-bit scans)
    uint64_t P, Q;
    uint32_t Lb, ftotal, split, fill, seg;
};

template <int kN>
__global__ __launch_bounds__(kK3Threads) void entropy_pack_kernel(FrameSet<EntropyArgs, kN> fs) {
    __shared__ PackLds S;
    const uint32_t set_f = set_member<kN>(fs.wg0, fs.n, blockIdx.x);  // (frame sets: kernels.hpp)
    const EntropyArgs& a = fs.a[set_f];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t wg = blockIdx.x - fs.wg0[set_f], G = fs.wg0[set_f + 1] - fs.wg0[set_f];
    const bool last = wg == G - 1;
    const bool eoi = last && (a.flags & kStripeLast);
    // the workgroup 1-fills its final byte: the image's end, or (restart) its segment's
    const WgTiles wt = wg_tiles(a.seg, wg);
    const bool fills = a.rst.mcus ? wt.last : eoi;
    JPGE_STAMP(0);
    // With pack_done (single-frame launches of a 1-lane encoder) every output byte is
    // stored write-through (sc1), so once a workgroup's stores have completed its bytes
    // are in memory, not in its XCD's L2; the pipeline streams them (nt).  Single bytes
    // (headers, markers, EOI) are always written through.
    const bool wthru = a.pack_done != nullptr;
    const __amdgpu_buffer_rsrc_t out_rs = __builtin_amdgcn_make_buffer_rsrc(
        a.out, 0, (int)(a.out_cap < 0x7FFFFFF0ull ? a.out_cap : 0x7FFFFFF0ull), 0x00020000);
    auto out_byte = [&](uint64_t i, uint32_t v) {  // (single bytes: headers, markers, EOI)
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, out_rs, (uint32_t)i, 0, kPackStoreAux);
    };
    if (wg == 0 && (a.flags & kStripeFirst)) {  // the headers (SOI .. SOS) travel behind the tables
        const uint8_t* hdr = reinterpret_cast<const uint8_t*>(a.tables + 1024);
        for (uint32_t i = tid; i < a.hdr_len; i += kK3Threads) out_byte(i, hdr[i]);
    }

    // ---- this workgroup's placement: from the scan kernel, or scanned here ----
    const RecView R{a.rec, G};
    if (a.flags & kExtPlace) {
        if (tid == 0) {
            const WgPlace w = a.place[wg];
            S.P = w.P;
            S.Q = w.Q;
            S.ftotal = w.ftotal;
            S.split = w.split;
            S.fill = w.fill;
            S.seg = w.seg;
            S.Lb = R(wg)[kRecBits];
        }
    } else {
        scan_records<kK3Waves>(a, R, S.wsum, tid, [&](uint32_t k, uint64_t p, uint64_t q, uint32_t o) {
            if (k != wg) return;
            const WgPlace w = make_place(R, k, p, q, o, a);
            S.P = w.P;
            S.Q = w.Q;
            S.ftotal = w.ftotal;
            S.split = w.split;
            S.fill = w.fill;
            S.seg = 0;
            S.Lb = R(k)[kRecBits];
        });
    }
    __syncthreads();
    JPGE_STAMP(1);

    // ---- shifted, stuffed copy R -> output ----
    const uint64_t P = S.P;
    const uint32_t b = (uint32_t)(P & 7), Lb = S.Lb, ftotal = S.ftotal;
    const uint32_t nc = (b + Lb) >> 3;  // complete output bytes
    const uint32_t eb = (b + Lb) & 7;   // bits in the byte after them
    const uint32_t n_own = nc + ((fills && eb) ? 1u : 0u);
    const uint32_t markers = a.rst.mcus ? S.seg + a.seg_markers0 : 0u;  // RST markers before this segment
    const uint64_t D0 = a.hdr_len + a.out_base + (P >> 3) + S.Q + 2ull * markers;
    const uint64_t ntot = (uint64_t)n_own + ftotal + (eoi ? 2u : 0u);
    const bool fits = D0 + ntot <= a.out_cap;
    if (fits && wt.first && markers && tid == 0) {  // RSTn ahead of the segment (not stuffed)
        uint8_t* const m = a.out + D0 - 2;
        const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(m, 0, 2, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0xFF, mrs, 0, 0, kPackStoreAux);
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(0xD0 + ((a.seg_index0 + S.seg - 1) & 7)), mrs, 1, 0,
                                             kPackStoreAux);  // RST(interval - 1 mod 8)
    }
    const uint32_t split = S.split, fill = S.fill;
    const uint32_t* R32 = reinterpret_cast<const uint32_t*>(a.ubuf + (uint64_t)wg * kEntropyRegionBytes);
    const uint32_t nwr = (Lb + 31) >> 5;
    auto rword = [&](int64_t m) -> uint32_t {
        return (m >= 0 && m < (int64_t)nwr) ? __builtin_bswap32(R32[m]) : 0u;
    };
    uint64_t d = D0;
    for (uint32_t c = 0; fits && c < n_own; c += kChunk) {
        const uint32_t j0 = c + kWin * tid;
        const uint32_t jhi = min(j0 + kWin, n_own);
        uint32_t y[kWinWords];
        uint32_t cff = 0;
        if (j0 < jhi) {
            // the window's 8 words as two 16-byte loads (j0 is a multiple of 32 and the
            // region keeps 128 bytes of slack past its worst case, so they stay inside
            // it; words at or past nwr are masked to 0 as rword does)
            const uint32_t w0 = j0 / 4;
            const uint4* R4 = reinterpret_cast<const uint4*>(R32 + w0);
            const uint4 lo = R4[0], hi = R4[1];
            const uint32_t raw[kWinWords] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            uint32_t prev = rword((int64_t)w0 - 1);
#pragma unroll
            for (int m = 0; m < kWinWords; ++m) {  // output word = R shifted right by b bits
                const uint32_t cur = w0 + m < nwr ? __builtin_bswap32(raw[m]) : 0u;
                y[m] = __builtin_amdgcn_alignbit(prev, cur, b);
                prev = cur;
            }
            if (j0 == 0 && b) y[0] = (y[0] & 0x00FFFFFFu) | (split << 24);
            if (fills && eb && n_own - 1 < j0 + kWin) {
                const uint32_t q = n_own - 1 - j0, sh = 24 - 8 * (q & 3);
#pragma unroll
                for (int m = 0; m < kWinWords; ++m)
                    if ((int)(q >> 2) == m) y[m] = (y[m] & ~(0xFFu << sh)) | (fill << sh);
            }
#pragma unroll
            for (int m = 0; m < kWinWords; ++m) {
                const int n = min((int)(jhi - j0) - 4 * m, 4);
                if (n > 0) cff += __builtin_popcount(ff_bytes(y[m]) & byte_range(0, n));
            }
        }
        uint32_t chunk_ff;
        const uint32_t excl = block_scan<kK3Waves, uint32_t, uint32_t, false, false>(cff, S.wsum, lane, wv, chunk_ff);  // (the previous round's barriers lead)
        const uint32_t cend = min(c + (uint32_t)kChunk, n_own);
        const uint32_t align = (uint32_t)(d & 3);
        if (j0 < jhi) {
            uint32_t o = align + (j0 - c) + excl;
            if (cff == 0 && jhi - j0 == (uint32_t)kWin) {
                // A full window without 0xFF (~88% of them): its 32 bytes go out as whole
                // LDS words, shifted to the window's byte offset, plus the bytes of the
                // words it shares with its neighbours (every byte has exactly one writer).
                // 8 or 7 word stores and 4 byte stores instead of 32 byte stores, each of
                // which conflicted 8 ways (lanes 32 bytes apart).
                uint32_t z[kWinWords];  // little-endian: byte 4m + i of the window in bits 8i of z[m]
#pragma unroll
                for (int m = 0; m < kWinWords; ++m) z[m] = __builtin_bswap32(y[m]);
                uint32_t* ob32 = reinterpret_cast<uint32_t*>(S.ob);
                const uint32_t r = o & 3u;
                if (r == 0) {
#pragma unroll
                    for (int m = 0; m < kWinWords; ++m) ob32[(o >> 2) + m] = z[m];
                } else {
#pragma unroll
                    for (uint32_t q = 0; q < 3; ++q)  // the head: window bytes 0 .. 3 - r
                        if (q < 4u - r) S.ob[o + q] = (uint8_t)(z[0] >> (8 * q));
                    const uint32_t wb = (o + 4u - r) >> 2;  // the first whole word
#pragma unroll
                    for (int m = 0; m < kWinWords - 1; ++m) ob32[wb + m] = __builtin_amdgcn_alignbyte(z[m + 1], z[m], 4u - r);
#pragma unroll
                    for (uint32_t q = 0; q < 3; ++q)  // the tail: window bytes 32 - r .. 31
                        if (q < r) S.ob[o + kWin - r + q] = (uint8_t)(z[kWinWords - 1] >> (8 * (4u - r + q)));
                }
            } else {
#pragma unroll
                for (int q = 0; q < kWin; ++q) {
                    if (j0 + q < jhi) {
                        const uint8_t v = (uint8_t)(y[q >> 2] >> (24 - 8 * (q & 3)));
                        S.ob[o++] = v;
                        if (v == 0xFF) S.ob[o++] = 0;
                    }
                }
            }
        }
        const uint32_t clen = (cend - c) + chunk_ff;
        __syncthreads();
        uint8_t* gout = a.out + (d - align);
        const uint32_t nw = (align + clen + 3) / 4;
        const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(gout, 0, (int)(4 * nw), 0x00020000);
        for (uint32_t w = tid; w < nw; w += kK3Threads) {
            const uint32_t s = 4 * w, e = s + 4;
            if (s >= align && e <= align + clen) {
                const uint32_t v = *reinterpret_cast<const uint32_t*>(S.ob + s);
                if (wthru) __builtin_amdgcn_raw_buffer_store_b32(v, ors, s, 0, kPackStoreAux);
                else __builtin_amdgcn_raw_buffer_store_b32(v, ors, s, 0, kPackStoreNt);
            } else {
                for (uint32_t q = max(s, align); q < min(e, align + clen); ++q)
                    __builtin_amdgcn_raw_buffer_store_b8(S.ob[q], ors, q, 0, kPackStoreAux);
            }
        }
        d += clen;
        if (c + kChunk < n_own) __syncthreads();  // ob is rewritten by the next round
    }
    if (last && tid == 0) {
        uint64_t len = 0;  // end of the image (EOI written) or of the stripe's bytes
        if (fits) {
            if (eoi) {  // EOI, Image.cpp:972
                uint8_t* const m = a.out + d;
                const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(m, 0, 2, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0xFF, mrs, 0, 0, kPackStoreAux);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0xD9, mrs, 1, 0, kPackStoreAux);
                d += 2;
            }
            len = d;
        }
        // the last workgroup's end offset bounds every workgroup's, so it alone decides
        // whether the output fits
        if (a.pack_done) {  // (left for the last workgroup to finish)
            __hip_atomic_store(reinterpret_cast<uint64_t*>(a.pack_done + 2), len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.pack_done + 4, fits ? 0u : 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (a.host_result) {  // (no fence needed: the host reads after the kernel)
            __hip_atomic_store(&a.host_result[0], len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&a.host_result[1], fits ? 0ull : 4ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&a.host_result[3], a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (a.pack_done) {
        // The length, flags and sequence word go into mapped host memory once EVERY
        // workgroup's output stores have completed (each counts itself after them; they
        // are write-through, so complete means in memory): the host may then use the
        // bytes before the kernel has formally ended.
        vm_drain();
        __syncthreads();
        if (tid == 0 && atomicAdd(a.pack_done, 1u) == G - 1 && a.host_result) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the last workgroup's end offset)
            const uint64_t len =
                __hip_atomic_load(reinterpret_cast<const uint64_t*>(a.pack_done + 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t nospace = __hip_atomic_load(a.pack_done + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.pack_done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (reusable without K1)
            __hip_atomic_store(&a.host_result[0], len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&a.host_result[1], (uint64_t)nospace, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&a.host_result[3], a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    JPGE_STAMP(2);
}

}  // namespace

// Workgroups: at most kEntropyMaxTilesPerWg tiles each (region size); about 384 in
// all (1.5 per CU: measured best beside the other lanes) unless overridden.  One segment (restart off):
// balanced tiles of <= 128 blocks (tile i of nt is blocks [i*nb/nt, (i+1)*nb/nt), so
// with nt >= 2 every tile holds >= 64 blocks), one or more per workgroup.  Every block
// codes >= 2 bits (a DC code and an EOB or AC code, each >= 1 bit), so each
// workgroup's stream holds >= 128 bits and its first and last 8 bits, which the
// placement reads, are defined.  Restart intervals of R MCUs: segments of bpm*R
// blocks (>= 3 blocks, >= 6 bits; each starts byte-aligned), each cut into
// balanced tiles of <= 128 blocks, a whole number of workgroups per segment.
SegLayout seg_layout(const Geometry& g, uint32_t restart_mcus, uint32_t wgs_override) {
    SegLayout L;
    const uint32_t nb = g.nblocks();
    const uint32_t want = wgs_override ? wgs_override : 384u;  // (pipeline: 384 +3% over 512; 768 -12%)
    const uint64_t S = (uint64_t)g.bpm * restart_mcus;
    if (!restart_mcus || S >= nb) {
        const uint32_t nt = (nb + kK3Blocks - 1) / kK3Blocks;
        uint32_t G = 1;
        if (nt > 1) {
            const uint32_t lo = (nt + kMaxTiles - 1) / kMaxTiles, hi = nt;
            // (the pipeline's default on frames under 768 tiles: 2 tiles per workgroup, not
            // one each: 1080p batch +8%)
            const uint32_t w = wgs_override ? want : (nt < 2u * want ? (nt + 1) / 2 : want);
            G = w < lo ? lo : (w > hi ? hi : w);
        }
        L.nseg = 1;
        L.sblk = L.lblk = nb;
        L.tps = L.ltps = nt;
        L.wps = L.lwps = G;
        return L;
    }
    L.nseg = (uint32_t)((nb + S - 1) / S);
    L.sblk = (uint32_t)S;
    L.lblk = nb - (L.nseg - 1) * L.sblk;
    const uint32_t per_seg = (want + L.nseg - 1) / L.nseg;
    auto part = [&](uint32_t blocks, uint32_t& tps, uint32_t& wps) {
        tps = (blocks + kK3Blocks - 1) / kK3Blocks;  // balanced tiles: >= 64 blocks each when tps > 1
        const uint32_t lo = (tps + kMaxTiles - 1) / kMaxTiles;
        wps = per_seg < lo ? lo : (per_seg > tps ? tps : per_seg);
    };
    part(L.sblk, L.tps, L.wps);
    part(L.lblk, L.ltps, L.lwps);
    return L;
}

// encode()'s gate (encoder.cpp): one workgroup waits for the host's word, then copies the
// tables and headers from mapped host memory to the device, ahead of the code kernel.  A
// time-out (~1 s) ends the wait whatever happens and flags the frame's result word
// (host_result[2]), so the call fails instead of coding with stale tables.
constexpr uint32_t kGateThreads = 512;
__global__ __launch_bounds__(kGateThreads) void gate_copy_kernel(const uint32_t* gate, uint32_t value, const uint4* src,
                                                                 uint4* dst, uint32_t n16, uint64_t* fail,
                                                                 uint64_t timeout_ticks) {
    __shared__ uint32_t open;
    if (threadIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t o = 1;
        while (__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != value) {
            __builtin_amdgcn_s_sleep(4);
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {  // (s_memrealtime: 100 MHz)
                o = 0;
                break;
            }
        }
        open = o;
    }
    __syncthreads();
    if (!open) {
        if (threadIdx.x == 0) __hip_atomic_store(fail, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // (the host's table stores precede its word)
    for (uint32_t i = threadIdx.x; i < n16; i += kGateThreads) dst[i] = src[i];
}

hipError_t launch_gate_copy(const uint32_t* gate, uint32_t value, const void* src, void* dst, uint32_t n16,
                            uint64_t* fail, uint64_t timeout_ticks, hipStream_t s) {
    hipLaunchKernelGGL(gate_copy_kernel, dim3(1), dim3(kGateThreads), 0, s, gate, value,
                       reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n16, fail, timeout_ticks);
    return hipGetLastError();
}

hipError_t launch_entropy(const EntropyArgs& a, hipStream_t s, const KTimer* tcode, const KTimer* tpack) {
    const hipError_t e = launch_entropy_code(a, s, tcode);
    return e != hipSuccess ? e : launch_entropy_pack(a, s, tpack);
}

hipError_t launch_entropy_code(const EntropyArgs& a, hipStream_t s, const KTimer* tcode) {
    const uint32_t G = a.seg.grid();
    return launch_timed(tcode, entropy_code_kernel<1>, dim3(G), dim3(kK3Threads), s, frame_set<1>(&a, 1, G));
}

hipError_t launch_entropy_pack(const EntropyArgs& a, hipStream_t s, const KTimer* tpack) {
    const uint32_t G = a.seg.grid();
    hipError_t e = hipSuccess;
    EntropyArgs b = a;
    b.dbg = a.dbg ? a.dbg + 65536 * kStampSlots : nullptr;  // (diag builds: the pack kernel's stamps)
    if (a.done) {  // placed by the code kernel's last workgroup
        if (!a.place || a.rst.mcus || G > kPlaceInCodeMaxWgs) return hipErrorInvalidValue;
        b.flags |= kExtPlace;
    } else if (G > kInlineScanMaxWgs || (a.flags & kExtPlace) || a.rst.mcus) {
        if (!a.place) return hipErrorInvalidValue;
        b.flags |= kExtPlace;
        if ((e = launch_place(b, G, s)) != hipSuccess) return e;
    }
    return launch_timed(tpack, entropy_pack_kernel<1>, dim3(G), dim3(kK3Threads), s, frame_set<1>(&b, 1, G));
}

hipError_t launch_entropy_set(const EntropyArgs* a, int n, hipStream_t s, const KTimer* tcode, const KTimer* tpack) {
    if (n < 1 || n > kMaxSet) return hipErrorInvalidValue;
    const uint32_t G = a[0].seg.grid();
    FrameSet<EntropyArgs> fs = frame_set(a, n, G);
    for (int f = 0; f < n; ++f) {  // one partition, each member placed by its code kernel's last workgroup
        const EntropyArgs& m = a[f];
        if (m.seg.grid() != G || !m.done || !m.place || m.rst.mcus || G > kPlaceInCodeMaxWgs) return hipErrorInvalidValue;
    }
    hipError_t e = launch_timed(tcode, entropy_code_kernel<kMaxSet>, dim3(G * n), dim3(kK3Threads), s, fs);
    if (e != hipSuccess) return e;
    for (int f = 0; f < n; ++f) {
        fs.a[f].flags |= kExtPlace;
        fs.a[f].dbg = a[f].dbg ? a[f].dbg + 65536 * kStampSlots : nullptr;
    }
    return launch_timed(tpack, entropy_pack_kernel<kMaxSet>, dim3(G * n), dim3(kK3Threads), s, fs);
}

hipError_t launch_entropy_code_summary(const EntropyArgs& a, hipStream_t s) {
    const uint32_t G = a.seg.grid();
    if (!a.summary) return hipErrorInvalidValue;
    hipLaunchKernelGGL(entropy_code_kernel<1>, dim3(G), dim3(kK3Threads), 0, s, frame_set<1>(&a, 1, G));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // (restart intervals: the stripe's placement is its own, computed now; its summary
    // is its byte length)
    hipLaunchKernelGGL(entropy_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, a, G, a.rst.mcus ? 0 : 1);
    return hipGetLastError();
}

hipError_t launch_entropy_place_pack(const EntropyArgs& a, hipStream_t s) {
    const uint32_t G = a.seg.grid();
    if (!a.place) return hipErrorInvalidValue;
    EntropyArgs b = a;
    b.flags |= kExtPlace;
    if (!a.rst.mcus) {  // (restart intervals: placed by launch_entropy_code_summary)
        const hipError_t e = launch_place(b, G, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(entropy_pack_kernel<1>, dim3(G), dim3(kK3Threads), 0, s, frame_set<1>(&b, 1, G));
    return hipGetLastError();
}

}  // namespace jpge
