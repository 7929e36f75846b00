// K2 stats_wave_kernel (gfx950): DC difference chain (Image.cpp:638-678) + zig-zag
// RLE + category coding (Coding.hpp:148-283) -> the four symbol histograms of
// writeJPEG's "texts" (Image.cpp:888-906) with first-occurrence keys, and the
// symbol records of every tile in stream order (kernels.hpp), which the entropy
// code kernel turns into bits once the tables exist: the run-length and category
// work is done once per frame.  Counters accumulate in LDS (bank-staggered copies
// split same-address atomics) and are flushed once per workgroup into kHistReplicas
// global replicas.  First-occurrence keys (text index of the symbol, huffman.hpp)
// are kept workgroup-relative in u32 LDS words and widened at the flush; the global
// key is stored inverted so atomicMax keeps the minimum.
#include <algorithm>
#include <cstddef>
#include <type_traits>

#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

// ---------------------------------------------------------------------------
// stats_wave_kernel: one wavefront per block at a time, lane p = zig-zag position p.
//
// A workgroup owns a contiguous run of record sub-streams (kernels.hpp: a quarter
// of an entropy tile, <= 32 blocks); its waves take them one at a time from an LDS
// counter and code each alone: no workgroup barrier between the prologue and the
// flush.  Per sub-stream a wave stages the blocks (natural order; the next
// sub-stream it takes is loaded into registers meanwhile) in its own LDS area,
// derives the per-block fields lane-parallel (lane j = block j: MCU, slot, text
// index, the DC difference to the chain predecessor, the DC record), then walks the
// blocks two at a time (their dependent chains interleave):
//   c    = the coefficient at zig-zag position p (one ds_read_i16 per lane)
//   M    = ballot(c != 0) without the DC: the block's AC non-zero mask, in SGPRs
//   rank = mbcnt(M): the record index of every non-zero (DC first, then AC in order)
//   run  = clz of M's bits below p: the zeros since the previous non-zero
//   cat  = frexp exponent of (float)c = bit length of |c| (getCategoryAndCode)
// and stores the block's records with one buffer store (consecutive addresses: the
// non-zeros, and lane 63 as the EOB when coefficient 63 is zero; lanes without a
// record store out of range, which the hardware drops).  Histogram counters are LDS
// atomics on the workgroup's copies (lane & 7: same-symbol lanes of one instruction
// land on different copies and banks), first-occurrence keys a read and a rare
// atomicMin.  A block with a run of 16+ zeros before a non-zero (rare)
// takes a wave scan for its ZRL records.  Each block's DC difference replaces its DC
// coefficient in the stage, so lane 0 codes the DC record with the block's records.
// Reference: DC chain Image.cpp:638-678, RLE + category Coding.hpp:148-283 and
// Image.cpp:680-735, texts Image.cpp:888-906.
constexpr int kWWaves = 8;  // (8-wave workgroups: 28.9 us alone at 4K vs 39.7 with 4; 16 waves: 148 GPix/s in the pipeline)
constexpr int kWWpe = 8;    // waves per SIMD the register allocation targets (<= 64 VGPRs: 4 workgroups per CU; 7 let the compiler take 69)
constexpr int kWThreads = 64 * kWWaves;
constexpr int kSubBlocks = (kEntropyTile + kRecSub - 1) / kRecSub;  // blocks of a sub-stream, at most
static_assert(kRecSub > 1 && kSubBlocks <= 64 && kSubBlocks % 8 == 0, "a sub-stream's blocks fit a wave");
constexpr int kWRows = kSubBlocks * 8 / 64;  // 16-byte block rows per lane = 8-block chunks per sub-stream
constexpr int kWCopies = 8;  // LDS counter copies (lane & 7)
// Counter / key words: table t's symbol s at kTabBase(t) + (s & 15) + 19 * (s >> 4).
// The stride 19 puts the frequent symbols (runs 0-4, sizes 1-5) on distinct banks
// (a stride of 16 put runs 0 and 2, or 1 and 3, of a size on one bank), and is
// injective for sizes up to 18.
constexpr uint32_t kRunStride = 19;
// A component's DC table follows its AC table at kRunStride * 16 words (run 16 of the
// AC layout), so lane 0 (the DC position) reaches it through the same word formula
// with a run of 16.
constexpr uint32_t kAcWords = 15 + kRunStride * 15 + 1;  // 301
constexpr uint32_t kDcOff = kRunStride * 16;             // 304
constexpr uint32_t kCompWords = kDcOff + 16;             // 320: Y (AC, DC), then C
static_assert(kAcWords <= kDcOff, "the DC table after the AC words");
__host__ __device__ constexpr uint32_t tab_base(uint32_t t) { return (t >> 1) * kCompWords + ((t & 1) ? 0 : kDcOff); }
constexpr uint32_t kWSyms = 2 * kCompWords;  // 640 words
// copy stride == 32 / copies (mod 32): the copies of a word sit on distinct banks
constexpr uint32_t kWBankStep = 32u / kWCopies;
constexpr uint32_t kWCopyWords = (kWSyms + 64 + 31 - kWBankStep) / 32 * 32 + kWBankStep;
static_assert(kWCopies <= 32 && kWCopyWords % 32 == kWBankStep && kWCopyWords >= kWSyms + 64, "copy stride");
constexpr uint32_t kWKeyWords = (kWSyms + 1 + 3) / 4 * 4;  // keys, then one shared dummy word
constexpr uint32_t kWMaxSubs = 1024;  // sub-streams per workgroup, at most (stats_grid)

struct K2WLds {
    alignas(16) uint32_t stage[kWWaves][8 * 32 + 32];   // each wave's 8-block chunk: int16 [block][64], natural order; 64 spare int16
    alignas(16) uint32_t cnt[kWCopies * kWCopyWords];    // counters [copy][word], then the dummies
    alignas(16) uint32_t key[kWKeyWords];                // first-occurrence keys (min), workgroup-relative
    uint32_t sb0[kWMaxSubs + 1];                         // the workgroup's sub-streams' first blocks, and the end
    uint32_t next;                                       // the next sub-stream to take
};

template <int kN>
__global__ __launch_bounds__(kWThreads) __attribute__((amdgpu_waves_per_eu(kWWpe))) void stats_wave_kernel(FrameSet<StatsArgs, kN> fs) {
    const uint32_t set_f = (kN == 1 ? 0u : set_member_rolled(fs.wg0, fs.n, blockIdx.x));  // (frame sets: kernels.hpp)
    const StatsArgs& a = fs.a[set_f];
    const uint32_t bid = blockIdx.x - fs.wg0[set_f], nbk = fs.wg0[set_f + 1] - fs.wg0[set_f];
    __shared__ K2WLds L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);

    const uint32_t bpm = a.g.bpm, mw = a.g.mw, yh = a.g.yh, yv = a.g.yv();
    const uint32_t yhs = (uint32_t)__builtin_ctz(yh);
    const uint32_t ybw = mw * yh;  // Y blocks per block row
    const uint32_t S = seg_tiles(a.seg) * kRecSub;
    // the workgroup's sub-streams [s_lo, s_hi) (64-bit divisions lane-parallel, on the VALU)
    uint32_t s_lo, s_hi;
    {
        const uint32_t w = bid + (uint32_t)(lane & 1);
        const uint32_t v = (uint32_t)((uint64_t)w * S / nbk);
        s_lo = __builtin_amdgcn_readlane(v, 0);
        s_hi = __builtin_amdgcn_readlane(v, 1);
    }
    const uint32_t ns = s_hi - s_lo;  // (<= kWMaxSubs: stats_grid)
    // this wave's first sub-stream (s_lo + wv) is requested before the LDS initialisation
    // and the workgroup's sub-stream table: its HBM latency overlaps them
    const uint32_t lane_u = (uint32_t)lane;
    uint4 cur[kWRows];
    int dcs = 0;  // lane l < nb + 6: the DC of block b0 - 6 + l of the fetched sub-stream (0 before the frame)
    auto load_row = [&](const __amdgpu_buffer_rsrc_t& rs, int i) {
        return as_u4(__builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(lane + 64 * i) * 16, 0, 0));
    };
    auto load_dcs_at = [&](uint32_t b0, uint32_t nb) {
        const int32_t g = (int32_t)(b0 + lane_u) - 6;  // (block numbers < 2^25: launch_stats)
        dcs = (lane_u < nb + 6 && g >= 0) ? a.coef[(uint64_t)(uint32_t)g * 64] : 0;
    };
    if ((uint32_t)wv < ns) {
        uint64_t b;
        uint32_t n;
        sub_tile(a.seg, s_lo + (uint32_t)wv, b, n);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int16_t*>(a.coef + b * 64), 0, n * 128, 0x00020000);
#pragma unroll
        for (int i = 0; i < kWRows; ++i) cur[i] = load_row(rs, i);
        load_dcs_at((uint32_t)b, n);
    }
    static_assert((kWCopies * kWCopyWords) % 4 == 0 && kWKeyWords % 4 == 0, "16-byte initialisation");
    for (int i = tid; i < (int)(kWCopies * kWCopyWords / 4); i += kWThreads)
        reinterpret_cast<uint4*>(L.cnt)[i] = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < (int)(kWKeyWords / 4); i += kWThreads)
        reinterpret_cast<uint4*>(L.key)[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (uint32_t i = tid; i <= ns; i += kWThreads) {  // their first blocks (block numbers < 2^32: launch_stats)
        uint64_t b;
        uint32_t n;
        sub_tile(a.seg, min(s_lo + i, S - 1), b, n);
        L.sb0[i] = (uint32_t)(s_lo + i < S ? b : b + n);
    }
    if (tid == 0) L.next = kWWaves;  // (sub-stream w is wave w's first)
    __syncthreads();
    // (single frames) the histogram export by the last workgroup to finish: every
    // workgroup counts itself once its flush atomics (device-coherent) have completed;
    // the one completing the count reads every workgroup's counts and keys
    auto export_if_last = [&]() {
        if (!a.done) return;
        vm_drain();
        __syncthreads();
        if (tid == 0) L.next = atomicAdd(a.done, 1u) == nbk - 1 ? 1u : 0u;
        __syncthreads();
        if (L.next) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            export_hist<kWThreads>(a.hist, a.host_cnt, a.host_key, a.host_seq, a.seq, tid);
        }
    };
    if (ns == 0) {
        export_if_last();
        return;
    }
    // key bases (keys are kept relative to them): the workgroup's first MCU row
    const uint32_t mrow0 = __builtin_amdgcn_readfirstlane((L.sb0[0] / bpm) / mw);
    const uint32_t ybase = mrow0 * yv * ybw, cbase = mrow0 * mw;
    JPGE_STAMP(0);
    uint64_t tq = JPGE_NOW();

    const uint32_t natoff = kZzToNat[lane];  // this lane's coefficient in a staged block (int16 index)
    const uint32_t k2p = 2u * (uint32_t)lane;
    uint32_t* const cnt = L.cnt + (uint32_t)(lane & (kWCopies - 1)) * kWCopyWords;
    const uint32_t shl = (uint32_t)(64 - lane) & 63u;
    const uint64_t lanes_ac = ~1ull;  // every lane but the DC
    const uint32_t dc_tab = lane == 0 ? 1u << 14 : 0u;  // (a record's table bits: 2t + 1 -> 2t)
    const uint32_t dc_run = lane == 0 ? 16u : 0u;  // (lane 0's run: its counter word is the DC table's, kDcOff)
    int16_t* st16 = reinterpret_cast<int16_t*>(L.stage[wv]);
    uint4* st4 = reinterpret_cast<uint4*>(L.stage[wv]);

    auto rows = [&](uint32_t si) {  // sub-stream si's coefficients through a buffer descriptor (zeros past its blocks)
        const uint32_t b0 = L.sb0[si], nb = L.sb0[si + 1] - b0;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(a.coef + (uint64_t)b0 * 64), 0, nb * 128,
                                                 0x00020000);
    };
    auto load_dcs = [&](uint32_t si) { load_dcs_at(L.sb0[si], L.sb0[si + 1] - L.sb0[si]); };
    uint32_t si = (uint32_t)wv;
    while (si < ns) {
        const uint32_t b0 = L.sb0[si], nb = L.sb0[si + 1] - b0;
        const uint32_t s = s_lo + si;
        // take the next sub-stream (its rows load chunk by chunk, as this one's are staged)
        uint32_t sn = 0;
        if (lane == 0) sn = atomicAdd(&L.next, 1u);
        sn = __builtin_amdgcn_readfirstlane(sn);
        const __amdgpu_buffer_rsrc_t rsn = rows(sn < ns ? sn : si);

        // ---- per block fields, lane j = block j ----
        const uint32_t g = b0 + (uint32_t)lane;
        const uint32_t m6 = g / bpm, k = g - m6 * bpm;
        const uint32_t mrow = m6 / mw, mcol = m6 - mrow * mw;
        const int comp = block_comp((int)k, bpm);
        // text index (the Y text in block raster order; all Cr after all Cb), relative to the bases
        const uint32_t rel = comp == 0 ? (mrow * yv + (k >> yhs)) * ybw + mcol * yh + (k & (yh - 1)) - ybase
                                       : (m6 - cbase) | (comp == 2 ? 0x80000000u : 0u);
        const uint32_t tsel = comp != 0;
        // the block loop reads one word per block: the AC key base, text index * 128 + d,
        // whose low bit d is the table select (a key is base + 2p: keys are compared only
        // within a table, where d is constant; a ZRL's key base + 2p - 1 still sorts
        // between positions p - 1 and p)
        const uint32_t acb = (rel & 0x80000000u) | ((rel & 0x7FFFFFFFu) << 7) | tsel;
        // DC difference to the chain predecessor: the previous Y slot, 3 blocks back for an
        // MCU's first Y block, bpm back for chroma; none in the first MCU; restarts reset it
        int dd;
        {
            const bool ynext = k >= 1 && k < bpm - 2;
            const int back = ynext ? 1 : (k == 0 ? 3 : (int)bpm);
            const bool none = !ynext && g < bpm;
            bool reset = false;
            if (a.rst.mcus && (k == 0 || k >= bpm - 2)) reset = (m6 + a.rst.mcu0) % a.rst.mcus == 0;
            const int dcv = __builtin_amdgcn_ds_bpermute((lane + 6) * 4, dcs);
            int pd = __builtin_amdgcn_ds_bpermute((lane + 6 - back) * 4, dcs);  // (lane - back >= -6)
            pd = reset ? 0 : none ? (comp == 0 ? a.seed.v[0] : comp == 1 ? a.seed.v[1] : a.seed.v[2]) : pd;
            dd = (int)(int16_t)dcv - (int)(int16_t)pd;
        }
        if (sn < ns) load_dcs(sn);
        if (si == (uint32_t)wv) JPGE_STAMP(1);  // (wave 0: its first sub-stream's data is in)
        JPGE_ACC(1, tq);

        // ---- the blocks ----
        uint16_t* srec = a.recs + (uint64_t)(s / kRecSub) * kTileRecords + (s % kRecSub) * kSubRecords;
        const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(srec, 0, kSubRecords * 2, 0x00020000);
        uint32_t base = 0;   // the block's first record (its DC) in the sub-stream
        // one block's fields (lane p: zig-zag position p)
        struct Blk {
            uint64_t M, em;     // AC non-zeros; the lanes with a record (lane 0: the DC; lane 63: non-zero, or the EOB)
            uint32_t rk, run;   // record index in the block (DC = 0; continuations before it counted), zeros before the coefficient
            uint64_t bg;        // the lanes whose extra bits need a continuation record (size >= 7; rare)
            uint32_t rec, w;    // the record; its counter / key word
            uint32_t Tj, acbj, acw;  // the block's AC table (record bits 14-15), key base, table base word
            bool zrl;           // a run of 16+ zeros before a non-zero
        };
        // kExact: runs exact (every length; the ZRL path).  Otherwise exact up to 31:
        // the leading zeros of the 32 mask bits below p, with a 1 below them (a window
        // without a non-zero, a run of 32+, reads 31); a block with a run of 16+ takes
        // the ZRL path, which recomputes it exactly, so the fast path codes runs < 16
        // and needs no mask of the run's low 4 bits.
        auto prep = [&](int c, uint32_t jb, auto exact) {
            constexpr bool kExact = decltype(exact)::value;
            Blk b;
            const uint64_t B1 = __ballot(c != 0) | 1ull;  // the AC non-zeros, and bit 0
            b.M = B1 & lanes_ac;
            b.acbj = __builtin_amdgcn_readlane(acb, jb);    // (+ 2p: the key; the EOB lane 63: text * 128 + 126 + d)
            const uint32_t d = b.acbj & 1u;                  // (scalar: 1 for the chroma tables)
            b.Tj = (1u << 14) + (d << 15);                   // the AC table, as a record's top bits
            b.acw = d * tab_base(3);                         // its first counter / key word (tab_base(1) = 0)
            b.rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(B1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B1, 0u));
            if constexpr (kExact) b.run = (uint32_t)__builtin_clzll(B1 << shl);  // (lane 0: unused)
            else b.run = (uint32_t)__builtin_clz((uint32_t)((B1 << shl) >> 32) | 1u);
            const uint32_t cat = (uint32_t)__builtin_amdgcn_frexp_expf((float)c);
            const uint32_t bits = extra_bits(c, (int)cat);
            // (the EOB lane: 0; the DC lane: 16)
            const uint32_t rr = __builtin_amdgcn_inverse_ballot_w64(b.M) ? (kExact ? b.run & 15u : b.run) : dc_run;
            // lane 0 (the DC position, where the stage holds the block's DC difference)
            // codes the block's DC symbol like an AC lane: its record (its table: the AC
            // table's number less one; the run of 16 sets a bit the table bits have; its
            // category where an AC record has its run) at the block's first record (rank
            // 0), its count in the DC table's word (kDcOff past the AC table's first), its
            // key as text index * 128 + d (the flush divides it back).  Stored after the
            // sub-stream, the DC records had rewritten lines already written back (K2 wrote
            // 1.24x its record bytes); counted after the sub-stream, they cost a pass of
            // their own.
            // a size above 6 keeps its extra bits' top 6 in the record and the rest in a
            // continuation right after it (kernels.hpp); the fast path writes every record
            // with its extra bits' low 6, and cont() rewrites such lanes' records from their
            // coefficients
            b.bg = __builtin_amdgcn_ballot_w64(cat > kRecXBits);
            uint32_t x = bits & 63u;
            if constexpr (kExact) {
                x = bits >> __builtin_elementwise_sub_sat(cat, kRecXBits);
                b.rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(b.bg >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b.bg, b.rk));
            }
            b.rec = ((b.Tj | (rr << 10) | (cat << 6)) ^ dc_tab) | x;
            b.w = b.acw + (uint32_t)cat + kRunStride * rr;
            b.em = B1 | (1ull << 63);
            b.zrl = (__ballot(b.run >= 16u) & b.M) != 0;
            return b;
        };
        // (fast path, a block with size >= 7 symbols: uniform, rare at Q90) each such record
        // keeps its extra bits' top 6, and its continuation right after it the rest: the
        // records after it move one further, the block's count grows by one
        auto cont = [&](uint64_t bg, int c, uint32_t Tj, uint32_t b0, uint32_t& rk, uint32_t& rec, uint32_t& n) {
            if (!bg) return;
            const uint32_t cat = (uint32_t)__builtin_amdgcn_frexp_expf((float)c);
            const uint32_t sh = __builtin_elementwise_sub_sat(cat, kRecXBits), bits = extra_bits(c, (int)cat);
            rec = (rec & ~63u) | (bits >> sh);
            rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(bg >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bg, rk));
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(Tj | (sh << 10) | (bits & ((1u << sh) - 1u))), rrs,
                                                  __builtin_amdgcn_inverse_ballot_w64(bg) ? (b0 + rk + 1u) * 2u : 0x80000000u, 0, 0);
            n += (uint32_t)__builtin_popcountll(bg);
        };
        // (general form, every block with ZRLs) block jb's records from
        // `base`, histogram and keys, all from its staged coefficient c; returns its record count
        auto emit = [&](int c, uint32_t jb, uint32_t base) -> uint32_t {
            Blk b = prep(c, jb, std::true_type{});
            uint32_t zt = 0;
            if (b.zrl) {  // ZRL records (F/0) before the non-zeros after 16+ zeros (rare)
                const uint32_t nzr = __builtin_amdgcn_inverse_ballot_w64(b.M) ? b.run >> 4 : 0u;
                const uint32_t zi = wave_scan_incl(nzr);
                zt = __builtin_amdgcn_readlane(zi, 63);
                b.rk += zi;
                if (nzr) {
                    const uint16_t zrec = (uint16_t)(b.Tj | (15u << 10));
                    for (uint32_t z = 1; z <= nzr; ++z) srec[base + b.rk - z] = zrec;
                    const uint32_t wz = b.acw + kRunStride * 15u;  // (symbol 0xF0)
                    atomicAdd(&cnt[wz], nzr);
                    const uint32_t kz = b.acbj + k2p - 1u;
                    if (kz < L.key[wz]) atomicMin(&L.key[wz], kz);
                }
            }
            if (__builtin_amdgcn_inverse_ballot_w64(b.em)) {
                srec[base + b.rk] = (uint16_t)b.rec;
                if (__builtin_amdgcn_inverse_ballot_w64(b.bg)) {  // (its extra bits past the record's 6)
                    const uint32_t cat = (uint32_t)__builtin_amdgcn_frexp_expf((float)c), sh = cat - kRecXBits;
                    srec[base + b.rk + 1] = (uint16_t)(b.Tj | (sh << 10) | (extra_bits(c, (int)cat) & ((1u << sh) - 1u)));
                }
                atomicAdd(&cnt[b.w], 1u);
                const uint32_t kk = b.acbj + k2p;
                if (kk < L.key[b.w]) atomicMin(&L.key[b.w], kk);
            }
            return (uint32_t)__builtin_popcountll(b.em) + zt + (uint32_t)__builtin_popcountll(b.bg);  // DC, non-zeros, EOB, ZRLs, continuations
        };
#pragma unroll
        for (int ch = 0; ch < kWRows; ++ch) {  // 8-block chunks: stage one, load the next sub-stream's into its registers
            const uint32_t j0 = 8u * ch;
            wave_order();
            if (j0 < nb) st4[lane] = cur[ch];
            cur[ch] = load_row(rsn, ch);
            // each block's DC difference over its DC coefficient (lane j: block j)
            // (every lane stores: the others into a slot of their own past the chunk)
            // (8 stores on one bank per chunk: a 72-int16 block stride put them on 8 banks,
            // but its staging index cost more than the conflicts, -0.4% in the pipeline)
            st16[(uint32_t)lane - j0 < 8u ? ((uint32_t)lane - j0) * 64u : 512u + (uint32_t)lane] = (int16_t)dd;
            wave_order();
            if (j0 >= nb) continue;
            const uint32_t j1 = min(nb, j0 + 8u);
            const int16_t* cp = st16 + natoff;  // this lane's coefficient of the pair's first block
            uint32_t jb = j0;
            // blocks jb, jb + 1 (their coefficients at cp[0], cp[64]) from `base`
            auto pair = [&](const int16_t* cp, uint32_t jb) {
                const int cA = cp[0], cB = cp[64];
                const Blk A = prep(cA, jb, std::false_type{}), B = prep(cB, jb + 1, std::false_type{});
                uint32_t baseB;
                if (!(A.zrl || B.zrl)) {
                    uint32_t recA = A.rec, recB = B.rec, rkA = A.rk, rkB = B.rk;
                    uint32_t nA = (uint32_t)__builtin_popcountll(A.em), nB = (uint32_t)__builtin_popcountll(B.em);
                    if (A.bg | B.bg) {
                        cont(A.bg, cp[0], A.Tj, base, rkA, recA, nA);
                        cont(B.bg, cp[64], B.Tj, base + nA, rkB, recB, nB);
                    }
                    // lanes without a record store out of range (dropped); their counter adds
                    // are masked off
                    baseB = base + nA;
                    const bool ia = __builtin_amdgcn_inverse_ballot_w64(A.em), ib = __builtin_amdgcn_inverse_ballot_w64(B.em);
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)recA, rrs, ia ? (base + rkA) * 2u : 0x80000000u, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)recB, rrs, ib ? (baseB + rkB) * 2u : 0x80000000u, 0, 0);
                    if (ia) atomicAdd(&cnt[A.w], 1u);
                    if (ib) atomicAdd(&cnt[B.w], 1u);
                    // (every lane reads its word: a lane without a record has c = 0, so its
                    // word is its table's first, and lane 0's is in range too)
                    const uint32_t kvA = L.key[A.w], kvB = L.key[B.w];
                    const uint32_t kkA = A.acbj + k2p, kkB = B.acbj + k2p;
                    // (rare: a first occurrence in this workgroup so far; the masks of the
                    // compares, which a bool's ballot would rebuild lane by lane)
                    const uint64_t fA = A.em & __builtin_amdgcn_ballot_w64(kkA < kvA);
                    const uint64_t fB = B.em & __builtin_amdgcn_ballot_w64(kkB < kvB);
                    if (fA | fB) {
                        if (__builtin_amdgcn_inverse_ballot_w64(fA)) atomicMin(&L.key[A.w], kkA);
                        if (__builtin_amdgcn_inverse_ballot_w64(fB)) atomicMin(&L.key[B.w], kkB);
                    }
                    base = baseB + nB;
                } else {  // (a ZRL block: both again from the stage, exactly)
                    baseB = base + emit(cp[0], jb, base);
                    base = baseB + emit(cp[64], jb + 1, baseB);
                }
            };
            // (a full chunk's 4 pairs unrolled: 3 times the kernel's code, 60 KB, for ~3 SALU
            // per block of loop control; not taken)
            for (; jb + 1 < j1; jb += 2, cp += 128) pair(cp, jb);
            if (jb < j1) base += emit(cp[0], jb, base);  // an odd last block
        }
        JPGE_ACC(2, tq);
        if (lane == 0) a.tcount[s] = base;
        si = sn;
        JPGE_ACC(3, tq);
    }
    JPGE_STAMP(2);
    __syncthreads();

    const int rep = bid % kHistReplicas;
    const uint64_t ncb = a.key_ncb ? a.key_ncb : a.g.nmcu();  // Cb blocks of the whole image
    // (a thread's two words; the global key's atomicMax unconditional: reading the key
    // first to skip needless atomics held every workgroup one global round trip longer,
    // K2 alone 68.6 -> 62.6 us per set of 4 4K frames without it)
    static_assert(1024 == 2 * kWThreads, "two flush words per thread");
    unsigned long long* gk = reinterpret_cast<unsigned long long*>(a.hist.key);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t i = (uint32_t)tid + (uint32_t)j * kWThreads;
        const uint32_t t = i >> 8, sy = i & 255u;
        if (!(t & 1) && sy >= 16) continue;  // (DC tables: categories < 16)
        const uint32_t w = tab_base(t) + (sy & 15u) + kRunStride * (sy >> 4);
        uint32_t c = 0;
#pragma unroll
        for (int cp = 0; cp < kWCopies; ++cp) c += L.cnt[cp * kWCopyWords + w];
        if (!c) continue;
        atomicAdd(&a.hist.cnt[rep * 1024 + i], c);
        const uint32_t k32 = L.key[w];
        uint64_t kb;  // (global texts: a stripe's bases are offset into the whole image)
        if (t < 2) kb = a.key_y0 + ybase;
        else kb = a.key_c0 + cbase + ((k32 & 0x80000000u) ? ncb : 0ull);
        // (AC keys: text index * 128 + 2p + delta + d; DC keys were kept as text index * 128 + d)
        const uint64_t gkey = (t & 1) ? kb * 128ull + (k32 & 0x7FFFFFFFu) : kb + ((k32 & 0x7FFFFFFFu) >> 7);
        atomicMax(&gk[i], (unsigned long long)~gkey);
    }
    export_if_last();
    JPGE_STAMP(3);
}

// Histogram export: one workgroup sums the replicas and writes the four final
// histograms and first-occurrence keys straight into mapped host memory, then the
// frame's sequence number (release-ordered after the data): the host polls that
// word instead of waiting on an event.  A kernel boundary orders it after
// stats_kernel; there is no device-to-host copy per frame.
// (Standalone form, for single frames and the pipeline's first frames; in steady
// state another frame's entropy code kernel carries the export.)
__global__ __launch_bounds__(1024) void hist_export_kernel(HistPtrs h, uint32_t* host_cnt, uint64_t* host_key,
                                                           uint64_t* host_seq, uint64_t seq) {
    export_hist<1024>(h, host_cnt, host_key, host_seq, seq, threadIdx.x);
}

}  // namespace

hipError_t launch_hist_export(const HistPtrs& h, uint32_t* host_cnt, uint64_t* host_key, uint64_t* host_seq,
                              uint64_t seq, hipStream_t s) {
    hipLaunchKernelGGL(hist_export_kernel, dim3(1), dim3(1024), 0, s, h, host_cnt, host_key, host_seq, seq);
    return hipGetLastError();
}

uint32_t stats_grid(const SegLayout& L, uint32_t wgs) {
    // workgroups of kWWaves waves over the record sub-streams: at least one sub-stream
    // per wave, at most kWMaxSubs per workgroup (its LDS table)
    const uint32_t subs = seg_tiles(L) * kRecSub;
    const uint32_t want = wgs ? wgs : 512u;
    const uint32_t cap = (subs + kWWaves - 1) / kWWaves;
    const uint32_t need = (subs + kWMaxSubs - 1) / kWMaxSubs;
    return std::max(std::max(1u, need), std::min(want, cap));
}

template <int kN>
static hipError_t launch_stats_fs(const FrameSet<StatsArgs, kN>& fs, hipStream_t s, const KTimer* t) {
    for (uint32_t f = 0; f < fs.n; ++f) {
        // (32-bit block numbers and buffer offsets)
        if ((uint64_t)fs.a[f].g.nblocks() * 128 >= (1ull << 32)) return hipErrorInvalidValue;
        if (fs.wg0[f + 1] - fs.wg0[f] != stats_grid(fs.a[f].seg, fs.a[f].wgs)) return hipErrorInvalidValue;
    }
    return launch_timed(t, stats_wave_kernel<kN>, dim3(fs.wg0[fs.n]), dim3(kWThreads), s, fs);
}

hipError_t launch_stats(const StatsArgs& a, hipStream_t s, const KTimer* t) {
    return launch_stats_fs(frame_set<1>(&a, 1, stats_grid(a.seg, a.wgs)), s, t);
}

hipError_t launch_stats_set(const StatsArgs* a, int n, hipStream_t s, const KTimer* t) {
    if (n < 1 || n > kMaxSet) return hipErrorInvalidValue;
    return launch_stats_fs(frame_set(a, n, stats_grid(a[0].seg, a[0].wgs)), s, t);
}

}  // namespace jpge
