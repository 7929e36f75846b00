// K2 stats_kernel (gfx950): DC difference chain (Image.cpp:638-678) + zig-zag RLE
// + category coding (Coding.hpp:148-283) -> the four symbol histograms of
// writeJPEG's "texts" (Image.cpp:888-906) with first-occurrence keys, and the
// symbol records of every tile in stream order (kernels.hpp), which the entropy
// code kernel turns into bits once the tables exist: the run-length and category
// work is done once per frame.
//
// Lane mapping (per step, below): a block row per lane, a block per lane, a
// non-zero per lane.  Persistent grid:
// each workgroup owns a contiguous run of 128-block tiles (the next one is loaded
// into registers while the current one is counted), accumulates into LDS
// (bank-staggered copies of the counters split same-address atomics) and flushes
// once into kHistReplicas global replicas.  First-occurrence keys (text index of
// the symbol, see huffman.hpp) are kept workgroup-relative in u32 LDS words and
// widened at the flush; the global key is stored inverted so atomicMax keeps the
// minimum.
#include <algorithm>
#include <cstddef>

#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

#ifndef K2_WAVE
#define K2_WAVE 1  // stats_wave_kernel (one wave per block, lane = zig-zag position); 0: the round-3 kernel
#endif
static_assert(K2_WAVE ? kRecSub > 1 : kRecSub == 1, "the round-3 kernel writes whole-tile record streams (K2_SUB=1)");

#if !K2_WAVE
#ifndef K2_STEP
#define K2_STEP 128
#endif
// Blocks per step: a tile is counted in steps of kK2Blocks.  64-block steps (34 KB,
// 63 VGPRs: 4 workgroups per CU) ran 3.5% slower in the pipeline than whole tiles at
// 3 per CU: the per-step barrier skeleton outweighs the occupancy.
constexpr int kK2Blocks = K2_STEP;
constexpr int kK2Threads = 512;
static_assert(kEntropyTile % kK2Blocks == 0, "steps divide a tile");
#ifndef K2_COPIES
#define K2_COPIES 4
#endif
constexpr int kHistCopies = K2_COPIES;
// Copy stride 512 + 4 words: LDS atomics bank by (word mod 32), so an unpadded
// stride (512) put every copy of a symbol on one bank and the copies only turned
// same-address serialisation into same-bank conflicts.  With +4 the copies of a
// symbol sit on banks s, s+4, ... (bank-conflict cycles halved).  4 copies, not 8:
// the 8.3 KB saved (with the shorter tile table) brings the workgroup to 52.7 KB,
// 3 per CU (6 waves per SIMD with <= 80 VGPRs): +5% in the pipeline, solo unchanged.
constexpr int kCopyWords = 2 * 256 + 4;
// DC counters: one wave's 64 lanes count a handful of categories; the same copies
// and bank stagger (stride 36 words) split them.
constexpr int kDcCopyWords = 2 * 16 + 4;

constexpr int kMaxNz = kK2Blocks * 63;  // AC non-zeros of a tile, at most
#ifndef K2_ZERO128
#define K2_ZERO128 1  // (counters and keys initialised in 16-byte stores: +0.4% over 3 pairs)
#endif
#ifndef K2_EARLY
#define K2_EARLY 1  // (first tile requested before the tile table: +0.7% in the pipeline, 3 pairs)
#endif
#ifndef K2_DROT
#define K2_DROT 128
#endif
#ifndef K2_PERCU
#define K2_PERCU 3
#endif
constexpr int kK2PerCu = K2_PERCU;        // resident workgroups per CU (stats_grid)
#ifndef K2_MAXRUN
#define K2_MAXRUN (kK2PerCu > 2 ? 128 : 256)
#endif
constexpr int kK2MaxRun = K2_MAXRUN;  // tiles per workgroup, at most (stats_grid)

// x / d and x % d for x < 2^24 (float reciprocal, corrected): the index arithmetic
// stays in 32-bit registers (a 64-bit division costs ~100 instructions per lane)
__device__ __forceinline__ uint32_t udiv24(uint32_t x, uint32_t d, float inv, uint32_t& r) {
    uint32_t q = (uint32_t)((float)x * inv);
    int32_t rr = (int32_t)(x - q * d);
    if (rr < 0) { --q; rr += (int32_t)d; }
    if (rr >= (int32_t)d) { ++q; rr -= (int32_t)d; }
    r = (uint32_t)rr;
    return q;
}

struct K2Lds {
    alignas(16) uint32_t nz[kMaxNz];                 // the tile's AC non-zeros in stream order: v & 0xFFFF | p << 16 | blk << 22
    uint32_t acnt[kHistCopies][kCopyWords];  // AC counters (Y-AC at 0, C-AC at 256), per copy
    uint32_t dcnt[kHistCopies][kDcCopyWords];  // DC counters (Y-DC at 0, C-DC at 16), per copy
    uint32_t key[4][256];                // workgroup-relative first-occurrence key (min)
    uint64_t bmask[kK2Blocks];           // AC non-zero mask (bit p = zig-zag position p); bit 0: ZRL block
    uint64_t lmask[kK2Blocks];           // ZRL block: the non-zeros after a run of 16+ zeros
    uint32_t nzbase[kK2Blocks];          // first non-zero of each block in nz
    // per block, read together by the symbol step: x = AC key base (text index * 128,
    // bit 31: Cr), y = (first record - first non-zero + 1) | chroma << 31
    uint2 binfo[kK2Blocks];
    int dcv[kK2Blocks];                  // DC of each block
    int prevdc[6];
    uint32_t wsum[kK2Threads / 64];
    uint32_t tot;                        // the tile's non-zeros
    // the workgroup's tiles: first block, and its MCU / slot / MCU row / column
    uint32_t tb0[kK2MaxRun + 1], tm6[kK2MaxRun], tk[kK2MaxRun], trow[kK2MaxRun], tcol[kK2MaxRun];
};


// K2 per tile, in four steps (barriers between them):
//  A  each lane holds one natural-order row of a block: its zig-zag positions, the
//     block's AC mask (OR over its 8 lanes), the DC;
//  B  one lane per block: non-zeros, EOB, ZRL test (a zero run of 16 before a later
//     non-zero), records; one scan gives every block's first non-zero and first record;
//  C  each row lane files its AC non-zeros into nz at their stream rank;
//  D  one lane per non-zero (all lanes busy whatever the block's density): run
//     (from the block mask), category, symbol, histogram, first-occurrence key, its
//     record at recbase + 1 + rank + ZRLs; one lane per block: DC and EOB.
template <int kN>
__global__ __launch_bounds__(kK2Threads) __attribute__((amdgpu_waves_per_eu(2 * kK2PerCu))) void stats_kernel(FrameSet<StatsArgs, kN> fs) {
    const uint32_t set_f = (kN == 1 ? 0u : set_member_rolled(fs.wg0, fs.n, blockIdx.x));  // (frame sets: kernels.hpp)
    const StatsArgs& a = fs.a[set_f];
    const uint32_t bid = blockIdx.x - fs.wg0[set_f], nbk = fs.wg0[set_f + 1] - fs.wg0[set_f];
    __shared__ K2Lds lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t mw = a.g.mw;
    // the entropy partition's tiles (seg_layout), a contiguous run per workgroup
    const uint32_t ntiles = seg_tiles(a.seg);
    const uint32_t t_first = (uint32_t)((uint64_t)bid * ntiles / nbk);
    const uint32_t t_last = (uint32_t)((uint64_t)(bid + 1) * ntiles / nbk);
#if K2_ZERO128
    // (counters and keys initialised in 16-byte stores: acnt and dcnt are contiguous)
    static_assert((kHistCopies * (kCopyWords + kDcCopyWords)) % 4 == 0 && offsetof(K2Lds, acnt) % 16 == 0 &&
                      offsetof(K2Lds, dcnt) == offsetof(K2Lds, acnt) + sizeof(lds.acnt) && offsetof(K2Lds, key) % 16 == 0,
                  "LDS initialisation in 16-byte stores");
    for (int i = tid; i < kHistCopies * (kCopyWords + kDcCopyWords) / 4; i += kK2Threads)
        reinterpret_cast<uint4*>(&lds.acnt[0][0])[i] = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < 1024 / 4; i += kK2Threads)
        reinterpret_cast<uint4*>(&lds.key[0][0])[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
#else
    for (int i = tid; i < kHistCopies * kCopyWords; i += kK2Threads) (&lds.acnt[0][0])[i] = 0;
    for (int i = tid; i < 1024; i += kK2Threads) (&lds.key[0][0])[i] = 0xFFFFFFFFu;
    for (int i = tid; i < kHistCopies * kDcCopyWords; i += kK2Threads) (&lds.dcnt[0][0])[i] = 0;
#endif
    JPGE_STAMP(0);
    // key bases: Y raster index of the first Y block row of this workgroup's first
    // MCU row, chroma raster index of that MCU row (keys are relative to them)
    const uint32_t bpm = a.g.bpm, yh = a.g.yh, yv = a.g.yv();  // MCU = yh x yv Y blocks + Cb + Cr
    const uint64_t ybw = (uint64_t)mw * yh;                    // Y blocks per block row
    const uint32_t yhs = (uint32_t)__builtin_ctz(yh);          // yh is 1, 2 or 4: k / yh = k >> yhs
    TileRegs<kK2Threads, kK2Blocks> regs;
    regs.init(tid);
#if K2_EARLY
    // the first tile's coefficients are requested before the tile table is built (its
    // 64-bit divisions and the barrier behind them would otherwise precede the load)
    if (t_first < t_last) {
        uint64_t b0;
        uint32_t nb;
        seg_tile(a.seg, t_first, b0, nb);
        regs.load(a.coef, b0, min((int)nb, kK2Blocks), tid);
    }
#endif
    // the tile table, computed once (64-bit arithmetic, one lane per tile)
    const uint32_t nrun = t_last - t_first;
    for (uint32_t i = tid; i <= nrun; i += kK2Threads) {
        uint64_t tb;
        uint32_t tn;
        seg_tile(a.seg, min(t_first + i, ntiles - 1), tb, tn);
        if (t_first + i >= ntiles) tb += tn;  // (the end of the last tile)
        lds.tb0[i] = (uint32_t)tb;
        if (i < nrun) {
            const uint32_t m6 = (uint32_t)(tb / bpm);
            lds.tm6[i] = m6;
            lds.tk[i] = (uint32_t)(tb - (uint64_t)m6 * bpm);
            lds.trow[i] = m6 / mw;
            lds.tcol[i] = m6 % mw;
        }
    }
#if K2_EARLY
    lds_barrier();  // (the table and the zeroed counters are in LDS; the first load stays in flight)
#else
    __syncthreads();
#endif
    const uint64_t fb0 = nrun ? lds.tb0[0] : 0;
    const uint32_t fnb = nrun ? lds.tb0[1] - lds.tb0[0] : 0;
    const uint32_t mrow0 = nrun ? lds.trow[0] : 0;
    const uint64_t ybase = (uint64_t)mrow0 * yv * ybw;
    const uint64_t cbase = (uint64_t)mrow0 * mw;
    const float inv_bpm = 1.0f / (float)bpm, inv_mw = 1.0f / (float)mw;
#if !K2_EARLY
    if (t_first < t_last) regs.load(a.coef, fb0, min((int)fnb, kK2Blocks), tid);
#else
    (void)fnb;
#endif
    constexpr int kPer = TileRegs<kK2Threads, kK2Blocks>::kPer;

    uint64_t tq = JPGE_NOW();
    for (uint32_t tile = t_first; tile < t_last; ++tile) {
        const uint32_t ti = tile - t_first;
        const uint64_t tb = lds.tb0[ti];
        const int tnb = (int)(lds.tb0[ti + 1] - lds.tb0[ti]);
        uint32_t* grec = a.recs + (uint64_t)tile * kTileRecords;
        uint32_t rec0 = 0;  // the tile's records before this step
      for (int s0 = 0; s0 < tnb; s0 += kK2Blocks) {
        const uint64_t b0 = tb + (uint64_t)s0;
        const int nb = min(tnb - s0, kK2Blocks);
        lds_barrier();  // the previous step's readers are done
        // ---- A: masks and DCs ----
        // (zlo/zhi made opaque per tile: the compiler would otherwise keep 8 zig-zag
        // positions and 8 64-bit masks derived from them live across the whole loop)
        asm volatile("" : "+v"(regs.zlo), "+v"(regs.zhi));
        uint64_t rowbits[kPer];  // zig-zag positions of this lane's non-zero AC values
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int q = tid + i * kK2Threads;
            const bool ok = q < nb * 8;
            const int blk = q >> 3, row = q & 7;
            const uint32_t w[4] = {regs.v[i].x, regs.v[i].y, regs.v[i].z, regs.v[i].w};
            uint64_t m = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int16_t c = (int16_t)(u & 1 ? w[u >> 1] >> 16 : w[u >> 1] & 0xFFFF);
                const uint32_t zp = ((u < 4 ? regs.zlo : regs.zhi) >> (8 * (u & 3))) & 0xFF;
                m |= (uint64_t)(c != 0) << zp;  // (rows past the tile were loaded as zeros)
            }
            rowbits[i] = m & ~1ull;
            m = or_lanes8(m);  // the block's 8 rows
            if (ok && row == 0) {
                lds.bmask[blk] = m & ~1ull;
                lds.dcv[blk] = (int16_t)(w[0] & 0xFFFF);
            }
        }
        if (tid < 6) lds.prevdc[tid] = regs.prev_dc;
        lds_barrier();
        JPGE_ACC(0, tq);
        // ---- B: per block counts, ZRL test, key index; one scan ----
        uint32_t cnt = 0;
        const int b = tid;
        const bool bact = b < nb;
        int comp = 0;
        uint32_t rel = 0;  // the block's text index (relative to the key bases; bit 31: Cr)
        int k = 0;         // its slot in its MCU
        uint32_t m6 = 0;   // its MCU
        if (bact) {
            uint64_t m = lds.bmask[b];
            const uint32_t n = (uint32_t)__builtin_popcountll(m);
            const bool eob = !(m >> 63);
            const uint64_t x = m | 1ull;
            const int last = 63 - __builtin_clzll(x);
            // a run of 16 zeros wholly before the last non-zero: a ZRL block
            uint64_t z = ~x & ((last ? (1ull << last) : 1ull) - 1ull);
            uint64_t r = z & (z >> 1);
            r &= r >> 2;
            r &= r >> 4;
            r &= r >> 8;
            uint32_t zrl = 0;
            if (r) {  // rare: the non-zeros after a run of 16+ zeros, and their ZRL count
                const uint64_t L = m & (r << 16);
                for (uint64_t t = L; t; t &= t - 1) {
                    const int p = __builtin_ctzll(t);
                    zrl += (uint32_t)(p - (63 - __builtin_clzll(x & ((1ull << p) - 1ull))) - 1) >> 4;
                }
                lds.bmask[b] = m | 1ull;  // flag: a ZRL block
                lds.lmask[b] = L;
            }
            cnt = (n << 16) | (1u + n + zrl + (eob ? 1u : 0u));
            // the block's MCU and slot, from the tile's (32-bit, small divisions)
            uint32_t kk;
            const uint32_t carry = udiv24(lds.tk[ti] + (uint32_t)(s0 + b), bpm, inv_bpm, kk);
            k = (int)kk;
            m6 = lds.tm6[ti] + carry;
            uint32_t mcol;
            const uint32_t mrow = lds.trow[ti] + udiv24(lds.tcol[ti] + carry, mw, inv_mw, mcol);
            comp = block_comp(k, bpm);
            // the block's text index (the Y text is in block raster order; all Cr after all Cb)
            if (comp == 0) {
                rel = (uint32_t)(((uint64_t)mrow * yv + ((uint32_t)k >> yhs)) * ybw + (uint64_t)mcol * yh +
                                 ((uint32_t)k & (yh - 1)) - ybase);
            } else {
                rel = (uint32_t)(m6 - cbase) | (comp == 2 ? 0x80000000u : 0u);
            }
        }
        uint32_t T;
        const uint32_t ex = block_scan<kK2Threads / 64, uint32_t, uint32_t, true, false>(cnt, lds.wsum, lane, wv, T);  // (A's barrier leads)
        if (bact) {
            lds.nzbase[b] = ex >> 16;
            lds.binfo[b] = make_uint2((rel & 0x80000000u) | ((rel & 0x7FFFFFFFu) << 7),
                                      (rec0 + (ex & 0xFFFF) + 1 - (ex >> 16)) | (comp ? 0x80000000u : 0u));
        }
        if (tid == 0) lds.tot = T >> 16;
        lds_barrier();
        JPGE_ACC(1, tq);
        // ---- C: the non-zeros at their stream rank ----
        asm volatile("" : "+v"(regs.zlo), "+v"(regs.zhi));
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int q = tid + i * kK2Threads;
            const int blk = q >> 3;
            uint64_t t = rowbits[i];
            if (t) {
                const uint64_t bm = lds.bmask[blk] & ~1ull;
                const uint32_t base = lds.nzbase[blk];
                const uint32_t w[4] = {regs.v[i].x, regs.v[i].y, regs.v[i].z, regs.v[i].w};
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int16_t c = (int16_t)(u & 1 ? w[u >> 1] >> 16 : w[u >> 1] & 0xFFFF);
                    const uint32_t zp = ((u < 4 ? regs.zlo : regs.zhi) >> (8 * (u & 3))) & 0xFF;
                    if (zp != 0 && c != 0) {
                        const uint32_t rank = (uint32_t)__builtin_popcountll(bm << (64u - zp));  // (zp >= 1)
                        lds.nz[base + rank] = ((uint32_t)c & 0xFFFFu) | (zp << 16) | ((uint32_t)blk << 22);
                    }
                }
            }
        }
        if (s0 + kK2Blocks < tnb)  // the rows are filed: load the next step's
            regs.load(a.coef, b0 + kK2Blocks, min(tnb - s0 - kK2Blocks, kK2Blocks), tid);
        else if (tile + 1 < t_last)
            regs.load(a.coef, lds.tb0[ti + 1], min((int)(lds.tb0[ti + 2] - lds.tb0[ti + 1]), kK2Blocks), tid);
        lds_barrier();
        JPGE_ACC(2, tq);
        // ---- D: symbols ----
        const uint32_t N = lds.tot;
        // (rotated by K2_DROT: the loop's partial last round falls first on the waves past
        // the block lanes, which code the DC and EOB records after it)
        for (uint32_t e = (tid + K2_DROT) & (kK2Threads - 1); e < N; e += kK2Threads) {
            const uint32_t ent = lds.nz[e];
            const int v = (int16_t)(ent & 0xFFFF);
            const int p = (int)((ent >> 16) & 63), blk = (int)(ent >> 22);
            const uint64_t m = lds.bmask[blk];
            // zeros since the previous non-zero (or the DC): the leading zeros of the mask
            // below p, shifted to the top (p >= 1)
            int run = __builtin_clzll((m | 1ull) << (64 - p));
            uint32_t zb = 0;  // ZRL records of this block up to and including this entry's
            if (m & 1ull) {   // a ZRL block (rare): the long runs at or before p
                for (uint64_t t = lds.lmask[blk] & (((1ull << p) - 1ull) | (1ull << p)); t; t &= t - 1) {
                    const int q = __builtin_ctzll(t);
                    zb += (uint32_t)(q - (63 - __builtin_clzll(m & ((1ull << q) - 1ull))) - 1) >> 4;
                }
            }
            const int nzr = run >> 4;
            run &= 15;
            const int cat = category(v);
            const int sym = (run << 4) | cat;
            const uint2 bi = lds.binfo[blk];
            const uint32_t acb = bi.x;
            const int tsel = (int)(bi.y >> 31);
            atomicAdd(&lds.acnt[lane & (kHistCopies - 1)][tsel * 256 + sym], 1u);
            const uint32_t kk = acb + 2u * p + 1u;
            uint32_t* kp = &lds.key[2 * tsel + 1][sym];
            if (kk < *kp) atomicMin(kp, kk);
            const uint32_t o = (bi.y & 0x7FFFFFFFu) + e + zb;  // recbase + 1 + rank + ZRLs
            if (nzr) {  // its ZRLs (F/0) just before it
                atomicAdd(&lds.acnt[lane & (kHistCopies - 1)][tsel * 256 + 0xF0], (uint32_t)nzr);
                uint32_t* kz = &lds.key[2 * tsel + 1][0xF0];
                if (kk - 1u < *kz) atomicMin(kz, kk - 1u);
                for (int z = 1; z <= nzr; ++z) grec[o - z] = rec_word(2 * tsel + 1, 0xF0, 0);
            }
            grec[o] = rec_word(2 * tsel + 1, (uint32_t)sym, extra_bits(v, cat));
        }
        if (bact) {  // one lane per block: DC and EOB
            const uint64_t m = lds.bmask[b];
            const int tsel = comp != 0;
            const uint32_t acb = (rel & 0x80000000u) | ((rel & 0x7FFFFFFFu) << 7);  // text index * 128
            // DC difference to the chain predecessor (Image.cpp:638-678)
            int pd;
            {
                bool reset = false;
                if (a.rst.mcus && (k == 0 || k >= (int)bpm - 2)) {
                    // exact 32-bit remainder: MCU numbers reach 2^26 (65535^2 at 4:4:4),
                    // beyond udiv24's float reciprocal (rare path: interval-boundary blocks)
                    reset = (m6 + a.rst.mcu0) % a.rst.mcus == 0;
                }
                // the predecessor (dc_pred_index): the previous Y slot, 3 blocks back for an
                // MCU's first Y block, bpm back for chroma; none in the first MCU
                const bool ynext = k >= 1 && k < (int)bpm - 2;
                const int back = ynext ? 1 : (k == 0 ? 3 : (int)bpm);
                const int64_t pg = (!ynext && b0 + b < bpm) ? -1 : (int64_t)(b0 + b) - back;
                pd = reset ? 0 : pg < 0 ? a.seed.v[block_comp(k, bpm)]
                               : pg >= (int64_t)b0 ? lds.dcv[pg - (int64_t)b0] : lds.prevdc[pg - ((int64_t)b0 - 6)];
            }
            const int dd = lds.dcv[b] - pd;
            const int dcat = category(dd);
            atomicAdd(&lds.dcnt[lane & (kHistCopies - 1)][tsel * 16 + dcat], 1u);
            uint32_t* kp = &lds.key[2 * tsel][dcat];
            if (rel < *kp) atomicMin(kp, rel);
            // the block's first record (from LDS: keeping the scan results live through
            // C and D costs VGPRs)
            const uint32_t recb = (lds.binfo[b].y & 0x7FFFFFFFu) - 1u + lds.nzbase[b];
            grec[recb] = rec_word(2 * tsel, (uint32_t)dcat, extra_bits(dd, dcat));
            if (!(m >> 63)) {  // EOB
                atomicAdd(&lds.acnt[lane & (kHistCopies - 1)][tsel * 256], 1u);
                uint32_t* ke = &lds.key[2 * tsel + 1][0];
                if (acb + 127u < *ke) atomicMin(ke, acb + 127u);
                const uint32_t eo = (b + 1 < nb ? (lds.binfo[b + 1].y & 0x7FFFFFFFu) - 1u + lds.nzbase[b + 1]
                                                : rec0 + (T & 0xFFFF)) - 1;  // the block's last record
                grec[eo] = rec_word(2 * tsel + 1, 0, 0);
            }
        }
        JPGE_ACC(3, tq);
        rec0 += T & 0xFFFF;
      }
        if (tid == 0) a.tcount[tile] = rec0;
    }
    __syncthreads();
    JPGE_STAMP(2);

    const int rep = bid % kHistReplicas;
    const uint64_t ncb = a.key_ncb ? a.key_ncb : a.g.nmcu();  // Cb blocks of the whole image
#pragma unroll
    for (int r = 0; r < 1024 / kK2Threads; ++r) {
        const int i = tid + r * kK2Threads;
        const int t = i >> 8, s = i & 255;
        const bool ac = t & 1;
        uint32_t c = 0;
        if (ac) {
            for (int cp = 0; cp < kHistCopies; ++cp) c += lds.acnt[cp][(t >> 1) * 256 + s];
        } else if (s < 16) {
            for (int cp = 0; cp < kHistCopies; ++cp) c += lds.dcnt[cp][(t >> 1) * 16 + s];
        }
        if (!c) continue;
        atomicAdd(&a.hist.cnt[(rep * 4 + t) * 256 + s], c);
        const uint32_t k32 = lds.key[t][s];
        uint64_t base;  // (global texts: a stripe's bases are offset into the whole image)
        if (t < 2) base = a.key_y0 + ybase;
        else base = a.key_c0 + cbase + ((k32 & 0x80000000u) ? ncb : 0ull);
        const uint64_t gkey = (ac ? base * 128ull : base) + (k32 & 0x7FFFFFFFu);
        const unsigned long long inv = ~gkey;
        unsigned long long* gk = reinterpret_cast<unsigned long long*>(&a.hist.key[t * 256 + s]);
        if (inv > *gk) atomicMax(gk, inv);
    }
    __syncthreads();
    JPGE_STAMP(3);
}
#endif  // !K2_WAVE

#if K2_WAVE
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
// atomics on the workgroup's copies (lane & 1: same-symbol lanes of one instruction
// land on different copies and banks), first-occurrence keys a read and a rare
// atomicMin; lanes without a record touch a dummy word of their own, so none of it
// needs an exec mask.  A block with a run of 16+ zeros before a non-zero (rare)
// takes a wave scan for its ZRL records.  Each block's DC difference replaces its DC
// coefficient in the stage, so lane 0 codes the DC record with the block's records.
// Reference: DC chain Image.cpp:638-678, RLE + category Coding.hpp:148-283 and
// Image.cpp:680-735, texts Image.cpp:888-906.
#ifndef K2W_WAVES
#define K2W_WAVES 8  // (8-wave workgroups: 28.9 us alone at 4K vs 39.7 with 4; 16 waves: 148 GPix/s in the pipeline)
#endif
#ifndef K2W_COPIES
#define K2W_COPIES 8
#endif
#ifndef K2W_WPE
#define K2W_WPE 8  // waves per SIMD the register allocation targets (<= 64 VGPRs: 4 workgroups per CU; 7 let the compiler take 69)
#endif
#ifndef K2W_DUMMY_ADD
#define K2W_DUMMY_ADD 0  // 1: lanes without a record add into a dummy word of their own instead of being masked off
#endif
constexpr int kWWaves = K2W_WAVES;
constexpr int kWThreads = 64 * kWWaves;
constexpr int kSubBlocks = (kEntropyTile + kRecSub - 1) / kRecSub;  // blocks of a sub-stream, at most
static_assert(kRecSub > 1 && kSubBlocks <= 64 && kSubBlocks % 8 == 0, "a sub-stream's blocks fit a wave");
constexpr int kWRows = kSubBlocks * 8 / 64;  // 16-byte block rows per lane = 8-block chunks per sub-stream
constexpr int kWCopies = K2W_COPIES;
// Counter / key words: table t's symbol s at kTabBase(t) + (s & 15) + 19 * (s >> 4).
// The stride 19 puts the frequent symbols (runs 0-4, sizes 1-5) on distinct banks
// (a stride of 16 put runs 0 and 2, or 1 and 3, of a size on one bank), and is
// injective for sizes up to 18.
constexpr uint32_t kRunStride = 19;
constexpr uint32_t kAcWords = 15 + kRunStride * 15 + 1;  // 301
__host__ __device__ constexpr uint32_t tab_base(uint32_t t) { return (t >> 1) * (16 + kAcWords) + (t & 1) * 16; }
constexpr uint32_t kWSyms = tab_base(3) + kAcWords;  // 634 words: Y-DC, Y-AC, C-DC, C-AC
constexpr uint32_t kWDummy = kWSyms;                  // + lane: the words of lanes without a record
// copy stride == 32 / copies (mod 32): the copies of a word sit on distinct banks
constexpr uint32_t kWBankStep = 32u / kWCopies;
constexpr uint32_t kWCopyWords = (kWSyms + 64 + 31 - kWBankStep) / 32 * 32 + kWBankStep;
static_assert(kWCopies <= 32 && kWCopyWords % 32 == kWBankStep && kWCopyWords >= kWSyms + 64, "copy stride");
constexpr uint32_t kWKeyWords = (kWSyms + 1 + 3) / 4 * 4;  // keys, then one shared dummy word
constexpr uint32_t kWMaxSubs = 1024;  // sub-streams per workgroup, at most (stats_grid)

// zig-zag position -> natural index (inverse of Coding.hpp:57-81)
static __constant__ uint8_t kZzToNat[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct K2WLds {
    alignas(16) uint32_t stage[kWWaves][8 * 32 + 32];   // each wave's 8-block chunk: int16 [block][64], natural order; 64 spare int16
    alignas(16) uint32_t cnt[kWCopies * kWCopyWords];    // counters [copy][word], then the dummies
    alignas(16) uint32_t key[kWKeyWords];                // first-occurrence keys (min), workgroup-relative
    uint32_t sb0[kWMaxSubs + 1];                         // the workgroup's sub-streams' first blocks, and the end
    uint32_t next;                                       // the next sub-stream to take
};

template <int kN>
__global__ __launch_bounds__(kWThreads) __attribute__((amdgpu_waves_per_eu(K2W_WPE))) void stats_wave_kernel(FrameSet<StatsArgs, kN> fs) {
    const uint32_t set_f = (kN == 1 ? 0u : set_member_rolled(fs.wg0, fs.n, blockIdx.x));  // (frame sets: kernels.hpp)
    const StatsArgs& a = fs.a[set_f];
    const uint32_t bid = blockIdx.x - fs.wg0[set_f], nbk = fs.wg0[set_f + 1] - fs.wg0[set_f];
    __shared__ K2WLds L;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    static_assert((kWCopies * kWCopyWords) % 4 == 0 && kWKeyWords % 4 == 0, "16-byte initialisation");
    for (int i = tid; i < (int)(kWCopies * kWCopyWords / 4); i += kWThreads)
        reinterpret_cast<uint4*>(L.cnt)[i] = make_uint4(0, 0, 0, 0);
    for (int i = tid; i < (int)(kWKeyWords / 4); i += kWThreads)
        reinterpret_cast<uint4*>(L.key)[i] = make_uint4(~0u, ~0u, ~0u, ~0u);

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
    for (uint32_t i = tid; i <= ns; i += kWThreads) {  // their first blocks (block numbers < 2^32: launch_stats)
        uint64_t b;
        uint32_t n;
        sub_tile(a.seg, min(s_lo + i, S - 1), b, n);
        L.sb0[i] = (uint32_t)(s_lo + i < S ? b : b + n);
    }
    if (tid == 0) L.next = kWWaves;  // (sub-stream w is wave w's first)
    __syncthreads();
    if (ns == 0) return;
    // key bases (keys are kept relative to them): the workgroup's first MCU row
    const uint32_t mrow0 = __builtin_amdgcn_readfirstlane((L.sb0[0] / bpm) / mw);
    const uint32_t ybase = mrow0 * yv * ybw, cbase = mrow0 * mw;
    JPGE_STAMP(0);
    uint64_t tq = JPGE_NOW();

    const uint32_t natoff = kZzToNat[lane];  // this lane's coefficient in a staged block (int16 index)
    const uint32_t k2p = 2u * (uint32_t)lane;
    uint32_t* const cnt = L.cnt + (uint32_t)(lane & (kWCopies - 1)) * kWCopyWords;
    const uint32_t dummy = kWDummy + (uint32_t)lane;  // this lane's dummy counter word
    const uint32_t shl = (uint32_t)(64 - lane) & 63u;
    const uint64_t lanes_ac = ~1ull;  // every lane but the DC
    const uint32_t dc_tab = lane == 0 ? 1u << 24 : 0u;  // (a record's table byte: 2t + 1 -> 2t)
    int16_t* st16 = reinterpret_cast<int16_t*>(L.stage[wv]);
    uint4* st4 = reinterpret_cast<uint4*>(L.stage[wv]);

    uint4 cur[kWRows];
    int dcs = 0;  // lane l < nb + 6: the DC of block b0 - 6 + l of the fetched sub-stream (0 before the frame)
    auto rows = [&](uint32_t si) {  // sub-stream si's coefficients through a buffer descriptor (zeros past its blocks)
        const uint32_t b0 = L.sb0[si], nb = L.sb0[si + 1] - b0;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(a.coef + (uint64_t)b0 * 64), 0, nb * 128,
                                                 0x00020000);
    };
    auto load_row = [&](const __amdgpu_buffer_rsrc_t& rs, int i) {
        return as_u4(__builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(lane + 64 * i) * 16, 0, 0));
    };
    auto load_dcs = [&](uint32_t si) {
        const uint32_t b0 = L.sb0[si], nb = L.sb0[si + 1] - b0;
        const int64_t g = (int64_t)b0 - 6 + lane;
        dcs = ((uint32_t)lane < nb + 6 && g >= 0) ? a.coef[(uint64_t)g * 64] : 0;
    };
    uint32_t si = (uint32_t)wv;
    if (si < ns) {
        const __amdgpu_buffer_rsrc_t rs = rows(si);
#pragma unroll
        for (int i = 0; i < kWRows; ++i) cur[i] = load_row(rs, i);
        load_dcs(si);
    }
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
        // the block loop reads two words per block: the AC key base (text index * 128 + 1;
        // a key is base + 2p), and the AC table as a record's top byte | its first counter word
        const uint32_t acb = (rel & 0x80000000u) | ((rel & 0x7FFFFFFFu) << 7) | 1u;
        const uint32_t tw = ((2u * tsel + 1u) << 24) | tab_base(2u * tsel + 1u);
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
        const int dcat = __builtin_amdgcn_frexp_expf((float)dd);
        const uint32_t drec = rec_word(2u * tsel, (uint32_t)dcat, extra_bits(dd, dcat));
        if (si == (uint32_t)wv) JPGE_STAMP(1);  // (wave 0: its first sub-stream's data is in)
        JPGE_ACC(1, tq);

        // ---- the blocks ----
        uint32_t* srec = a.recs + (uint64_t)(s / kRecSub) * kTileRecords + (s % kRecSub) * kSubRecords;
        const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(srec, 0, kSubRecords * 4, 0x00020000);
        uint32_t base = 0;   // the block's first record (its DC) in the sub-stream
        // one block's fields (lane p: zig-zag position p)
        struct Blk {
            uint64_t M, em;     // AC non-zeros; the lanes with a record (+ lane 63: non-zero, or the EOB)
            uint32_t rk, run;   // record index in the block (DC = 0), zeros before the coefficient
            uint32_t rec, w;    // the record; its counter / key word
            uint32_t Tj, acbj, acw;  // the block's AC table (top byte), key base, table base word
            bool zrl;           // a run of 16+ zeros before a non-zero
        };
        auto prep = [&](int c, uint32_t jb) {
            Blk b;
            const uint64_t B1 = __ballot(c != 0) | 1ull;  // the AC non-zeros, and bit 0
            b.M = B1 & lanes_ac;
            const uint32_t twj = __builtin_amdgcn_readlane(tw, jb);
            b.Tj = twj & 0xFF000000u;                       // the AC table, as a record's top byte
            b.acw = twj & 0xFFFFu;                          // its first counter / key word
            b.acbj = __builtin_amdgcn_readlane(acb, jb);    // (+ 2p: the key; the EOB lane 63: text * 128 + 127)
            b.rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(B1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B1, 0u));
            b.run = (uint32_t)__builtin_clzll(B1 << shl);  // (lane 0: unused)
            const int cat = __builtin_amdgcn_frexp_expf((float)c);
            const uint32_t bits = extra_bits(c, cat);
            const uint32_t rr = __builtin_amdgcn_inverse_ballot_w64(b.M) ? (b.run & 15u) : 0u;  // (the EOB lane, the DC lane: 0)
            // lane 0 (the DC position, where the stage holds the block's DC difference)
            // codes the block's DC record (its table: the AC table's number less one),
            // stored with the block's other records at its first record (rank 0): stored
            // after the sub-stream, the DC records rewrote lines already written back (K2
            // wrote 1.24x its record bytes)
            b.rec = (b.Tj | (((rr << 4) | (uint32_t)cat) << 16) | bits) ^ dc_tab;
            b.w = b.acw + (uint32_t)cat + kRunStride * rr;
            b.em = b.M | (1ull << 63);
            b.zrl = (__ballot(b.run >= 16u) & b.M) != 0;
            return b;
        };
        // (general form, every block with ZRLs) its records from `base`, histogram and
        // keys; returns its record count
        auto emit = [&](Blk b, uint32_t base) -> uint32_t {
            uint32_t zt = 0;
            if (b.zrl) {  // ZRL records (F/0) before the non-zeros after 16+ zeros (rare)
                const uint32_t nzr = __builtin_amdgcn_inverse_ballot_w64(b.M) ? b.run >> 4 : 0u;
                const uint32_t zi = wave_scan_incl(nzr);
                zt = __builtin_amdgcn_readlane(zi, 63);
                b.rk += zi;
                if (nzr) {
                    const uint32_t zrec = b.Tj | (0xF0u << 16);
                    for (uint32_t z = 1; z <= nzr; ++z) srec[base + b.rk - z] = zrec;
                    const uint32_t wz = b.acw + kRunStride * 15u;  // (symbol 0xF0)
                    atomicAdd(&cnt[wz], nzr);
                    const uint32_t kz = b.acbj + k2p - 1u;
                    if (kz < L.key[wz]) atomicMin(&L.key[wz], kz);
                }
            }
            if (lane == 0) srec[base] = b.rec;  // (the DC record)
            if (__builtin_amdgcn_inverse_ballot_w64(b.em)) {
                srec[base + b.rk] = b.rec;
                atomicAdd(&cnt[b.w], 1u);
                const uint32_t kk = b.acbj + k2p;
                if (kk < L.key[b.w]) atomicMin(&L.key[b.w], kk);
            }
            return 1u + (uint32_t)__builtin_popcountll(b.em) + zt;  // DC, the non-zeros and the EOB, the ZRLs
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
            const int16_t* cp = st16 + natoff;  // (the pair after the chunk's last reads past it: unused)
            int cnA = cp[0], cnB = cp[64];
            uint32_t jb = j0;
            for (; jb + 1 < j1; jb += 2) {
                const int cA = cnA, cB = cnB;
                cp += 128;
                cnA = cp[0];
                cnB = cp[64];
                const Blk A = prep(cA, jb), B = prep(cB, jb + 1);
                uint32_t baseB;
                if (!(A.zrl || B.zrl)) {
                    // lanes without a record store out of range (dropped); their counter adds
                    // go to a dummy word of their own (K2W_DUMMY_ADD) or are masked off
                    baseB = base + 1u + (uint32_t)__builtin_popcountll(A.em);
                    const bool ia = __builtin_amdgcn_inverse_ballot_w64(A.em), ib = __builtin_amdgcn_inverse_ballot_w64(B.em);
                    // (lane 0: the DC record, at rank 0)
                    __builtin_amdgcn_raw_buffer_store_b32(A.rec, rrs, ia || lane == 0 ? (base + A.rk) * 4u : 0x80000000u, 0, 0);
                    __builtin_amdgcn_raw_buffer_store_b32(B.rec, rrs, ib || lane == 0 ? (baseB + B.rk) * 4u : 0x80000000u, 0, 0);
#if K2W_DUMMY_ADD
                    atomicAdd(&cnt[ia ? A.w : dummy], 1u);
                    atomicAdd(&cnt[ib ? B.w : dummy], 1u);
#else
                    if (ia) atomicAdd(&cnt[A.w], 1u);
                    if (ib) atomicAdd(&cnt[B.w], 1u);
#endif
                    // (every lane reads its word: a lane without a record has c = 0, so its
                    // word is its table's first, and lane 0's is in range too)
                    const uint32_t kvA = L.key[A.w], kvB = L.key[B.w];
                    const uint32_t kkA = A.acbj + k2p, kkB = B.acbj + k2p;
                    const bool fa = ia && kkA < kvA, fb = ib && kkB < kvB;
                    if (__ballot(fa || fb)) {  // (rare: a first occurrence in this workgroup so far)
                        if (fa) atomicMin(&L.key[A.w], kkA);
                        if (fb) atomicMin(&L.key[B.w], kkB);
                    }
                    base = baseB + 1u + (uint32_t)__builtin_popcountll(B.em);
                } else {
                    baseB = base + emit(A, base);
                    base = baseB + emit(B, baseB);
                }
            }
            if (jb < j1) base += emit(prep(cnA, jb), base);  // an odd last block
        }
        JPGE_ACC(2, tq);
        if ((uint32_t)lane < nb) {  // the DC symbols' counts and keys (their records went with their blocks)
            const uint32_t w = ((drec >> 25) ? tab_base(2) : tab_base(0)) + ((drec >> 16) & 0xFFu);
            const uint32_t rk = (acb & 0x80000000u) | ((acb & 0x7FFFFFFFu) >> 7);  // the text index
            atomicAdd(&cnt[w], 1u);
            if (rk < L.key[w]) atomicMin(&L.key[w], rk);
        }
        if (lane == 0) a.tcount[s] = base;
        si = sn;
        JPGE_ACC(3, tq);
    }
    JPGE_STAMP(2);
    __syncthreads();
#ifdef K2W_FLUSH  // (ablation builds only: 0 no flush, 1 counts only; outputs invalid)
    if (K2W_FLUSH == 0) return;
#endif

    const int rep = bid % kHistReplicas;
    const uint64_t ncb = a.key_ncb ? a.key_ncb : a.g.nmcu();  // Cb blocks of the whole image
    for (int i = tid; i < 1024; i += kWThreads) {
        const uint32_t t = (uint32_t)i >> 8, sy = (uint32_t)i & 255u;
        if (!(t & 1) && sy >= 16) continue;  // (DC tables: categories < 16)
        const uint32_t w = tab_base(t) + (sy & 15u) + kRunStride * (sy >> 4);
        uint32_t c = 0;
#pragma unroll
        for (int cp = 0; cp < kWCopies; ++cp) c += L.cnt[cp * kWCopyWords + w];
        if (!c) continue;
        atomicAdd(&a.hist.cnt[rep * 1024 + i], c);
#ifdef K2W_FLUSH
        if (K2W_FLUSH == 1) continue;
#endif
        const uint32_t k32 = L.key[w];
        uint64_t kb;  // (global texts: a stripe's bases are offset into the whole image)
        if (t < 2) kb = a.key_y0 + ybase;
        else kb = a.key_c0 + cbase + ((k32 & 0x80000000u) ? ncb : 0ull);
        const uint64_t gkey = ((t & 1) ? kb * 128ull : kb) + (k32 & 0x7FFFFFFFu);
        const unsigned long long inv = ~gkey;
        unsigned long long* gk = reinterpret_cast<unsigned long long*>(&a.hist.key[i]);
        if (inv > *gk) atomicMax(gk, inv);
    }
    JPGE_STAMP(3);
}
#endif  // K2_WAVE

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

#if K2_WAVE
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
#else
uint32_t stats_grid(const SegLayout& L, uint32_t wgs) {
    const uint32_t tiles = seg_tiles(L);
    // persistent over contiguous runs of at most kK2MaxRun tiles: kK2PerCu per CU by
    // default, or wgs (kept within the tile-table bound and the tile count)
    const uint32_t want = wgs ? wgs : 256u * kK2PerCu;
    const uint32_t g = tiles < want ? tiles : want;
    const uint32_t need = (tiles + kK2MaxRun - 1) / kK2MaxRun;
    if (g >= need) return g;
    // more workgroups than asked for (the tile-table bound): whole multiples of the 256
    // CUs, so every CU holds as many (16384^2 beside other lanes: 384 workgroups ran
    // 174 GPix/s, 512 ran 193)
    const uint32_t r = (need + 255u) / 256u * 256u;
    return r < tiles ? r : tiles;
}

template <int kN>
static hipError_t launch_stats_fs(const FrameSet<StatsArgs, kN>& fs, hipStream_t s, const KTimer* t) {
    for (uint32_t f = 0; f < fs.n; ++f)
        if (fs.wg0[f + 1] - fs.wg0[f] != stats_grid(fs.a[f].seg, fs.a[f].wgs)) return hipErrorInvalidValue;
    return launch_timed(t, stats_kernel<kN>, dim3(fs.wg0[fs.n]), dim3(kK2Threads), s, fs);
}
#endif

hipError_t launch_stats(const StatsArgs& a, hipStream_t s, const KTimer* t) {
    return launch_stats_fs(frame_set<1>(&a, 1, stats_grid(a.seg, a.wgs)), s, t);
}

hipError_t launch_stats_set(const StatsArgs* a, int n, hipStream_t s, const KTimer* t) {
    if (n < 1 || n > kMaxSet) return hipErrorInvalidValue;
    return launch_stats_fs(frame_set(a, n, stats_grid(a[0].seg, a[0].wgs)), s, t);
}

}  // namespace jpge
