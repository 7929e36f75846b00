// K2 stats_kernel (gfx950): DC difference chain (Image.cpp:638-678) + zig-zag RLE
// + category coding (Coding.hpp:148-283) -> the four symbol histograms of
// writeJPEG's "texts" (Image.cpp:888-906) with first-occurrence keys, and the
// symbol records of every tile in stream order (kernels.hpp), which the entropy
// code kernel turns into bits once the tables exist: the run-length and category
// work is done once per frame.
//
// Lane mapping: PartView (device_common.hpp), four lanes per block, one wave per
// 16 zig-zag positions of 64 blocks.  Persistent grid:
// each workgroup owns a contiguous run of 128-block tiles (the next one is loaded
// into registers while the current one is counted), accumulates into LDS
// (8 bank-staggered copies of the AC counters cap same-address atomics at 8 lanes) and flushes
// once into kHistReplicas global replicas.  First-occurrence keys (text index of
// the symbol, see huffman.hpp) are kept workgroup-relative in u32 LDS words and
// widened at the flush; the global key is stored inverted so atomicMax keeps the
// minimum.
#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

constexpr int kK2Blocks = kStatsTile;
constexpr int kK2Threads = kK2Blocks * kPartsPerBlock;
constexpr int kHistCopies = 8;
// Copy stride 512 + 4 words: LDS atomics bank by (word mod 32), so an unpadded
// stride (512) put every copy of a symbol on one bank and the copies only turned
// same-address serialisation into same-bank conflicts.  With +4 the 8 copies of a
// symbol sit on banks s, s+4, ..., s+28 (bank-conflict cycles halved; 16 copies at
// +2 removed only 7% more and cost LDS occupancy in the pipeline).
constexpr int kCopyWords = 2 * 256 + 4;
// DC counters: one wave's 64 lanes count a handful of categories; the same copies
// and bank stagger (stride 36 words) split them.
constexpr int kDcCopyWords = 2 * 16 + 4;

struct K2Lds {
    int16_t zz[kK2Blocks * kZzStride];
    uint32_t acnt[kHistCopies][kCopyWords];  // AC counters (Y-AC at 0, C-AC at 256), per copy
    uint32_t dcnt[kHistCopies][kDcCopyWords];  // DC counters (Y-DC at 0, C-DC at 16), per copy
    uint32_t key[4][256];                // workgroup-relative first-occurrence key (min)
    uint64_t bmask[kK2Blocks];
    int prevdc[6];
    uint32_t pcnt[kK2Threads];           // records of every part (stream order), then their offsets
    uint32_t wsum[kK2Threads / 64];
    uint32_t recs[kTileRecords];         // the tile's symbol records, stream order
};

// Record words (kernels.hpp): table << 24 | symbol << 16 | extra bits.
__device__ __forceinline__ uint32_t rec_word(uint32_t table, uint32_t sym, uint32_t bits) {
    return (table << 24) | (sym << 16) | bits;
}

__global__ __launch_bounds__(kK2Threads) void stats_kernel(StatsArgs a) {
    __shared__ K2Lds lds;
    const int tid = threadIdx.x;
    const uint32_t mw = a.g.mw;
    // the entropy partition's tiles (seg_layout), a contiguous run per workgroup
    const uint32_t ntiles = seg_tiles(a.seg);
    const uint32_t t_first = (uint32_t)((uint64_t)blockIdx.x * ntiles / gridDim.x);
    const uint32_t t_last = (uint32_t)((uint64_t)(blockIdx.x + 1) * ntiles / gridDim.x);
    for (int i = tid; i < kHistCopies * kCopyWords; i += kK2Threads) (&lds.acnt[0][0])[i] = 0;
    for (int i = tid; i < 1024; i += kK2Threads) (&lds.key[0][0])[i] = 0xFFFFFFFFu;
    for (int i = tid; i < kHistCopies * kDcCopyWords; i += kK2Threads) (&lds.dcnt[0][0])[i] = 0;
    JPGE_STAMP(0);
    // key bases: Y raster index of the first Y block row of this workgroup's first
    // MCU row, chroma raster index of that MCU row (keys are relative to them)
    const uint32_t bpm = a.g.bpm, yh = a.g.yh, yv = a.g.yv();  // MCU = yh x yv Y blocks + Cb + Cr
    const uint64_t ybw = (uint64_t)mw * yh;                    // Y blocks per block row
    const uint32_t yhs = (uint32_t)__builtin_ctz(yh);          // yh is 1, 2 or 4: k / yh = k >> yhs
    uint64_t fb0 = 0;
    uint32_t fnb = 0;
    if (t_first < t_last) seg_tile(a.seg, t_first, fb0, fnb);
    const uint32_t mrow0 = (uint32_t)(fb0 / bpm) / mw;
    const uint64_t ybase = (uint64_t)mrow0 * yv * ybw;
    const uint64_t cbase = (uint64_t)mrow0 * mw;
    const int lane = tid & 63, wv = tid >> 6;
    const int blk = block_of(wv, lane), part = part_of(wv);
    TileRegs<kK2Threads, kK2Blocks> regs;
    regs.init(tid);
    if (t_first < t_last) regs.load(a.coef, fb0, (int)fnb, tid);

    uint64_t tq = JPGE_NOW();
    for (uint32_t tile = t_first; tile < t_last; ++tile) {
        uint64_t b0;
        uint32_t nbu;
        seg_tile(a.seg, tile, b0, nbu);
        const int nb = (int)nbu;
        lds_barrier();  // previous tile's readers are done with zz / bmask / recs
        regs.stage(nb, lds.zz, lds.bmask, lds.prevdc, tid);
        if (tile + 1 < t_last) {  // (stays in flight across the LDS-only barriers below)
            uint64_t nb0;
            uint32_t nnb;
            seg_tile(a.seg, tile + 1, nb0, nnb);
            regs.load(a.coef, nb0, (int)nnb, tid);
        }
        lds_barrier();
        JPGE_STAMP(1);
        JPGE_ACC(0, tq);
        const bool active = blk < nb;
        const uint64_t g = b0 + blk;
        const int k = (int)(g % bpm);
        const uint64_t m6 = g / bpm;
        const int comp = block_comp(k, bpm);
        uint32_t rel;  // index of this block in its symbol text, relative to the bases
        int tsel;
        if (comp == 0) {
            // raster index of Y slot k of MCU m6 (the Y text is in block raster order)
            const uint32_t mrow = (uint32_t)(m6 / mw), mcol = (uint32_t)(m6 % mw);
            rel = (uint32_t)(((uint64_t)mrow * yv + ((uint32_t)k >> yhs)) * ybw + (uint64_t)mcol * yh +
                             ((uint32_t)k & (yh - 1)) - ybase);
            tsel = 0;
        } else {
            rel = (uint32_t)(m6 - cbase) | (comp == 2 ? 0x80000000u : 0u);  // all Cr after all Cb
            tsel = 1;
        }
        const uint64_t mask = lds.bmask[blk];
        PartView pv;
        pv.load(lds.zz, mask, blk, part, active);
        const bool eob = active && part == 3 && !(mask >> 63);
        // this part's records: DC, its ZRLs (only the first run of a 16-position part
        // can reach 16) and run/size symbols, EOB — then its offset in the tile's stream
        {
            uint32_t n = 0;
            if (active) {
                n = (part == 0 ? 1u : 0u) + (uint32_t)__builtin_popcount(pv.m16) + (eob ? 1u : 0u);
                if (pv.m16) n += (uint32_t)(16 * part + __builtin_ctz(pv.m16) - pv.last - 1) >> 4;
            }
            lds.pcnt[blk * 4 + part] = n;
        }
        lds_barrier();
        uint32_t T;  // the tile's records
        const uint32_t ex = block_scan<kK2Threads / 64, uint32_t, uint32_t, true>(lds.pcnt[tid], lds.wsum, lane, wv, T);
        lds.pcnt[tid] = ex;
        lds_barrier();
        JPGE_ACC(1, tq);
        uint32_t o = lds.pcnt[blk * 4 + part];
        if (active && part == 0) {  // DC symbol (difference to the chain predecessor)
            const int dd = lds.zz[blk * kZzStride] - pred_dc(b0, blk, lds.zz, lds.prevdc, a.seed, a.rst, bpm);
            const int dcat = category(dd);
            atomicAdd(&lds.dcnt[lane & (kHistCopies - 1)][tsel * 16 + dcat], 1u);
            uint32_t* kp = &lds.key[2 * tsel][dcat];
            if (rel < *kp) atomicMin(kp, rel);
            const uint32_t db = (uint32_t)(dd < 0 ? dd + (1 << dcat) - 1 : dd) & ((1u << dcat) - 1);
            lds.recs[o++] = rec_word(2 * tsel, (uint32_t)dcat, db);
        }
        const uint32_t acb = (rel & 0x80000000u) | ((rel & 0x7FFFFFFFu) << 7);  // text index * 128
        uint32_t* cnt = &lds.acnt[lane & (kHistCopies - 1)][tsel * 256];
        uint32_t* key = lds.key[2 * tsel + 1];
        const uint32_t tac = 2 * tsel + 1;
        for_each_ac(pv, part, [&](int p, int run, int v) {
            const int cat = category(v);
            const int sym = ((run & 15) << 4) | cat;
            atomicAdd(&cnt[sym], 1u);
            const uint32_t kk = acb + 2u * p + 1u;
            if (kk < key[sym]) atomicMin(&key[sym], kk);
            if (run >= 16) {
                atomicAdd(&cnt[0xF0], (uint32_t)(run >> 4));
                if (kk - 1u < key[0xF0]) atomicMin(&key[0xF0], kk - 1u);
                for (int r = run; r >= 16; r -= 16) lds.recs[o++] = rec_word(tac, 0xF0, 0);
            }
            lds.recs[o++] = rec_word(tac, (uint32_t)sym, (uint32_t)(v + (v >> 31)) & ((1u << cat) - 1));
        });
        if (eob) {
            atomicAdd(&cnt[0], 1u);
            if (acb + 127u < key[0]) atomicMin(&key[0], acb + 127u);
            lds.recs[o] = rec_word(tac, 0, 0);
        }
        lds_barrier();
        JPGE_ACC(2, tq);
        // the tile's records to HBM, coalesced (16 bytes per lane)
        {
            uint4* dst = reinterpret_cast<uint4*>(a.recs + (uint64_t)tile * kTileRecords);
            const uint4* src = reinterpret_cast<const uint4*>(lds.recs);
            for (uint32_t i = tid; 4 * i < T; i += kK2Threads) dst[i] = src[i];
            if (tid == 0) a.tcount[tile] = T;
        }
        JPGE_ACC(3, tq);
    }
    __syncthreads();
    JPGE_STAMP(2);

    const int rep = blockIdx.x % kHistReplicas;
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

uint32_t stats_grid(const SegLayout& L) {
    const uint32_t tiles = seg_tiles(L);
    return tiles < 512 ? tiles : 512;  // 2 per CU, persistent over contiguous tiles
}

hipError_t launch_stats(const StatsArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(stats_kernel, dim3(stats_grid(a.seg)), dim3(kK2Threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace jpge
