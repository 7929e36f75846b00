// jpge HIP kernels for gfx950 (MI355X, CDNA4, wave64).
//
//   K1 fdct_kernel   RGB8 -> YCbCr -> 4:2:0 (S420_m) -> Arai FDCT (fp64) -> quantise
//                    -> int16 coefficients (natural order, MCU-interleaved blocks).
//                    One wavefront owns a tile of 4 MCUs (64x16 px) staged in LDS for
//                    the column pass, the transpose and the row pass; each lane stores
//                    one 16-byte row of a block straight from registers.
//                    Reference: Image.cpp:112-147, 198-235, 540-636; Dct.hpp:47-215;
//                    Coding.hpp:84-97.
//   K2 stats_kernel  DC difference chain (Image.cpp:638-678) + zig-zag RLE + category
//                    coding (Coding.hpp:148-283) -> the four symbol histograms of
//                    writeJPEG's "texts" (Image.cpp:888-906) with first-occurrence keys;
//                    also the per-block AC non-zero masks for K3.  Thread = block.
//   K3 entropy_kernel Huffman emission (Image.cpp:737-829) in MCU interleave order
//                    (:957-968), 1-fill and 0xFF00 stuffing (BitstreamGeneric.hpp:
//                    213-248) in ONE pass with two decoupled look-back scans (bit
//                    offsets, then stuffed-byte offsets).  Thread = block.
//
// Bit-exactness: every fp64 operation of the reference is reproduced in order with
// no contraction (compiled with -ffp-contract=off plus the pragma below); the colour
// conversion of 8-bit input uses FMA chains only where every partial result is exact
// (all terms are multiples of 2^-27 far inside 53 bits).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "constants.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace jpge {
namespace {

// ---- colour constants, Image.cpp:131-134 (float literals widened) ----
constexpr double kYr = (double).299f, kYg = (double).587f, kYb = (double).114f;
constexpr double kCbR = (double)-.1687f, kCbG = (double)-.3312f, kCbB = (double).5f;
constexpr double kCrR = (double).5f, kCrG = (double)-.4186f, kCrB = (double)-.0813f;

// natural (row-major) index -> zig-zag position (inverse of Coding.hpp:57-81)
__constant__ uint8_t kNatToZz[64] = {
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42,
    3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24, 31, 40, 44, 53,
    10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// Orders LDS traffic between lanes of ONE wavefront (a wave's DS ops execute in
// order; this stops the compiler from moving them across the point).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int category(int v) {  // getCategoryAndCode, Coding.hpp:197-230
    const int av = v < 0 ? -v : v;
    return av ? 32 - __builtin_clz((unsigned)av) : 0;
}

// One 8-point Arai pass, Dct.hpp:62-131 (same op order for both passes).
__device__ __forceinline__ void arai8(const double x[8], double o[8]) {
    double z0 = x[0] + x[7], z1 = x[1] + x[6], z2 = x[2] + x[5], z3 = x[3] + x[4];
    double z4 = -x[4] + x[3], z5 = -x[5] + x[2], z6 = -x[6] + x[1], z7 = -x[7] + x[0];
    double r0 = z0 + z3, r1 = z1 + z2, r2 = z1 - z2, r3 = z0 - z3;
    double r4 = -z4 - z5, r5 = z5 + z6, r6 = z6 + z7, r7 = z7;
    double t0 = r0 + r1, t1 = r0 - r1, t2 = r2 + r3;
    double tmp = (r4 + r6) * kA5;
    t2 = t2 * kA1;
    double t4 = r4 * kA2, t5 = r5 * kA3, t6 = r6 * kA4;
    double u4 = -t4 - tmp, u6 = t6 - tmp;
    double v2 = t2 + r3, v3 = r3 - t2, v5 = t5 + r7, v7 = r7 - t5;
    double w4 = u4 + v7, w5 = v5 + u6, w6 = -u6 + v5, w7 = v7 - u4;
    o[0] = t0 * kS0; o[4] = t1 * kS4; o[2] = v2 * kS2; o[6] = v3 * kS6;
    o[5] = w4 * kS5; o[1] = w5 * kS1; o[7] = w6 * kS7; o[3] = w7 * kS3;
}

// quantize, Coding.hpp:92-94: (int)std::round(d / q) — correctly rounded fp64
// division, then round half away from zero.  Fast path: r = d * (1/q) is within
// ~2 ulp of the true quotient, so round(r) == round(fl(d/q)) unless r lies within
// 2^-30 of a half-integer (|q| >= 1, |d/q| < 2^20 keep that bound far above the
// error); those rare cases take the exact division.  Integer boundaries are
// harmless: a quotient on either side of k rounds to k either way.
__device__ __forceinline__ int quant1(double d, double q, double invq) {
    const double r = d * invq;
    const double a = __builtin_fabs(r);
    const double fl = __builtin_floor(a);
    const double f = a - fl;
    if (__builtin_fabs(f - 0.5) < 0x1p-30 || a >= 0x1p20) return (int)round(d / q);
    const int n = (int)fl + (f > 0.5 ? 1 : 0);
    return r < 0 ? -n : n;
}

// ===========================================================================
// K1 — colour + 4:2:0 + FDCT + quantise
// ===========================================================================
constexpr int kK1Threads = 256;  // 4 waves, one 4-MCU tile each
constexpr int kRgbPitch = 66;    // u32 per staged pixel row: Y column reads conflict-free
constexpr int kTmpBlock = 72;    // doubles per transpose block (rows of 9 doubles)
constexpr int kTmpRow = 9;

struct K1WaveLds {
    uint32_t rgbx[16 * kRgbPitch];  // packed R | G<<8 | B<<16
    double tmp[8 * kTmpBlock];      // pass-1 output, transposed
};
constexpr int kQRow = 9;  // padded q-table rows: lanes reading rows j=0..7 hit distinct banks
struct K1Lds {
    K1WaveLds w[4];
    double q[2][8 * kQRow];     // luma, chroma
    double invq[2][8 * kQRow];  // 1/q (correctly rounded)
};

__device__ __forceinline__ double ycc_exact_y(uint32_t p) {
    const double r = (double)(p & 0xFF), g = (double)((p >> 8) & 0xFF), b = (double)(p >> 16);
    // (0 + ((.299 r + .587 g) + .114 b)) - 128 : every partial result is exact
    return __builtin_fma(kYb, b, __builtin_fma(kYg, g, __builtin_fma(kYr, r, -128.0)));
}

__device__ __forceinline__ double ycc_ref_y(uint32_t p, double scale) {
    const double r = (double)(p & 0xFF) * scale, g = (double)((p >> 8) & 0xFF) * scale,
                 b = (double)(p >> 16) * scale;
    return (0.0 + ((kYr * r + kYg * g) + kYb * b)) - 128;
}

__device__ __forceinline__ double ycc_ref_c(uint32_t p, double scale, double kr, double kg, double kb) {
    const double r = (double)(p & 0xFF) * scale, g = (double)((p >> 8) & 0xFF) * scale,
                 b = (double)(p >> 16) * scale;
    return (128.0 + ((kr * r + kg * g) + kb * b)) - 128;
}

template <bool kExact>
__global__ __launch_bounds__(kK1Threads) void fdct_kernel(FdctArgs a) {
    __shared__ K1Lds lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    K1WaveLds& W = lds.w[wv];
    for (int i = tid; i < 128; i += kK1Threads) {
        const int c = i >> 6, e = i & 63, o = (e >> 3) * kQRow + (e & 7);
        lds.q[c][o] = a.qtab[i];
        lds.invq[c][o] = 1.0 / a.qtab[i];
    }
    __syncthreads();

    const uint32_t mw = a.g.mw;
    const uint32_t tiles_per_row = (mw + 3) / 4;
    const uint32_t ntiles = tiles_per_row * a.g.mh;
    const uint32_t nwaves = gridDim.x * 4;
    const double scale = 255.0 / (double)a.maxval;  // Image.cpp:465
    const bool aligned = (((uintptr_t)a.rgb | a.stride) & 15) == 0;
    const int r16 = lane >> 2, c16 = lane & 3;  // staging: lane -> (pixel row, 16-px chunk)
    const int b8 = lane >> 3, j = lane & 7;     // DCT: lane -> (block of the round, column)

    // 48-byte RGB run of this lane for tile t, if the tile is on the aligned fast path
    auto fast_load = [&](uint32_t t, uint4& v0, uint4& v1, uint4& v2) -> bool {
        const uint32_t mrow = t / tiles_per_row, mcol0 = (t % tiles_per_row) * 4;
        const uint32_t y = mrow * 16 + r16, xs = mcol0 * 16 + c16 * 16;
        if (!(aligned && y < a.g.height && xs + 16 <= a.g.width)) return false;
        const uint4* src = reinterpret_cast<const uint4*>(a.rgb + (uint64_t)y * a.stride + (uint64_t)xs * 3);
        v0 = src[0]; v1 = src[1]; v2 = src[2];
        return true;
    };
    uint32_t t = blockIdx.x * 4 + wv;
    uint4 c0 = {}, c1 = {}, c2 = {};
    bool cfast = t < ntiles && fast_load(t, c0, c1, c2);

    for (; t < ntiles; t += nwaves) {
        const uint32_t mrow = t / tiles_per_row;
        const uint32_t mcol0 = (t % tiles_per_row) * 4;
        const int nvalid = (int)min(4u, mw - mcol0);
        const uint32_t y = mrow * 16 + r16, xs = mcol0 * 16 + c16 * 16;
        // prefetch the next tile of this wave while this one is transformed
        uint4 n0 = {}, n1 = {}, n2 = {};
        const bool nfast = t + nwaves < ntiles && fast_load(t + nwaves, n0, n1, n2);

        // ---- stage 16 px per lane as packed u32 ----
        uint32_t px[16];
        if (cfast) {
            const uint4 v0 = c0, v1 = c1, v2 = c2;
            const uint32_t wd[13] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w, 0u};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int b0 = 3 * i, d = b0 >> 2, sh = 8 * (b0 & 3);
                px[i] = (sh ? __builtin_amdgcn_alignbit(wd[d + 1], wd[d], sh) : wd[d]) & 0xFFFFFFu;
            }
        } else {  // right/bottom edge replication (Image.cpp:498-531) as clamped addressing
            const uint32_t sy = min(y, a.g.height - 1);
            for (int i = 0; i < 16; ++i) {
                const uint32_t sx = min(xs + i, a.g.width - 1);
                const uint8_t* p = a.rgb + (uint64_t)sy * a.stride + (uint64_t)sx * 3;
                px[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
            }
        }
        uint32_t* dst = &W.rgbx[r16 * kRgbPitch + c16 * 16];
#pragma unroll
        for (int i = 0; i < 16; i += 2) *reinterpret_cast<uint2*>(dst + i) = make_uint2(px[i], px[i + 1]);
        wave_lds_sync();

        // ---- rounds: Y blocks 0-7, Y blocks 8-15, then Cb x4 + Cr x4 ----
#pragma unroll 1
        for (int round = 0; round < 3; ++round) {
            double x[8];
            int m, slot, qb;
            if (round < 2) {
                const int yb = round * 8 + b8, sub = yb & 3;
                m = yb >> 2;
                const int col = m * 16 + (sub & 1) * 8 + j, row0 = (sub >> 1) * 8;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t p = W.rgbx[(row0 + i) * kRgbPitch + col];
                    x[i] = kExact ? ycc_exact_y(p) : ycc_ref_y(p, scale);
                }
                slot = sub;
                qb = 0;
            } else {
                const int comp = b8 >> 2;
                m = b8 & 3;
                const double kr = comp ? kCrR : kCbR, kg = comp ? kCrG : kCbG, kb = comp ? kCrB : kCbB;
                const int col = m * 16 + 2 * j;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint2 t0 = *reinterpret_cast<const uint2*>(&W.rgbx[(2 * i) * kRgbPitch + col]);
                    const uint2 t1 = *reinterpret_cast<const uint2*>(&W.rgbx[(2 * i + 1) * kRgbPitch + col]);
                    if (kExact) {
                        // ((a+b)+(c+d))/4 of the exact per-pixel values equals the exact
                        // value of the channel sums
                        const uint32_t s = (t0.x & 0xFF00FFu) + (t0.y & 0xFF00FFu) + (t1.x & 0xFF00FFu) +
                                           (t1.y & 0xFF00FFu);
                        const double sr = (double)(s & 0xFFFF), sb = (double)(s >> 16);
                        const double sg = (double)(((t0.x >> 8) & 0xFF) + ((t0.y >> 8) & 0xFF) +
                                                   ((t1.x >> 8) & 0xFF) + ((t1.y >> 8) & 0xFF));
                        x[i] = __builtin_fma(kb, sb, __builtin_fma(kg, sg, kr * sr)) * 0.25;
                    } else {
                        // subsample(S420_m), Image.cpp:207-224: ((0+a+b) + (0+c+d)) / 4
                        double top = 0.0, bot = 0.0;
                        top += ycc_ref_c(t0.x, scale, kr, kg, kb);
                        top += ycc_ref_c(t0.y, scale, kr, kg, kb);
                        bot += ycc_ref_c(t1.x, scale, kr, kg, kb);
                        bot += ycc_ref_c(t1.y, scale, kr, kg, kb);
                        x[i] = (top + bot) / 4;
                    }
                }
                slot = 4 + comp;
                qb = 1;
            }
            // column pass, written transposed (Dct.hpp:124-131); row pass
            double o[8];
            arai8(x, o);
            double* tb = &W.tmp[b8 * kTmpBlock];
#pragma unroll
            for (int k = 0; k < 8; ++k) tb[j * kTmpRow + k] = o[k];
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = tb[i * kTmpRow + j];
            arai8(x, o);  // o[u] = y(j, u)
            int qv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                qv[u] = quant1(o[u], lds.q[qb][j * kQRow + u], lds.invq[qb][j * kQRow + u]);
            if (m < nvalid) {
                const uint64_t blk = ((uint64_t)mrow * mw + mcol0 + m) * 6 + slot;
                uint4 pk;
                pk.x = (uint32_t)(qv[0] & 0xFFFF) | ((uint32_t)qv[1] << 16);
                pk.y = (uint32_t)(qv[2] & 0xFFFF) | ((uint32_t)qv[3] << 16);
                pk.z = (uint32_t)(qv[4] & 0xFFFF) | ((uint32_t)qv[5] << 16);
                pk.w = (uint32_t)(qv[6] & 0xFFFF) | ((uint32_t)qv[7] << 16);
                *reinterpret_cast<uint4*>(a.coef + blk * 64 + j * 8) = pk;
            }
            wave_lds_sync();
        }
        c0 = n0; c1 = n1; c2 = n2;
        cfast = nfast;
    }
}


// ===========================================================================
// Shared pieces of K2 / K3
// ===========================================================================
constexpr int kZzStride = 72;    // int16 per staged block (144 B: spreads LDS banks)
constexpr int kPartsPerBlock = 4;  // lanes cooperating on one block's non-zero coefficients

// natural-order global blocks -> zig-zag-ordered LDS blocks
template <int kThreads>
__device__ __forceinline__ void stage_blocks_zz(const int16_t* __restrict__ coef, uint64_t b0, int nb, int16_t* zz,
                                                int tid) {
    const uint4* src = reinterpret_cast<const uint4*>(coef + b0 * 64);
    for (int q = tid; q < nb * 8; q += kThreads) {
        const uint4 v = src[q];
        const int blk = q >> 3, row = q & 7;
        int16_t* d = zz + blk * kZzStride;
        const uint8_t* z = &kNatToZz[row * 8];
        d[z[0]] = (int16_t)(v.x & 0xFFFF); d[z[1]] = (int16_t)(v.x >> 16);
        d[z[2]] = (int16_t)(v.y & 0xFFFF); d[z[3]] = (int16_t)(v.y >> 16);
        d[z[4]] = (int16_t)(v.z & 0xFFFF); d[z[5]] = (int16_t)(v.z >> 16);
        d[z[6]] = (int16_t)(v.w & 0xFFFF); d[z[7]] = (int16_t)(v.w >> 16);
    }
}

// DC predecessor of flat block g (Image.cpp:638-678): the Y chain runs in MCU
// order, Cb and Cr each over their own blocks; a chain's first block predicts 0.
__device__ __forceinline__ int64_t dc_pred_index(uint64_t g) {
    const int k = (int)(g % 6);
    if (k >= 1 && k <= 3) return (int64_t)g - 1;
    if (g < 6) return -1;
    return (int64_t)g - (k == 0 ? 3 : 6);
}

// position of the k-th (0-based) set bit of m (k < popcount(m))
__device__ __forceinline__ int kth_set_bit(uint64_t m, int k) {
    uint32_t w = (uint32_t)m;
    int pos = 0, c = __builtin_popcount(w);
    if (k >= c) { k -= c; w = (uint32_t)(m >> 32); pos = 32; }
    c = __builtin_popcount(w & 0xFFFFu);
    if (k >= c) { k -= c; w >>= 16; pos += 16; }
    c = __builtin_popcount(w & 0xFFu);
    if (k >= c) { k -= c; w >>= 8; pos += 8; }
    c = __builtin_popcount(w & 0xFu);
    if (k >= c) { k -= c; w >>= 4; pos += 4; }
    for (; k > 0; --k) w &= w - 1;
    return pos + __builtin_ctz(w);
}

// One lane's share of a block's AC symbols: the non-zero coefficients with rank
// [lo, hi) in zig-zag order.  `last` is the zig-zag position of the non-zero just
// before the first one of this share (0 = the DC position), `m` the mask of the
// positions still to visit, `cnt` how many of them belong to this share.
struct Share {
    uint64_t m;
    int last, cnt;
    __device__ __forceinline__ void init(uint64_t mask, int part) {
        const int n = __builtin_popcountll(mask);
        const int per = (n + kPartsPerBlock - 1) / kPartsPerBlock;
        const int lo = min(n, part * per), hi = min(n, lo + per);
        cnt = hi - lo;
        if (lo == 0) {
            m = mask;
            last = 0;
        } else {
            last = kth_set_bit(mask, lo - 1);
            m = last >= 63 ? 0ull : mask & ~((2ull << last) - 1);
        }
    }
};

// ===========================================================================
// K2 — symbol statistics (4 lanes per block)
// ===========================================================================
constexpr int kK2Blocks = kStatsTile;
constexpr int kK2Threads = kK2Blocks * kPartsPerBlock;
constexpr int kHistCopies = 8;  // LDS copies of the AC counters: caps same-address atomics at 8 lanes

struct K2Lds {
    int16_t zz[kK2Blocks * kZzStride];
    uint32_t acnt[kHistCopies][2][256];  // AC counters (Y-AC, C-AC), per copy
    uint32_t dcnt[2][16];                // DC counters (Y-DC, C-DC)
    uint32_t key[4][256];                // workgroup-relative first-occurrence key (min)
    uint64_t bmask[kK2Blocks];
};

__global__ __launch_bounds__(kK2Threads) void stats_kernel(StatsArgs a) {
    __shared__ K2Lds lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t nblocks = a.g.nblocks(), mw = a.g.mw;
    const uint64_t b0 = (uint64_t)blockIdx.x * kK2Blocks;
    const int nb = (int)min((uint64_t)kK2Blocks, nblocks - b0);
    for (int i = tid; i < kHistCopies * 512; i += kK2Threads) (&lds.acnt[0][0][0])[i] = 0;
    for (int i = tid; i < 1024; i += kK2Threads) (&lds.key[0][0])[i] = 0xFFFFFFFFu;
    if (tid < 32) (&lds.dcnt[0][0])[tid] = 0;
    stage_blocks_zz<kK2Threads>(a.coef, b0, nb, lds.zz, tid);
    __syncthreads();

    // AC masks: lane p tests zig-zag position p; each wave covers 16 blocks
    constexpr int kPerWave = kK2Blocks / (kK2Threads / 64);
    for (int i = 0; i < kPerWave; ++i) {
        const int blk = wv * kPerWave + i;
        if (blk >= nb) break;
        const int v = lds.zz[blk * kZzStride + lane];
        const uint64_t m = __ballot(lane != 0 && v != 0);
        if (lane == 0) {
            lds.bmask[blk] = m;
            a.mask[b0 + blk] = m;
        }
    }
    __syncthreads();

    const int blk = tid / kPartsPerBlock, part = tid % kPartsPerBlock;
    // key bases: Y raster index of the first Y block row of this tile's first MCU
    // row, chroma raster index of that MCU row (keys are relative inside the tile)
    const uint32_t mrow0 = (uint32_t)(b0 / 6) / mw;
    const uint64_t ybase = 2ull * mrow0 * (2ull * mw);
    const uint64_t cbase = (uint64_t)mrow0 * mw;
    if (blk < nb) {
        const uint64_t g = b0 + blk;
        const int k = (int)(g % 6);
        const uint64_t m6 = g / 6;
        const uint32_t mrow = (uint32_t)(m6 / mw), mcol = (uint32_t)(m6 % mw);
        uint32_t rel;  // index of this block in its symbol text, relative to the tile base
        int tsel;
        if (k < 4) {
            rel = (uint32_t)((2ull * mrow + (k >> 1)) * (2ull * mw) + 2ull * mcol + (k & 1) - ybase);
            tsel = 0;
        } else {
            rel = (uint32_t)(m6 - cbase) | (k == 5 ? 0x80000000u : 0u);  // all Cr after all Cb
            tsel = 1;
        }
        const int16_t* zb = &lds.zz[blk * kZzStride];
        const uint64_t mask = lds.bmask[blk];
        if (part == 0) {  // DC symbol (difference to the chain predecessor)
            const int64_t pg = dc_pred_index(g);
            int prev = 0;
            if (pg >= (int64_t)b0) prev = lds.zz[(pg - b0) * kZzStride];
            else if (pg >= 0) prev = a.coef[(uint64_t)pg * 64];
            const int dcat = category(zb[0] - prev);
            atomicAdd(&lds.dcnt[tsel][dcat], 1u);
            uint32_t* kp = &lds.key[2 * tsel][dcat];
            if (rel < *kp) atomicMin(kp, rel);
        }
        const uint32_t acb = (rel & 0x80000000u) | ((rel & 0x7FFFFFFFu) << 7);  // text index * 128
        uint32_t* cnt = lds.acnt[(tid >> 2) & (kHistCopies - 1)][tsel];
        uint32_t* key = lds.key[2 * tsel + 1];
        Share sh;
        sh.init(mask, part);
        for (int i = 0; i < sh.cnt; ++i) {
            const int p = __builtin_ctzll(sh.m);
            sh.m &= sh.m - 1;
            const int run = p - sh.last - 1;
            sh.last = p;
            const int sym = ((run & 15) << 4) | category(zb[p]);
            atomicAdd(&cnt[sym], 1u);
            const uint32_t kk = acb + 2u * p + 1u;
            if (kk < key[sym]) atomicMin(&key[sym], kk);
            if (run >= 16) {
                atomicAdd(&cnt[0xF0], (uint32_t)(run >> 4));
                if (kk - 1u < key[0xF0]) atomicMin(&key[0xF0], kk - 1u);
            }
        }
        if (part == kPartsPerBlock - 1 && !(mask >> 63)) {  // EOB
            atomicAdd(&cnt[0], 1u);
            if (acb + 127u < key[0]) atomicMin(&key[0], acb + 127u);
        }
    }
    __syncthreads();

    const int rep = blockIdx.x % kHistReplicas;
    const uint64_t ncb = a.g.nmcu();
    for (int i = tid; i < 1024; i += kK2Threads) {
        const int t = i >> 8, s = i & 255;
        const bool ac = t & 1;
        uint32_t c = 0;
        if (ac) {
            for (int cp = 0; cp < kHistCopies; ++cp) c += lds.acnt[cp][t >> 1][s];
        } else if (s < 16) {
            c = lds.dcnt[t >> 1][s];
        }
        if (!c) continue;
        atomicAdd(&a.hist.cnt[(rep * 4 + t) * 256 + s], c);
        const uint32_t k32 = lds.key[t][s];
        uint64_t base;
        if (t < 2) base = ybase;
        else base = (k32 & 0x80000000u) ? ncb + cbase : cbase;
        const uint64_t gkey = (ac ? base * 128ull : base) + (k32 & 0x7FFFFFFFu);
        const unsigned long long inv = ~gkey;
        unsigned long long* gk = reinterpret_cast<unsigned long long*>(&a.hist.key[t * 256 + s]);
        if (inv > *gk) atomicMax(gk, inv);
    }
}

// ===========================================================================
// K3 — entropy coding with two decoupled look-back scans (4 lanes per block)
// ===========================================================================
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// Decoupled look-back run by one whole wave: each pass inspects 64 predecessors.
// Records are self-contained 8-byte {flag, value} granules (one relaxed agent-scope
// store each), so no payload fence is needed.  Returns the exclusive prefix.
__device__ uint64_t lookback_wave(uint64_t* rec, uint32_t tile, uint64_t agg, uint64_t* err, int lane) {
    if (tile == 0) {
        if (lane == 0) st_relaxed(&rec[0], kFlagIncl | agg);
        return 0;
    }
    if (lane == 0) st_relaxed(&rec[tile], kFlagAgg | agg);
    uint64_t excl = 0;
    int64_t end = tile;
    uint32_t spins = 0;
    for (;;) {
        const int64_t idx = end - 1 - lane;
        const uint64_t r = idx >= 0 ? ld_relaxed(&rec[idx]) : kFlagIncl;
        const uint64_t f = r & ~kValMask;
        const uint64_t incl = __ballot(f == kFlagIncl);
        const uint64_t notready = __ballot(f == 0);
        const int first = incl ? __builtin_ctzll(incl) : 64;
        const uint64_t upto = first >= 63 ? ~0ull : ((2ull << first) - 1);
        if (notready & upto) {
            if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(err), 1ull);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += wave_sum64(lane <= first ? (r & kValMask) : 0ull);
        if (first < 64) break;
        end -= 64;
    }
    if (lane == 0) st_relaxed(&rec[tile], kFlagIncl | (excl + agg));
    return excl;
}

// MSB-first bit sink over big-endian 32-bit words (LDS, or the global fallback
// slot); a lane's first and last words may be shared with its neighbours, so
// every word is OR-ed in.
template <typename W>
struct BitSink {
    W* st;
    uint32_t word;
    int fill;      // bits placed in the current word (leading bits belong to others)
    uint64_t acc;  // right-aligned pending bits of the current word
    __device__ __forceinline__ void init(W* s, uint32_t pos) {
        st = s; word = pos >> 5; fill = (int)(pos & 31); acc = 0;
    }
    __device__ __forceinline__ void put(uint32_t v, int n) {  // n <= 32
        acc = (acc << n) | v;
        fill += n;
        if (fill >= 32) {
            fill -= 32;
            atomicOr(&st[word++], (uint32_t)(acc >> fill));
            acc &= (1ull << fill) - 1;
        }
    }
    __device__ __forceinline__ void flush() {
        if (fill > 0) atomicOr(&st[word], (uint32_t)(acc << (32 - fill)));
    }
};

template <typename W>
__device__ __forceinline__ uint32_t stage_byte(const W* st, uint32_t i) {
    return (st[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
}

constexpr int kK3Threads = kEntropyTile * kPartsPerBlock;
constexpr int kK3Waves = kK3Threads / 64;
constexpr int kStageCapBytes = kEntropyTile * 96;  // typical tiles; larger ones use the global slot
constexpr int kOutLdsBytes = kEntropyTile * kZzStride * 2;

struct EntropyShare {
    const int16_t* zb;
    const uint32_t* tdc;
    const uint32_t* tac;
    uint64_t mask;
    int part, dcdiff;
    bool active;
};

// Bits of this lane's share (DC for part 0, its non-zero run/size symbols, EOB
// for the last part), computed (pass 1) or emitted (pass 2) in stream order.
template <bool kEmit, typename W>
__device__ __forceinline__ uint32_t share_bits(const EntropyShare& e, BitSink<W>* bs) {
    if (!e.active) return 0;
    uint32_t nbits = 0;
    if (e.part == 0) {
        const int dcat = category(e.dcdiff);
        const uint32_t ent = e.tdc[dcat];
        nbits += (ent >> 16) + dcat;
        if (kEmit) {
            const uint32_t db = (uint32_t)(e.dcdiff < 0 ? e.dcdiff + (1 << dcat) - 1 : e.dcdiff) & ((1u << dcat) - 1);
            bs->put(((ent & 0xFFFF) << dcat) | db, (int)(ent >> 16) + dcat);
        }
    }
    const uint32_t zrl = e.tac[0xF0];
    Share sh;
    sh.init(e.mask, e.part);
    for (int i = 0; i < sh.cnt; ++i) {
        const int p = __builtin_ctzll(sh.m);
        sh.m &= sh.m - 1;
        int run = p - sh.last - 1;
        sh.last = p;
        const int v = e.zb[p];
        const int cat = category(v);
        if (kEmit) {
            while (run >= 16) { bs->put(zrl & 0xFFFF, (int)(zrl >> 16)); run -= 16; }
            const uint32_t ent = e.tac[(run << 4) | cat];
            const uint32_t vb = (uint32_t)(v < 0 ? v + (1 << cat) - 1 : v) & ((1u << cat) - 1);
            bs->put(((ent & 0xFFFF) << cat) | vb, (int)(ent >> 16) + cat);
        } else {
            nbits += (uint32_t)(run >> 4) * (zrl >> 16) + (e.tac[((run & 15) << 4) | cat] >> 16) + cat;
        }
    }
    if (e.part == kPartsPerBlock - 1 && !(e.mask >> 63)) {  // EOB
        const uint32_t ent = e.tac[0];
        nbits += ent >> 16;
        if (kEmit) bs->put(ent & 0xFFFF, (int)(ent >> 16));
    }
    return nbits;
}

// block-wide exclusive scan of one u32 per thread (thread order)
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* wsum, int lane, int wv, uint32_t& total) {
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    __syncthreads();
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < kK3Waves; ++w) {
        const uint32_t s = wsum[w];
        if (w < wv) base += s;
        total += s;
    }
    return base + incl - v;
}

template <typename W>
__device__ __forceinline__ void entropy_tail(const EntropyArgs& a, W* stage, int16_t* zz, uint32_t* wsum,
                                             uint64_t* s_ffprefix, const EntropyShare& es, uint32_t tile,
                                             bool last_tile, uint64_t P, uint32_t excl_bits, uint32_t total,
                                             int tid, int lane, int wv) {
    const uint32_t lead = (uint32_t)(P & 7);
    const uint32_t endbit = lead + total;
    const uint32_t nwords = (endbit + 31) / 32 + 1;
    for (uint32_t i = tid; i < nwords; i += kK3Threads) stage[i] = 0;
    __syncthreads();

    // ---- pass 2: emit (doHuffmanEncoding + MCU concatenation, Image.cpp:737-968) ----
    {
        BitSink<W> bs;
        bs.init(stage, lead + excl_bits);
        share_bits<true>(es, &bs);
        if (es.active) bs.flush();
    }
    __syncthreads();

    // ---- boundary byte: publish own tail, merge the predecessor's; 1-fill at the end ----
    if (tid == 0) {
        if (!last_tile) {
            const uint32_t tb = (endbit & 7) ? stage_byte(stage, endbit >> 3) : 0u;
            __hip_atomic_store(&a.tails[tile], 0x80000000u | ((endbit & 7) << 8) | tb, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else if (endbit & 7) {  // Bitstream::fill(), BitstreamGeneric.hpp:243-248
            const uint32_t bi = endbit >> 3;
            stage[bi >> 2] |= (0xFFu >> (endbit & 7)) << (24 - 8 * (bi & 3));
        }
        if (lead && tile > 0) {
            uint32_t t = 0, spins = 0;
            while (!((t = __hip_atomic_load(&a.tails[tile - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 31)) {
                if (++spins > kSpinLimit) {
                    atomicOr(reinterpret_cast<unsigned long long*>(a.result + 1), 2ull);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            stage[0] |= (t & 0xFF) << 24;
        }
    }
    __syncthreads();

    // ---- 0xFF count over the bytes this tile owns (byte owner = tile of its last bit) ----
    const uint32_t nown = (endbit >> 3) + ((last_tile && (endbit & 7)) ? 1u : 0u);
    const uint32_t per = (nown + kK3Threads - 1) / kK3Threads;
    const uint32_t lo = min(nown, (uint32_t)tid * per), hi = min(nown, lo + per);
    uint32_t nff = 0;
    for (uint32_t i = lo; i < hi; ++i) nff += stage_byte(stage, i) == 0xFF;
    uint32_t ftotal;
    const uint32_t ff_before = block_scan(nff, wsum, lane, wv, ftotal);

    // ---- look-back 2: stuffed-byte offset ----
    if (wv == 0) {
        const uint64_t pre = lookback_wave(a.lb_ff, tile, ftotal, a.result + 1, lane);
        if (lane == 0) *s_ffprefix = pre;
    }
    __syncthreads();
    const uint64_t D0 = a.hdr_len + (P >> 3) + *s_ffprefix;  // first output byte of this tile
    const uint32_t ntot = nown + ftotal + (last_tile ? 2u : 0u);
    if (D0 + ntot > a.out_cap) {
        if (tid == 0) atomicOr(reinterpret_cast<unsigned long long*>(a.result + 1), 4ull);
        return;
    }
    const uint32_t align = (uint32_t)(D0 & 3);
    if (align + ntot <= (uint32_t)kOutLdsBytes) {
        // stuff into LDS (reusing the coefficient buffer), then aligned 4-byte stores
        uint8_t* ob = reinterpret_cast<uint8_t*>(zz);
        uint32_t o = align + lo + ff_before;
        for (uint32_t i = lo; i < hi; ++i) {
            const uint8_t b = (uint8_t)stage_byte(stage, i);
            ob[o++] = b;
            if (b == 0xFF) ob[o++] = 0;
        }
        if (last_tile && tid == 0) {
            ob[align + nown + ftotal] = 0xFF;
            ob[align + nown + ftotal + 1] = 0xD9;
        }
        __syncthreads();
        uint8_t* gout = a.out + (D0 - align);
        const uint32_t nw = (align + ntot + 3) / 4;
        for (uint32_t w = tid; w < nw; w += kK3Threads) {
            const uint32_t s = 4 * w, e = s + 4;
            if (s >= align && e <= align + ntot) {
                *reinterpret_cast<uint32_t*>(gout + s) = *reinterpret_cast<const uint32_t*>(ob + s);
            } else {
                for (uint32_t q = max(s, align); q < min(e, align + ntot); ++q) gout[q] = ob[q];
            }
        }
    } else {
        uint64_t o = D0 + lo + ff_before;
        for (uint32_t i = lo; i < hi; ++i) {
            const uint8_t b = (uint8_t)stage_byte(stage, i);
            a.out[o++] = b;
            if (b == 0xFF) a.out[o++] = 0;
        }
        if (last_tile && tid == 0) {
            a.out[D0 + nown + ftotal] = 0xFF;
            a.out[D0 + nown + ftotal + 1] = 0xD9;
        }
    }
    if (last_tile && tid == 0) a.result[0] = D0 + ntot;
}

__global__ __launch_bounds__(kK3Threads) void entropy_kernel(EntropyArgs a) {
    __shared__ int16_t zz[kEntropyTile * kZzStride];  // reused as the stuffed-output buffer
    __shared__ uint32_t stage[kStageCapBytes / 4 + 2];
    __shared__ uint32_t tab[4 * 256];
    __shared__ uint32_t wsum[kK3Waves];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_prefix, s_ffprefix;

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(a.ticket, 1u);
    for (int i = tid; i < 1024; i += kK3Threads) tab[i] = a.tables[i];
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t nblocks = a.g.nblocks();
    const uint32_t ntiles = (nblocks + kEntropyTile - 1) / kEntropyTile;
    const bool last_tile = tile == ntiles - 1;
    const uint64_t b0 = (uint64_t)tile * kEntropyTile;
    const int nb = (int)min((uint64_t)kEntropyTile, nblocks - b0);
    stage_blocks_zz<kK3Threads>(a.coef, b0, nb, zz, tid);
    __syncthreads();

    const int blk = tid / kPartsPerBlock;
    EntropyShare es;
    es.part = tid % kPartsPerBlock;
    es.active = blk < nb;
    es.zb = &zz[blk * kZzStride];
    const uint64_t g = b0 + blk;
    const int k = (int)(g % 6);
    es.tdc = &tab[(k < 4 ? 0 : 2) * 256];
    es.tac = &tab[(k < 4 ? 1 : 3) * 256];
    es.mask = 0;
    es.dcdiff = 0;
    if (es.active) {
        es.mask = a.mask[g];
        if (es.part == 0) {
            const int64_t pg = dc_pred_index(g);
            int prev = 0;
            if (pg >= (int64_t)b0) prev = zz[(pg - b0) * kZzStride];
            else if (pg >= 0) prev = a.coef[(uint64_t)pg * 64];
            es.dcdiff = es.zb[0] - prev;
        }
    }

    // ---- pass 1: bit length of this lane's share, tile-local scan ----
    const uint32_t nbits = share_bits<false, uint32_t>(es, nullptr);
    uint32_t total;
    const uint32_t excl_bits = block_scan(nbits, wsum, lane, wv, total);

    // ---- look-back 1: global bit offset of this tile ----
    if (wv == 0) {
        const uint64_t pre = lookback_wave(a.lb_bits, tile, total, a.result + 1, lane);
        if (lane == 0) s_prefix = pre;
    }
    __syncthreads();
    const uint64_t P = s_prefix;
    const uint32_t need = ((uint32_t)(P & 7) + total + 31) / 32 * 4 + 8;
    if (need <= min(a.stage_cap, (uint32_t)kStageCapBytes)) {
        entropy_tail(a, stage, zz, wsum, &s_ffprefix, es, tile, last_tile, P, excl_bits, total, tid, lane, wv);
    } else {
        uint32_t* slot = a.scratch + (uint64_t)tile * kScratchWordsPerTile;
        entropy_tail(a, slot, zz, wsum, &s_ffprefix, es, tile, last_tile, P, excl_bits, total, tid, lane, wv);
    }
}

}  // namespace

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s) {
    const uint32_t tiles = ((a.g.mw + 3) / 4) * a.g.mh;
    const uint32_t wgs = (tiles + 3) / 4;
    const uint32_t grid = wgs < 1024 ? wgs : 1024;  // 4 workgroups per CU, persistent
    if (a.maxval == 255)
        hipLaunchKernelGGL(fdct_kernel<true>, dim3(grid), dim3(kK1Threads), 0, s, a);
    else
        hipLaunchKernelGGL(fdct_kernel<false>, dim3(grid), dim3(kK1Threads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_stats(const StatsArgs& a, hipStream_t s) {
    const uint32_t grid = (a.g.nblocks() + kK2Blocks - 1) / kK2Blocks;
    hipLaunchKernelGGL(stats_kernel, dim3(grid), dim3(kK2Threads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_entropy(const EntropyArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(entropy_kernel, dim3(entropy_tiles(a.g)), dim3(kK3Threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace jpge
