// jpge HIP kernels for gfx950 (MI355X, CDNA4, wave64).
//
//   K1 fdct_kernel     RGB8 -> YCbCr -> 4:2:0 (S420_m) -> Arai FDCT (fp64) ->
//                      quantise -> int16 zig-zag coefficients, AC non-zero masks,
//                      DC values, and the Y-AC / C-AC symbol histograms with
//                      first-occurrence keys.  One wavefront owns a tile of 4 MCUs
//                      (64x16 px); the tile is staged in LDS for the column and
//                      row passes.  Reference: Image.cpp:112-147, 198-235,
//                      540-636, Dct.hpp:47-215, Coding.hpp:84-97.
//   K2 dc_stats_kernel DC difference chain (Y in MCU order, Cb/Cr in block
//                      order, Image.cpp:638-678) -> Y-DC / C-DC histograms.
//   K3 entropy_kernel  DC diff + zig-zag RLE + category coding (Coding.hpp:
//                      148-283) + Huffman emission (Image.cpp:737-829) + MCU
//                      interleave (:957-968) + 1-fill + 0xFF00 stuffing
//                      (BitstreamGeneric.hpp:213-248), as ONE kernel with two
//                      decoupled look-back scans (bit offsets, then stuffed-byte
//                      offsets).  One thread owns one 8x8 block.
//
// Bit-exactness: every fp64 operation of the reference is reproduced in order
// with no contraction (this file is compiled with -ffp-contract=off and the
// pragma below); colour conversion of 8-bit input uses FMA chains only where the
// result is provably exact (all terms are multiples of 2^-27 well inside 53 bits).
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

__constant__ uint8_t kNaturalToZigzag[64] = {
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42,
    3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24, 31, 40, 44, 53,
    10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// Orders LDS traffic between lanes of ONE wavefront (DS ops of a wave execute
// in order; this only stops the compiler from moving them).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
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
// division, then round half away from zero.
__device__ __forceinline__ int quant1(double d, double q) { return (int)round(d / q); }

// ---------------------------------------------------------------------------
// K1
// ---------------------------------------------------------------------------
constexpr int kK1Threads = 256;             // 4 waves, one tile (4 MCUs) each
constexpr int kRgbPitch = 66;               // u32 per staged pixel row (bank spread)
constexpr int kTmpBlock = 72;               // doubles per transposition block (9-double rows)
constexpr int kTmpRow = 9;

struct K1WaveLds {
    uint32_t rgbx[16 * kRgbPitch];          // packed R | G<<8 | B<<16
    double tmp[8 * kTmpBlock];              // pass-1 output, transposed
    int16_t zz[24 * 64];                    // quantised, zig-zag, MCU-interleaved
};
struct K1Lds {
    K1WaveLds w[4];
    double q[128];
    uint32_t hcnt[2][256];                  // Y-AC, C-AC
    unsigned long long hkey[2][256];        // ~first key (max == earliest)
};

__device__ __forceinline__ void ycc_exact_y(uint32_t p, double& y) {
    const double r = (double)(p & 0xFF), g = (double)((p >> 8) & 0xFF), b = (double)(p >> 16);
    // (0 + ((.299 r + .587 g) + .114 b)) - 128 ; every partial result is exact.
    y = __builtin_fma(kYb, b, __builtin_fma(kYg, g, __builtin_fma(kYr, r, -128.0)));
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
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = tid >> 6;
    K1WaveLds& W = lds.w[wv];

    for (int i = tid; i < 128; i += kK1Threads) lds.q[i] = a.qtab[i];
    for (int i = tid; i < 512; i += kK1Threads) {
        (&lds.hcnt[0][0])[i] = 0;
        (&lds.hkey[0][0])[i] = 0;
    }
    __syncthreads();

    const uint32_t mw = a.g.mw, mh = a.g.mh;
    const uint32_t tiles_per_row = (mw + 3) / 4;
    const uint32_t ntiles = tiles_per_row * mh;
    const uint32_t nwaves = gridDim.x * 4;
    const double scale = 255.0 / (double)a.maxval;  // Image.cpp:465

    for (uint32_t t = blockIdx.x * 4 + wv; t < ntiles; t += nwaves) {
        const uint32_t mrow = t / tiles_per_row;
        const uint32_t mcol0 = (t % tiles_per_row) * 4;
        const int nvalid = (int)min(4u, mw - mcol0);
        const uint32_t x0 = mcol0 * 16, y0 = mrow * 16;

        // ---- stage RGB: lane -> (row lane/4, 16 px chunk lane%4) ----
        {
            const int r = lane >> 2, c = lane & 3;
            const uint32_t y = y0 + r, xs = x0 + c * 16;
            uint32_t px[16];
            const bool fast = (y < a.g.height) && (xs + 16 <= a.g.width) &&
                              (((uintptr_t)a.rgb | a.stride) & 15) == 0;
            if (fast) {
                const uint4* src = reinterpret_cast<const uint4*>(a.rgb + (uint64_t)y * a.stride + (uint64_t)xs * 3);
                uint4 v0 = src[0], v1 = src[1], v2 = src[2];
                uint32_t wd[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    // bytes 3i..3i+2 of the 48-byte run
                    const int b0 = 3 * i;
                    const uint64_t pair = ((uint64_t)wd[(b0 >> 2) + ((b0 >> 2) < 11 ? 1 : 0)] << 32) | wd[b0 >> 2];
                    px[i] = (uint32_t)(pair >> (8 * (b0 & 3))) & 0xFFFFFFu;
                }
            } else {
                // edge replication (Image.cpp:498-531) as clamped addressing
                const uint32_t sy = min(y, a.g.height - 1);
                for (int i = 0; i < 16; ++i) {
                    const uint32_t sx = min(xs + i, a.g.width - 1);
                    const uint8_t* p = a.rgb + (uint64_t)sy * a.stride + (uint64_t)sx * 3;
                    px[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
                }
            }
            uint32_t* dst = &W.rgbx[r * kRgbPitch + c * 16];
#pragma unroll
            for (int i = 0; i < 16; i += 2)
                *reinterpret_cast<uint2*>(dst + i) = make_uint2(px[i], px[i + 1]);
        }
        wave_lds_sync();

        // ---- three rounds of 8 blocks x 8 columns: Y, Y, then Cb/Cr ----
        const int b8 = lane >> 3, j = lane & 7;
#pragma unroll 1
        for (int round = 0; round < 3; ++round) {
            double x[8];
            int slot, qbase;
            if (round < 2) {
                const int yb = round * 8 + b8, m = yb >> 2, sub = yb & 3;
                const int col = m * 16 + (sub & 1) * 8 + j, row0 = (sub >> 1) * 8;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t p = W.rgbx[(row0 + i) * kRgbPitch + col];
                    if (kExact) ycc_exact_y(p, x[i]);
                    else x[i] = ycc_ref_y(p, scale);
                }
                slot = m * 6 + sub;
                qbase = 0;
            } else {
                const int comp = b8 >> 2, m = b8 & 3;
                const double kr = comp ? kCrR : kCbR, kg = comp ? kCrG : kCbG, kb = comp ? kCrB : kCbB;
                const int col = m * 16 + 2 * j;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint2 t0 = *reinterpret_cast<const uint2*>(&W.rgbx[(2 * i) * kRgbPitch + col]);
                    const uint2 t1 = *reinterpret_cast<const uint2*>(&W.rgbx[(2 * i + 1) * kRgbPitch + col]);
                    if (kExact) {
                        // ((a+b)+(c+d))/4 of exact per-pixel values == exact value of
                        // the channel sums; every partial is exact.
                        const uint32_t s = (t0.x & 0xFF00FFu) + (t0.y & 0xFF00FFu) + (t1.x & 0xFF00FFu) + (t1.y & 0xFF00FFu);
                        const double sr = (double)(s & 0xFFFF), sb = (double)(s >> 16);
                        const double sg = (double)(((t0.x >> 8) & 0xFF) + ((t0.y >> 8) & 0xFF) +
                                                   ((t1.x >> 8) & 0xFF) + ((t1.y >> 8) & 0xFF));
                        x[i] = __builtin_fma(kb, sb, __builtin_fma(kg, sg, kr * sr)) * 0.25;
                    } else {
                        // subsample(S420_m), Image.cpp:207-224: ((a + b) + (c + d)) / 4
                        const double va = ycc_ref_c(t0.x, scale, kr, kg, kb);
                        const double vb = ycc_ref_c(t0.y, scale, kr, kg, kb);
                        const double vc = ycc_ref_c(t1.x, scale, kr, kg, kb);
                        const double vd = ycc_ref_c(t1.y, scale, kr, kg, kb);
                        double top = 0.0;
                        top += va;
                        top += vb;
                        double bot = 0.0;
                        bot += vc;
                        bot += vd;
                        x[i] = (top + bot) / 4;
                    }
                }
                slot = m * 6 + 4 + comp;
                qbase = 64;
            }
            // pass 1 over the column, result written transposed (Dct.hpp:124-131)
            double o[8];
            arai8(x, o);
            double* tb = &W.tmp[b8 * kTmpBlock];
#pragma unroll
            for (int k = 0; k < 8; ++k) tb[j * kTmpRow + k] = o[k];
            wave_lds_sync();
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = tb[i * kTmpRow + j];
            arai8(x, o);  // o[u] = y(j, u)
            int16_t* zb = &W.zz[slot * 64];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                zb[kNaturalToZigzag[j * 8 + u]] = (int16_t)quant1(o[u], lds.q[qbase + j * 8 + u]);
            wave_lds_sync();
        }

        // ---- per-block AC masks and DC values (lane p = zig-zag position) ----
        const int nblk = nvalid * 6;
        uint64_t my_mask = 0;
        int my_dc = 0;
        for (int b = 0; b < nblk; ++b) {
            const int v = W.zz[b * 64 + lane];
            const uint64_t m = __ballot(lane != 0 && v != 0);
            const int d = __shfl(v, 0);
            if (lane == b) { my_mask = m; my_dc = d; }
        }

        // ---- AC symbol histogram (RLE_AC + encode_category, Coding.hpp:148-283) ----
        if (a.do_hist && lane < nblk) {
            const int m = lane / 6, k = lane % 6;
            const int tsel = k < 4 ? 0 : 1;
            uint64_t ridx;  // block index in the reference's symbol text order (Image.cpp:892-906)
            if (k < 4) {
                const uint64_t by = 2ull * mrow + (k >> 1), bx = 2ull * (mcol0 + m) + (k & 1);
                ridx = by * (2ull * mw) + bx;
            } else {
                ridx = (uint64_t)mrow * mw + mcol0 + m + (k == 5 ? (uint64_t)mw * mh : 0ull);
            }
            const unsigned long long kb = ridx * 128ull;
            uint64_t msk = my_mask;
            int last = 0;
            while (msk) {
                const int p = __builtin_ctzll(msk);
                msk &= msk - 1;
                const int v = W.zz[lane * 64 + p];
                const int run = p - last - 1;
                last = p;
                const int av = v < 0 ? -v : v;
                const int cat = 32 - __builtin_clz((unsigned)av);
                const int sym = ((run & 15) << 4) | cat;
                atomicAdd(&lds.hcnt[tsel][sym], 1u);
                atomicMax(&lds.hkey[tsel][sym], ~(kb + 2ull * p + 1ull));
                if (run >= 16) {
                    atomicAdd(&lds.hcnt[tsel][0xF0], (unsigned)(run >> 4));
                    atomicMax(&lds.hkey[tsel][0xF0], ~(kb + 2ull * p));
                }
            }
            if (last < 63) {
                atomicAdd(&lds.hcnt[tsel][0], 1u);
                atomicMax(&lds.hkey[tsel][0], ~(kb + 127ull));
            }
        }

        // ---- store coefficients / masks / DC (MCU-contiguous) ----
        const uint64_t mcu0 = (uint64_t)mrow * mw + mcol0;
        const uint4* zsrc = reinterpret_cast<const uint4*>(W.zz);
        uint4* zdst = reinterpret_cast<uint4*>(a.coef + mcu0 * 384);
        const int nchunks = nvalid * 48;  // 768 B per MCU
        for (int q = lane; q < nchunks; q += 64) zdst[q] = zsrc[q];
        if (lane < nblk) {
            a.mask[mcu0 * 6 + lane] = my_mask;
            a.dc[mcu0 * 6 + lane] = (int16_t)my_dc;
        }
        wave_lds_sync();
    }

    __syncthreads();
    if (a.do_hist) {
        const int rep = blockIdx.x % kHistReplicas;
        for (int i = tid; i < 512; i += kK1Threads) {
            const int tsel = i >> 8, s = i & 255, gt = tsel ? 3 : 1;
            const uint32_t c = lds.hcnt[tsel][s];
            if (c) {
                atomicAdd(&a.hist.cnt[(rep * 4 + gt) * 256 + s], c);
                const unsigned long long kk = lds.hkey[tsel][s];
                unsigned long long* gk = reinterpret_cast<unsigned long long*>(&a.hist.key[gt * 256 + s]);
                if (kk > *gk) atomicMax(gk, kk);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// K2 — DC difference statistics
// ---------------------------------------------------------------------------
__device__ __forceinline__ int category(int v) {
    const int av = v < 0 ? -v : v;
    return av ? 32 - __builtin_clz((unsigned)av) : 0;
}

__global__ __launch_bounds__(256) void dc_stats_kernel(const int16_t* __restrict__ dc, Geometry g, HistPtrs h) {
    __shared__ uint32_t hc[2][16];
    __shared__ unsigned long long hk[2][16];
    const int tid = threadIdx.x;
    if (tid < 32) { (&hc[0][0])[tid] = 0; (&hk[0][0])[tid] = 0; }
    __syncthreads();
    const uint32_t nmcu = g.nmcu(), mw = g.mw;
    const uint64_t ncb = nmcu;
    for (uint32_t m = blockIdx.x * 256 + tid; m < nmcu; m += gridDim.x * 256) {
        const int16_t* d = dc + (uint64_t)m * 6;
        const int py = m ? dc[(uint64_t)(m - 1) * 6 + 3] : 0;
        const int pcb = m ? dc[(uint64_t)(m - 1) * 6 + 4] : 0;
        const int pcr = m ? dc[(uint64_t)(m - 1) * 6 + 5] : 0;
        const uint32_t mrow = m / mw, mcol = m % mw;
        int prev = py;
        for (int k = 0; k < 4; ++k) {
            const int c = category(d[k] - prev);
            prev = d[k];
            const uint64_t by = 2ull * mrow + (k >> 1), bx = 2ull * mcol + (k & 1);
            const unsigned long long key = by * 2ull * mw + bx;  // Y-DC text: block raster order
            atomicAdd(&hc[0][c], 1u);
            atomicMax(&hk[0][c], ~key);
        }
        const int ccb = category(d[4] - pcb), ccr = category(d[5] - pcr);
        atomicAdd(&hc[1][ccb], 1u);
        atomicMax(&hk[1][ccb], ~(unsigned long long)m);             // Cb blocks first ...
        atomicAdd(&hc[1][ccr], 1u);
        atomicMax(&hk[1][ccr], ~(unsigned long long)(ncb + m));     // ... then Cr blocks
    }
    __syncthreads();
    if (tid < 32) {
        const int tsel = tid >> 4, s = tid & 15, gt = tsel ? 2 : 0;
        const uint32_t c = hc[tsel][s];
        if (c) {
            const int rep = blockIdx.x % kHistReplicas;
            atomicAdd(&h.cnt[(rep * 4 + gt) * 256 + s], c);
            unsigned long long* gk = reinterpret_cast<unsigned long long*>(&h.key[gt * 256 + s]);
            const unsigned long long kk = hk[tsel][s];
            if (kk > *gk) atomicMax(gk, kk);
        }
    }
}

// ---------------------------------------------------------------------------
// K3 — entropy coding with two decoupled look-back scans
// ---------------------------------------------------------------------------
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 24;

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Single-lane decoupled look-back; records are self-contained 8-byte granules
// {flag, value} written by one store, so no payload fence is needed.
__device__ uint64_t lookback(uint64_t* rec, uint32_t tile, uint64_t agg, uint64_t* err) {
    if (tile == 0) { st_relaxed(&rec[0], kFlagIncl | agg); return 0; }
    st_relaxed(&rec[tile], kFlagAgg | agg);
    uint64_t excl = 0;
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    while (j >= 0) {
        const uint64_t r = ld_relaxed(&rec[j]);
        const uint64_t f = r & ~kValMask;
        if (f == 0) {
            if (++spins > kSpinLimit) { atomicOr(reinterpret_cast<unsigned long long*>(err), 1ull); break; }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        excl += r & kValMask;
        if (f == kFlagIncl) break;
        --j;
    }
    st_relaxed(&rec[tile], kFlagIncl | (excl + agg));
    return excl;
}

// MSB-first bit sink over big-endian 32-bit LDS words; the first word of a
// thread's run may be shared with the previous thread, so words are OR-ed.
struct BitSink {
    uint32_t* st;
    uint32_t word;
    int fill;       // bits already placed in the current word (leading bits are others')
    uint64_t acc;   // right-aligned pending bits of the current word
    __device__ __forceinline__ void init(uint32_t* s, uint64_t pos) {
        st = s; word = (uint32_t)(pos >> 5); fill = (int)(pos & 31); acc = 0;
    }
    __device__ __forceinline__ void put(uint32_t v, int n) {  // n <= 32
        if (n == 0) return;
        acc = (acc << n) | v;
        fill += n;
        if (fill >= 32) {
            fill -= 32;
            atomicOr(&st[word++], (uint32_t)(acc >> fill));
            acc &= (fill ? ((1ull << fill) - 1) : 0ull);
        }
    }
    __device__ __forceinline__ void flush() {
        if (fill > 0) atomicOr(&st[word], (uint32_t)(acc << (32 - fill)));
    }
};

__device__ __forceinline__ uint32_t stage_byte(const uint32_t* st, uint32_t i) {
    return (st[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
}

constexpr int kK3Threads = kEntropyTile;
constexpr int kStageWords = kEntropyTile * kStageBytesPerBlock / 4 + 2;

__global__ __launch_bounds__(kK3Threads) void entropy_kernel(EntropyArgs a) {
    __shared__ int16_t coef[kEntropyTile * 64];
    __shared__ uint32_t stage[kStageWords];
    __shared__ uint32_t tab[4 * 256];
    __shared__ uint32_t wsum[kK3Threads / 64];
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

    // coefficients of the tile: contiguous [nb][64] int16 (16-byte chunks)
    {
        const uint4* src = reinterpret_cast<const uint4*>(a.coef + b0 * 64);
        uint4* dst = reinterpret_cast<uint4*>(coef);
        for (int q = tid; q < nb * 8; q += kK3Threads) dst[q] = src[q];
    }
    const bool active = tid < nb;
    const uint64_t g = b0 + tid;
    const int k = (int)(g % 6);
    const uint64_t m = g / 6;
    uint64_t msk = 0;
    int dcdiff = 0;
    if (active) {
        msk = a.mask[g];
        // DC predecessor (Image.cpp:638-678): Y chain in MCU order, Cb/Cr per component.
        const int cur = a.dc[g];
        int prev = 0;
        if (k >= 1 && k <= 3) prev = a.dc[g - 1];
        else if (m > 0) prev = a.dc[g - (k == 0 ? 3 : 6)];
        dcdiff = cur - prev;
    }
    const uint32_t* tdc = &tab[(k < 4 ? 0 : 2) * 256];
    const uint32_t* tac = &tab[(k < 4 ? 1 : 3) * 256];
    __syncthreads();

    // ---- pass 1: bit length of this block ----
    uint32_t nbits = 0;
    const int16_t* cb = &coef[tid * 64];
    if (active) {
        const int dcat = category(dcdiff);
        nbits = (tdc[dcat] >> 16) + dcat;
        uint64_t mm = msk;
        int last = 0;
        const uint32_t zrl = tac[0xF0] >> 16;
        while (mm) {
            const int p = __builtin_ctzll(mm);
            mm &= mm - 1;
            const int run = p - last - 1;
            last = p;
            const int cat = category(cb[p]);
            nbits += (uint32_t)(run >> 4) * zrl + (tac[((run & 15) << 4) | cat] >> 16) + cat;
        }
        if (last < 63) nbits += tac[0] >> 16;
    }

    // ---- tile-local exclusive scan of block lengths ----
    uint32_t incl = nbits;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
    for (int w = 0; w < kK3Threads / 64; ++w) {
        if (w < wv) wbase += wsum[w];
        total += wsum[w];
    }
    const uint32_t excl_bits = wbase + incl - nbits;

    // ---- look-back 1: global bit offset ----
    if (tid == 0) s_prefix = lookback(a.lb_bits, tile, total, a.result + 1);
    __syncthreads();
    const uint64_t P = s_prefix;
    const uint32_t lead = (uint32_t)(P & 7);
    const uint32_t endbit = lead + total;
    const uint32_t nwords = (endbit + 31) / 32 + 1;
    for (uint32_t i = tid; i < nwords; i += kK3Threads) stage[i] = 0;
    __syncthreads();

    // ---- pass 2: emit (doHuffmanEncoding + MCU concatenation) ----
    if (active) {
        BitSink bs;
        bs.init(stage, lead + excl_bits);
        const int dcat = category(dcdiff);
        const uint32_t dce = tdc[dcat];
        const uint32_t dbits = dcdiff < 0 ? (uint32_t)(dcdiff + (1 << dcat) - 1) : (uint32_t)dcdiff;
        bs.put(dce & 0xFFFF, (int)(dce >> 16));
        bs.put(dcat ? (dbits & ((1u << dcat) - 1)) : 0u, dcat);
        uint64_t mm = msk;
        int last = 0;
        const uint32_t zrl = tac[0xF0];
        while (mm) {
            const int p = __builtin_ctzll(mm);
            mm &= mm - 1;
            int run = p - last - 1;
            last = p;
            while (run >= 16) { bs.put(zrl & 0xFFFF, (int)(zrl >> 16)); run -= 16; }
            const int v = cb[p];
            const int cat = category(v);
            const uint32_t e = tac[(run << 4) | cat];
            const uint32_t vb = v < 0 ? (uint32_t)(v + (1 << cat) - 1) : (uint32_t)v;
            bs.put(e & 0xFFFF, (int)(e >> 16));
            bs.put(vb & ((1u << cat) - 1), cat);
        }
        if (last < 63) { const uint32_t e = tac[0]; bs.put(e & 0xFFFF, (int)(e >> 16)); }
        bs.flush();
    }
    __syncthreads();

    // ---- boundary byte: publish own tail, merge predecessor's tail; 1-fill at the end ----
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
                if (++spins > kSpinLimit) { atomicOr(reinterpret_cast<unsigned long long*>(a.result + 1), 2ull); break; }
                __builtin_amdgcn_s_sleep(1);
            }
            stage[0] |= (t & 0xFF) << 24;
        }
    }
    __syncthreads();

    // ---- 0xFF count over the bytes this tile owns ----
    const uint32_t nown = (endbit >> 3) + ((last_tile && (endbit & 7)) ? 1u : 0u);
    const uint32_t per = (nown + kK3Threads - 1) / kK3Threads;
    const uint32_t lo = min(nown, (uint32_t)tid * per), hi = min(nown, lo + per);
    uint32_t nff = 0;
    for (uint32_t i = lo; i < hi; ++i) nff += stage_byte(stage, i) == 0xFF;
    uint32_t fincl = nff;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(fincl, d);
        if (lane >= d) fincl += o;
    }
    __syncthreads();
    if (lane == 63) wsum[wv] = fincl;
    __syncthreads();
    uint32_t fbase = 0, ftotal = 0;
    for (int w = 0; w < kK3Threads / 64; ++w) {
        if (w < wv) fbase += wsum[w];
        ftotal += wsum[w];
    }
    const uint32_t ff_before = fbase + fincl - nff;

    // ---- look-back 2: stuffed-byte offset ----
    if (tid == 0) s_ffprefix = lookback(a.lb_ff, tile, ftotal, a.result + 1);
    __syncthreads();
    const uint64_t Q = s_ffprefix;
    const uint64_t base = a.hdr_len + (P >> 3) + Q;
    const uint64_t end_total = base + nown + ftotal + (last_tile ? 2 : 0);
    if (end_total > a.out_cap) {
        if (tid == 0) atomicOr(reinterpret_cast<unsigned long long*>(a.result + 1), 4ull);
        return;
    }
    uint64_t o = base + lo + ff_before;
    for (uint32_t i = lo; i < hi; ++i) {
        const uint8_t b = (uint8_t)stage_byte(stage, i);
        a.out[o++] = b;
        if (b == 0xFF) a.out[o++] = 0;
    }
    if (last_tile && tid == 0) {
        const uint64_t e = base + nown + ftotal;
        a.out[e] = 0xFF;
        a.out[e + 1] = 0xD9;
        a.result[0] = e + 2;
    }
}

}  // namespace

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s) {
    const uint32_t tiles = ((a.g.mw + 3) / 4) * a.g.mh;
    const uint32_t wgs_needed = (tiles + 3) / 4;
    const uint32_t grid = wgs_needed < 1024 ? wgs_needed : 1024;
    if (a.maxval == 255)
        hipLaunchKernelGGL(fdct_kernel<true>, dim3(grid), dim3(kK1Threads), 0, s, a);
    else
        hipLaunchKernelGGL(fdct_kernel<false>, dim3(grid), dim3(kK1Threads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_dc_stats(const int16_t* dc, const Geometry& g, HistPtrs h, hipStream_t s) {
    uint32_t grid = (g.nmcu() + 255) / 256;
    if (grid > 512) grid = 512;
    hipLaunchKernelGGL(dc_stats_kernel, dim3(grid), dim3(256), 0, s, dc, g, h);
    return hipGetLastError();
}

hipError_t launch_entropy(const EntropyArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(entropy_kernel, dim3(entropy_tiles(a.g)), dim3(kK3Threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace jpge
