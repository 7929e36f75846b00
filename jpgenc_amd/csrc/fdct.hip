// K1 fdct_kernel (gfx950): RGB8 -> YCbCr -> 4:2:0 (S420_m) -> Arai FDCT (fp64)
// -> quantise -> int16 coefficients (natural order, MCU-interleaved blocks).
//
// One wavefront owns a tile of 4 MCUs (64x16 px) staged in LDS for the column
// pass, the transpose and the row pass; each lane stores one 16-byte row of a
// block straight from registers.  Persistent grid: a wave walks tiles with a
// stride of all waves, prefetching its next tile's RGB run during the transform.
// Reference: Image.cpp:112-147, 198-235, 540-636; Dct.hpp:47-215; Coding.hpp:84-97.
//
// Bit-exactness: every fp64 operation of the reference is reproduced in order with
// no contraction (-ffp-contract=off plus the pragma in device_common.hpp); the
// colour conversion of 8-bit input uses FMA chains only where every partial result
// is exact (all terms are multiples of 2^-27 far inside 53 bits).
#include "constants.hpp"
#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

// ---- colour constants, Image.cpp:131-134 (float literals widened) ----
constexpr double kYr = (double).299f, kYg = (double).587f, kYb = (double).114f;
constexpr double kCbR = (double)-.1687f, kCbG = (double)-.3312f, kCbB = (double).5f;
constexpr double kCrR = (double).5f, kCrG = (double)-.4186f, kCrB = (double)-.0813f;

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
// 2^-52 |r| of the true quotient and |r| <= |d| < 2^15 (q >= 1, 8-bit samples), so
// unless r lies within 2^-30 of a half-integer, rint(r) (ties-to-even, but r is no
// tie) equals the reference's integer; integer boundaries are harmless (a quotient
// on either side of k rounds to k either way).  e = r - rint(r) is exact, so a lane
// near a half-integer is flagged by |e| > 0.5 - 2^-30 and the whole row is redone
// by exact division (rare; one branch per row).
__device__ __forceinline__ int quant_fast(double d, double invq, bool& near_half) {
    const double r = d * invq;
    const double k = __builtin_rint(r);
    near_half |= __builtin_fabs(r - k) > 0.5 - 0x1p-30;
    return (int)k;
}

__device__ __forceinline__ int quant_exact(double d, double q) { return (int)round(d / q); }

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
    for (uint32_t i = blockIdx.x * kK1Threads + tid; i < a.zero_words; i += gridDim.x * kK1Threads) a.zero[i] = 0;
    if (blockIdx.x == 0)  // carried: another frame's tables + headers, host -> device
        for (uint32_t i = tid; i < a.imp_n16; i += kK1Threads) a.imp_dst[i] = a.imp_src[i];
    if (tid < 128) {
        const int c = tid >> 6, e = tid & 63, o = (e >> 3) * kQRow + (e & 7);
        const double q = (double)a.q[tid];  // Image.cpp:611-636 divides by the entry as double
        lds.q[c][o] = q;
        lds.invq[c][o] = 1.0 / q;
    }
    __syncthreads();
    JPGE_STAMP(0);

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
            bool near_half = false;
#pragma unroll
            for (int u = 0; u < 8; ++u) qv[u] = quant_fast(o[u], lds.invq[qb][j * kQRow + u], near_half);
            if (__builtin_amdgcn_ballot_w64(near_half)) {  // wave-uniform: a real branch, not predication
#pragma unroll
                for (int u = 0; u < 8; ++u) qv[u] = quant_exact(o[u], lds.q[qb][j * kQRow + u]);
            }
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
    __syncthreads();
    JPGE_STAMP(7);
}

}  // namespace

uint32_t fdct_grid(const Geometry& g) {
    const uint32_t tiles = ((g.mw + 3) / 4) * g.mh;
    const uint32_t wgs = (tiles + 3) / 4;
    return wgs < 1024 ? wgs : 1024;  // 4 workgroups per CU, persistent
}

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s) {
    const uint32_t grid = fdct_grid(a.g);
    if (a.maxval == 255)
        hipLaunchKernelGGL(fdct_kernel<true>, dim3(grid), dim3(kK1Threads), 0, s, a);
    else
        hipLaunchKernelGGL(fdct_kernel<false>, dim3(grid), dim3(kK1Threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace jpge
