// K1 fdct_kernel (gfx950): RGB8 -> YCbCr -> 4:2:0 (S420_m) -> Arai FDCT (fp64)
// -> quantise -> int16 coefficients (natural order, MCU-interleaved blocks).
//
// One wavefront owns a tile of 4 MCUs (64x16 px) staged in LDS for the column
// pass, the transpose and the row pass; each lane stores one 16-byte row of a
// block straight from registers.  Persistent workgroups (8 waves, two per CU, alone) own a
// contiguous run of tiles; its waves take tiles from an LDS counter (the SIMD
// favours its oldest wave, so static shares finish unevenly) and prefetch the next
// tile's RGB run during the transform.  Three rounds per tile (chroma, Y MCUs 0-1,
// Y MCUs 2-3), each round's LDS reads issued in one batch during the previous
// round's row pass.  Pixels and coefficients go through buffer descriptors so that
// every tile issues the same loads and stores (no branches around them) and the
// in-order wait for the prefetch never drains a just-issued store; the stores are
// write-through (sc1), so the kernel ends without dirty L2 lines to flush.
// Reference: Image.cpp:112-147, 198-235, 540-636; Dct.hpp:47-215; Coding.hpp:84-97.
//
// Bit-exactness: every fp64 operation of the reference is reproduced in order with
// no contraction (-ffp-contract=off plus the pragma in device_common.hpp); the
// colour conversion of 8-bit input uses FMA chains only where every partial result
// is exact (all terms are multiples of 2^-27 far inside 53 bits).
#include <cstring>

#include "arai.hpp"
#include "device_common.hpp"

namespace jpge {
namespace {
using namespace dev;

// ---- colour constants, Image.cpp:131-134 (float literals widened) ----
constexpr double kYr = (double).299f, kYg = (double).587f, kYb = (double).114f;
constexpr double kCbR = (double)-.1687f, kCbG = (double)-.3312f, kCbB = (double).5f;
constexpr double kCrR = (double).5f, kCrG = (double)-.4186f, kCrB = (double)-.0813f;

// quantize, Coding.hpp:92-94, of the row pass's output o = w * s_u (Dct.hpp:124-131):
// (int)std::round(o / q) — two correctly rounded fp64 operations, then round half
// away from zero.  Fast path in one fp64 instruction per coefficient: the exact
// product x = w * c, c = fl(s_u / q), is within 2^-40 of the reference's quotient
// fl(fl(w s_u) / q) (|x| < 2^11: 8-bit samples, q >= 1), and
// y = fma(w, c, 1.5 * 2^36 + 0x8001 * 2^-16) rounds it once onto the 2^-16 grid (the
// addend lies on the grid, and y stays in [2^36, 2^37)), so the low word of y is
// t = n + 0x8001 with n = round(x * 2^16) (two's complement, mod 2^32):
//   - t >> 16 (its high half) is floor(x + 1/2), the reference's integer unless x
//     lies within 2^-15 of a half-integer — where the reference's quotient could sit
//     on the other side of it;
//   - those are exactly the t whose low half is 0, 1 or 2: one 16-bit min over the
//     row's 8 values finds them, and such a row is redone the reference's way
//     (quant_exact; rare, one wave-uniform branch per row).
// Integer boundaries are harmless (a quotient on either side of k rounds to k).
constexpr double kQuantMagic = 103079215104.50002;  // 1.5 * 2^36 + 0x8001 * 2^-16 (bits 0x4238000000008001)
static_assert(kQuantMagic - 103079215104.0 == 0x8001 * 0x1p-16, "the magic addend is exact");
__device__ __forceinline__ uint32_t quant_fix16(double w, double c) {
    return (uint32_t)__builtin_bit_cast(uint64_t, __builtin_fma(w, c, kQuantMagic));
}

__device__ __forceinline__ int quant_exact(double w, double s, double q) { return (int)round((w * s) / q); }

// One row of 8 quantised coefficients as int16 x 8 (natural order): the fast path,
// or the reference's two divisions when any lane of the wave has a near-half row.
// qrow: this lane's 8 quantisers (LDS).
__device__ __forceinline__ u32x4 quant_row(const double o[8], const double c[8], const double* qrow) {
    uint32_t t[8];
    uint16_t m = 0xFFFF;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        t[u] = quant_fix16(o[u], c[u]);
        m = __builtin_elementwise_min(m, (uint16_t)t[u]);  // v_min_u16 on the low half
    }
    if (__builtin_amdgcn_ballot_w64(m <= 2)) {  // wave-uniform: a real branch, not predication
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = (uint32_t)quant_exact(o[u], kS[u], qrow[u]) << 16;
    }
    u32x4 pk;  // the high halves, two per word
    pk.x = __builtin_amdgcn_perm(t[1], t[0], 0x07060302u);
    pk.y = __builtin_amdgcn_perm(t[3], t[2], 0x07060302u);
    pk.z = __builtin_amdgcn_perm(t[5], t[4], 0x07060302u);
    pk.w = __builtin_amdgcn_perm(t[7], t[6], 0x07060302u);
    return pk;
}

constexpr uint32_t kOob = 0xFFFFFF00u;  // buffer offset past every descriptor's range
constexpr int kK1StoreAux = 16;  // sc1: write-through coefficient stores (no dirty L2 lines at the kernel's end)
constexpr uint32_t kK1SharedCap = 512;  // shared-shape workgroups per launch, at most (2 per CU: measured
                                        // +1.5% in the pipeline over 1024, which filled every CU)

// Workgroup shapes: whole-CU, one 16-wave workgroup per CU (4 waves per SIMD), whose
// waves balance their tiles among themselves — for large frames with the GPU to
// itself (two 8-wave workgroups per CU: equal at 4K, 4% slower at 16384^2); 4 waves,
// four per CU alone (smaller frames, launch_fdct) or at most two per CU beside other
// lanes' kernels (a whole-CU workgroup waits for a whole CU to drain).
constexpr int kK1WavesSolo = 16;
constexpr int kK1WavesShared = 4;  // (pipeline: 8 waves x 256 -1.4%, 8 x 512 -3.3%, 2 x 1024 -2.3%)
constexpr int kRgbPitch = 66;    // u32 per staged pixel row: Y column reads conflict-free
constexpr int kTmpBlock = 72;    // doubles per transpose block (rows of 9 doubles)
constexpr int kTmpRow = 9;

struct K1WaveLds {
    uint32_t rgbx[16 * kRgbPitch];  // packed R | G<<8 | B<<16
    double tmp[8 * kTmpBlock];      // pass-1 output, transposed
};
constexpr int kQRow = 9;  // padded q-table rows: lanes reading rows j=0..7 hit distinct banks

template <int kWaves>
struct K1Lds {
    K1WaveLds w[kWaves];
    uint32_t next;  // next tile of the workgroup's run to hand out
    double q[2][8 * kQRow];     // luma, chroma
    double invq[2][8 * kQRow];  // s_u / q (correctly rounded), u = column
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

// exact chroma of one 8-bit pixel: (128 + v) - 128 == v, v exact
__device__ __forceinline__ double ycc_exact_c(uint32_t p, double kr, double kg, double kb) {
    const double r = (double)(p & 0xFF), g = (double)((p >> 8) & 0xFF), b = (double)(p >> 16);
    return __builtin_fma(kb, b, __builtin_fma(kg, g, kr * r));
}

// The prologue reads its constants without vector loads: a vector load issued after
// the first tile's pixel loads waits for them (the vector memory counter retires in
// order), which held every workgroup's prologue for the start-up burst (~3.5 us).
// kS[u] as a select over the constants (no load from the constant table):
__device__ __forceinline__ double arai_scale(int u) {
    double r = kS[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) r = u == i ? kS[i] : r;
    return r;
}
// quantiser entry tid (< 128) of the kernel arguments, through scalar loads (the
// array is 16-byte aligned in FdctArgs):
__device__ __forceinline__ uint32_t q_entry(const FdctArgs& a, int tid) {
    const uint32_t* qw = reinterpret_cast<const uint32_t*>(a.q);
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) w = (tid >> 2) == i ? qw[i] : w;
    return (w >> (8 * (tid & 3))) & 0xFF;
}

// v_permlane32_swap on a double pair: lanes 32-63 of a trade places with lanes 0-31
// of b (a keeps its low half, b its high half).
__device__ __forceinline__ void swap_halves(double& a, double& b) {
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
    a = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]);
    b = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);
}

template <bool kExact, int kWaves, int kFilt, int kN>
__global__ __launch_bounds__(kWaves * 64) void fdct_kernel(FrameSet<FdctArgs, kN> fs) {
    const uint32_t set_f = set_member<kN>(fs.wg0, fs.n, blockIdx.x);  // (frame sets: kernels.hpp)
    const FdctArgs& a = fs.a[set_f];
    const uint32_t bid = blockIdx.x - fs.wg0[set_f], nbk = fs.wg0[set_f + 1] - fs.wg0[set_f];
    // the arguments the tile loop reads, loaded once into scalar registers: a set
    // member's arguments sit at a computed kernarg offset, and the compiler otherwise
    // reloads them per tile (scalar loads whose lgkmcnt waits also wait for LDS traffic)
    const uint8_t* rgb_ = a.rgb;
    uint64_t stride_ = a.stride;
    uint32_t gw_ = a.g.width, gh_ = a.g.height;
    asm volatile("" : "+s"(rgb_), "+s"(stride_), "+s"(gw_), "+s"(gh_));
    constexpr int kK1Threads = kWaves * 64;
    __shared__ K1Lds<kWaves> lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;  // wv: 0..15
    K1WaveLds& W = lds.w[wv];
    JPGE_STAMP(1);
    const uint32_t mw = a.g.mw;
    const uint32_t tiles_per_row = (mw + 3) / 4;
    const uint32_t ntiles = tiles_per_row * a.g.mh;
    const double scale = 255.0 / (double)a.maxval;  // Image.cpp:465
    const bool aligned = (((uintptr_t)rgb_ | stride_) & 15) == 0;
    const int r16 = lane >> 2, c16 = lane & 3;  // staging: lane -> (pixel row, 16-px chunk)
    const int b8 = lane >> 3, j = lane & 7;     // DCT: lane -> (block of the round, column)

    // Pixels and coefficients move through buffer descriptors: an out-of-range
    // offset (kOob) makes a load return zeros and drops a store, so every tile
    // issues the same 3 loads and 3 stores with no branch around them, and the
    // wait for the prefetched pixels leaves the previous tile's stores in flight.
    const __amdgpu_buffer_rsrc_t rgb_rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(rgb_), 0, (int)(uint32_t)((uint64_t)stride_ * (gh_ - 1) + 3ull * gw_),
        0x00020000);
    const __amdgpu_buffer_rsrc_t coef_rs =
        __builtin_amdgcn_make_buffer_rsrc(a.coef, 0, (int)(uint32_t)((uint64_t)a.g.nblocks() * 128), 0x00020000);

    // Dynamic tiles.  One workgroup per CU owns a contiguous run of n_p tiles; each
    // of its 16 waves takes its first tile by rank, then grabs more from an LDS
    // counter until the run is exhausted.  The SIMD issues the oldest ready wave
    // first, so waves progress unequally: grabbing lets the faster ones take more
    // tiles, and all waves of a CU finish within about a tile of each other.
    const uint32_t tb_p = (uint32_t)((uint64_t)ntiles * bid / nbk);
    const uint32_t n_p = (uint32_t)((uint64_t)ntiles * (bid + 1) / nbk) - tb_p;
    auto grab = [&]() -> uint32_t {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&lds.next, 1u);
        return __builtin_amdgcn_readfirstlane(v);
    };

    // 48-byte RGB run of this lane for partition tile k, if the tile is on the aligned
    // fast path (else zeros, and the staging takes the clamped edge path)
    // (tile numbers are wave-uniform: the tile's row and column come from scalar
    // arithmetic, and only this lane's fixed offset within the tile is per lane)
    const uint32_t lane_off = (uint32_t)r16 * (uint32_t)stride_ + (uint32_t)c16 * 48u;
    auto fast_load = [&](uint32_t k, uint4& v0, uint4& v1, uint4& v2) -> bool {
        const uint32_t t = tb_p + k;
        const uint32_t mrow = t / tiles_per_row, mcol0 = (t % tiles_per_row) * 4;
        const uint32_t y = mrow * 16 + r16, xs = mcol0 * 16 + c16 * 16;
        const bool ok = k < n_p && aligned && y < gh_ && xs + 16 <= gw_;
        const uint32_t base = (uint32_t)((uint64_t)(mrow * 16) * stride_ + (uint64_t)mcol0 * 48);  // (uniform)
        const uint32_t off = ok ? base + lane_off : kOob;
        v0 = as_u4(__builtin_amdgcn_raw_buffer_load_b128(rgb_rs, off, 0, 0));
        v1 = as_u4(__builtin_amdgcn_raw_buffer_load_b128(rgb_rs, off + 16, 0, 0));
        v2 = as_u4(__builtin_amdgcn_raw_buffer_load_b128(rgb_rs, off + 32, 0, 0));
        return ok;
    };
    // The last round's 16-byte coefficient row (kOob: none) is stored during the
    // next tile, after its staging: the staging's wait for the prefetched pixels
    // then finds only long-issued stores ahead of them in the in-order counter.
    u32x4 pend;
    uint32_t poff = kOob;
    auto store_pending = [&] { __builtin_amdgcn_raw_buffer_store_b128(pend, coef_rs, poff, 0, kK1StoreAux); };
    uint32_t k = __builtin_amdgcn_readfirstlane((uint32_t)wv);  // this wave's current tile of the run
    uint4 c0, c1, c2;
    bool cfast = fast_load(k, c0, c1, c2);  // issued before the prologue's own memory traffic

    for (uint32_t i = bid * kK1Threads + tid; i < a.zero_words; i += nbk * kK1Threads) a.zero[i] = 0;
    if (bid == 0)  // carried: another frame's tables + headers, host -> device
        for (uint32_t i = tid; i < a.imp_n16; i += kK1Threads) a.imp_dst[i] = a.imp_src[i];
    if (tid == 0) lds.next = kWaves;
    if (tid < 128) {
        const int c = tid >> 6, e = tid & 63, o = (e >> 3) * kQRow + (e & 7);
        const double q = (double)q_entry(a, tid);  // Image.cpp:611-636 divides by the entry as double
        lds.q[c][o] = q;
        lds.invq[c][o] = arai_scale(e & 7) / q;
    }
    // LDS-only barrier: the prologue's shared state is in LDS (a full __syncthreads
    // would also wait for the first tile's pixels, issued above)
    lds_barrier();
    JPGE_STAMP(0);
    uint32_t kn = k < n_p ? grab() : n_p;  // the next tile (its pixels are prefetched a tile ahead)

    // Round inputs, read from LDS in one batch per round (issued during the previous
    // round's row pass): 8 pixel words of a Y column, or the 2x2 pixel pairs of 8
    // chroma samples, and the lane's 8 reciprocal quantisers.
    const int ycolbase = (b8 >> 2) * 16 + (b8 & 1) * 8 + j;  // Y round: column of the lane's block
    const int yrow0 = ((b8 >> 1) & 1) * 8;
    const int ccomp = b8 >> 2, cm = b8 & 3;
    const int ccol = cm * 16 + 2 * j;
    double* tb = &W.tmp[b8 * kTmpBlock];
    auto load_y = [&](int round, uint32_t p[8]) {
        const int col = round * 32 + ycolbase;
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = W.rgbx[(yrow0 + i) * kRgbPitch + col];
    };
    // Exact colour (8-bit input): a Cb lane and its Cr partner 32 lanes up read the same
    // pixels, so each reads half of them (rows 8h..8h+7, its 4 samples), converts them for
    // both components, and the pair trades the other component's values (swap_halves).
    const int crow0 = kExact ? 8 * ccomp : 0;
    auto load_c = [&](uint2 c[16]) {
        constexpr int n = kExact ? 8 : 16;
#pragma unroll
        for (int i = 0; i < n; ++i)
            c[i] = *reinterpret_cast<const uint2*>(&W.rgbx[(crow0 + i) * kRgbPitch + ccol]);
    };
    auto load_iq = [&](int qb, double iq[8]) {
#pragma unroll
        for (int u = 0; u < 8; ++u) iq[u] = lds.invq[qb][j * kQRow + u];
    };
    auto y_inputs = [&](const uint32_t p[8], double x[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = kExact ? ycc_exact_y(p[i]) : ycc_ref_y(p[i], scale);
    };
    auto c_inputs = [&](const uint2 c[16], double x[8]) {
        if constexpr (kExact) {
            // channel sums of this lane's 4 samples (exact integers), then both components:
            // the chroma of 8-bit input is exact, and each filter's
            // 1/4, 1/2 or 1 is folded into the constants (every product stays exact):
            //   S420_m  ((a+b)+(c+d))/4 of the 2x2 pixels, Image.cpp:207-224;
            //   S420_lm (a+c)/2 of the two rows' left pixels, Image.cpp:218-224, 297-306;
            //   S420    the top-left pixel (the masks' zero terms add zeros), Image.cpp:279-286
            constexpr double f = kFilt == kFiltS420 ? 1.0 : kFilt == kFiltS420lm ? 0.5 : 0.25;
            double vb[4], vr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint2 t0 = c[2 * i], t1 = c[2 * i + 1];
                uint32_t sr = t0.x & 0xFF, sg = (t0.x >> 8) & 0xFF, sb = t0.x >> 16;
                if (kFilt != kFiltS420) {
                    sr += t1.x & 0xFF;
                    sg += (t1.x >> 8) & 0xFF;
                    sb += t1.x >> 16;
                }
                if (kFilt == kFiltS420m) {
                    sr += (t0.y & 0xFF) + (t1.y & 0xFF);
                    sg += ((t0.y >> 8) & 0xFF) + ((t1.y >> 8) & 0xFF);
                    sb += (t0.y >> 16) + (t1.y >> 16);
                }
                const double dr = (double)sr, dg = (double)sg, db = (double)sb;
                vb[i] = __builtin_fma(kCbB * f, db, __builtin_fma(kCbG * f, dg, (kCbR * f) * dr));
                vr[i] = __builtin_fma(kCrB * f, db, __builtin_fma(kCrG * f, dg, (kCrR * f) * dr));
            }
            // lanes < 32 (Cb) keep Cb of samples 0-3 and receive Cb of 4-7; lanes >= 32 (Cr)
            // receive Cr of 0-3 and keep Cr of 4-7
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                swap_halves(vb[i], vr[i]);
                x[i] = vb[i];
                x[4 + i] = vr[i];
            }
            return;
        }
        const double kr = ccomp ? kCrR : kCbR, kg = ccomp ? kCrG : kCbG, kb = ccomp ? kCrB : kCbB;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint2 t0 = c[2 * i], t1 = c[2 * i + 1];
            // other maxvals: the reference's per-pixel op order
            if (kFilt == kFiltS420) {
                // subsample(S420), Image.cpp:279-286: mask {1, 0} on even rows only, the
                // top-left sample (the mask's 0 * b adds a zero)
                x[i] = ycc_ref_c(t0.x, scale, kr, kg, kb);
            } else if (kFilt == kFiltS420lm) {
                // subsample(S420_lm), Image.cpp:297-306, 218-224: (a + c) / 2 of the left
                // samples of both rows
                double v = ycc_ref_c(t0.x, scale, kr, kg, kb);
                v += ycc_ref_c(t1.x, scale, kr, kg, kb);
                x[i] = v / 2;
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
    };

    uint32_t ndone = 0;
    for (; k < n_p; ++ndone) {
        const uint32_t t = tb_p + k;
        const uint32_t mrow = t / tiles_per_row;
        const uint32_t mcol0 = (t % tiles_per_row) * 4;
        const int nvalid = (int)min(4u, mw - mcol0);
        const uint32_t y = mrow * 16 + r16, xs = mcol0 * 16 + c16 * 16;

        JPGE_STAMP(2 + min(ndone, 4u));
        // ---- stage 16 px per lane as packed u32 ----
        // (the prefetched registers are consumed on every path, so no later wait on
        // them can also drain the previous tile's coefficient stores)
        uint32_t px[16];
        {
            const uint4 v0 = c0, v1 = c1, v2 = c2;
            const uint32_t wd[13] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w, 0u};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int b0 = 3 * i, d = b0 >> 2, sh = 8 * (b0 & 3);
                // bytes b0..b0+2 of the run, zero-extended (perm selector 0x0c = 0x00)
                const uint32_t o8 = (uint32_t)(sh / 8);
                px[i] = __builtin_amdgcn_perm(wd[d + 1], wd[d], 0x0C000000u | ((o8 + 2) << 16) | ((o8 + 1) << 8) | o8);
            }
        }
        if (!cfast) {  // right/bottom edge replication (Image.cpp:498-531) as clamped addressing
            const uint32_t sy = min(y, gh_ - 1);
            for (int i = 0; i < 16; ++i) {
                const uint32_t sx = min(xs + i, gw_ - 1);
                const uint8_t* p = rgb_ + (uint64_t)sy * stride_ + (uint64_t)sx * 3;
                px[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
            }
        }
        uint32_t* dst = &W.rgbx[r16 * kRgbPitch + c16 * 16];
#pragma unroll
        for (int i = 0; i < 16; i += 2) *reinterpret_cast<uint2*>(dst + i) = make_uint2(px[i], px[i + 1]);
        wave_order();
        // prefetch the next tile of this wave (into the registers just staged) while
        // this one is transformed
        store_pending();
        cfast = fast_load(kn, c0, c1, c2);
        const uint32_t kn2 = kn < n_p ? grab() : n_p;

        // ---- rounds: Cb x4 + Cr x4, Y blocks 0-7 (MCUs 0, 1), Y blocks 8-15 (MCUs 2, 3) ----
        // A round: inputs -> column pass -> transposed LDS write (Dct.hpp:124-131) ->
        // row pass -> quantise -> one 16-byte row store.  A wave's LDS operations run
        // in issue order, so only the compiler needs fencing between them.
        // The chroma round's inputs are read now; each later round's during the
        // previous round's row pass.
        uint32_t p[8];
        uint2 cc[16];
        double iq[8];
        load_c(cc);
        load_iq(1, iq);
        wave_order();
        auto finish = [&](double x[8], int m, int slot, int qb, u32x4& pk, uint32_t& off, auto&& prefetch_next) {
            double o[8];
            arai8(x, o);
#pragma unroll
            for (int k = 0; k < 8; ++k) tb[j * kTmpRow + k] = o[k];
            wave_order();
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = tb[i * kTmpRow + j];
            double iqc[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) iqc[u] = iq[u];
            wave_order();
            prefetch_next();  // next round's inputs: after this round's LDS reads
            arai8_unscaled(x, o);  // y(j, u) = o[u] * s_u
            pk = quant_row(o, iqc, &lds.q[qb][j * kQRow]);
            const uint32_t blk = (mrow * mw + mcol0 + m) * 6 + slot;
            off = m < nvalid ? blk * 128 + j * 16 : kOob;
        };
        {
            double x[8];
            c_inputs(cc, x);
            u32x4 pk;
            uint32_t off;
            finish(x, cm, 4 + ccomp, 1, pk, off, [&] {
                load_y(0, p);
                load_iq(0, iq);
            });
            __builtin_amdgcn_raw_buffer_store_b128(pk, coef_rs, off, 0, kK1StoreAux);
        }
        {
            double x[8];
            y_inputs(p, x);
            u32x4 pk;
            uint32_t off;
            finish(x, b8 >> 2, b8 & 3, 0, pk, off, [&] { load_y(1, p); });
            __builtin_amdgcn_raw_buffer_store_b128(pk, coef_rs, off, 0, kK1StoreAux);
        }
        {
            double x[8];
            y_inputs(p, x);
            finish(x, 2 + (b8 >> 2), b8 & 3, 0, pend, poff, [] {});
        }
        wave_order();  // the next tile's staging overwrites the transpose buffer
        k = kn;
        kn = kn2;
    }
    store_pending();
    __syncthreads();
    JPGE_STAMP(7);
}

// ---- MCUs one block row high: 4:4:4, 4:2:2, 4:1:1 (applySubsampling S444, S422,
// S411, Image.cpp:257-278; the MCU is kYh Y blocks across + Cb + Cr) ----
// Same machinery as fdct_kernel: a wave owns a tile of 128x8 px (16 Y blocks,
// 16 / kYh MCUs; a lane stages one 16-px run of one row), in rounds of 8 blocks
// (lane = (block of the round, column)): Y blocks 0-7, Y blocks 8-15, then the
// chroma blocks — 4:4:4: Cb 0-7, Cb 8-15, Cr 0-7, Cr 8-15; 4:2:2: Cb 0-7, Cr 0-7;
// 4:1:1: Cb 0-3 + Cr 0-3 in one round.  S422 / S411 keep the first sample of each
// 2 / 4 along a row (mask {1,0} / {1,0,0,0}, every scanline; the mask's zero terms
// add zeros).  Chroma is converted per pixel: for 8-bit input (128 + v) - 128 == v
// exactly, and v = fma(kb, b, fma(kg, g, kr r)) is exact.
constexpr int kRgbPitch444 = 130;  // u32 per staged row of 128 px (+2: even, for uint2 stores)
static_assert(8 * kRgbPitch444 <= 16 * kRgbPitch, "the 4:4:4 tile fits the 4:2:0 staging area");

template <bool kExact, int kWaves, int kYh, int kN>
__global__ __launch_bounds__(kWaves * 64) void fdct_row8_kernel(FrameSet<FdctArgs, kN> fs) {
    const uint32_t set_f = set_member<kN>(fs.wg0, fs.n, blockIdx.x);  // (frame sets: kernels.hpp)
    const FdctArgs& a = fs.a[set_f];
    const uint32_t bid = blockIdx.x - fs.wg0[set_f], nbk = fs.wg0[set_f + 1] - fs.wg0[set_f];
    // the arguments the tile loop reads, loaded once into scalar registers: a set
    // member's arguments sit at a computed kernarg offset, and the compiler otherwise
    // reloads them per tile (scalar loads whose lgkmcnt waits also wait for LDS traffic)
    const uint8_t* rgb_ = a.rgb;
    uint64_t stride_ = a.stride;
    uint32_t gw_ = a.g.width, gh_ = a.g.height;
    asm volatile("" : "+s"(rgb_), "+s"(stride_), "+s"(gw_), "+s"(gh_));
    constexpr int kK1Threads = kWaves * 64;
    constexpr uint32_t kMcus = 16 / kYh;            // MCUs per tile
    constexpr int kBpm = kYh + 2;                   // blocks per MCU
    constexpr int kRounds = 2 + 4 / kYh;            // 2 Y rounds + the chroma rounds
    __shared__ K1Lds<kWaves> lds;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    K1WaveLds& W = lds.w[wv];
    JPGE_STAMP(1);
    const uint32_t mw = a.g.mw;
    const uint32_t tiles_per_row = (mw + kMcus - 1) / kMcus;
    const uint32_t ntiles = tiles_per_row * a.g.mh;
    const double scale = 255.0 / (double)a.maxval;  // Image.cpp:465
    const bool aligned = (((uintptr_t)rgb_ | stride_) & 15) == 0;
    const int r8 = lane >> 3, c8 = lane & 7;  // staging: lane -> (pixel row, 16-px chunk)
    const int b8 = lane >> 3, j = lane & 7;   // DCT: lane -> (block of the round, column)

    const __amdgpu_buffer_rsrc_t rgb_rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(rgb_), 0, (int)(uint32_t)((uint64_t)stride_ * (gh_ - 1) + 3ull * gw_),
        0x00020000);
    const __amdgpu_buffer_rsrc_t coef_rs =
        __builtin_amdgcn_make_buffer_rsrc(a.coef, 0, (int)(uint32_t)((uint64_t)a.g.nblocks() * 128), 0x00020000);

    // dynamic tiles over the workgroup's contiguous run, as in fdct_kernel
    const uint32_t tb_p = (uint32_t)((uint64_t)ntiles * bid / nbk);
    const uint32_t n_p = (uint32_t)((uint64_t)ntiles * (bid + 1) / nbk) - tb_p;
    auto grab = [&]() -> uint32_t {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(&lds.next, 1u);
        return __builtin_amdgcn_readfirstlane(v);
    };
    const uint32_t lane_off = (uint32_t)r8 * (uint32_t)stride_ + (uint32_t)c8 * 48u;  // (as in fdct_kernel)
    auto fast_load = [&](uint32_t k, uint4& v0, uint4& v1, uint4& v2) -> bool {
        const uint32_t t = tb_p + k;
        const uint32_t mrow = t / tiles_per_row, mcol0 = (t % tiles_per_row) * kMcus;
        const uint32_t y = mrow * 8 + r8, xs = mcol0 * 8 * kYh + c8 * 16;
        const bool ok = k < n_p && aligned && y < gh_ && xs + 16 <= gw_;
        const uint32_t base = (uint32_t)((uint64_t)(mrow * 8) * stride_ + (uint64_t)mcol0 * 24 * kYh);  // (uniform)
        const uint32_t off = ok ? base + lane_off : kOob;
        v0 = as_u4(__builtin_amdgcn_raw_buffer_load_b128(rgb_rs, off, 0, 0));
        v1 = as_u4(__builtin_amdgcn_raw_buffer_load_b128(rgb_rs, off + 16, 0, 0));
        v2 = as_u4(__builtin_amdgcn_raw_buffer_load_b128(rgb_rs, off + 32, 0, 0));
        return ok;
    };
    u32x4 pend;
    uint32_t poff = kOob;
    auto store_pending = [&] { __builtin_amdgcn_raw_buffer_store_b128(pend, coef_rs, poff, 0, kK1StoreAux); };
    uint32_t k = __builtin_amdgcn_readfirstlane((uint32_t)wv);
    uint4 c0, c1, c2;
    bool cfast = fast_load(k, c0, c1, c2);

    for (uint32_t i = bid * kK1Threads + tid; i < a.zero_words; i += nbk * kK1Threads) a.zero[i] = 0;
    if (bid == 0)
        for (uint32_t i = tid; i < a.imp_n16; i += kK1Threads) a.imp_dst[i] = a.imp_src[i];
    if (tid == 0) lds.next = kWaves;
    if (tid < 128) {
        const int c = tid >> 6, e = tid & 63, o = (e >> 3) * kQRow + (e & 7);
        const double q = (double)q_entry(a, tid);
        lds.q[c][o] = q;
        lds.invq[c][o] = arai_scale(e & 7) / q;
    }
    // LDS-only barrier: the prologue's shared state is in LDS (a full __syncthreads
    // would also wait for the first tile's pixels, issued above)
    lds_barrier();
    JPGE_STAMP(0);
    uint32_t kn = k < n_p ? grab() : n_p;

    double* tb = &W.tmp[b8 * kTmpBlock];
    auto load_px = [&](int round, uint32_t p[8]) {  // column j of the round's block b8
        int col;
        if (round < 2 || kYh == 1) col = ((round & 1) * 8 + b8) * 8 + j;  // full resolution
        else if (kYh == 2) col = b8 * 16 + 2 * j;                          // S422: left of each pair
        else col = (b8 & 3) * 32 + 4 * j;                                  // S411: first of each 4
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = W.rgbx[i * kRgbPitch444 + col];
    };
    auto load_iq = [&](int qb, double iq[8]) {
#pragma unroll
        for (int u = 0; u < 8; ++u) iq[u] = lds.invq[qb][j * kQRow + u];
    };

    for (; k < n_p;) {
        const uint32_t t = tb_p + k;
        const uint32_t mrow = t / tiles_per_row;
        const uint32_t mcol0 = (t % tiles_per_row) * kMcus;
        const int nvalid = (int)min(kMcus, mw - mcol0);
        const uint32_t y = mrow * 8 + r8, xs = mcol0 * 8 * kYh + c8 * 16;

        uint32_t px[16];
        {
            const uint4 v0 = c0, v1 = c1, v2 = c2;
            const uint32_t wd[13] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w, 0u};
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int b0 = 3 * i, d = b0 >> 2;
                const uint32_t o8 = (uint32_t)(b0 & 3);
                px[i] = __builtin_amdgcn_perm(wd[d + 1], wd[d], 0x0C000000u | ((o8 + 2) << 16) | ((o8 + 1) << 8) | o8);
            }
        }
        if (!cfast) {  // edge replication (Image.cpp:498-531) as clamped addressing
            const uint32_t sy = min(y, gh_ - 1);
            for (int i = 0; i < 16; ++i) {
                const uint32_t sx = min(xs + i, gw_ - 1);
                const uint8_t* p = rgb_ + (uint64_t)sy * stride_ + (uint64_t)sx * 3;
                px[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
            }
        }
        uint32_t* dst = &W.rgbx[r8 * kRgbPitch444 + c8 * 16];
#pragma unroll
        for (int i = 0; i < 16; i += 2) *reinterpret_cast<uint2*>(dst + i) = make_uint2(px[i], px[i + 1]);
        wave_order();
        store_pending();
        cfast = fast_load(kn, c0, c1, c2);
        const uint32_t kn2 = kn < n_p ? grab() : n_p;

        uint32_t p[8];
        double iq[8];
        load_px(0, p);
        load_iq(0, iq);
        wave_order();
#pragma unroll
        for (int round = 0; round < kRounds; ++round) {
            // the lane's block: component, MCU of the tile, slot in the MCU
            int comp, m, slot;
            if (round < 2) {
                const int bx = round * 8 + b8;  // Y block of the tile
                comp = 0; m = bx / kYh; slot = bx % kYh;
            } else {
                comp = kYh == 1 ? 1 + ((round - 2) >> 1) : kYh == 2 ? round - 1 : 1 + (b8 >> 2);
                m = kYh == 1 ? (round & 1) * 8 + b8 : kYh == 2 ? b8 : (b8 & 3);
                slot = kYh + comp - 1;
            }
            const int qb = comp ? 1 : 0;
            double x[8];
            if (comp == 0) {
#pragma unroll
                for (int i = 0; i < 8; ++i) x[i] = kExact ? ycc_exact_y(p[i]) : ycc_ref_y(p[i], scale);
            } else {
                const double kr = comp == 2 ? kCrR : kCbR, kg = comp == 2 ? kCrG : kCbG, kb = comp == 2 ? kCrB : kCbB;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    x[i] = kExact ? ycc_exact_c(p[i], kr, kg, kb) : ycc_ref_c(p[i], scale, kr, kg, kb);
            }
            double o[8];
            arai8(x, o);
#pragma unroll
            for (int u = 0; u < 8; ++u) tb[j * kTmpRow + u] = o[u];
            wave_order();
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = tb[i * kTmpRow + j];
            double iqc[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) iqc[u] = iq[u];
            wave_order();
            if (round + 1 < kRounds) {  // the next round's inputs, after this round's LDS reads
                load_px(round + 1, p);
                if (round == 1) load_iq(1, iq);
            }
            arai8_unscaled(x, o);
            const u32x4 pk = quant_row(o, iqc, &lds.q[qb][j * kQRow]);
            const uint32_t blk = (mrow * mw + mcol0 + m) * kBpm + slot;
            const uint32_t off = m < nvalid ? blk * 128 + j * 16 : kOob;
            if (round < kRounds - 1) {
                __builtin_amdgcn_raw_buffer_store_b128(pk, coef_rs, off, 0, kK1StoreAux);
            } else {
                pend = pk;
                poff = off;
            }
        }
        wave_order();  // the next tile's staging overwrites the transpose buffer
        k = kn;
        kn = kn2;
    }
    store_pending();
    __syncthreads();
    JPGE_STAMP(7);
}

}  // namespace

// Alone on the GPU, frames with fewer than kK1WholeCuTiles tiles (a 4K frame has
// 8 100) run the 4-wave shape at 4 workgroups per CU, larger ones the whole-CU shape:
// measured 15.5-15.6 vs 16.2-16.3 us at 4K, but 340-349 vs 317-326 us at 16384^2
// (262 144 tiles), where the whole-CU workgroups' shared tile counter balances ~64
// tiles per wave.
constexpr uint32_t kK1WholeCuTiles = 65536;
uint32_t k1_tiles(const Geometry& g) {
    const uint32_t per = g.row8() ? 16 / g.yh : 4;  // MCUs per tile
    return ((g.mw + per - 1) / per) * g.mh;
}
bool k1_whole_cu(const Geometry& g, bool solo) { return solo && k1_tiles(g) >= kK1WholeCuTiles; }

template <int kYh, int kN>
hipError_t launch_row8(const FrameSet<FdctArgs, kN>& fs, uint32_t grid, hipStream_t s, const KTimer* t) {
    const FdctArgs& a = fs.a[0];
    const bool ex = a.maxval == 255;
    if (k1_whole_cu(a.g, a.solo)) {
        if (ex) return launch_timed(t, fdct_row8_kernel<true, kK1WavesSolo, kYh, kN>, dim3(grid), dim3(kK1WavesSolo * 64), s, fs);
        else return launch_timed(t, fdct_row8_kernel<false, kK1WavesSolo, kYh, kN>, dim3(grid), dim3(kK1WavesSolo * 64), s, fs);
    } else {
        if (ex) return launch_timed(t, fdct_row8_kernel<true, kK1WavesShared, kYh, kN>, dim3(grid), dim3(kK1WavesShared * 64), s, fs);
        else return launch_timed(t, fdct_row8_kernel<false, kK1WavesShared, kYh, kN>, dim3(grid), dim3(kK1WavesShared * 64), s, fs);
    }
}

template <int kFilt, int kN>
hipError_t launch_420(const FrameSet<FdctArgs, kN>& fs, uint32_t grid, hipStream_t s, const KTimer* t) {
    const FdctArgs& a = fs.a[0];
    const bool ex = a.maxval == 255;
    if (k1_whole_cu(a.g, a.solo)) {
        if (ex) return launch_timed(t, fdct_kernel<true, kK1WavesSolo, kFilt, kN>, dim3(grid), dim3(kK1WavesSolo * 64), s, fs);
        else return launch_timed(t, fdct_kernel<false, kK1WavesSolo, kFilt, kN>, dim3(grid), dim3(kK1WavesSolo * 64), s, fs);
    } else {
        if (ex) return launch_timed(t, fdct_kernel<true, kK1WavesShared, kFilt, kN>, dim3(grid), dim3(kK1WavesShared * 64), s, fs);
        else return launch_timed(t, fdct_kernel<false, kK1WavesShared, kFilt, kN>, dim3(grid), dim3(kK1WavesShared * 64), s, fs);
    }
}

uint32_t fdct_grid(const Geometry& g, bool solo, uint32_t override_wgs) {
    const uint32_t tiles = k1_tiles(g);
    if (k1_whole_cu(g, solo)) {  // one whole-CU workgroup per CU (MI355X: 256 CUs)
        const uint32_t cap = 256u * (16u / (uint32_t)kK1WavesSolo);
        return tiles < cap ? tiles : cap;
    }
    // the 4-wave shape, a tile per wave at a time: four per CU alone, at most
    // kK1SharedCap beside other lanes
    const uint32_t wgs = (tiles + kK1WavesShared - 1) / kK1WavesShared;
    const uint32_t cap = override_wgs ? override_wgs : solo ? 1024u : kK1SharedCap;
    return wgs < cap ? wgs : cap;
}

// A set of frames of one geometry, colour path and workgroup shape (one launch).
template <int kN>
static hipError_t launch_fdct_fs(const FrameSet<FdctArgs, kN>& fs, hipStream_t s, const KTimer* t) {
    const FdctArgs& a = fs.a[0];
    for (uint32_t f = 0; f < fs.n; ++f) {
        const FdctArgs& m = fs.a[f];
        // 32-bit buffer offsets: the frame's pixels and coefficients must stay below kOob
        // (a 16384^2 frame needs 805 MB of each)
        if ((uint64_t)m.stride * m.g.height >= kOob || (uint64_t)m.g.nblocks() * 128 >= kOob) return hipErrorInvalidValue;
        if (std::memcmp(&m.g, &a.g, sizeof(Geometry)) != 0 || (m.maxval == 255) != (a.maxval == 255) ||
            m.solo != a.solo || fs.wg0[f + 1] - fs.wg0[f] != fdct_grid(m.g, m.solo, m.wgs))
            return hipErrorInvalidValue;
    }
    const uint32_t grid = fs.wg0[fs.n];
    // the kernels assume these shapes (kernels.hpp Geometry)
    if (a.g.row8()) {
        switch (a.g.yh) {
            // (launch_timed returns the launch's error: hipGetLastError has already consumed it)
            case 1: return a.g.bpm != 3 ? hipErrorInvalidValue : launch_row8<1, kN>(fs, grid, s, t);
            case 2: return a.g.bpm != 4 ? hipErrorInvalidValue : launch_row8<2, kN>(fs, grid, s, t);
            case 4: return a.g.bpm != 6 ? hipErrorInvalidValue : launch_row8<4, kN>(fs, grid, s, t);
            default: return hipErrorInvalidValue;
        }
    }
    if (a.g.yh != 2 || a.g.bpm != 6) return hipErrorInvalidValue;
    switch (a.g.cfilt) {
        case kFiltS420m: return launch_420<kFiltS420m, kN>(fs, grid, s, t);
        case kFiltS420lm: return launch_420<kFiltS420lm, kN>(fs, grid, s, t);
        case kFiltS420: return launch_420<kFiltS420, kN>(fs, grid, s, t);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fdct(const FdctArgs& a, hipStream_t s, const KTimer* t) {
    return launch_fdct_fs(frame_set<1>(&a, 1, fdct_grid(a.g, a.solo, a.wgs)), s, t);
}

hipError_t launch_fdct_set(const FdctArgs* a, int n, hipStream_t s, const KTimer* t) {
    if (n < 1 || n > kMaxSet) return hipErrorInvalidValue;
    return launch_fdct_fs(frame_set(a, n, fdct_grid(a[0].g, a[0].solo, a[0].wgs)), s, t);
}

}  // namespace jpge
