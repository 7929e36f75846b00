// Device helpers shared by the jpge kernels (fdct.hip, stats.hip, entropy.hip).
// Included only by HIP translation units.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace jpge {
// Launch `kernel` on s, through hipExtLaunchKernel with the timer's events when
// one is given (KTimer, kernels.hpp), else as a plain launch.
template <typename F, typename... Args>
inline hipError_t launch_timed(const KTimer* t, F kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
    if (t && t->start && t->stop)
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, t->start, t->stop, 0, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
    return hipGetLastError();
}
}  // namespace jpge

#pragma clang fp contract(off)

namespace jpge {
namespace dev {

// Diagnostic phase stamps (JPGE_STAMPS builds only; otherwise they compile to
// nothing): thread 0 of each workgroup records s_memrealtime (100 MHz, chip-wide)
// at phase boundaries into a.dbg[blockIdx.x * kStampSlots + i] (slots 0-7), and
// accumulated sub-phase durations into slots 8-15 (JPGE_ACC).  Never part of an
// output.
#ifdef JPGE_STAMPS
#define JPGE_NOW() __builtin_amdgcn_s_memrealtime()
#define JPGE_STAMP(i)                                                                                    \
    do {                                                                                                 \
        if (a.dbg && threadIdx.x == 0) a.dbg[blockIdx.x * kStampSlots + (i)] = JPGE_NOW();              \
    } while (0)
#define JPGE_ACC(i, t)                                                                                   \
    do {                                                                                                 \
        const uint64_t now_ = JPGE_NOW();                                                                \
        if (a.dbg && threadIdx.x == 0) a.dbg[blockIdx.x * kStampSlots + 8 + (i)] += now_ - (t);        \
        (t) = now_;                                                                                      \
    } while (0)
#else
#define JPGE_NOW() 0ull
#define JPGE_STAMP(i) \
    do {              \
    } while (0)
#define JPGE_ACC(i, t) \
    do {               \
        (void)(t);     \
    } while (0)
#endif

// buffer-descriptor loads return 4 x u32 as a vector type
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 as_u4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 as_u2(u32x2 v) { return make_uint2(v.x, v.y); }

// natural (row-major) index -> zig-zag position (inverse of Coding.hpp:57-81)
static __constant__ uint8_t kNatToZz[64] = {
    0, 1, 5, 6, 14, 15, 27, 28, 2, 4, 7, 13, 16, 26, 29, 42,
    3, 8, 12, 17, 25, 30, 41, 43, 9, 11, 18, 24, 31, 40, 44, 53,
    10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
    21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// zig-zag position -> natural index (Coding.hpp:57-81)
static __constant__ uint8_t kZzToNat[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Orders LDS traffic between lanes of ONE wavefront (a wave's DS ops execute in
// order; this stops the compiler from moving them across the point).
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
// The same ordering without the wait: a wave's DS instructions execute in issue
// order, so a read issued after another lane's write sees it; only the compiler
// must not move LDS accesses across this point.
__device__ __forceinline__ void wave_order() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// getCategoryAndCode, Coding.hpp:197-230: bit length of |v| (0 for v == 0)
__device__ __forceinline__ int category(int v) {
    const int av = v < 0 ? -v : v;
    return av ? 32 - __builtin_clz((unsigned)av) : 0;
}

// Symbol record words (kernels.hpp): table << 24 | symbol << 16 | extra bits.
__device__ __forceinline__ uint32_t rec_word(uint32_t table, uint32_t sym, uint32_t bits) {
    return (table << 24) | (sym << 16) | bits;
}
__device__ __forceinline__ uint32_t extra_bits(int v, int cat) {  // getCategoryAndCode, Coding.hpp:214-221
    return (uint32_t)(v + (v >> 31)) & ((1u << cat) - 1);
}

constexpr int kPartsPerBlock = 4;  // lanes cooperating on one block's non-zero coefficients

// DC predecessor of flat block g (Image.cpp:638-678): the Y chain runs in MCU
// order, Cb and Cr each over their own blocks; a chain's first block predicts 0.
// The predecessor is at most 6 blocks back (bpm <= 6).  In every mode the Y chain
// runs in MCU order over the MCU's bpm - 2 Y slots, so an MCU's first Y block
// follows the previous MCU's last (3 blocks back: past Cr and Cb), and each chroma
// block follows the same slot of the previous MCU.
__device__ __forceinline__ int64_t dc_pred_index(uint64_t g, uint32_t bpm) {
    const int k = (int)(g % bpm);
    if (k >= 1 && k < (int)bpm - 2) return (int64_t)g - 1;
    if (g < bpm) return -1;
    return (int64_t)g - (k == 0 ? 3 : bpm);
}

// One tile of kBlocks coefficient blocks (natural order in HBM) held in registers
// between its load and its LDS staging, so a persistent workgroup can fetch tile
// t+1 while it codes tile t.  Lane q of the tile carries row q&7 of block q>>3;
// lanes < 6 also carry the DC of the 6 blocks before the tile (DC predecessors).
// The zig-zag positions of a lane's row (row = tid & 7 for every tile) are read
// from the constant table once, into registers: a global load inside the tile loop
// would make the in-order vmcnt wait for it also wait for the prefetched tile.
template <int kThreads, int kBlocks>
struct TileRegs {
    static constexpr int kPer = kBlocks * 8 / kThreads;
    static_assert(kPer * kThreads == kBlocks * 8 && kThreads % 8 == 0, "tile rows must divide over the threads");
    uint4 v[kPer];
    int prev_dc;
    uint32_t zlo, zhi;  // zig-zag positions of this lane's row, 4 per word

    __device__ __forceinline__ void init(int tid) {
        const uint32_t* z = reinterpret_cast<const uint32_t*>(&kNatToZz[(tid & 7) * 8]);
        zlo = z[0];
        zhi = z[1];
    }

    __device__ __forceinline__ void load(const int16_t* __restrict__ coef, uint64_t b0, int nb, int tid) {
        const uint4* src = reinterpret_cast<const uint4*>(coef + b0 * 64);
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            const int q = tid + i * kThreads;
            v[i] = q < nb * 8 ? src[q] : make_uint4(0, 0, 0, 0);
        }
        prev_dc = (tid < 6 && b0 + tid >= 6) ? coef[(b0 - 6 + tid) * 64] : 0;
    }
};

// Workgroup barrier for LDS traffic only: waits for this wave's LDS operations, not
// for its global loads or stores.  __syncthreads() is a workgroup fence as well,
// whose s_waitcnt vmcnt(0) also waits for every prefetch in flight — a tile or
// round loaded ahead would then arrive before the barrier passes and hide nothing.
// Use only where the data other waves read after the barrier is in LDS.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wait for this lane's outstanding global stores (so a following barrier publishes
// them to the rest of the workgroup).
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Histogram export: sum the replicas and write the four final histograms and
// first-occurrence keys into mapped host memory, then the frame's sequence number
// (release-ordered after the data): the host polls that word.  One workgroup.
template <int kThreads>
__device__ __forceinline__ void export_hist(const HistPtrs& h, uint32_t* host_cnt, uint64_t* host_key,
                                            uint64_t* host_seq, uint64_t seq, int tid) {
    for (int t = tid; t < 1024; t += kThreads) {  // (table, symbol) = (t >> 8, t & 255)
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < kHistReplicas; ++r) c += h.cnt[r * 1024 + t];
        host_cnt[t] = c;
        host_key[t] = h.key[t];
    }
    __syncthreads();
    if (tid == 0) {
        __threadfence_system();
        __hip_atomic_store(host_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Inclusive scan of one u32 per lane over the wave in DPP moves (row shifts, then
// the row broadcasts of lanes 15 and 31): no LDS traffic, no waits.
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)x;
}

// OR over each aligned group of 8 lanes: DPP quad permutes for lanes 1 and 2 apart
// (VALU only), a ds_swizzle (xor 4; no memory access) for 4 apart.
__device__ __forceinline__ uint32_t or_lanes8(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    v |= (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F);              // xor 4 (bitmask mode)
    return v;
}
__device__ __forceinline__ uint64_t or_lanes8(uint64_t v) {
    return ((uint64_t)or_lanes8((uint32_t)(v >> 32)) << 32) | or_lanes8((uint32_t)v);
}

// block-wide exclusive scan of one value per thread (thread order); wsum holds
// kWaves values of T.  kLdsSync: LDS-only barriers (lds_barrier), so global loads in
// flight stay in flight.  kLead: a barrier before wsum is written, for callers whose
// previous reads of wsum are not already behind one (without it: one barrier).
template <int kWaves, typename T, typename W, bool kLdsSync = false, bool kLead = true>
__device__ __forceinline__ T block_scan(T v, W* wsum, int lane, int wv, T& total) {
    static_assert(sizeof(W) == 4 && (sizeof(T) == 4 || sizeof(T) == 8), "scan word types");
    T* ws = reinterpret_cast<T*>(wsum);
    T incl = v;
    if constexpr (sizeof(T) == 4) {
        incl = (T)wave_scan_incl((uint32_t)v);  // DPP: no LDS permutes on the chain
    } else {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const T o = __shfl_up(incl, d);
            if (lane >= d) incl += o;
        }
    }
    if constexpr (kLead) {
        if (kLdsSync) lds_barrier();
        else __syncthreads();
    }
    // (wv is the wave's number, uniform: in an SGPR the wave's base is summed on the
    // scalar unit; as a VGPR it took a move and a select per wave sum, every call)
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    if (lane == 63) ws[wvu] = incl;
    if (kLdsSync) lds_barrier();
    else __syncthreads();
    T base = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const T s = ws[w];
        if (w < wvu) base += s;
        total += s;
    }
    return base + incl - v;
}

}  // namespace dev
}  // namespace jpge
