// Segment concatenation (gfx950): n device byte runs written back to back into one
// device buffer, in one launch per up to kConcatMax segments.  Config 4's gather
// (jpgenc_amd/gather.py) packs a rank's .jpg bytes with it before the
// one transfer to rank 0; the reference has no counterpart (a single-process
// encoder), the bytes are unchanged.
//
// Byte copy at HBM speed with arbitrary source and destination alignments: a thread
// writes one aligned 16-byte destination word.  For a word wholly inside its segment
// the source bytes are a 16-byte window at a fixed shift from an aligned pair of
// source words, and that shift is the same for every word of the segment (the
// destination words are 16 apart), so each thread does two 16-byte buffer loads and
// four v_alignbyte under a workgroup-uniform switch.  The (at most two) destination
// words a segment shares with its neighbours are written byte by byte: every byte has
// exactly one writer.  Sources go through buffer descriptors bounded by the segment's
// last aligned 16 bytes, so a load past them reads zeros, never another page.
// HBM-bound: 2 bytes of traffic per byte copied.
#include "device_common.hpp"
#include "kernels.hpp"

namespace jpge {
namespace {
using namespace dev;

constexpr uint32_t kConcatThreads = 256;
constexpr uint32_t kConcatWords = 4096;  // destination words per workgroup (64 KB)

__global__ __launch_bounds__(kConcatThreads) void concat_kernel(ConcatArgs a) {
    // this workgroup's segment: the last k with chunk0[k] <= blockIdx.x (scalar search)
    const uint32_t bx = blockIdx.x;
    uint32_t k = 0;
    while (k + 1 < a.n && a.chunk0[k + 1] <= bx) ++k;
    const uint32_t chunk = bx - a.chunk0[k];
    const uint8_t* src = a.src[k];
    const uint64_t len = a.len[k];
    uint8_t* const dst = a.dst + a.off[k];  // the segment's first destination byte
    // destination words overlapping the segment: [w0, w1) of 16 bytes at an aligned base
    const uintptr_t d0 = reinterpret_cast<uintptr_t>(dst);
    const uintptr_t wbase = d0 & ~(uintptr_t)15;
    const uint64_t nw = (d0 + len + 15 - wbase) >> 4;
    // the source window: rel(w) = s0 + (wbase + 16 w - d0) from the aligned source base
    const uintptr_t s = reinterpret_cast<uintptr_t>(src);
    const uint8_t* const sbase = reinterpret_cast<const uint8_t*>(s & ~(uintptr_t)15);
    const uint32_t s0 = (uint32_t)(s & 15);
    const uint32_t lead = (uint32_t)(d0 - wbase);     // bytes of word 0 before the segment
    const uint32_t sh = (s0 + 16u - lead) & 15u;       // the window's shift (uniform)
    const uint32_t dw = sh >> 2, b = sh & 3u;
    // The descriptor ends at the 16-byte boundary after the run: a load holding a needed
    // byte is then wholly in range (the range check drops whole dwords, so a bound at
    // the run's last byte would zero the valid bytes of a straddling dword), and the
    // <= 15 bytes read past the run share its last aligned 16 bytes (never another page).
    // (descriptor sizes are 32-bit: segments are far below 4 GB, launch_concat checks)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(sbase), 0, (int)((s0 + len + 15) & ~(uint64_t)15), 0x00020000);
    const uint64_t w_lo = (uint64_t)chunk * kConcatWords;
    const uint64_t w_hi = w_lo + kConcatWords < nw ? w_lo + kConcatWords : nw;
    for (uint64_t w = w_lo + threadIdx.x; w < w_hi; w += kConcatThreads) {
        const uintptr_t da = wbase + 16 * w;
        const bool inside = da >= d0 && da + 16 <= d0 + len;
        if (inside) {
            // source offset of this word's first byte from sbase: s0 + (da - d0)
            const uint32_t rel = s0 + (uint32_t)(da - d0);
            const uint32_t A = rel - sh;  // (aligned: rel == sh mod 16)
            const u32x4 x = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, A, 0, 0));
            const u32x4 y = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, A + 16, 0, 0));
            const uint32_t W[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
            uint32_t o[4];
            switch (dw) {  // (uniform over the workgroup)
                case 0:
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(W[i + 1], W[i], b);
                    break;
                case 1:
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(W[i + 2], W[i + 1], b);
                    break;
                case 2:
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(W[i + 3], W[i + 2], b);
                    break;
                default:
#pragma unroll
                    for (int i = 0; i < 4; ++i) o[i] = __builtin_amdgcn_alignbyte(W[i + 4], W[i + 3], b);
                    break;
            }
            *reinterpret_cast<uint4*>(da) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {  // a word shared with a neighbour segment (or the buffer's edge): its bytes
            for (uint32_t j = 0; j < 16; ++j) {
                const uintptr_t p = da + j;
                if (p >= d0 && p < d0 + len) *reinterpret_cast<uint8_t*>(p) = src[p - d0];
            }
        }
    }
}

}  // namespace

hipError_t launch_concat(const ConcatArgs& a, uint32_t nchunks, hipStream_t s) {
    if (a.n == 0 || a.n > kConcatMax) return hipErrorInvalidValue;
    for (uint32_t k = 0; k < a.n; ++k)
        if (a.len[k] >= (1ull << 31)) return hipErrorInvalidValue;
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(concat_kernel, dim3(nchunks), dim3(kConcatThreads), 0, s, a);
    return hipGetLastError();
}

uint32_t concat_chunks(uint64_t len, uintptr_t dst) {
    const uintptr_t wbase = dst & ~(uintptr_t)15;
    const uint64_t nw = len ? (dst + len + 15 - wbase) >> 4 : 0;
    return (uint32_t)((nw + kConcatWords - 1) / kConcatWords);
}

}  // namespace jpge
