// Plane stage kernels (gfx950): the reference's Image stage methods on fp64 planes,
// for the drop-in facade's stage entries and for encoding an Image whose planes no
// longer come from an RGB8 frame (jpge_encode_planes).  The fused RGB8 path (K1,
// fdct.hip) is the hot path; these kernels reproduce the same arithmetic on
// arbitrary double planes, operation for operation:
//   plane_color_kernel      convertToColorSpace   Image.cpp:112-179
//   plane_subsample_kernel  subsample             Image.cpp:198-235 (masks :256-309)
//   plane_block_kernel      dctArai / dctMat / dctDirect (Dct.hpp:47-276) per 8x8
//                           block, optionally followed by quantize (Coding.hpp:84-97),
//                           into a double plane, an int plane, or the int16 MCU
//                           layout K2/K3 consume (writeJPEG's blocks, Image.cpp:540-636)
//   plane_quant_kernel      quantize per block    Coding.hpp:84-97
// All elementwise / blockwise over HBM, coalesced along rows: HBM-bound, no MFMA.
#include "arai.hpp"
#include "device_common.hpp"
#include "planes.hpp"

namespace jpge {
namespace {
using namespace dev;

// Image.cpp:131-134 (float literals, widened in the double arithmetic)
constexpr float kFlat[3] = {.0f, 256 / 2.f, 256 / 2.f};
constexpr float kYv[3] = {.299f, .587f, .114f};
constexpr float kCb[3] = {-.1687f, -.3312f, .5f};
constexpr float kCr[3] = {.5f, -.4186f, -.0813f};
// Image.cpp:159-162
constexpr float kRr[3] = {1.f, .0f, 1.402f};
constexpr float kRg[3] = {1.f, -.344f, -.714f};
constexpr float kRb[3] = {1.f, 1.772f, .0f};

__global__ __launch_bounds__(256) void plane_color_kernel(PlaneColorArgs a) {
    for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < a.n; x += (size_t)gridDim.x * blockDim.x) {
        const double p0 = a.in0[x], p1 = a.in1[x], p2 = a.in2[x];
        if (a.to_ycc) {  // Image.cpp:141-143
            a.out0[x] = kFlat[0] + (kYv[0] * p0 + kYv[1] * p1 + kYv[2] * p2) - 128;
            a.out1[x] = kFlat[1] + (kCb[0] * p0 + kCb[1] * p1 + kCb[2] * p2) - 128;
            a.out2[x] = kFlat[2] + (kCr[0] * p0 + kCr[1] * p1 + kCr[2] * p2) - 128;
        } else {  // Image.cpp:165-171
            const double y = p0 + 128, cb = p1 + 128, cr = p2 + 128;
            a.out0[x] = (kRr[0] * y + kRr[1] * cb + kRr[2] * cr);
            a.out1[x] = (kRg[0] * y + kRg[1] * cb + kRg[2] * cr);
            a.out2[x] = (kRb[0] * y + kRb[1] * cb + kRb[2] * cr);
        }
    }
}

// Image::subsample for one output sample.  The reference walks rows in steps of 2
// (or 1: `--y` when the mask neither skips a scanline nor averages), sums each run
// of `m` samples weighted by the mask row starting from 0, and for the averaging
// masks adds the next scanline's sum and divides by 4 (S420_m) or 2 (S420_lm).
__global__ __launch_bounds__(256) void plane_subsample_kernel(PlaneSubsampleArgs a) {
    const size_t n = (size_t)a.out_rows * a.out_cols;
    for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < n; o += (size_t)gridDim.x * blockDim.x) {
        const uint32_t oy = (uint32_t)(o / a.out_cols), ox = (uint32_t)(o % a.out_cols);
        const uint32_t y = a.row_step == 2 ? 2 * oy : oy;
        const uint32_t x = ox * a.m;
        const double* r0 = a.in + (size_t)y * a.cols + x;
        double top = 0;
        for (uint32_t k = 0; k < a.m; ++k) top += (double)a.mask[k] * r0[k];
        double v = top;
        if (a.avg_div) {
            const double* r1 = r0 + a.cols;
            double bot = 0;
            for (uint32_t k = 0; k < a.m; ++k) bot += (double)a.mask[k] * r1[k];
            v = (top + bot) / a.avg_div;
        }
        a.out[o] = v;
    }
}

// Where the 8 values of block b's row j come from / go to.
struct BlockPos {
    const double* src;  // row 0 of the block in its plane
    size_t pitch;       // plane row pitch (elements)
    int qsel;           // quantiser: 0 luma, 1 chroma
    size_t dst;         // sink index of row 0 (plane element, or coefficient)
    size_t dpitch;
};

// Block b of the sink's enumeration.  Planes: blocks in raster order of one plane.
// MCU layout (writeJPEG 4:2:0): b = m * 6 + k, Y00 Y01 Y10 Y11 Cb Cr, natural order
// inside a block (the coefficient layout of K1, kernels.hpp).
__device__ __forceinline__ BlockPos block_pos(const PlaneBlockArgs& a, size_t b) {
    BlockPos p;
    if (!a.mcu) {
        const uint32_t bw = a.cols / 8;
        const size_t by = b / bw, bx = b % bw;
        p.src = a.in0 + by * 8 * a.cols + bx * 8;
        p.pitch = a.cols;
        p.qsel = a.qsel;
        p.dst = by * 8 * a.cols + bx * 8;
        p.dpitch = a.cols;
        return p;
    }
    const size_t m = b / 6;
    const int k = (int)(b % 6);
    const uint32_t mw = a.cols / 16;
    const size_t mr = m / mw, mc = m % mw;
    if (k < 4) {
        p.src = a.in0 + (mr * 16 + (k >> 1) * 8) * a.cols + mc * 16 + (k & 1) * 8;
        p.pitch = a.cols;
        p.qsel = 0;
    } else {
        const size_t cc = a.cols / 2;
        p.src = (k == 4 ? a.in1 : a.in2) + mr * 8 * cc + mc * 8;
        p.pitch = cc;
        p.qsel = 1;
    }
    p.dst = b * 64;
    p.dpitch = 8;
    return p;
}

// 8 lanes per block (lane j of the block owns column j in the first pass and row j
// of the result), 32 blocks per 256-thread workgroup.
template <int kMode>
__global__ __launch_bounds__(256) void plane_block_kernel(PlaneBlockArgs a) {
    __shared__ double tmp[32][8][9];
    __shared__ double qt[2][64];
    const int t = threadIdx.x, lb = t >> 3, j = t & 7;
    for (int i = t; i < 128; i += 256) qt[i >> 6][i & 63] = a.q[i];
    __syncthreads();
    const size_t b = (size_t)blockIdx.x * 32 + lb;
    const bool ok = b < a.nblocks;
    const BlockPos p = block_pos(a, ok ? b : 0);
    double o[8];
    if (kMode == kDctArai) {
        // Dct.hpp:52-132: column j -> temp(j, k); then column j of temp -> y(j, k)
        double x[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = ok ? p.src[i * p.pitch + j] : 0.0;
        arai8(x, o);
#pragma unroll
        for (int k = 0; k < 8; ++k) tmp[lb][j][k] = o[k];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = tmp[lb][i][j];
        arai8(x, o);  // o[k] = y(j, k)
    } else if (kMode == kDctMatrix) {
        // Dct.hpp:264-276: first = X * A^T, Y = A * first (uBLAS prod: k ascending)
        double xr[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) xr[k] = ok ? p.src[j * p.pitch + k] : 0.0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) s += xr[k] * a.A[c * 8 + k];
            tmp[lb][j][c] = s;  // first(j, c)
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) s += a.A[j * 8 + k] * tmp[lb][k][c];
            o[c] = s;  // Y(j, c)
        }
    } else {
        // Dct.hpp:238-262: Y(jj, i) = sum_x sum_y X(y, x) A(i, x) A(jj, y); lane j owns
        // i = j (its outputs are column j of Y), written through LDS as rows
        double xs[64];
#pragma unroll
        for (int i = 0; i < 64; ++i) xs[i] = ok ? p.src[(i >> 3) * p.pitch + (i & 7)] : 0.0;
        for (int jj = 0; jj < 8; ++jj) {
            double s = 0.0;
            for (int x = 0; x < 8; ++x)
                for (int y = 0; y < 8; ++y) s += xs[y * 8 + x] * a.A[j * 8 + x] * a.A[jj * 8 + y];
            tmp[lb][jj][j] = s;
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 8; ++c) o[c] = tmp[lb][j][c];
    }
    if (!ok) return;
    // row j of the block's result -> the sink
    if (a.sink == kSinkDouble) {
#pragma unroll
        for (int c = 0; c < 8; ++c) a.out_d[p.dst + j * p.dpitch + c] = o[c];
        return;
    }
    // quantize, Coding.hpp:92-94: (int)std::round(m / table), natural index
    int qv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) qv[c] = (int)round(o[c] / qt[p.qsel][j * 8 + c]);
    if (a.sink == kSinkInt) {
#pragma unroll
        for (int c = 0; c < 8; ++c) a.out_i[p.dst + j * p.dpitch + c] = qv[c];
    } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) a.out_h[p.dst + j * p.dpitch + c] = (int16_t)qv[c];
    }
}

__global__ __launch_bounds__(256) void plane_quant_kernel(PlaneQuantArgs a) {
    const size_t n = (size_t)a.rows * a.cols;
    for (size_t x = blockIdx.x * (size_t)blockDim.x + threadIdx.x; x < n; x += (size_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(x / a.cols) & 7, c = (uint32_t)(x % a.cols) & 7;
        a.out[x] = (int)round(a.in[x] / a.q[r * 8 + c]);
    }
}

uint32_t stride_grid(size_t n) {
    const size_t g = (n + 255) / 256;
    return (uint32_t)(g < 8192 ? (g ? g : 1) : 8192);
}

}  // namespace

hipError_t launch_plane_color(const PlaneColorArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(plane_color_kernel, dim3(stride_grid(a.n)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_plane_subsample(const PlaneSubsampleArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(plane_subsample_kernel, dim3(stride_grid((size_t)a.out_rows * a.out_cols)), dim3(256), 0, s,
                       a);
    return hipGetLastError();
}

hipError_t launch_plane_block(const PlaneBlockArgs& a, int mode, hipStream_t s) {
    const dim3 grid((uint32_t)((a.nblocks + 31) / 32));
    if (a.nblocks == 0) return hipSuccess;
    switch (mode) {
        case kDctArai: hipLaunchKernelGGL(plane_block_kernel<kDctArai>, grid, dim3(256), 0, s, a); break;
        case kDctMatrix: hipLaunchKernelGGL(plane_block_kernel<kDctMatrix>, grid, dim3(256), 0, s, a); break;
        case kDctSimple: hipLaunchKernelGGL(plane_block_kernel<kDctSimple>, grid, dim3(256), 0, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_plane_quant(const PlaneQuantArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(plane_quant_kernel, dim3(stride_grid((size_t)a.rows * a.cols)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace jpge
