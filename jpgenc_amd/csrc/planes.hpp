// Parameter blocks of the plane stage kernels (planes.hip): the reference's Image
// stage methods on fp64 planes (row-major, `cols` elements per row).
#pragma once
#include <cstddef>
#include <cstdint>

#include <hip/hip_runtime_api.h>

namespace jpge {

// DCT modes, Image::DCTMode (Image.hpp:54-59)
constexpr int kDctSimple = 0, kDctMatrix = 1, kDctArai = 2;
// block kernel sinks
constexpr int kSinkDouble = 0, kSinkInt = 1, kSinkMcu16 = 2;

struct PlaneColorArgs {  // convertToColorSpace, Image.cpp:112-179
    const double *in0, *in1, *in2;
    double *out0, *out1, *out2;
    size_t n;
    int to_ycc;  // 1: RGB -> YCbCr, 0: YCbCr -> RGB
};

struct PlaneSubsampleArgs {  // Image::subsample, Image.cpp:198-235
    const double* in;
    double* out;
    uint32_t cols;                 // input row length
    uint32_t out_rows, out_cols;
    uint32_t m;                    // mask row length (2, or 4 for S411)
    uint8_t mask[4];               // mask row weights
    uint32_t row_step;             // 2: rows in pairs (S420, S420_m, S420_lm), 1: every row (S422, S411)
    uint32_t avg_div;              // 4 (S420_m), 2 (S420_lm), 0: no averaging
};

struct PlaneBlockArgs {  // dctArai / dctMat / dctDirect per 8x8 block, then optionally quantize
    const double *in0, *in1, *in2;  // plane (in0), or Y, Cb, Cr for the MCU sink
    uint32_t cols;                  // plane row length (MCU sink: the Y plane's; chroma = cols / 2)
    uint64_t nblocks;               // blocks of the plane, or 6 x MCUs
    int mcu;                        // 1: blocks in writeJPEG's MCU order (4:2:0)
    int qsel;                       // plane sink: quantiser 0 luma / 1 chroma
    int sink;                       // kSink*
    double q[128];                  // luma, chroma quantisers (natural order) as doubles
    double A[64];                   // Dct.hpp:220-235 matrix A (Matrix / Simple modes)
    double* out_d;
    int32_t* out_i;
    int16_t* out_h;
};

struct PlaneQuantArgs {  // quantize, Coding.hpp:84-97, over a plane of blocks
    const double* in;
    int32_t* out;
    uint32_t rows, cols;
    double q[64];
};

hipError_t launch_plane_color(const PlaneColorArgs& a, hipStream_t s);
hipError_t launch_plane_subsample(const PlaneSubsampleArgs& a, hipStream_t s);
hipError_t launch_plane_block(const PlaneBlockArgs& a, int mode, hipStream_t s);
hipError_t launch_plane_quant(const PlaneQuantArgs& a, hipStream_t s);

}  // namespace jpge
