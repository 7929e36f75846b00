// VALU issue-rate probe (diagnostic): times long unrolled chains of one fp64 /
// conversion instruction kind over 8 independent accumulators per lane, a full
// chip of waves, and prints cycles per wave-instruction.  Used to decide which
// instructions the transform kernel should avoid.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kIters = 4096;

template <int K>
__global__ __launch_bounds__(256) void probe(double* out, double seed, uint32_t useed) {
    double v[8];
    uint32_t u[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = seed + threadIdx.x + i;
        u[i] = useed + threadIdx.x * 7 + i;
    }
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (K == 0) v[i] = v[i] + 1.0000001;             // v_add_f64
            if constexpr (K == 1) v[i] = v[i] * 1.0000001;             // v_mul_f64
            if constexpr (K == 2) v[i] = __builtin_fma(v[i], 1.0000001, 0.5);  // v_fma_f64
            if constexpr (K == 3) v[i] = v[i] + (double)(u[i] += 3);  // v_cvt_f64_u32 + add + int add
            if constexpr (K == 4) v[i] = __builtin_rint(v[i]) + 0.25;  // v_rndne_f64 + add
            if constexpr (K == 5) u[i] += (uint32_t)(int)v[i] + 1;     // v_cvt_i32_f64 + adds
            if constexpr (K == 6) u[i] = (u[i] ^ 0x9E3779B9u) + (u[i] >> 3);  // 3 int32 ops
            if constexpr (K == 7) v[0] = v[0] + 1.0000001;                // dependent add_f64 chain
            if constexpr (K == 8) v[i & 1] = v[i & 1] + 1.0000001;        // two chains
            if constexpr (K == 9) v[i & 3] = v[i & 3] + 1.0000001;        // four chains
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i] + u[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 256 * 8;  // 256*8: 8 waves per SIMD
    double* out;
    hipMalloc(&out, sizeof(double) * grid * 256);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"add_f64", "mul_f64", "fma_f64", "cvt_f64_u32+add_f64+add_u32", "rndne_f64+add_f64",
                           "cvt_i32_f64+2 add_u32", "3 int32 ops", "add_f64 1 chain", "add_f64 2 chains", "add_f64 4 chains"};
    auto run = [&](auto kern, const char* name) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 1.0, 3u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            // wave-instructions per SIMD: waves per SIMD (grid*4/1024) * iters * 8
            const double winst = (double)grid * 4 / 1024 * kIters * 8;
            if (rep) std::printf("%-32s %8.3f ms  %6.2f ns per wave-op per SIMD  (%.2f cycles at 2.4 GHz)\n", name, ms,
                                 ms * 1e6 / winst, ms * 1e6 / winst * 2.4);
        }
    };
    run(probe<0>, names[0]);
    run(probe<1>, names[1]);
    run(probe<2>, names[2]);
    run(probe<3>, names[3]);
    run(probe<4>, names[4]);
    run(probe<5>, names[5]);
    run(probe<6>, names[6]);
    run(probe<7>, names[7]);
    run(probe<8>, names[8]);
    run(probe<9>, names[9]);
    return 0;
}
