// The Arai-Agui-Nakajima 8-point forward DCT pass of Dct.hpp:62-131 on the
// device (fp64, the reference's operation order, no contraction), shared by the
// fused transform kernel (fdct.hip) and the plane stage kernels (planes.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "constants.hpp"

#pragma clang fp contract(off)

namespace jpge {
namespace dev {

// One 8-point Arai pass, Dct.hpp:62-131 (same op order for both passes), up to
// the final scaling: o[k] = w[k] * kS_k.
__device__ __forceinline__ void arai8_unscaled(const double x[8], double w[8]) {
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
    w[0] = t0; w[4] = t1; w[2] = v2; w[6] = v3;
    w[5] = w4; w[1] = w5; w[7] = w6; w[3] = w7;
}
constexpr double kS[8] = {kS0, kS1, kS2, kS3, kS4, kS5, kS6, kS7};
__device__ __forceinline__ void arai8(const double x[8], double o[8]) {
    double w[8];
    arai8_unscaled(x, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = w[k] * kS[k];
}

}  // namespace dev
}  // namespace jpge
