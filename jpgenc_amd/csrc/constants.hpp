// Arai FDCT constants, Dct.hpp:21-43 — cos(k*pi/16) as evaluated by glibc at
// static initialisation with Boost's pi/root_two.  Hard-coded
// bit patterns: device cos() must never be used for them.  Shared by the
// kernels and by jpge_arai_constants() so the tests can pin them.
#pragma once

namespace jpge {
constexpr double kA1 = 0x1.6a09e667f3bcdp-1;  // c4
constexpr double kA2 = 0x1.1517a7bdb3894p-1;  // c2 - c6
constexpr double kA3 = 0x1.6a09e667f3bcdp-1;  // c4
constexpr double kA4 = 0x1.4e7ae9144f0fcp+0;  // c6 + c2
constexpr double kA5 = 0x1.87de2a6aea964p-2;  // c6
constexpr double kS0 = 0x1.6a09e667f3bccp-2;  // 1 / (2 sqrt 2)
constexpr double kS1 = 0x1.0503ed17cba53p-2;  // 1 / (4 c_k)
constexpr double kS2 = 0x1.1517a7bdb3895p-2;
constexpr double kS3 = 0x1.33e37a1e0173ep-2;
constexpr double kS4 = 0x1.6a09e667f3bccp-2;
constexpr double kS5 = 0x1.ccc9aefb18d57p-2;
constexpr double kS6 = 0x1.4e7ae9144f0fbp-1;
constexpr double kS7 = 0x1.480d9d073b426p+0;
}  // namespace jpge
