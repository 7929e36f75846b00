// Host check of K1's quantiser fast path (fdct.hip quant_fix16 / quant_row): for every
// quantiser 1..255 and every Arai column scale, random and adversarial row outputs w,
// y = fma(w, fl(s_u / q), 1.5 * 2^36 + 0x8001 * 2^-16) must give the reference's
// (int)round(fl(w * s_u) / q) (Coding.hpp:92-94 after Dct.hpp:124-131) in the high half
// of its low word whenever the low half exceeds 2; lanes at or below 2 take the exact
// path on the GPU.  IEEE fma on the host is the GPU's v_fma_f64.  Exit 0 = no mismatch.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "constants.hpp"

int main(int argc, char** argv) {
    const int per = argc > 1 ? atoi(argv[1]) : 4000;
    const double kS[8] = {jpge::kS0, jpge::kS1, jpge::kS2, jpge::kS3, jpge::kS4, jpge::kS5, jpge::kS6, jpge::kS7};
    const double magic = 103079215104.50002;
    std::mt19937_64 rng(2024);
    std::uniform_real_distribution<double> uni(-1.0, 1.0);
    long checked = 0, exact_path = 0, bad = 0;
    for (int q = 1; q <= 255; ++q)
        for (int u = 0; u < 8; ++u) {
            const double s = kS[u], c = s / q;
            const double wmax = 2040.0 / s;  // |w s| < 2^11 (8-bit samples)
            for (int i = 0; i < per; ++i) {
                double w;
                switch (i % 4) {
                    case 0: w = uni(rng) * wmax; break;  // anywhere
                    case 1: {  // near a half-integer quotient
                        const double k = std::floor(uni(rng) * 2040.0 / q) + 0.5;
                        w = (k * q) / s + uni(rng) * 1e-9 * wmax;
                        break;
                    }
                    case 2: {  // exactly on a half-integer of the unrounded quotient's neighbourhood
                        const double k = std::floor(uni(rng) * 2040.0 / q) + 0.5;
                        w = std::nextafter((k * q) / s, uni(rng) > 0 ? INFINITY : -INFINITY);
                        break;
                    }
                    default: w = std::round(uni(rng) * wmax * 8.0) / 8.0;  // dyadic values
                }
                const int ref = (int)std::round((w * s) / q);
                const double y = std::fma(w, c, magic);
                uint64_t bits;
                std::memcpy(&bits, &y, 8);
                const uint32_t t = (uint32_t)bits;
                ++checked;
                if ((t & 0xFFFF) <= 2) {
                    ++exact_path;
                    continue;
                }
                const int fast = (int16_t)(t >> 16);
                if (fast != ref && ++bad <= 10)
                    std::printf("mismatch q=%d u=%d w=%.17g: fast %d ref %d\n", q, u, w, fast, ref);
            }
        }
    std::printf("%ld values, %ld on the exact path, %ld mismatches\n", checked, exact_path, bad);
    return bad ? 1 : 0;
}
