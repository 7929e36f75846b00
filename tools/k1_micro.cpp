// K1 micro-benchmark (diagnostic, not part of the product or tests): times
// launch_fdct alone over a ring of distinct HBM-resident frames with HIP events
// and prints a checksum of the coefficients, so kernel variants can be compared
// for speed and output.  Build: see tools/k1_micro.sh.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#include "kernels.hpp"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const uint32_t W = argc > 1 ? atoi(argv[1]) : 3840, H = argc > 2 ? atoi(argv[2]) : 2160;
    const int nf = argc > 3 ? atoi(argv[3]) : 16, iters = argc > 4 ? atoi(argv[4]) : 20;
    const int quality = argc > 5 ? atoi(argv[5]) : 90;
    jpge::Geometry g;
    g.width = W;
    g.height = H;
    g.mw = (W + 15) / 16;
    g.mh = (H + 15) / 16;
    const size_t stride = (size_t)W * 3;
    const size_t fbytes = stride * H, cbytes = (size_t)g.nblocks() * 64 * 2;
    std::vector<uint8_t> host(fbytes);
    uint8_t* rgb;
    int16_t* coef;
    CK(hipMalloc(&rgb, fbytes * nf));
    CK(hipMalloc(&coef, cbytes * nf));
    for (int f = 0; f < nf; ++f) {
        uint64_t s = 1000 + f;
        for (uint32_t y = 0; y < H; ++y)
            for (uint32_t x = 0; x < W; ++x) {
                const uint64_t r = splitmix(s);
                for (int c = 0; c < 3; ++c) {
                    int v = (int)((x * (3 + c) + y * (5 - c)) / 7 % 256) + (int)((r >> (8 * c)) & 31) - 16;
                    host[(size_t)y * stride + x * 3 + c] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
                }
            }
        CK(hipMemcpy(rgb + fbytes * f, host.data(), fbytes, hipMemcpyHostToDevice));
    }
    // IJG-scaled reference tables (Image.cpp:850-869 at Q50)
    static const int lum[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
    static const int chr[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
    const int sc = quality < 50 ? 5000 / quality : 200 - 2 * quality;
    jpge::FdctArgs a{};
    a.stride = stride;
    a.g = g;
    a.maxval = argc > 6 ? atoi(argv[6]) : 255;
    a.solo = getenv("K1_SHARED") == nullptr;
    for (int i = 0; i < 64; ++i) {
        int t = (lum[i] * sc + 50) / 100, u = (chr[i] * sc + 50) / 100;
        a.q[i] = (uint8_t)(t < 1 ? 1 : t > 255 ? 255 : t);
        a.q[64 + i] = (uint8_t)(u < 1 ? 1 : u > 255 ? 255 : u);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // kernel-exact times of every timed launch (events bound to the dispatch, KTimer)
    std::vector<hipEvent_t> kev(2 * iters * nf);
    for (auto& e : kev) CK(hipEventCreate(&e));
    int kn = -1;
    auto run = [&](int f) {
        a.rgb = rgb + fbytes * f;
        a.coef = coef + (cbytes / 2) * f;
        jpge::KTimer t{};
        if (kn >= 0) t = jpge::KTimer{kev[2 * kn], kev[2 * kn + 1]}, ++kn;
        CK(jpge::launch_fdct(a, 0, kn >= 0 ? &t : nullptr));
    };
    for (int w = 0; w < 3; ++w)
        for (int f = 0; f < nf; ++f) run(f);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    kn = 0;
    for (int it = 0; it < iters; ++it)
        for (int f = 0; f < nf; ++f) run(f);
    kn = -1;
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / (iters * nf);
    {
        std::vector<double> k;
        for (int i = 0; i < iters * nf; ++i) {
            float m;
            CK(hipEventElapsedTime(&m, kev[2 * i], kev[2 * i + 1]));
            k.push_back(1000.0 * m);
        }
        std::sort(k.begin(), k.end());
        double sum = 0;
        for (double v : k) sum += v;
        std::printf("kernel-exact: mean %.2f us  min %.2f  median %.2f  max %.2f\n", sum / k.size(), k[0],
                    k[k.size() / 2], k.back());
    }
#ifdef JPGE_STAMPS
    {  // per-workgroup phase stamps of one more launch (s_memrealtime, 100 MHz)
        const uint32_t G = jpge::fdct_grid(g, a.solo);
        uint64_t* dbg;
        CK(hipMalloc(&dbg, (size_t)G * jpge::kStampSlots * 8));
        CK(hipMemset(dbg, 0, (size_t)G * jpge::kStampSlots * 8));
        a.dbg = dbg;
        run(0);
        CK(hipDeviceSynchronize());
        std::vector<uint64_t> st((size_t)G * jpge::kStampSlots);
        CK(hipMemcpy(st.data(), dbg, st.size() * 8, hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull;
        for (uint32_t w = 0; w < G; ++w) t0 = std::min(t0, st[w * jpge::kStampSlots + 1]);
        const char* nm[8] = {"prologue done", "start", "tile0", "tile1", "tile2", "tile3", "tile4+", "end"};
        for (int k = 0; k < 8; ++k) {
            std::vector<double> v;
            for (uint32_t w = 0; w < G; ++w) {
                const uint64_t x = st[w * jpge::kStampSlots + k];
                if (x) v.push_back((x - t0) * 0.01);
            }
            if (v.empty()) continue;
            std::sort(v.begin(), v.end());
            std::printf("  %-14s n=%5zu  min %6.2f  p10 %6.2f  med %6.2f  p90 %6.2f  max %6.2f us\n", nm[k], v.size(), v[0],
                        v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
        }
        for (int k = 2; k < 8; k += 5) {  // by blockIdx % 8 (the XCD under round-robin dispatch)
            std::printf("  %-8s by XCD:", nm[k]);
            for (uint32_t x = 0; x < 8; ++x) {
                std::vector<double> v;
                for (uint32_t w = x; w < G; w += 8) {
                    const uint64_t y = st[w * jpge::kStampSlots + k];
                    if (y) v.push_back((y - t0) * 0.01);
                }
                std::sort(v.begin(), v.end());
                if (!v.empty()) std::printf(" %5.1f/%5.1f", v[v.size() / 2], v.back());
            }
            std::printf("  (median/max us)\n");
        }
        a.dbg = nullptr;
    }
#endif
    std::vector<int16_t> hc(cbytes / 2);
    uint64_t h = 1469598103934665603ull;
    for (int f = 0; f < nf; f += 5) {
        CK(hipMemcpy(hc.data(), coef + (cbytes / 2) * f, cbytes, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < hc.size(); ++i) h = (h ^ (uint16_t)hc[i]) * 1099511628211ull;
    }
    const double bytes = 6.0 * W * H;
    std::printf("K1 %ux%u q%d maxval %d: %.2f us/launch  %.1f GB/s  frac %.3f  checksum %016llx\n", W, H, quality,
                a.maxval, us, bytes / us / 1e3, bytes / us / 1e3 / 8000.0, (unsigned long long)h);
    return 0;
}
