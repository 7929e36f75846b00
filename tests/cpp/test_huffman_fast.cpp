// Cross-check of jpge's array emulation of the reference's Huffman construction
// (huffman.cpp build_table / build_code_lengths: hash order, binary heap, package
// DAG) against the same algorithm run on std::unordered_map / std::priority_queue
// (build_table_std / build_code_lengths_std, which tests/test_host.py pins to the
// reference's own Huffman.cpp).  Random histograms with heavy ties, random first-
// occurrence orders, symbol texts with negative and large ints.  Exit 0 = all equal.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "huffman.hpp"

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    int bad = 0;
    jpge::HuffTable t, u;
    for (int it = 0; it < iters; ++it) {
        uint32_t cc[256] = {0};
        uint64_t kk[256];
        const int ns = 1 + (int)(rng() % 256);
        const int mode = it % 7;
        const uint32_t maxc = mode == 0 ? 2 : mode == 1 ? 20 : mode == 2 ? 1000 : mode == 3 ? 3000000 : 2000000000u / 256;
        std::vector<int> perm(256);
        for (int i = 0; i < 256; ++i) perm[i] = i;
        std::shuffle(perm.begin(), perm.end(), rng);
        for (int i = 0; i < ns; ++i) cc[perm[i]] = 1 + (uint32_t)(rng() % maxc);
        if (mode == 5)  // log-uniform counts, like a frame's: ties among the rare symbols and their packages
            for (int i = 0; i < ns; ++i)
                cc[perm[i]] = (uint32_t)std::exp(std::uniform_real_distribution<double>(0.0, 20.0)(rng));
        if (mode == 6)  // a few powers of two and small counts: whole levels of tied packages, whose order repeats
            for (int i = 0; i < ns; ++i)
                cc[perm[i]] = rng() % 3 ? 1u + (uint32_t)(rng() % 4) : 1u << (rng() % 16);
        for (int s = 0; s < 256; ++s) kk[s] = rng() % (mode == 4 ? 300 : 100000000);  // (ties in keys: symbol order)
        const bool a = jpge::build_table(cc, kk, t), b = jpge::build_table_std(cc, kk, u);
        if (a != b || std::memcmp(&t, &u, sizeof t) != 0) {
            if (++bad <= 5) std::printf("table mismatch: iteration %d, %d symbols\n", it, ns);
        }
    }
    for (int it = 0; it < iters / 4; ++it) {  // symbol texts: arbitrary ints (the facade's generateHuffmanCode)
        const int ns = 1 + (int)(rng() % 300), len = 1 + (int)(rng() % 3000);
        std::vector<int> alpha(ns);
        for (auto& x : alpha) x = (int)(rng() % 200001) - 100000;
        std::sort(alpha.begin(), alpha.end());
        alpha.erase(std::unique(alpha.begin(), alpha.end()), alpha.end());
        std::vector<std::pair<int, int>> fc;
        std::vector<int> seen;
        for (int i = 0; i < len; ++i) {
            const int s = alpha[(size_t)(rng() % alpha.size()) * (rng() % 4 ? 1 : 0)];
            auto p = std::find(seen.begin(), seen.end(), s);
            if (p == seen.end()) {
                seen.push_back(s);
                fc.emplace_back(s, 1);
            } else {
                fc[p - seen.begin()].second++;
            }
        }
        std::vector<std::vector<int>> x, y;
        jpge::build_code_lengths(fc, x);
        jpge::build_code_lengths_std(fc, y);
        if (x != y && ++bad <= 10) std::printf("code-length mismatch: text %d, %zu symbols\n", it, fc.size());
    }
    std::printf("%d mismatches\n", bad);
    return bad ? 1 : 0;
}
