// Host table-build timing: the four Huffman tables of each frame of a recorded
// histogram set, built with build_table (the per-frame path), checked against
// build_table_std (standard containers).  Input: counts (frames x 1024 u32) and
// first-occurrence keys (frames x 1024 u64) as written by bench/tools; prints the median
// and minimum per frame over `reps` passes.
//   g++ -O2 -std=c++17 -Ijpgenc_amd/csrc tools/table_bench.cpp jpgenc_amd/csrc/huffman.cpp -o /tmp/tb
//   /tmp/tb counts.bin keys.bin [reps]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "huffman.hpp"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    FILE* fc = fopen(argv[1], "rb");
    FILE* fk = fopen(argv[2], "rb");
    if (!fc || !fk) return 2;
    std::vector<uint32_t> cnt;
    std::vector<uint64_t> key;
    uint32_t c[1024];
    uint64_t k[1024];
    while (fread(c, 4, 1024, fc) == 1024 && fread(k, 8, 1024, fk) == 1024) {
        cnt.insert(cnt.end(), c, c + 1024);
        key.insert(key.end(), k, k + 1024);
    }
    const int nf = (int)(cnt.size() / 1024);
    // correctness first
    for (int f = 0; f < nf; ++f)
        for (int t = 0; t < 4; ++t) {
            jpge::HuffTable a, b;
            const bool oa = jpge::build_table(&cnt[f * 1024 + t * 256], &key[f * 1024 + t * 256], a);
            const bool ob = jpge::build_table_std(&cnt[f * 1024 + t * 256], &key[f * 1024 + t * 256], b);
            if (oa != ob || memcmp(a.bits, b.bits, 17) || memcmp(a.huffval, b.huffval, 256) || memcmp(a.len, b.len, 256) ||
                memcmp(a.code, b.code, sizeof a.code)) {
                fprintf(stderr, "mismatch frame %d table %d\n", f, t);
                return 1;
            }
        }
    std::vector<double> per(nf, 1e30);
    for (int r = 0; r < reps; ++r)
        for (int f = 0; f < nf; ++f) {
            jpge::HuffTable out[4];
            const auto t0 = std::chrono::steady_clock::now();
            for (int t = 0; t < 4; ++t) jpge::build_table(&cnt[f * 1024 + t * 256], &key[f * 1024 + t * 256], out[t]);
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            per[f] = std::min(per[f], us);
        }
    std::vector<double> s = per;
    std::sort(s.begin(), s.end());
    double sum = 0;
    for (double v : per) sum += v;
    printf("%d frames: per frame (4 tables) min-over-passes: median %.2f us, mean %.2f us, min %.2f us\n", nf,
           s[nf / 2], sum / nf, s[0]);
    return 0;
}
