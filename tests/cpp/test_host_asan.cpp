// Host-code driver for the sanitizer build (`make asan`, run by tests/test_asan.py):
// every host-only entry point of libjpge's C ABI on valid, adversarial and corrupted
// inputs, built with -fsanitize=address,undefined.  It checks the outcomes it can
// check cheaply (round trips, statuses); its main product is the sanitizer's verdict
// on the host code: the PPM tokenizer, the per-frame Huffman builder
// (heap pops with their one-step look-ahead at every heap size, the hash-order
// emulation), the decode utilities, stripe placement and the coding primitives.
//
// Usage: test_host_asan <ppm dir> [file.jpg ...]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <algorithm>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "jpge.h"

static int g_checks = 0, g_fail = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        ++g_checks;                                                           \
        if (!(c)) {                                                           \
            ++g_fail;                                                         \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
        }                                                                     \
    } while (0)

static std::vector<uint8_t> read_file(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

// PPM front end: every reference test image, each prefix of the small ones, and
// random corruptions (bytes flipped, tokens replaced) must parse or fail cleanly.
static void ppm(const std::string& dir, std::mt19937_64& rng) {
    DIR* d = opendir(dir.c_str());
    CHECK(d != nullptr);
    if (!d) return;
    std::vector<std::string> files;
    while (dirent* e = readdir(d)) {
        const std::string n = e->d_name;
        if (n.size() > 4 && n.substr(n.size() - 4) == ".ppm") files.push_back(dir + "/" + n);
    }
    closedir(d);
    CHECK(!files.empty());
    for (const auto& p : files) {
        const std::vector<uint8_t> buf = read_file(p);
        uint32_t w = 0, h = 0;
        int mv = 0;
        CHECK(jpge_ppm_info(buf.data(), buf.size(), &w, &h, &mv) == JPGE_OK);
        std::vector<uint8_t> rgb((size_t)w * h * 3);
        CHECK(jpge_parse_ppm(buf.data(), buf.size(), rgb.data(), rgb.size(), &w, &h, &mv) == JPGE_OK);
        // too small an output: refused, nothing written past cap
        if (!rgb.empty()) {
            std::vector<uint8_t> small(rgb.size() - 1);
            CHECK(jpge_parse_ppm(buf.data(), buf.size(), small.data(), small.size(), &w, &h, &mv) != JPGE_OK);
        }
        // every prefix (exact-size copies, so a read past the end is caught)
        const size_t lim = buf.size() < 4096 ? buf.size() : 4096;
        for (size_t n = 0; n < lim; ++n) {
            std::vector<uint8_t> pre(buf.begin(), buf.begin() + (long)n);
            std::vector<uint8_t> out(rgb.size() + 1);
            uint32_t pw, ph;
            int pm;
            (void)jpge_ppm_info(pre.data(), pre.size(), &pw, &ph, &pm);
            (void)jpge_parse_ppm(pre.data(), pre.size(), out.data(), out.size(), &pw, &ph, &pm);
        }
        // corruptions
        for (int it = 0; it < 200; ++it) {
            std::vector<uint8_t> c = buf;
            const int edits = 1 + (int)(rng() % 4);
            for (int e = 0; e < edits && !c.empty(); ++e) {
                const size_t at = rng() % (c.size() < 64 ? c.size() : 64 + rng() % (c.size() - 63));
                static const char* toks[] = {" ", "\n", "#x\n", "-1", "65536", "0", "99999999999", "P3", "P6", "P7", "\t"};
                if (rng() & 1) {
                    c[at] = (uint8_t)rng();
                } else {
                    const char* t = toks[rng() % (sizeof(toks) / sizeof(*toks))];
                    c.insert(c.begin() + (long)at, t, t + std::strlen(t));
                }
            }
            uint32_t cw = 0, ch = 0;
            int cm = 0;
            if (jpge_ppm_info(c.data(), c.size(), &cw, &ch, &cm) == JPGE_OK && (uint64_t)cw * ch <= (1u << 22)) {
                std::vector<uint8_t> out((size_t)cw * ch * 3);
                (void)jpge_parse_ppm(c.data(), c.size(), out.data(), out.size(), &cw, &ch, &cm);
            }
        }
    }
}

// Huffman tables from histograms: sizes 1..256 symbols, heavy ties (counts from a
// small range, so package weights tie at every level), skewed counts (codes limited
// to 15 bits), and the text form round-tripped through jpge_huffman_decode.
static void huffman(std::mt19937_64& rng) {
    for (int it = 0; it < 3000; ++it) {
        uint32_t counts[256] = {0};
        uint64_t first[256];
        for (int s = 0; s < 256; ++s) first[s] = ~0ull;
        const int n = 1 + (int)(it % 256);
        const int mode = (int)(rng() % 4);
        std::vector<int> syms(256);
        for (int s = 0; s < 256; ++s) syms[s] = s;
        std::shuffle(syms.begin(), syms.end(), rng);
        for (int i = 0; i < n; ++i) {
            uint32_t c;
            switch (mode) {
                case 0: c = 1 + (uint32_t)(rng() % 3); break;                            // ties everywhere
                case 1: c = 1 + (uint32_t)(rng() % 1000); break;                         // mixed
                case 2: c = i < 2 ? 1u << (20 + i) : 1 + (uint32_t)(rng() % 2); break;   // deep trees
                default: c = (uint32_t)1 << (rng() % 24); break;                         // powers of two
            }
            counts[syms[i]] = c;
            first[syms[i]] = (uint64_t)(rng() % (1ull << 40));
        }
        uint8_t bits[16], huffval[256], len[256];
        uint32_t code[256];
        int nsym = 0;
        CHECK(jpge_huffman_table(counts, first, bits, huffval, &nsym, code, len) == JPGE_OK);
        CHECK(nsym == n);
        int tot = 0;
        for (int l = 0; l < 16; ++l) tot += bits[l];
        CHECK(tot == n);
        for (int i = 0; i < nsym; ++i) CHECK(len[huffval[i]] >= 1 && len[huffval[i]] <= 16);
    }
    // the text form and its decoder
    for (int it = 0; it < 300; ++it) {
        const int alpha = 1 + (int)(rng() % 300);
        const size_t n = 1 + rng() % 2000;
        std::vector<int> text(n);
        for (auto& t : text) t = (int)(rng() % (uint64_t)alpha) - alpha / 2;
        std::vector<int> syms(n), lens(n);
        std::vector<uint32_t> codes(n);
        int nsym = 0;
        CHECK(jpge_huffman_text(text.data(), n, syms.data(), lens.data(), codes.data(), &nsym) == JPGE_OK);
        // encode with the table, decode back
        std::vector<uint8_t> buf(n * 4 + 8, 0);
        uint64_t nbits = 0;
        std::vector<uint32_t> tsym(nsym), tcode(nsym);
        std::vector<uint8_t> tlen(nsym);
        for (int i = 0; i < nsym; ++i) {
            tsym[i] = (uint32_t)syms[i];
            tcode[i] = codes[i];
            tlen[i] = (uint8_t)lens[i];
        }
        for (int t : text) {
            int k = 0;
            while (k < nsym && syms[k] != t) ++k;
            CHECK(k < nsym);
            if (k == nsym) return;
            for (int b = lens[k] - 1; b >= 0; --b, ++nbits)
                if ((codes[k] >> b) & 1) buf[nbits >> 3] |= (uint8_t)(0x80 >> (nbits & 7));
        }
        std::vector<uint8_t> exact(buf.begin(), buf.begin() + (long)((nbits + 7) / 8));
        std::vector<int> dec(n);
        size_t got = 0;
        CHECK(jpge_huffman_decode(exact.data(), nbits, tsym.data(), tcode.data(), tlen.data(), nsym, dec.data(), n,
                                  &got) == JPGE_OK);
        CHECK(got == n && dec == text);
        // a short output buffer and a count-only call
        if (n > 1) (void)jpge_huffman_decode(exact.data(), nbits, tsym.data(), tcode.data(), tlen.data(), nsym,
                                             dec.data(), n / 2, &got);
        (void)jpge_huffman_decode(exact.data(), nbits, tsym.data(), tcode.data(), tlen.data(), nsym, nullptr, 0, &got);
    }
}

// .jpg decode utility on encoder streams, their truncations and corruptions.
static void decode(const std::vector<std::string>& jpgs, std::mt19937_64& rng) {
    for (const auto& p : jpgs) {
        const std::vector<uint8_t> jpg = read_file(p);
        jpge_decoded info;
        CHECK(jpge_decode_coeffs(jpg.data(), jpg.size(), &info, nullptr, nullptr, nullptr, 0, 0) == JPGE_OK);
        std::vector<int16_t> y(info.y_blocks * 64), cb(info.c_blocks * 64), cr(info.c_blocks * 64);
        CHECK(jpge_decode_coeffs(jpg.data(), jpg.size(), &info, y.data(), cb.data(), cr.data(), info.y_blocks,
                                 info.c_blocks) == JPGE_OK);
        // too small planes: refused
        if (info.y_blocks > 1) {
            std::vector<int16_t> ys((info.y_blocks - 1) * 64);
            CHECK(jpge_decode_coeffs(jpg.data(), jpg.size(), &info, ys.data(), cb.data(), cr.data(), info.y_blocks - 1,
                                     info.c_blocks) != JPGE_OK);
        }
        for (int it = 0; it < 120; ++it) {
            std::vector<uint8_t> c(jpg.begin(), jpg.begin() + (long)(it < 40 ? rng() % jpg.size() : jpg.size()));
            if (it >= 40 && !c.empty())
                for (int e = 0; e < 3; ++e) c[rng() % c.size()] = (uint8_t)rng();
            jpge_decoded ci;
            if (jpge_decode_coeffs(c.data(), c.size(), &ci, nullptr, nullptr, nullptr, 0, 0) != JPGE_OK) continue;
            if (ci.y_blocks > (1u << 20) || ci.c_blocks > (1u << 20)) continue;
            std::vector<int16_t> a(ci.y_blocks * 64), b(ci.c_blocks * 64), d(ci.c_blocks * 64);
            (void)jpge_decode_coeffs(c.data(), c.size(), &ci, a.data(), b.data(), d.data(), ci.y_blocks, ci.c_blocks);
        }
    }
    // the inverse DCT on random blocks
    std::uniform_real_distribution<double> u(-1024.0, 1024.0);
    for (int it = 0; it < 200; ++it) {
        double in[64], out[64];
        for (double& v : in) v = u(rng);
        jpge_idct8x8(in, out);
    }
}

// Stripe placement over random summaries (whole-frame and restart stripes).
static void stripes(std::mt19937_64& rng) {
    for (int it = 0; it < 2000; ++it) {
        const int n = 1 + (int)(rng() % 16);
        const bool restart = rng() & 1;
        std::vector<jpge_stripe_summary> all(n);
        for (auto& s : all) {
            std::memset(&s, 0, sizeof(s));
            s.bits = 8 + rng() % 100000;
            for (auto& f : s.ff) f = (uint32_t)(rng() % 64);
            s.head = (uint32_t)(rng() & 0xFF);
            s.tail = (uint32_t)(rng() & 0xFF);
            s.restart = restart;
        }
        size_t prev = 0, total = 0, off = 0;
        for (int i = 0; i < n; ++i) {
            CHECK(jpge_stripe_place(all.data(), n, i, 600, &off, &total) == JPGE_OK);
            CHECK(i == 0 ? off == 0 : off >= prev);
            prev = off;
        }
        CHECK(jpge_stripe_place(all.data(), n, n, 600, &off, &total) != JPGE_OK);
        CHECK(jpge_stripe_place(all.data(), n, -1, 600, &off, &total) != JPGE_OK);
        CHECK(jpge_stripe_place(nullptr, n, 0, 600, &off, &total) != JPGE_OK);
    }
}

// Coding primitives and small helpers.
static void coding(std::mt19937_64& rng) {
    for (int q = 1; q <= 100; ++q) {
        uint8_t qy[64], qc[64];
        CHECK(jpge_quality_tables(q, qy, qc) == JPGE_OK);
    }
    CHECK(jpge_quality_tables(0, nullptr, nullptr) != JPGE_OK);
    for (uint32_t w : {1u, 7u, 16u, 33u, 1920u})
        for (uint32_t h : {1u, 9u, 16u, 17u, 1080u}) {
            std::vector<uint8_t> f((size_t)w * h * 3 + 5);
            for (int kind = 0; kind < 3; ++kind) CHECK(jpge_synth_rgb8(rng(), w, h, kind, f.data(), (size_t)w * 3) == JPGE_OK);
            CHECK(jpge_max_jpeg_bytes(w, h) > 600);
        }
    for (int it = 0; it < 2000; ++it) {
        int v = (int)(rng() % 8192) - 4096;
        if (it < 40) v = it - 20;
        uint16_t cat = 99;
        uint32_t code = 0;
        CHECK(jpge_category_code(v, &cat, &code) == JPGE_OK);
        CHECK(cat <= 13);
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: test_host_asan <ppm dir> [file.jpg ...]\n");
        return 2;
    }
    std::mt19937_64 rng(12345);
    std::vector<std::string> jpgs(argv + 2, argv + argc);
    ppm(argv[1], rng);
    huffman(rng);
    decode(jpgs, rng);
    stripes(rng);
    coding(rng);
    std::printf("%d checks, %d failed\n", g_checks, g_fail);
    return g_fail ? 1 : 0;
}
