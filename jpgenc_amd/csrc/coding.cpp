// Coding.hpp's per-block primitives as C-ABI host functions (include/jpge.h), for the
// facade's free functions (jpge_image.hpp) and their known-answer tests.  The GPU
// encode path does not call these: K1-K3 compute the same quantities in their
// kernels (fdct.hip, stats.hip, entropy.hip).
#include <cmath>
#include <cstdlib>
#include <initializer_list>

#include "jpge.h"

namespace {
// zig-zag position -> natural index (the table of Coding.hpp:69-77)
constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
}  // namespace

extern "C" {

int jpge_zigzag_index(int i) { return (i < 0 || i >= 64) ? -1 : kZigzag[i]; }

int jpge_zigzag_block(const int32_t in[64], int32_t out[64]) {
    if (!in || !out) return JPGE_E_ARG;
    for (int p = 0; p < 64; ++p) out[p] = in[kZigzag[p]];
    return JPGE_OK;
}

int jpge_quantize_block(const double block[64], const double table[64], int32_t out[64]) {
    if (!block || !table || !out) return JPGE_E_ARG;
    for (int i = 0; i < 64; ++i) out[i] = static_cast<int>(std::round(block[i] / table[i]));
    return JPGE_OK;
}

int jpge_rle_ac(const int32_t* data, size_t n, int zigzag_scan, uint8_t* runs, int32_t* values, size_t cap,
                size_t* npairs) {
    if (!data || !npairs || n < 2 || (zigzag_scan && n != 64) || (cap && (!runs || !values))) return JPGE_E_ARG;
    size_t k = 0;
    auto emit = [&](unsigned run, int32_t v) {
        if (k < cap) {
            runs[k] = (uint8_t)run;
            values[k] = v;
        }
        ++k;
    };
    emit(0, data[0]);  // the DC pair, run 0
    unsigned zeros = 0;
    for (size_t i = 1; i < n; ++i) {
        const int32_t v = data[zigzag_scan ? kZigzag[i] : i];
        if (v == 0) {
            ++zeros;
            continue;
        }
        while (zeros > 15) {  // ZRL: sixteen zeros
            emit(15, 0);
            zeros -= 16;
        }
        emit(zeros, v);
        zeros = 0;
    }
    if (zeros > 0) emit(0, 0);  // EOB
    *npairs = k;
    return k > cap ? JPGE_E_NOSPACE : JPGE_OK;
}

int jpge_category_code(int32_t value, uint16_t* category, uint32_t* bits) {
    if (!category || !bits) return JPGE_E_ARG;
    const uint32_t a = (uint32_t)std::abs((long)value);
    if (a >= (1u << 15)) return JPGE_E_RANGE;
    uint16_t c = 0;
    while ((a >> c) != 0) ++c;
    *category = c;
    *bits = value > 0 ? (uint32_t)value : (c ? ((1u << c) - 1u) - a : 0u);
    return JPGE_OK;
}

int jpge_encode_category(const uint8_t* runs, const int32_t* values, size_t n, uint8_t* symbols, uint32_t* codes,
                         uint8_t* code_lens) {
    if (n && (!runs || !values || !symbols || !codes || !code_lens)) return JPGE_E_ARG;
    for (size_t i = 0; i < n; ++i) {
        uint16_t c;
        uint32_t b;
        if (runs[i] > 15) return JPGE_E_ARG;
        if (const int e = jpge_category_code(values[i], &c, &b)) return e;
        symbols[i] = (uint8_t)((runs[i] << 4) | c);
        codes[i] = b;
        code_lens[i] = (uint8_t)c;
    }
    return JPGE_OK;
}

int jpge_dc_difference(int32_t* y, uint32_t rows, uint32_t cols, int32_t* cb, int32_t* cr, uint32_t crows,
                       uint32_t ccols) {
    if (!y || !cb || !cr || rows % 16 || cols % 16 || crows % 8 || ccols % 8) return JPGE_E_ARG;
    int32_t b = 0;
    auto step = [&](int32_t* p) {
        const int32_t t = *p;
        *p = t - b;
        b = t;
    };
    for (uint32_t h = 0; h < rows; h += 16)  // Y in MCU order, Image.cpp:640-659
        for (uint32_t w = 0; w < cols; w += 16) {
            step(&y[(size_t)h * cols + w]);
            step(&y[(size_t)h * cols + w + 8]);
            step(&y[(size_t)(h + 8) * cols + w]);
            step(&y[(size_t)(h + 8) * cols + w + 8]);
        }
    for (int32_t* c : {cb, cr}) {  // Image.cpp:661-677
        b = 0;
        for (uint32_t h = 0; h < crows; h += 8)
            for (uint32_t w = 0; w < ccols; w += 8) step(&c[(size_t)h * ccols + w]);
    }
    return JPGE_OK;
}

}  // extern "C"
