// =============================================================================
// jpge ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A clean-room CPU restatement of the Nuos/jpgEnc encode path (reference at
// /root/reference, read-only).  Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py may load this library, and only as a checker or
// as the timed CPU baseline.  The product (jpgenc_amd/, libjpge.so) never links,
// loads or calls it.
//
// Parity pinning (see DESIGN.md "Oracle"):
//   * every stage is checked against the reference's own known-answer tests
//     (src/test/{DctTest,CodingTest,ImageTest,BitstreamGenericTest}.cpp), restated
//     as JSON fixtures under tests/golden/;
//   * the Huffman table construction and the Bitstream byte layout are checked
//     against the reference's own src/Huffman.cpp + include/BitstreamGeneric.hpp,
//     compiled unmodified from /root/reference into oracle/_ref/ (oracle/Makefile);
//   * Image.cpp / Dct.hpp / Coding.hpp need Boost (absent from this image), so the
//     whole-file writeJPEG bytes cannot be produced by the reference here: the
//     full-file path is pinned by composition of the pinned stages.
//
// Semantics follow the reference exactly (fp64, IEEE op order, no contraction —
// build with -ffp-contract=off), including libstdc++ unordered_map /
// priority_queue iteration order in the Huffman builder.
// =============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// ---------------------------------------------------------------------------
// Arai constants: Dct.hpp:21-43 (cos of k*pi/16 evaluated by glibc at static
// init; pi and sqrt(2) are Boost's correctly rounded doubles).
// ---------------------------------------------------------------------------
struct AraiK {
    double c[8], a1, a2, a3, a4, a5, s[8];
    AraiK() {
        const double pi = 3.141592653589793115997963468544185161590576171875;  // boost pi<double>
        const double root_two = 1.4142135623730951454746218587388284504413604736328125;
        for (int k = 1; k < 8; ++k) c[k] = std::cos(k * pi / 16);
        c[0] = 0;
        a1 = c[4]; a2 = c[2] - c[6]; a3 = c[4]; a4 = c[6] + c[2]; a5 = c[6];
        s[0] = 1 / (2 * root_two);
        for (int k = 1; k < 8; ++k) s[k] = 1 / (4 * c[k]);
    }
};
const AraiK& K() { static AraiK k; return k; }

// One 8-point Arai pass, Dct.hpp:53-131 (identical op sequence for both passes).
// in[i] = x_i ; writes out[k] for the scaled frequency k.
inline void arai_pass(const double x[8], double out[8]) {
    const AraiK& k = K();
    double z0 = x[0] + x[7], z1 = x[1] + x[6], z2 = x[2] + x[5], z3 = x[3] + x[4];
    double z4 = -x[4] + x[3], z5 = -x[5] + x[2], z6 = -x[6] + x[1], z7 = -x[7] + x[0];
    double r0 = z0 + z3, r1 = z1 + z2, r2 = z1 - z2, r3 = z0 - z3;
    double r4 = -z4 - z5, r5 = z5 + z6, r6 = z6 + z7, r7 = z7;
    double t0 = r0 + r1, t1 = r0 - r1, t2 = r2 + r3, t3 = r3, t4 = r4, t5 = r5, t6 = r6, t7 = r7;
    double tmp = (t4 + t6) * k.a5;
    t2 *= k.a1; t4 *= k.a2; t5 *= k.a3; t6 *= k.a4;
    double u4 = -t4 - tmp, u6 = t6 - tmp;
    double v2 = t2 + t3, v3 = t3 - t2, v5 = t5 + t7, v7 = t7 - t5;
    double w4 = u4 + v7, w5 = v5 + u6, w6 = -u6 + v5, w7 = v7 - u4;
    out[0] = t0 * k.s[0]; out[4] = t1 * k.s[4]; out[2] = v2 * k.s[2]; out[6] = v3 * k.s[6];
    out[5] = w4 * k.s[5]; out[1] = w5 * k.s[1]; out[7] = w6 * k.s[7]; out[3] = w7 * k.s[3];
}

// dctArai, Dct.hpp:47-215: pass over columns of x -> temp (transposed), then over
// columns of temp -> y.  blk/out are row-major 8x8.
inline void dct_arai(const double* blk, int stride, double* out, int ostride) {
    double temp[64];
    double col[8], res[8];
    for (int j = 0; j < 8; ++j) {
        for (int i = 0; i < 8; ++i) col[i] = blk[i * stride + j];
        arai_pass(col, res);
        for (int k = 0; k < 8; ++k) temp[j * 8 + k] = res[k];
    }
    for (int j = 0; j < 8; ++j) {
        for (int i = 0; i < 8; ++i) col[i] = temp[i * 8 + j];
        arai_pass(col, res);
        for (int k = 0; k < 8; ++k) out[j * ostride + k] = res[k];
    }
}

// Zig-zag scan index -> natural (row-major) index: Coding.hpp:57-81 (the
// reference's lookup, verified by DctTest.cpp:103-106).
const int kZigzagToNatural[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// getCategoryAndCode, Coding.hpp:197-230.  Returns category (0 for v == 0) and
// the offset bits written MSB-first in `cat` bits.
inline int category(int v, uint32_t* bits) {
    if (v == 0) { *bits = 0; return 0; }
    long bound = 2;
    for (int cat = 1; cat < 16; ++cat, bound <<= 1) {
        long upper = bound - 1, lower = bound >> 1;
        long a = std::labs((long)v);
        if (a >= lower && a <= upper) {
            *bits = (uint32_t)(v < 0 ? upper - a : (long)v);
            return cat;
        }
    }
    *bits = 0;  // reference asserts (unreachable for |v| < 32768)
    return 0;
}

struct Sym { uint8_t symbol; uint8_t nbits; uint32_t bits; };

// RLE_AC(matrix<int>) Coding.hpp:148-183 + encode_category Coding.hpp:265-283.
// blk: natural-order quantised block (DC already difference-coded).
inline void rle_block(const int* blk, std::vector<Sym>& out) {
    uint32_t bits;
    int cat = category(blk[0], &bits);
    out.push_back({(uint8_t)cat, (uint8_t)cat, bits});
    unsigned zeros = 0;
    for (int i = 1; i < 64; ++i) {
        int v = blk[kZigzagToNatural[i]];
        if (v == 0) { ++zeros; continue; }
        while (zeros > 15) { out.push_back({0xF0, 0, 0}); zeros -= 16; }
        cat = category(v, &bits);
        out.push_back({(uint8_t)((zeros << 4) | cat), (uint8_t)cat, bits});
        zeros = 0;
    }
    if (zeros > 0) out.push_back({0x00, 0, 0});
}

// ---------------------------------------------------------------------------
// Huffman table construction — Huffman.cpp:3-66 + Huffman.hpp:114-174, with the
// same standard-library containers so that unordered_map iteration order and
// priority_queue tie-breaking (libstdc++) match the reference build.
// ---------------------------------------------------------------------------
struct Pkg {
    int weight;
    std::vector<int> syms;  // sorted ascending (std::merge of sorted lists)
};
struct PkgGreater {
    bool operator()(const Pkg& a, const Pkg& b) const { return a.weight > b.weight; }
};

struct Table {
    std::vector<std::vector<int>> by_len;   // [0..16], DHT order
    std::unordered_map<int, std::pair<uint32_t, int>> code;  // symbol -> (code value, length)
};

Table build_table(const std::vector<int>& text) {
    Table t;
    std::unordered_map<int, int> counts;
    for (int s : text) ++counts[s];
    std::vector<std::pair<int, int>> freq;  // (symbol, count) in map iteration order
    for (auto& kv : counts) freq.push_back(kv);

    if (counts.size() == 1) {  // Huffman.cpp:17-25
        t.by_len.assign(17, {});
        t.by_len[1] = {text[0]};
        t.code[text[0]] = {0u, 1};
        return t;
    }
    const int L = 15;
    typedef std::priority_queue<Pkg, std::vector<Pkg>, PkgGreater> Level;
    Level base;
    for (auto& f : freq) base.push(Pkg{f.second, {f.first}});
    std::vector<Level> levels;
    for (int i = 0; i < L; ++i) levels.push_back(base);
    levels.push_back(Level());
    for (int i = 0; i < L; ++i) {
        Level& lv = levels[i];
        Level& nx = levels[i + 1];
        while (lv.size() > 1) {
            Pkg p1 = lv.top(); lv.pop();
            Pkg p2 = lv.top(); lv.pop();
            Pkg m;
            m.weight = p1.weight + p2.weight;
            std::merge(p1.syms.begin(), p1.syms.end(), p2.syms.begin(), p2.syms.end(),
                       std::back_inserter(m.syms));
            nx.push(std::move(m));
        }
    }
    std::unordered_map<int, int> lens;
    Level& fin = levels[L];
    while (!fin.empty()) {
        Pkg p = fin.top(); fin.pop();
        for (int s : p.syms) lens[s]++;
    }
    t.by_len.assign(L + 2, {});
    for (auto& kv : lens) t.by_len[kv.second].push_back(kv.first);
    // preventOnlyOnesCode, Huffman.cpp:37-48
    int last = (int)t.by_len.size() - 1;
    while (last > 0 && t.by_len[last].empty()) --last;
    int s = t.by_len[last].back();
    t.by_len[last].pop_back();
    t.by_len[last + 1].push_back(s);
    // generateCodes, Huffman.cpp:50-66
    uint32_t c = 0;
    for (int len = 1; len < (int)t.by_len.size(); ++len) {
        for (int sym : t.by_len[len]) { t.code[sym] = {c, len}; ++c; }
        c <<= 1;
    }
    return t;
}

// ---------------------------------------------------------------------------
// MSB-first bit writer with the Bitstream_Generic<uint8_t> layout
// (BitstreamGeneric.hpp:127-146 push, :243-248 fill, :213-224 0xFF stuffing).
// ---------------------------------------------------------------------------
struct BitWriter {
    std::vector<uint8_t> bytes;
    uint64_t nbits = 0;
    void put(uint32_t v, int n) {  // lowest n bits of v, MSB first
        for (int i = n - 1; i >= 0; --i) {
            if ((nbits & 7) == 0) bytes.push_back(0);
            if ((v >> i) & 1) bytes.back() |= (uint8_t)(0x80 >> (nbits & 7));
            ++nbits;
        }
    }
    void fill() {  // fill(): pad with ones; an empty stream gets a whole 0xFF byte
        if (nbits == 0) { put(0xFF, 8); return; }
        while (nbits & 7) put(1, 1);
    }
    void stuff_into(std::vector<uint8_t>& out) const {
        if (nbits == 0) return;
        for (uint8_t b : bytes) { out.push_back(b); if (b == 0xFF) out.push_back(0); }
    }
};

// IJG quality scaling of the Annex-K tables (the reference itself is fixed at
// quality 50, Image.cpp:850-869; Q50 returns the tables unchanged).
const int kLuma[64] = {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                       14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                       18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                       49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int kChroma[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                         24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

void scaled_tables(int q, uint8_t qy[64], uint8_t qc[64]) {
    if (q < 1) q = 1;
    if (q > 100) q = 100;
    int s = q < 50 ? 5000 / q : 200 - 2 * q;
    for (int i = 0; i < 64; ++i) {
        int a = (kLuma[i] * s + 50) / 100, b = (kChroma[i] * s + 50) / 100;
        qy[i] = (uint8_t)std::min(255, std::max(1, a));
        qc[i] = (uint8_t)std::min(255, std::max(1, b));
    }
}

// ---------------------------------------------------------------------------
// The pipeline state (Image.hpp:101-114 as flat row-major arrays).
// ---------------------------------------------------------------------------
struct Frame {
    int rw = 0, rh = 0;        // real (unpadded) size
    int W = 0, H = 0;          // padded to multiples of 16 (Image.cpp:480-531)
    int sw = 0, sh = 0;        // subsampled chroma size
    std::vector<double> R, G, B;
    std::vector<double> Y, Cb, Cr;
    std::vector<double> dY, dCb, dCr;
    std::vector<int> qY, qCb, qCr;
};

// loadPPM padding: Image.cpp:480-531 (right, bottom, corner edge replication).
void load_planes(Frame& f, const uint8_t* rgb, int w, int h, int maxval) {
    f.rw = w; f.rh = h;
    f.W = (w % 16) ? w + 16 - w % 16 : w;
    f.H = (h % 16) ? h + 16 - h % 16 : h;
    const double scale = 255. / maxval;  // Image.cpp:465
    f.R.assign((size_t)f.W * f.H, 0); f.G = f.R; f.B = f.R;
    for (int y = 0; y < f.H; ++y) {
        int sy = std::min(y, h - 1);
        for (int x = 0; x < f.W; ++x) {
            int sx = std::min(x, w - 1);
            const uint8_t* p = rgb + ((size_t)sy * w + sx) * 3;
            size_t o = (size_t)y * f.W + x;
            f.R[o] = p[0] * scale; f.G[o] = p[1] * scale; f.B[o] = p[2] * scale;
        }
    }
}

// convertToColorSpace(YCbCr): Image.cpp:131-144 (float literals widened to double).
void to_ycc(Frame& f) {
    static const float Flat[] = {.0f, 256 / 2.f, 256 / 2.f};
    static const float Yv[] = {.299f, .587f, .114f};
    static const float Cbv[] = {-.1687f, -.3312f, .5f};
    static const float Crv[] = {.5f, -.4186f, -.0813f};
    size_t n = (size_t)f.W * f.H;
    f.Y.resize(n); f.Cb.resize(n); f.Cr.resize(n);
    for (size_t x = 0; x < n; ++x) {
        double r = f.R[x], g = f.G[x], b = f.B[x];
        f.Y[x] = Flat[0] + (Yv[0] * r + Yv[1] * g + Yv[2] * b) - 128;
        f.Cb[x] = Flat[1] + (Cbv[0] * r + Cbv[1] * g + Cbv[2] * b) - 128;
        f.Cr[x] = Flat[2] + (Crv[0] * r + Crv[1] * g + Crv[2] * b) - 128;
    }
}

// subsample(S420_m): Image.cpp:198-235 -> ((a+b) + (c+d)) / 4.
void subsample420m(const std::vector<double>& in, int W, int H, std::vector<double>& out) {
    int sw = W / 2, sh = H / 2;
    out.assign((size_t)sw * sh, 0);
    for (int y = 0; y < sh; ++y)
        for (int x = 0; x < sw; ++x) {
            double top = 0, bot = 0;
            top += 1 * in[(size_t)(2 * y) * W + 2 * x];
            top += 1 * in[(size_t)(2 * y) * W + 2 * x + 1];
            bot += 1 * in[(size_t)(2 * y + 1) * W + 2 * x];
            bot += 1 * in[(size_t)(2 * y + 1) * W + 2 * x + 1];
            double v = top;
            v += bot;
            v /= 4;
            out[(size_t)y * sw + x] = v;
        }
}

// Image::subsample, Image.cpp:198-235, for every mask applySubsampling builds
// (Image.cpp:256-309): mask row m of a scanline, summed from 0 in mask order; with
// averaging the next scanline's sum is added and the result divided by 4 (S420_m)
// or 2; without scanline_jump and without averaging every scanline is visited
// (the --y at :229).  mode: 422 S422, 411 S411, 4200 S420, 4201 S420_lm, 420 S420_m,
// 444 S444 (identity, :257-261).
void subsample_mode(const std::vector<double>& chan, int W, int H, int mode, std::vector<double>& out) {
    std::vector<uint8_t> row;
    bool jump = false, averaging = false;
    int vdiv = 2, hdiv = 2;
    switch (mode) {
        case 422: row = {1, 0}; vdiv = 1; hdiv = 2; break;
        case 411: row = {1, 0, 0, 0}; vdiv = 1; hdiv = 4; break;
        case 4200: row = {1, 0}; jump = true; break;
        case 420: row = {1, 1}; averaging = true; break;
        case 4201: row = {1, 0}; averaging = true; break;
        default: out = chan; return;
    }
    const int rs = (int)row.size();
    out.assign((size_t)(H / vdiv) * (W / hdiv), 0);
    size_t idx = 0, idx2 = 0;
    for (int y = 0; y < H;) {
        for (int x = 0; x < W; x += rs) {
            double v = 0;
            for (int m = 0; m < rs; ++m) v += row[m] * chan[(size_t)y * W + x + m];
            out[idx++] = v;
        }
        if (!jump && averaging) {
            for (int x = 0; x < W; x += rs) {
                double v = 0;
                for (int m = 0; m < rs; ++m) v += row[m] * chan[(size_t)(y + 1) * W + x + m];
                (out[idx2++] += v) /= (mode == 420 ? 4 : 2);
            }
        }
        y += (!jump && !averaging) ? 1 : 2;  // y += 2 after the --y of :229
    }
}

void dct_plane(const std::vector<double>& in, int W, int H, std::vector<double>& out) {
    out.assign((size_t)W * H, 0);
#pragma omp parallel for schedule(static)
    for (int h = 0; h < H; h += 8)
        for (int w = 0; w < W; w += 8)
            dct_arai(&in[(size_t)h * W + w], W, &out[(size_t)h * W + w], W);
}

// quantize, Coding.hpp:84-97: (int)round(d / (double)q), natural order.
void quant_plane(const std::vector<double>& in, int W, int H, const uint8_t q[64],
                 std::vector<int>& out) {
    out.assign((size_t)W * H, 0);
#pragma omp parallel for schedule(static)
    for (int h = 0; h < H; h += 8)
        for (int w = 0; w < W; w += 8)
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 8; ++j) {
                    size_t o = (size_t)(h + i) * W + w + j;
                    out[o] = (int)std::round(in[o] / (double)q[i * 8 + j]);
                }
}

void run_to_quant(Frame& f, const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy,
                  const uint8_t* qc) {
    load_planes(f, rgb, w, h, maxval);
    to_ycc(f);
    f.R.clear(); f.G.clear(); f.B.clear();
    f.sw = f.W / 2; f.sh = f.H / 2;
    std::vector<double> cb, cr;
    subsample420m(f.Cr, f.W, f.H, cr);
    subsample420m(f.Cb, f.W, f.H, cb);
    f.Cb.swap(cb); f.Cr.swap(cr);
    dct_plane(f.Y, f.W, f.H, f.dY);
    dct_plane(f.Cb, f.sw, f.sh, f.dCb);
    dct_plane(f.Cr, f.sw, f.sh, f.dCr);
    quant_plane(f.dY, f.W, f.H, qy, f.qY);
    quant_plane(f.dCb, f.sw, f.sh, qc, f.qCb);
    quant_plane(f.dCr, f.sw, f.sh, qc, f.qCr);
}

// applyDCdifferenceCoding, Image.cpp:638-678.
void dc_diff(Frame& f) {
    int b = 0;
    for (int h = 0; h < f.H; h += 16)
        for (int w = 0; w < f.W; w += 16) {
            const int off[4][2] = {{0, 0}, {0, 8}, {8, 0}, {8, 8}};
            for (auto& o : off) {
                int& v = f.qY[(size_t)(h + o[0]) * f.W + w + o[1]];
                int t = v; v = t - b; b = t;
            }
        }
    for (std::vector<int>* pl : {&f.qCb, &f.qCr}) {
        b = 0;
        for (int h = 0; h < f.sh; h += 8)
            for (int w = 0; w < f.sw; w += 8) {
                int& v = (*pl)[(size_t)h * f.sw + w];
                int t = v; v = t - b; b = t;
            }
    }
}

// Restart-interval variant (not in the reference, which never emits DRI/RSTn): the
// same chains with every predictor reset to 0 at the first MCU of each interval of R
// MCUs (ITU T.81 F.1.2.3; MCU raster order is each chain's order at 4:2:0).
void dc_diff_restart(Frame& f, int R) {
    int bY = 0, bCb = 0, bCr = 0, m = 0;
    const int cbw = f.sw / 8;
    for (int h = 0; h < f.H; h += 16)
        for (int w = 0; w < f.W; w += 16, ++m) {
            if (m % R == 0) bY = bCb = bCr = 0;
            const int off[4][2] = {{0, 0}, {0, 8}, {8, 0}, {8, 8}};
            for (auto& o : off) {
                int& v = f.qY[(size_t)(h + o[0]) * f.W + w + o[1]];
                int t = v; v = t - bY; bY = t;
            }
            const size_t c = (size_t)(h / 2) * f.sw + w / 2;
            (void)cbw;
            int& vb = f.qCb[c]; int tb = vb; vb = tb - bCb; bCb = tb;
            int& vr = f.qCr[c]; int tr = vr; vr = tr - bCr; bCr = tr;
        }
}

// S444 variant (not in the reference's writeJPEG, which hard-codes S420_m at
// Image.cpp:842): applySubsampling(S444) (Image.cpp:257-261) leaves Cb and Cr at full
// resolution, and the MCU is one 8x8 block of each component.  The planes are cropped
// to whole blocks, ceil(w/8)*8 x ceil(h/8)*8, of the reference's 16-padded planes
// (edge replication either way: a decoder expects ceil(w/8) x ceil(h/8) MCUs).
void run_to_quant444(Frame& f, const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy,
                     const uint8_t* qc) {
    load_planes(f, rgb, w, h, maxval);
    to_ycc(f);
    f.R.clear(); f.G.clear(); f.B.clear();
    const int W8 = (w + 7) / 8 * 8, H8 = (h + 7) / 8 * 8;
    for (std::vector<double>* p : {&f.Y, &f.Cb, &f.Cr}) {
        std::vector<double> o((size_t)W8 * H8);
        for (int y = 0; y < H8; ++y)
            for (int x = 0; x < W8; ++x) o[(size_t)y * W8 + x] = (*p)[(size_t)y * f.W + x];
        p->swap(o);
    }
    f.W = f.sw = W8;
    f.H = f.sh = H8;
    dct_plane(f.Y, W8, H8, f.dY);
    dct_plane(f.Cb, W8, H8, f.dCb);
    dct_plane(f.Cr, W8, H8, f.dCr);
    quant_plane(f.dY, W8, H8, qy, f.qY);
    quant_plane(f.dCb, W8, H8, qc, f.qCb);
    quant_plane(f.dCr, W8, H8, qc, f.qCr);
}

// DC chains at 4:4:4 (Image.cpp:638-678 applied per component): each component's
// blocks in raster order, which is MCU order; restart R > 0 resets all three at the
// first MCU of every interval.
void dc_diff444(Frame& f, int R) {
    int b[3] = {0, 0, 0}, m = 0;
    std::vector<int>* pl[3] = {&f.qY, &f.qCb, &f.qCr};
    for (int h = 0; h < f.H; h += 8)
        for (int w = 0; w < f.W; w += 8, ++m) {
            if (R && m % R == 0) b[0] = b[1] = b[2] = 0;
            for (int c = 0; c < 3; ++c) {
                int& v = (*pl[c])[(size_t)h * f.W + w];
                int t = v; v = t - b[c]; b[c] = t;
            }
        }
}

// Sampling shape of a subsampling mode: Y blocks across (yh) and down (yv) an MCU;
// one Cb and one Cr block per MCU in every mode.
bool mode_shape(int mode, int& yh, int& yv) {
    switch (mode) {
        case 420: case 4200: case 4201: yh = 2; yv = 2; return true;
        case 444: yh = 1; yv = 1; return true;
        case 422: yh = 2; yv = 1; return true;
        case 411: yh = 4; yv = 1; return true;
        default: return false;
    }
}

// Generic subsampling-mode path (the modes of applySubsampling, Image.cpp:237-319,
// that writeJPEG cannot emit).  At 420 and 444 it reproduces the
// pinned paths above (a CPU test checks this).  The planes are edge-replicated to
// whole MCUs of 8yh x 8yv px (Image.cpp:480-531 replicates to 16 px; 4:1:1 needs 32
// across), converted (to_ycc), chroma-subsampled (subsample_mode), transformed and
// quantised.
void run_to_quant_mode(Frame& f, const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy,
                       const uint8_t* qc, int mode) {
    int yh, yv;
    mode_shape(mode, yh, yv);
    load_planes(f, rgb, w, h, maxval);
    to_ycc(f);
    f.R.clear(); f.G.clear(); f.B.clear();
    const int MW = 8 * yh, MH = 8 * yv;
    const int W = (w + MW - 1) / MW * MW, H = (h + MH - 1) / MH * MH;
    for (std::vector<double>* p : {&f.Y, &f.Cb, &f.Cr}) {
        std::vector<double> o((size_t)W * H);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x)
                o[(size_t)y * W + x] = (*p)[(size_t)std::min(y, f.H - 1) * f.W + std::min(x, f.W - 1)];
        p->swap(o);
    }
    f.W = W; f.H = H;
    f.sw = W / yh; f.sh = H / yv;
    std::vector<double> cb, cr;
    subsample_mode(f.Cr, W, H, mode, cr);
    subsample_mode(f.Cb, W, H, mode, cb);
    f.Cb.swap(cb); f.Cr.swap(cr);
    dct_plane(f.Y, W, H, f.dY);
    dct_plane(f.Cb, f.sw, f.sh, f.dCb);
    dct_plane(f.Cr, f.sw, f.sh, f.dCr);
    quant_plane(f.dY, W, H, qy, f.qY);
    quant_plane(f.dCb, f.sw, f.sh, qc, f.qCb);
    quant_plane(f.dCr, f.sw, f.sh, qc, f.qCr);
}

// The Y block (v, u) of MCU (i, j), u across, v down, in a plane of W px.
inline size_t y_block_origin(const Frame& f, int yh, int yv, int i, int j, int v, int u) {
    return (size_t)((i * yv + v) * 8) * f.W + (size_t)(j * yh + u) * 8;
}

// DC chains (Image.cpp:638-678) in MCU order: Y over the MCU's yh*yv blocks row by
// row (the MCU-order chain of :640-659), Cb and Cr over their blocks, whose raster
// order is MCU order in every mode; restart R > 0 resets the three at the first MCU
// of every interval.
void dc_diff_mode(Frame& f, int yh, int yv, int R) {
    int b[3] = {0, 0, 0}, m = 0;
    for (int i = 0; i < f.sh / 8; ++i)
        for (int j = 0; j < f.sw / 8; ++j, ++m) {
            if (R && m % R == 0) b[0] = b[1] = b[2] = 0;
            for (int v = 0; v < yv; ++v)
                for (int u = 0; u < yh; ++u) {
                    int& x = f.qY[y_block_origin(f, yh, yv, i, j, v, u)];
                    int t = x; x = t - b[0]; b[0] = t;
                }
            for (int c = 1; c < 3; ++c) {
                int& x = (c == 1 ? f.qCb : f.qCr)[(size_t)(i * 8) * f.sw + j * 8];
                int t = x; x = t - b[c]; b[c] = t;
            }
        }
}

void block_syms(const std::vector<int>& plane, int W, int H, std::vector<std::vector<Sym>>& out) {
    int bw = W / 8, bh = H / 8;
    out.assign((size_t)bw * bh, {});
    int blk[64];
    for (int by = 0; by < bh; ++by)
        for (int bx = 0; bx < bw; ++bx) {
            for (int i = 0; i < 8; ++i)
                for (int j = 0; j < 8; ++j) blk[i * 8 + j] = plane[(size_t)(by * 8 + i) * W + bx * 8 + j];
            rle_block(blk, out[(size_t)by * bw + bx]);
        }
}

void put_u16(std::vector<uint8_t>& o, int v) { o.push_back((uint8_t)(v >> 8)); o.push_back((uint8_t)v); }

// JFIF segments, JpegSegments.hpp:55-377 as used by Image.cpp:933-972.
void write_headers(std::vector<uint8_t>& o, int rw, int rh, const uint8_t qy[64], const uint8_t qc[64],
                   const Table* t[4], int restart = 0, uint8_t ysamp = 0x22) {
    const uint8_t soi_app0[] = {0xFF, 0xD8, 0xFF, 0xE0, 0, 16, 'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
    o.insert(o.end(), soi_app0, soi_app0 + sizeof(soi_app0));
    const uint8_t* qt[2] = {qy, qc};
    for (int id = 0; id < 2; ++id) {  // DQT: zigzag<Byte> Coding.hpp:30-54
        o.push_back(0xFF); o.push_back(0xDB); put_u16(o, 67); o.push_back((uint8_t)id);
        for (int i = 0; i < 64; ++i) o.push_back(qt[id][kZigzagToNatural[i]]);
    }
    o.push_back(0xFF); o.push_back(0xC0); put_u16(o, 17); o.push_back(8);
    put_u16(o, rh & 0xFFFF); put_u16(o, rw & 0xFFFF); o.push_back(3);
    const uint8_t comp[9] = {1, ysamp, 0, 2, 0x11, 1, 3, 0x11, 1};  // Y: (H << 4) | V sampling factors
    o.insert(o.end(), comp, comp + 9);
    const uint8_t info[4] = {0x00, 0x10, 0x01, 0x11};
    for (int k = 0; k < 4; ++k) {
        size_t n = 0;
        for (int l = 1; l <= 16; ++l) n += t[k]->by_len[l].size();
        o.push_back(0xFF); o.push_back(0xC4); put_u16(o, (int)(2 + 17 + n)); o.push_back(info[k]);
        for (int l = 1; l <= 16; ++l) o.push_back((uint8_t)t[k]->by_len[l].size());
        for (int l = 1; l <= 16; ++l)
            for (int s : t[k]->by_len[l]) o.push_back((uint8_t)s);
    }
    if (restart) {  // DRI, ITU T.81 B.2.4.4 (restart variant only)
        o.push_back(0xFF); o.push_back(0xDD); put_u16(o, 4); put_u16(o, restart);
    }
    const uint8_t sos[] = {0xFF, 0xDA, 0, 12, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 0x3F, 0};
    o.insert(o.end(), sos, sos + sizeof(sos));
}

void emit_block(BitWriter& bw, const std::vector<Sym>& s, const Table& dc, const Table& ac) {
    for (size_t i = 0; i < s.size(); ++i) {
        const Table& t = i == 0 ? dc : ac;
        auto it = t.code.find(s[i].symbol);
        if (it != t.code.end()) bw.put(it->second.first, it->second.second);
        bw.put(s[i].bits, s[i].nbits);
    }
}

// restart = 0: writeJPEG (Image.cpp:831-976).  restart = R > 0: the restart-interval
// variant — DC chains reset per interval, and after every interval but the last the
// stream is 1-filled, stuffed and followed by RSTn (n = interval index mod 8).
// s444: the S444 variant (run_to_quant444; Y 1x1 in SOF0; MCU = Y, Cb, Cr).
int encode_frame(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                 std::vector<uint8_t>& out, int restart = 0, bool s444 = false) {
    if (w <= 0 || h <= 0 || maxval <= 0 || maxval > 255 || restart < 0 || restart > 65535) return -1;
    Frame f;
    if (s444) {
        run_to_quant444(f, rgb, w, h, maxval, qy, qc);
        dc_diff444(f, restart);
    } else {
        run_to_quant(f, rgb, w, h, maxval, qy, qc);
        if (restart) dc_diff_restart(f, restart);
        else dc_diff(f);
    }
    std::vector<std::vector<Sym>> sY, sCb, sCr;
    block_syms(f.qY, f.W, f.H, sY);
    block_syms(f.qCb, f.sw, f.sh, sCb);
    block_syms(f.qCr, f.sw, f.sh, sCr);
    // symbol texts, Image.cpp:888-906
    std::vector<int> ydc, yac, cdc, cac;
    for (auto& b : sY) { ydc.push_back(b[0].symbol); for (size_t i = 1; i < b.size(); ++i) yac.push_back(b[i].symbol); }
    for (auto* pl : {&sCb, &sCr})
        for (auto& b : *pl) { cdc.push_back(b[0].symbol); for (size_t i = 1; i < b.size(); ++i) cac.push_back(b[i].symbol); }
    Table tyd = build_table(ydc), tya = build_table(yac), tcd = build_table(cdc), tca = build_table(cac);
    const Table* tabs[4] = {&tyd, &tya, &tcd, &tca};
    out.clear();
    write_headers(out, f.rw, f.rh, qy, qc, tabs, restart, s444 ? 0x11 : 0x22);
    // MCU interleave, Image.cpp:957-968 (at 4:4:4 one block of each component)
    BitWriter bw;
    int ybw = f.W / 8, cbw = f.sw / 8, cbh = f.sh / 8;
    int mcu = 0;
    for (int i = 0; i < cbh; ++i)
        for (int j = 0; j < cbw; ++j, ++mcu) {
            if (restart && mcu > 0 && mcu % restart == 0) {  // end of an interval
                bw.fill();
                bw.stuff_into(out);
                out.push_back(0xFF); out.push_back((uint8_t)(0xD0 + ((mcu / restart - 1) & 7)));
                bw = BitWriter();
            }
            if (s444) {
                emit_block(bw, sY[(size_t)i * ybw + j], tyd, tya);
            } else {
                emit_block(bw, sY[(size_t)(2 * i) * ybw + 2 * j], tyd, tya);
                emit_block(bw, sY[(size_t)(2 * i) * ybw + 2 * j + 1], tyd, tya);
                emit_block(bw, sY[(size_t)(2 * i + 1) * ybw + 2 * j], tyd, tya);
                emit_block(bw, sY[(size_t)(2 * i + 1) * ybw + 2 * j + 1], tyd, tya);
            }
            emit_block(bw, sCb[(size_t)i * cbw + j], tcd, tca);
            emit_block(bw, sCr[(size_t)i * cbw + j], tcd, tca);
        }
    bw.fill();
    bw.stuff_into(out);
    out.push_back(0xFF); out.push_back(0xD9);
    return 0;
}

// The generic subsampling-mode encode (run_to_quant_mode / dc_diff_mode): texts in
// block raster order per component (Image.cpp:888-906), MCUs of yh*yv Y blocks
// (row by row) + Cb + Cr (the interleave of Image.cpp:957-968 generalised), SOF0
// declaring Y as yh x yv.
int encode_frame_mode(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                      std::vector<uint8_t>& out, int restart, int mode) {
    int yh, yv;
    if (!mode_shape(mode, yh, yv)) return -1;
    if (w <= 0 || h <= 0 || maxval <= 0 || maxval > 255 || restart < 0 || restart > 65535) return -1;
    Frame f;
    run_to_quant_mode(f, rgb, w, h, maxval, qy, qc, mode);
    dc_diff_mode(f, yh, yv, restart);
    std::vector<std::vector<Sym>> sY, sCb, sCr;
    block_syms(f.qY, f.W, f.H, sY);
    block_syms(f.qCb, f.sw, f.sh, sCb);
    block_syms(f.qCr, f.sw, f.sh, sCr);
    std::vector<int> ydc, yac, cdc, cac;
    for (auto& b : sY) { ydc.push_back(b[0].symbol); for (size_t i = 1; i < b.size(); ++i) yac.push_back(b[i].symbol); }
    for (auto* pl : {&sCb, &sCr})
        for (auto& b : *pl) { cdc.push_back(b[0].symbol); for (size_t i = 1; i < b.size(); ++i) cac.push_back(b[i].symbol); }
    Table tyd = build_table(ydc), tya = build_table(yac), tcd = build_table(cdc), tca = build_table(cac);
    const Table* tabs[4] = {&tyd, &tya, &tcd, &tca};
    out.clear();
    write_headers(out, f.rw, f.rh, qy, qc, tabs, restart, (uint8_t)((yh << 4) | yv));
    BitWriter bw;
    const int ybw = f.W / 8, cbw = f.sw / 8, cbh = f.sh / 8;
    int mcu = 0;
    for (int i = 0; i < cbh; ++i)
        for (int j = 0; j < cbw; ++j, ++mcu) {
            if (restart && mcu > 0 && mcu % restart == 0) {
                bw.fill();
                bw.stuff_into(out);
                out.push_back(0xFF); out.push_back((uint8_t)(0xD0 + ((mcu / restart - 1) & 7)));
                bw = BitWriter();
            }
            for (int v = 0; v < yv; ++v)
                for (int u = 0; u < yh; ++u) emit_block(bw, sY[(size_t)(i * yv + v) * ybw + j * yh + u], tyd, tya);
            emit_block(bw, sCb[(size_t)i * cbw + j], tcd, tca);
            emit_block(bw, sCr[(size_t)i * cbw + j], tcd, tca);
        }
    bw.fill();
    bw.stuff_into(out);
    out.push_back(0xFF); out.push_back(0xD9);
    return 0;
}

// PPM parsing, Image.cpp:326-474 (PPMFileBuffer::read_word incl. '#' handling,
// fast_atoi, magic check, maxval).
struct PpmReader {
    const uint8_t* f; size_t pos = 0, eof;
    PpmReader(const uint8_t* p, size_t n) : f(p), eof(n) {}
    uint8_t rb() { return pos < eof ? f[pos++] : (pos++, 0); }
    std::string word() {
        uint8_t c = rb();
        if (isspace(c)) { while (pos < eof && isspace(f[pos])) ++pos; c = rb(); }
        size_t first = pos - 1;
        for (;;) {
            if (c == '#') { while (pos < eof && f[pos++] != '\n') {} first = pos; }
            else if (isspace(c)) return std::string((const char*)f + first, pos - 1 - first);
            else if (pos >= eof) return std::string((const char*)f + first, std::min(pos, eof) - first);
            c = rb();
        }
    }
};

}  // namespace

// =============================================================================
// C ABI (ctypes) — test infrastructure only.
// =============================================================================
extern "C" {

int orc_quality_tables(int q, uint8_t* qy, uint8_t* qc) { scaled_tables(q, qy, qc); return 0; }

void orc_arai_constants(double* c8, double* a5, double* s8) {
    const AraiK& k = K();
    for (int i = 0; i < 8; ++i) { c8[i] = k.c[i]; s8[i] = k.s[i]; }
    a5[0] = k.a1; a5[1] = k.a2; a5[2] = k.a3; a5[3] = k.a4; a5[4] = k.a5;
}

void orc_dct_arai(const double* in64, double* out64) { dct_arai(in64, 8, out64, 8); }

void orc_quantize(const double* in64, const int* q64, int* out64) {
    for (int i = 0; i < 64; ++i) out64[i] = (int)std::round(in64[i] / (double)q64[i]);
}

void orc_ycc(double r, double g, double b, double* out3) {
    Frame f; f.W = 1; f.H = 1; f.R = {r}; f.G = {g}; f.B = {b};
    to_ycc(f);
    out3[0] = f.Y[0]; out3[1] = f.Cb[0]; out3[2] = f.Cr[0];
}

// subsample(S420_m) of an arbitrary W x H plane (the KAT applies it to RGB planes).
void orc_subsample420m(const double* in, int W, int H, double* out) {
    std::vector<double> v(in, in + (size_t)W * H), o;
    subsample420m(v, W, H, o);
    memcpy(out, o.data(), o.size() * 8);
}

int orc_zigzag_to_natural(int i) { return kZigzagToNatural[i]; }

int orc_category(int v, uint32_t* bits) { return category(v, bits); }

// RLE of a natural-order block (RLE_AC(matrix)): returns the number of pairs;
// runs[k], vals[k] are RLE_PAIR(num_zeros_before, value); sym/nbits/bits the
// encode_category output.
int orc_rle_block(const int* blk64, int* runs, int* vals, int* syms, int* nbits, uint32_t* bits) {
    std::vector<Sym> s;
    rle_block(blk64, s);
    // recover RLE pairs from the symbols: run = sym >> 4, value from category/offset
    for (size_t k = 0; k < s.size(); ++k) {
        syms[k] = s[k].symbol; nbits[k] = s[k].nbits; bits[k] = s[k].bits;
        runs[k] = k == 0 ? 0 : (s[k].symbol >> 4);
        int cat = s[k].nbits;
        int v = 0;
        if (cat) { uint32_t o = s[k].bits; v = (o >> (cat - 1)) ? (int)o : -(int)(((1u << cat) - 1) - o); }
        vals[k] = v;
    }
    return (int)s.size();
}

// Huffman tables from a symbol text.  Outputs: n distinct symbols;
// dht_syms[k]/dht_lens[k] in SymbolsPerLength (DHT) order; codes[k] the code value.
int orc_huffman(const int* text, int n, int* dht_syms, int* dht_lens, uint32_t* codes) {
    std::vector<int> t(text, text + n);
    Table tb = build_table(t);
    int k = 0;
    for (int len = 1; len < (int)tb.by_len.size(); ++len)
        for (int s : tb.by_len[len]) {
            dht_syms[k] = s; dht_lens[k] = len; codes[k] = tb.code[s].first; ++k;
        }
    return k;
}

// Pack (value, nbits) pairs MSB-first, then fill + 0xFF stuffing.  Returns bytes
// written (stuffed) and the raw bit count.
int64_t orc_pack_bits(const uint32_t* vals, const int* nbits, int n, int do_fill, uint8_t* out,
                      int64_t cap, int64_t* raw_bits) {
    BitWriter bw;
    for (int i = 0; i < n; ++i) bw.put(vals[i], nbits[i]);
    if (do_fill) bw.fill();
    *raw_bits = (int64_t)bw.nbits;
    std::vector<uint8_t> o;
    bw.stuff_into(o);
    if ((int64_t)o.size() > cap) return -(int64_t)o.size();
    memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

// PPM parse following loadPPM; returns 0 and fills w/h/maxval/samples
// (w*h*3 ints, unscaled), -1 open/format error, -2 truncated.
int orc_parse_ppm(const uint8_t* buf, size_t n, int* w, int* h, int* maxval, int* samples, size_t cap) {
    PpmReader r(buf, n);
    std::string magic = r.word();
    if (magic != "P3" && magic != "P6") return -1;
    *w = atoi(r.word().c_str());
    *h = atoi(r.word().c_str());
    *maxval = atoi(r.word().c_str());
    size_t cnt = (size_t)(*w) * (*h) * 3;
    if (!samples) return 0;
    if (cnt > cap) return -3;
    if (magic == "P6") {
        if (r.pos + cnt > n) return -2;
        for (size_t i = 0; i < cnt; ++i) samples[i] = r.rb();
    } else {
        for (size_t i = 0; i < cnt; ++i) {
            std::string wd = r.word();
            int v = 0;
            for (char c : wd) v = v * 10 + (c - '0');  // fast_atoi, Image.cpp:326-333
            samples[i] = v;
        }
    }
    return 0;
}

// Stage dump: quantised coefficients before DC differencing, per component,
// blocks in raster order, 64 natural-order values per block.
int orc_stage_coeffs(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                     int16_t* outY, int16_t* outCb, int16_t* outCr) {
    Frame f;
    run_to_quant(f, rgb, w, h, maxval, qy, qc);
    auto dump = [](const std::vector<int>& pl, int W, int H, int16_t* o) {
        int bw = W / 8, bh = H / 8;
        for (int by = 0; by < bh; ++by)
            for (int bx = 0; bx < bw; ++bx)
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 8; ++j)
                        o[((size_t)by * bw + bx) * 64 + i * 8 + j] = (int16_t)pl[(size_t)(by * 8 + i) * W + bx * 8 + j];
    };
    dump(f.qY, f.W, f.H, outY);
    dump(f.qCb, f.sw, f.sh, outCb);
    dump(f.qCr, f.sw, f.sh, outCr);
    return 0;
}

// Stage dump: YCbCr planes after colour conversion + S420_m (doubles).
int orc_stage_ycc(const uint8_t* rgb, int w, int h, int maxval, double* Y, double* Cb, double* Cr) {
    Frame f;
    load_planes(f, rgb, w, h, maxval);
    to_ycc(f);
    std::vector<double> cb, cr;
    subsample420m(f.Cb, f.W, f.H, cb);
    subsample420m(f.Cr, f.W, f.H, cr);
    memcpy(Y, f.Y.data(), f.Y.size() * 8);
    memcpy(Cb, cb.data(), cb.size() * 8);
    memcpy(Cr, cr.data(), cr.size() * 8);
    return 0;
}

// Symbol histograms + first-occurrence order of the four texts (Image.cpp:888-906):
// counts[t*256+s], first[t*256+s] = index of the first occurrence in text t (-1 if absent).
int orc_stage_hist(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                   uint32_t* counts, int64_t* first) {
    Frame f;
    run_to_quant(f, rgb, w, h, maxval, qy, qc);
    dc_diff(f);
    std::vector<std::vector<Sym>> sY, sCb, sCr;
    block_syms(f.qY, f.W, f.H, sY);
    block_syms(f.qCb, f.sw, f.sh, sCb);
    block_syms(f.qCr, f.sw, f.sh, sCr);
    for (int i = 0; i < 4 * 256; ++i) { counts[i] = 0; first[i] = -1; }
    int64_t pos[4] = {0, 0, 0, 0};
    auto add = [&](int t, int s) {
        if (first[t * 256 + s] < 0) first[t * 256 + s] = pos[t];
        counts[t * 256 + s]++; pos[t]++;
    };
    for (auto& b : sY) { add(0, b[0].symbol); for (size_t i = 1; i < b.size(); ++i) add(1, b[i].symbol); }
    for (auto* pl : {&sCb, &sCr})
        for (auto& b : *pl) { add(2, b[0].symbol); for (size_t i = 1; i < b.size(); ++i) add(3, b[i].symbol); }
    return 0;
}

// Full encode of interleaved RGB samples (w*h*3 bytes) with explicit tables.
// Returns the .jpg length, or -(needed) if cap is too small, or -1 on bad args.
int64_t orc_encode_rgb(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                       uint8_t* out, int64_t cap) {
    std::vector<uint8_t> o;
    if (encode_frame(rgb, w, h, maxval, qy, qc, o) != 0) return -1;
    if ((int64_t)o.size() > cap) return -(int64_t)o.size();
    memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

// The restart-interval variant (restart MCUs per interval; 0 = orc_encode_rgb).
int64_t orc_encode_rgb_restart(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                               int restart, uint8_t* out, int64_t cap) {
    std::vector<uint8_t> o;
    if (encode_frame(rgb, w, h, maxval, qy, qc, o, restart) != 0) return -1;
    if ((int64_t)o.size() > cap) return -(int64_t)o.size();
    memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

// Any variant: restart MCUs per interval (0 = none); subsampling 420 (S420_m) or 444
// through the pinned paths, 422 / 411 / 4200 (S420) / 4201 (S420_lm) through the
// generic one; generic = 1 forces the generic path (consistency tests).
int64_t orc_encode_rgb_mode(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                            int restart, int subsampling, int generic, uint8_t* out, int64_t cap) {
    int yh, yv;
    if (!mode_shape(subsampling, yh, yv)) return -1;
    std::vector<uint8_t> o;
    const bool pinned = !generic && (subsampling == 420 || subsampling == 444);
    const int st = pinned ? encode_frame(rgb, w, h, maxval, qy, qc, o, restart, subsampling == 444)
                          : encode_frame_mode(rgb, w, h, maxval, qy, qc, o, restart, subsampling);
    if (st != 0) return -1;
    if ((int64_t)o.size() > cap) return -(int64_t)o.size();
    memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
}

int64_t orc_encode_rgb_ex(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                          int restart, int subsampling, uint8_t* out, int64_t cap) {
    return orc_encode_rgb_mode(rgb, w, h, maxval, qy, qc, restart, subsampling, 0, out, cap);
}

// Stage dump of the generic path: quantised coefficients before DC differencing,
// Y plane of ceil(w/8yh)*yh x ceil(h/8yv)*yv blocks and the two chroma planes of
// ceil(w/8yh) x ceil(h/8yv) blocks, raster order, natural order inside a block.
int orc_stage_coeffs_mode(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                          int mode, int16_t* outY, int16_t* outCb, int16_t* outCr) {
    int yh, yv;
    if (!mode_shape(mode, yh, yv)) return -1;
    Frame f;
    run_to_quant_mode(f, rgb, w, h, maxval, qy, qc, mode);
    auto dump = [](const std::vector<int>& pl, int W, int H, int16_t* o) {
        const int bw = W / 8, bh = H / 8;
        for (int by = 0; by < bh; ++by)
            for (int bx = 0; bx < bw; ++bx)
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 8; ++j)
                        o[((size_t)by * bw + bx) * 64 + i * 8 + j] = (int16_t)pl[(size_t)(by * 8 + i) * W + bx * 8 + j];
    };
    dump(f.qY, f.W, f.H, outY);
    dump(f.qCb, f.sw, f.sh, outCb);
    dump(f.qCr, f.sw, f.sh, outCr);
    return 0;
}

// subsample_mode of an arbitrary W x H plane (Image::subsample for one mode).
int orc_subsample_mode(const double* in, int W, int H, int mode, double* out) {
    std::vector<double> v(in, in + (size_t)W * H), o;
    subsample_mode(v, W, H, mode, o);
    memcpy(out, o.data(), o.size() * 8);
    return (int)o.size();
}

// Stage dump of the S444 variant: quantised coefficients before DC differencing,
// three planes of ceil(w/8) x ceil(h/8) blocks in raster order.
int orc_stage_coeffs444(const uint8_t* rgb, int w, int h, int maxval, const uint8_t* qy, const uint8_t* qc,
                        int16_t* outY, int16_t* outCb, int16_t* outCr) {
    Frame f;
    run_to_quant444(f, rgb, w, h, maxval, qy, qc);
    const int bw = f.W / 8, bh = f.H / 8;
    const std::vector<int>* pl[3] = {&f.qY, &f.qCb, &f.qCr};
    int16_t* o[3] = {outY, outCb, outCr};
    for (int c = 0; c < 3; ++c)
        for (int by = 0; by < bh; ++by)
            for (int bx = 0; bx < bw; ++bx)
                for (int i = 0; i < 8; ++i)
                    for (int j = 0; j < 8; ++j)
                        o[c][((size_t)by * bw + bx) * 64 + i * 8 + j] =
                            (int16_t)(*pl[c])[(size_t)(by * 8 + i) * f.W + bx * 8 + j];
    return 0;
}

int orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

}  // extern "C"
