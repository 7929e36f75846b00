// Decode-side verification utilities: the reference's
// huffmanDecode (Huffman.cpp:78-146) and inverseDctMat (Dct.hpp:278-306), plus a
// baseline entropy decoder that turns a jpge .jpg (any subsampling mode, restart
// intervals) back into its quantised coefficients, so that round trips can be
// checked at sizes the CPU oracle cannot encode in test time.  Host code: these
// utilities verify streams; they are not on the encode path.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/jpge.h"
#include "host_io.hpp"

namespace {

// MSB-first bit reader over entropy-coded bytes with JPEG byte stuffing (FF 00 ->
// FF).  A marker (FF xx, xx != 0) ends the data: reading past it yields 1-bits
// (T.81 F.2.2.5) and sets `marker`.
struct BitReader {
    const uint8_t* p;
    size_t n, pos;
    uint32_t acc = 0;
    int cnt = 0;
    int marker = -1;  // the marker that stopped the reader
    BitReader(const uint8_t* d, size_t len, size_t start) : p(d), n(len), pos(start) {}
    void refill() {
        while (cnt <= 24) {
            uint32_t b = 0xFF;
            if (marker < 0 && pos < n) {
                b = p[pos];
                if (b == 0xFF) {
                    const uint32_t nx = pos + 1 < n ? p[pos + 1] : 0xD9;
                    if (nx == 0x00) pos += 2;
                    else { marker = (int)nx; b = 0xFF; }  // leave pos at the marker
                } else {
                    ++pos;
                }
            }
            acc |= b << (24 - cnt);
            cnt += 8;
        }
    }
    uint32_t peek(int k) { refill(); return acc >> (32 - k); }
    void skip(int k) { acc <<= k; cnt -= k; }
    uint32_t get(int k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        skip(k);
        return v;
    }
    // drop the partial byte and step over an RSTn marker (restart interval boundary)
    bool restart(int expect) {
        acc = 0; cnt = 0;
        if (marker != 0xD0 + expect) return false;
        pos += 2;
        marker = -1;
        return true;
    }
};

// Canonical decoding table from a DHT (bits[1..16], huffval): T.81 F.2.2.3.
struct DecTable {
    int32_t maxcode[18];
    int32_t valptr[17];
    int32_t mincode[17];
    uint8_t val[256];
    bool ok = false;
    void build(const uint8_t bits[16], const uint8_t* huffval, int nsym) {
        std::memcpy(val, huffval, (size_t)nsym);
        int32_t code = 0, k = 0;
        for (int l = 1; l <= 16; ++l) {
            valptr[l] = k;
            mincode[l] = code;
            code += bits[l - 1];
            k += bits[l - 1];
            maxcode[l] = bits[l - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7FFFFFFF;
        ok = true;
    }
    int decode(BitReader& br) const {
        const uint32_t w = br.peek(16);
        for (int l = 1; l <= 16; ++l) {
            const int32_t c = (int32_t)(w >> (16 - l));
            if (maxcode[l] >= 0 && c <= maxcode[l]) {
                br.skip(l);
                return val[valptr[l] + c - mincode[l]];
            }
        }
        return -1;
    }
};

// value bits of category s (getCategoryAndCode, Coding.hpp:197-230, inverted)
inline int extend(uint32_t v, int s) { return s == 0 ? 0 : (v >> (s - 1)) ? (int)v : (int)v - (1 << s) + 1; }

inline uint32_t be16(const uint8_t* q) { return ((uint32_t)q[0] << 8) | q[1]; }

}  // namespace

extern "C" {

int jpge_huffman_decode(const uint8_t* bits, uint64_t nbits, const uint32_t* table_syms, const uint32_t* table_codes,
                        const uint8_t* table_lens, int nsym, int* text, size_t cap, size_t* n) {
    // huffmanDecode, Huffman.cpp:91-146: at each position take max_code_length bits
    // (fewer at the end, the rest 1-filled) and pick the first code, in order of the
    // 1-filled codes, that is >= them.  For a prefix code that is the code the bits
    // start with.
    if (!bits || !table_syms || !table_codes || !table_lens || !n || nsym <= 0 || nsym > (1 << 15)) return JPGE_E_ARG;  // (package_merge: <= 2^15 symbols, Huffman.hpp:115)
    struct Entry { uint32_t filled; int len; int sym; };
    std::vector<Entry> e;
    int maxlen = 0;
    for (int i = 0; i < nsym; ++i) {
        const int l = table_lens[i];
        if (l < 1 || l > 32) return JPGE_E_ARG;
        const uint32_t msb = l == 32 ? table_codes[i] : table_codes[i] << (32 - l);
        const uint32_t fill = l == 32 ? 0u : (uint32_t)((1ull << (32 - l)) - 1);  // fillRestWithOnes
        e.push_back({msb | fill, l, (int)table_syms[i]});
        if (l > maxlen) maxlen = l;
    }
    std::sort(e.begin(), e.end(), [](const Entry& a, const Entry& b) { return a.filled < b.filled; });
    size_t k = 0;
    uint64_t pos = 0;
    while (pos < nbits) {
        const int take = (int)std::min<uint64_t>((uint64_t)maxlen, nbits - pos);
        uint32_t w = 0;
        for (int i = 0; i < take; ++i) {
            const uint64_t b = pos + (uint64_t)i;
            w |= (uint32_t)((bits[b >> 3] >> (7 - (b & 7))) & 1u) << (31 - i);
        }
        w |= take == 32 ? 0u : (uint32_t)((1ull << (32 - take)) - 1);
        size_t idx = e.size();
        for (size_t i = 0; i < e.size(); ++i)
            if (e[i].filled >= w) { idx = i; break; }
        if (idx == e.size()) return JPGE_E_FORMAT;  // no code matches (the reference asserts)
        if (text) {
            if (k >= cap) return JPGE_E_NOSPACE;
            text[k] = e[idx].sym;
        }
        ++k;
        pos += (uint64_t)e[idx].len;
    }
    *n = k;
    return JPGE_OK;
}

void jpge_idct8x8(const double in[64], double out[64]) {
    // inverseDctMat, Dct.hpp:278-306: A(k, n) = C(k) sqrt(2/N) cos((2n+1) k pi / 2N),
    // res = (A^T X) A, each product summed over the inner index in order from 0.
    const double pi = 3.141592653589793115997963468544185161590576171875;  // boost pi<double>
    const double root_two = 1.4142135623730951454746218587388284504413604736328125;
    const double scale = std::sqrt(2. / 8);
    double A[64], first[64];
    for (int k = 0; k < 8; ++k)
        for (int n = 0; n < 8; ++n) {
            const double co = k == 0 ? 1. / root_two : 1.;
            const double cos_term = (2. * n + 1.) * ((k * pi) / (2. * 8));
            A[k * 8 + n] = co * scale * std::cos(cos_term);
        }
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) {
            double t = 0;
            for (int k = 0; k < 8; ++k) t += A[k * 8 + i] * in[k * 8 + j];
            first[i * 8 + j] = t;
        }
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) {
            double t = 0;
            for (int k = 0; k < 8; ++k) t += first[i * 8 + k] * A[k * 8 + j];
            out[i * 8 + j] = t;
        }
}

int jpge_decode_coeffs(const uint8_t* jpg, size_t len, jpge_decoded* info, int16_t* y, int16_t* cb, int16_t* cr,
                       size_t cap_y_blocks, size_t cap_c_blocks) {
    if (!jpg || !info || len < 4) return JPGE_E_ARG;
    std::memset(info, 0, sizeof(*info));
    if (jpg[0] != 0xFF || jpg[1] != 0xD8) return JPGE_E_FORMAT;
    DecTable dc[4], ac[4];
    int hs[3] = {0, 0, 0}, vs[3] = {0, 0, 0}, tq[3] = {0, 0, 0}, td[3] = {0, 0, 0}, ta[3] = {0, 0, 0};
    uint8_t qt[4][64] = {};
    uint32_t restart = 0;
    size_t pos = 2;
    bool sof = false;
    for (;;) {  // header segments up to SOS (JpegSegments.hpp:55-358)
        if (pos + 4 > len || jpg[pos] != 0xFF) return JPGE_E_FORMAT;
        const uint8_t m = jpg[pos + 1];
        const uint32_t sl = be16(jpg + pos + 2);
        const uint8_t* s = jpg + pos + 4;
        if (pos + 2 + sl > len || sl < 2) return JPGE_E_FORMAT;
        if (m == 0xDB) {  // DQT: 8-bit tables, zig-zag order
            for (uint32_t o = 0; o + 65 <= sl - 2; o += 65) {
                const int id = s[o] & 3;
                for (int i = 0; i < 64; ++i) qt[id][jpge::kZigzagToNatural[i]] = s[o + 1 + i];
            }
        } else if (m == 0xC0) {  // SOF0
            if (sl < 17 || s[0] != 8 || s[5] != 3) return JPGE_E_FORMAT;
            info->height = be16(s + 1);
            info->width = be16(s + 3);
            for (int c = 0; c < 3; ++c) {
                hs[c] = s[7 + 3 * c] >> 4;
                vs[c] = s[7 + 3 * c] & 15;
                tq[c] = s[8 + 3 * c] & 3;
            }
            sof = true;
        } else if (m == 0xC4) {  // DHT
            uint32_t o = 0;
            while (o + 17 <= sl - 2) {
                const int tc = s[o] >> 4, th = s[o] & 3;
                int nsym = 0;
                for (int l = 0; l < 16; ++l) nsym += s[o + 1 + l];
                if (nsym > 256 || o + 17 + (uint32_t)nsym > sl - 2) return JPGE_E_FORMAT;
                (tc ? ac : dc)[th].build(s + o + 1, s + o + 17, nsym);
                o += 17 + (uint32_t)nsym;
            }
        } else if (m == 0xDD) {  // DRI
            if (sl < 4) return JPGE_E_FORMAT;
            restart = be16(s);
        } else if (m == 0xDA) {  // SOS: three components, in frame order
            if (!sof || sl < 2 + 1 + 2 * 3 + 3 || s[0] != 3) return JPGE_E_FORMAT;
            for (int c = 0; c < 3; ++c) {
                td[c] = s[2 + 2 * c] >> 4;
                ta[c] = s[2 + 2 * c] & 15;
                if (td[c] > 3 || ta[c] > 3) return JPGE_E_FORMAT;
            }
            pos += 2 + sl;
            break;
        } else if (m < 0xE0 && m != 0xFE) {
            return JPGE_E_FORMAT;  // not baseline, or not a jpge stream
        }
        pos += 2 + sl;
    }
    // the sampling shapes jpge emits: chroma 1x1, Y yh x yv
    const int yh = hs[0], yv = vs[0];
    if (hs[1] != 1 || vs[1] != 1 || hs[2] != 1 || vs[2] != 1 || yh < 1 || yh > 4 || yv < 1 || yv > 2 ||
        yh * yv > 4 || !info->width || !info->height)
        return JPGE_E_FORMAT;
    for (int c = 0; c < 3; ++c)
        if (!dc[td[c]].ok || !ac[ta[c]].ok) return JPGE_E_FORMAT;
    const uint32_t mw = (info->width + 8 * yh - 1) / (8 * yh), mh = (info->height + 8 * yv - 1) / (8 * yv);
    info->yh = (uint32_t)yh;
    info->yv = (uint32_t)yv;
    info->restart = restart;
    info->y_blocks = (size_t)mw * yh * mh * yv;
    info->c_blocks = (size_t)mw * mh;
    std::memcpy(info->qy, qt[tq[0]], 64);
    std::memcpy(info->qc, qt[tq[1]], 64);
    if (!y) return JPGE_OK;  // size query
    if (!cb || !cr || cap_y_blocks < info->y_blocks || cap_c_blocks < info->c_blocks) return JPGE_E_NOSPACE;

    BitReader br(jpg, len, pos);
    int pred[3] = {0, 0, 0};
    const uint32_t ybw = mw * (uint32_t)yh;
    int16_t blk[64];
    auto block = [&](int c, int16_t* dst) -> bool {
        const int s = dc[td[c]].decode(br);
        if (s < 0 || s > 11) return false;
        pred[c] += extend(br.get(s), s);
        std::memset(blk, 0, sizeof(blk));
        blk[0] = (int16_t)pred[c];
        for (int k = 1; k < 64;) {
            const int rs = ac[ta[c]].decode(br);
            if (rs < 0) return false;
            const int r = rs >> 4, sz = rs & 15;
            if (sz == 0) {
                if (r != 15) break;  // EOB
                k += 16;             // ZRL
                continue;
            }
            k += r;
            if (k > 63) return false;
            blk[jpge::kZigzagToNatural[k]] = (int16_t)extend(br.get(sz), sz);
            ++k;
        }
        std::memcpy(dst, blk, sizeof(blk));
        return true;
    };
    for (uint32_t m = 0; m < mw * mh; ++m) {
        if (restart && m && m % restart == 0) {  // RSTn: byte-align, reset the predictions
            if (!br.restart((int)((m / restart - 1) & 7))) return JPGE_E_FORMAT;
            pred[0] = pred[1] = pred[2] = 0;
        }
        const uint32_t i = m / mw, j = m % mw;
        for (int v = 0; v < yv; ++v)
            for (int u = 0; u < yh; ++u)
                if (!block(0, y + ((size_t)(i * yv + v) * ybw + j * yh + u) * 64)) return JPGE_E_FORMAT;
        if (!block(1, cb + (size_t)m * 64) || !block(2, cr + (size_t)m * 64)) return JPGE_E_FORMAT;
    }
    // the stream ends with the 1-filled final byte and EOI
    br.acc = 0;
    br.cnt = 0;
    br.refill();
    if (br.marker != 0xD9) return JPGE_E_FORMAT;
    return JPGE_OK;
}

}  // extern "C"
