#include "host_io.hpp"
#include "host_par.hpp"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <thread>

namespace jpge {

const uint8_t kZigzagToNatural[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

namespace {

// Tokenizer with the reference's exact behaviour (Image.cpp:349-389), bounds-checked.
class Tokens {
  public:
    Tokens(const uint8_t* p, size_t n) : p_(p), n_(n) {}
    size_t pos() const { return pos_; }
    uint8_t byte() { return pos_ < n_ ? p_[pos_++] : (pos_++, 0); }
    std::string word() {
        uint8_t c = byte();
        if (std::isspace(c)) {
            while (pos_ < n_ && std::isspace(p_[pos_])) ++pos_;
            c = byte();
        }
        size_t first = pos_ - 1;
        for (;;) {
            if (c == '#') {
                while (pos_ < n_ && p_[pos_++] != '\n') {}
                first = pos_;
            } else if (std::isspace(c)) {
                return std::string(reinterpret_cast<const char*>(p_) + first, pos_ - 1 - first);
            } else if (pos_ >= n_) {
                size_t end = std::min(pos_, n_);
                return first < end ? std::string(reinterpret_cast<const char*>(p_) + first, end - first)
                                   : std::string();
            }
            c = byte();
        }
    }

  private:
    const uint8_t* p_;
    size_t n_, pos_ = 0;
};

bool to_int(const std::string& s, long& v) {
    if (s.empty()) return false;
    char* end = nullptr;
    v = std::strtol(s.c_str(), &end, 10);
    return end != s.c_str();
}

const uint8_t kLuma[64] = {16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                           14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                           18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                           49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kChroma[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                             24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                             99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                             99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

void put16(std::vector<uint8_t>& o, uint32_t v) {
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

// splitmix64 (integer-only PRNG so the frames are identical on every host).
inline uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

inline int tri(int x, int period) {  // triangle wave 0..255
    int p = x % period;
    if (p < 0) p += period;
    int h = period / 2;
    return (p < h ? p : period - p) * 255 / (h ? h : 1);
}

// loadP3PPM's fast_atoi (Image.cpp:393-408): digits accumulated without validation.
// The reference's int overflows (undefined) on long tokens; here an accumulator that
// leaves +-2^40 stops at -1, which every caller rejects as out of range, and every
// token that stays inside that range gets the reference's value.
inline long fast_atoi(const std::string& wd) {
    long v = 0;
    for (char c : wd) {
        v = v * 10 + (c - '0');
        if (v > (1l << 40) || v < -(1l << 40)) return -1;
    }
    return v;
}

}  // namespace

int parse_ppm(const uint8_t* buf, size_t n, PpmImage& out) {
    Tokens t(buf, n);
    std::string magic = t.word();
    if (magic != "P3" && magic != "P6") return kErrFormat;
    long w = 0, h = 0, mv = 0;
    if (!to_int(t.word(), w) || !to_int(t.word(), h) || !to_int(t.word(), mv)) return kErrFormat;
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535) return kErrFormat;
    if (mv < 1 || mv > 255) return kErrRange;  // Image.cpp:462 asserts maxval < 256
    out.width = (uint32_t)w;
    out.height = (uint32_t)h;
    out.maxval = (int)mv;
    const size_t cnt = (size_t)w * (size_t)h * 3;
    out.rgb.resize(cnt);
    if (magic == "P6") {  // loadP6PPM, Image.cpp:411-418
        if (t.pos() + cnt > n) return kErrTruncated;
        std::memcpy(out.rgb.data(), buf + t.pos(), cnt);
        for (size_t i = 0; i < cnt; ++i)
            if (out.rgb[i] > mv) return kErrRange;
    } else {  // loadP3PPM, Image.cpp:393-408 (fast_atoi, no validation)
        for (size_t i = 0; i < cnt; ++i) {
            std::string wd = t.word();
            if (wd.empty() && t.pos() >= n) return kErrTruncated;
            const long v = fast_atoi(wd);
            if (v < 0 || v > mv) return kErrRange;
            out.rgb[i] = (uint8_t)v;
        }
    }
    return kOk;
}

int parse_ppm_inplace(uint8_t* buf, size_t n, uint32_t& width, uint32_t& height, int& maxval, size_t& offset) {
    Tokens t(buf, n);
    std::string magic = t.word();
    if (magic != "P3" && magic != "P6") return kErrFormat;
    long w = 0, h = 0, mv = 0;
    if (!to_int(t.word(), w) || !to_int(t.word(), h) || !to_int(t.word(), mv)) return kErrFormat;
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535) return kErrFormat;
    if (mv < 1 || mv > 255) return kErrRange;
    width = (uint32_t)w;
    height = (uint32_t)h;
    maxval = (int)mv;
    const size_t cnt = (size_t)w * (size_t)h * 3;
    if (magic == "P6") {  // loadP6PPM, Image.cpp:411-418: the samples are the frame
        if (t.pos() + cnt > n) return kErrTruncated;
        offset = t.pos();
        if (mv < 255)
            for (size_t i = 0; i < cnt; ++i)
                if (buf[offset + i] > mv) return kErrRange;
        return kOk;
    }
    // loadP3PPM, Image.cpp:393-408: sample i is written over the text at byte i, which
    // the tokenizer has passed (every earlier sample took >= 2 characters)
    for (size_t i = 0; i < cnt; ++i) {
        std::string wd = t.word();
        if (wd.empty() && t.pos() >= n) return kErrTruncated;
        const long v = fast_atoi(wd);
        if (v < 0 || v > mv) return kErrRange;
        buf[i] = (uint8_t)v;
    }
    offset = 0;
    return kOk;
}

int load_ppm_file(const std::string& path, PpmImage& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return kErrIo;
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return parse_ppm(buf.data(), buf.size(), out);
}

void quality_tables(int q, uint8_t qy[64], uint8_t qc[64]) {
    q = std::min(100, std::max(1, q));
    const int s = q < 50 ? 5000 / q : 200 - 2 * q;
    for (int i = 0; i < 64; ++i) {
        qy[i] = (uint8_t)std::min(255, std::max(1, (kLuma[i] * s + 50) / 100));
        qc[i] = (uint8_t)std::min(255, std::max(1, (kChroma[i] * s + 50) / 100));
    }
}

std::vector<uint8_t> jfif_headers(uint32_t rw, uint32_t rh, const uint8_t qy[64], const uint8_t qc[64],
                                  const HuffTable* const tables[4], uint32_t restart_mcus, uint8_t ysamp) {
    std::vector<uint8_t> o;
    o.reserve(700);
    // sSOI + sAPP0 (JpegSegments.hpp:55-109): JFIF 1.1, no units, density 1x1.
    static const uint8_t kSoiApp0[20] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F',
                                         0x00, 0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    o.insert(o.end(), kSoiApp0, kSoiApp0 + 20);
    // sDQT x2 (JpegSegments.hpp:259-319): one table per segment, zig-zag order.
    const uint8_t* qt[2] = {qy, qc};
    for (int id = 0; id < 2; ++id) {
        o.push_back(0xFF); o.push_back(0xDB); put16(o, 67); o.push_back((uint8_t)id);
        for (int i = 0; i < 64; ++i) o.push_back(qt[id][kZigzagToNatural[i]]);
    }
    // sSOF0 (JpegSegments.hpp:112-164): height before width, unpadded size;
    // Y 2x2 on table 0, Cb/Cr 1x1 on table 1 (Image.cpp:940-945); the other
    // subsampling modes declare Y as ysamp = (H << 4) | V.
    o.push_back(0xFF); o.push_back(0xC0); put16(o, 17); o.push_back(8);
    put16(o, rh & 0xFFFF); put16(o, rw & 0xFFFF);
    const uint8_t comp[10] = {3, 1, ysamp, 0, 2, 0x11, 1, 3, 0x11, 1};
    o.insert(o.end(), comp, comp + 10);
    // sDHT x4 (JpegSegments.hpp:167-256), Image.cpp:946-949.
    static const uint8_t kInfo[4] = {0x00, 0x10, 0x01, 0x11};
    for (int k = 0; k < 4; ++k) {
        const HuffTable& t = *tables[k];
        o.push_back(0xFF); o.push_back(0xC4); put16(o, (uint32_t)(2 + 17 + t.nsym)); o.push_back(kInfo[k]);
        for (int l = 1; l <= 16; ++l) o.push_back(t.bits[l]);
        o.insert(o.end(), t.huffval, t.huffval + t.nsym);
    }
    if (restart_mcus) {  // DRI (ITU T.81 B.2.4.4): restart interval in MCUs
        o.push_back(0xFF); o.push_back(0xDD); put16(o, 4); put16(o, restart_mcus & 0xFFFF);
    }
    // sSOS (JpegSegments.hpp:322-358): Y tables 0/0, Cb and Cr 1/1, Ss 0 Se 63 AhAl 0.
    static const uint8_t kSos[14] = {0xFF, 0xDA, 0x00, 0x0C, 0x03, 0x01, 0x00, 0x02, 0x11, 0x03, 0x11, 0x00, 0x3F, 0x00};
    o.insert(o.end(), kSos, kSos + 14);
    return o;
}

namespace {
int synth_threads(uint32_t h) {  // test-data synthesis: a few threads for large frames
    const unsigned hw = std::thread::hardware_concurrency();
    return h < 256 ? 1 : (int)std::min(8u, hw ? hw : 1u);
}
}  // namespace

void synth_rgb8(uint64_t seed, uint32_t w, uint32_t h, int kind, uint8_t* out, size_t stride) {
    const uint64_t s = mix(seed);
    if (kind == 2) {
        const uint8_t c[3] = {(uint8_t)s, (uint8_t)(s >> 8), (uint8_t)(s >> 16)};
        for (uint32_t y = 0; y < h; ++y)
            for (uint32_t x = 0; x < w; ++x) std::memcpy(out + (size_t)y * stride + x * 3, c, 3);
        return;
    }
    const int px = (int)(s % 977) + 200, py = (int)((s >> 10) % 743) + 150;
    const int tx = (int)((s >> 20) % 23) + 9, ty = (int)((s >> 30) % 19) + 7;
    parallel_for((long)h, synth_threads(h), [&](long yy) {
        const int y = (int)yy;
        uint8_t* row = out + (size_t)y * stride;
        for (uint32_t xu = 0; xu < w; ++xu) {
            const int x = (int)xu;
            const uint64_t r = mix(s ^ ((uint64_t)y << 32) ^ (uint64_t)x);
            if (kind == 1) {
                row[x * 3] = (uint8_t)r; row[x * 3 + 1] = (uint8_t)(r >> 8); row[x * 3 + 2] = (uint8_t)(r >> 16);
                continue;
            }
            // approx. gaussian noise, sigma ~ 12: sum of 4 uniform bytes
            int noise = ((int)(r & 0xFF) + (int)((r >> 8) & 0xFF) + (int)((r >> 16) & 0xFF) + (int)((r >> 24) & 0xFF) - 510) / 6;
            int texture = ((x / tx + y / ty) & 1) ? 18 : -18;
            int v[3];
            v[0] = (tri(x, px) * 3 + tri(y, py)) / 4;
            v[1] = (tri(x + y, px + py) + tri(y * 2, py)) / 2;
            v[2] = (tri(x - y, px) + 255 - tri(y, py / 2 + 1)) / 2;
            for (int c = 0; c < 3; ++c) {
                int val = v[c] + noise + (c == 1 ? texture : texture / 2) + (int)((r >> (32 + 8 * c)) & 7) - 3;
                row[x * 3 + c] = (uint8_t)std::min(255, std::max(0, val));
            }
        }
    });
}

}  // namespace jpge
