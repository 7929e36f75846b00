// Drop-in C++ facade with the reference's entry points: Image.hpp (Image, loadPPM,
// fast_atoi), Coding.hpp (from_vector, zigzag, quantize, RLE_PAIR, RLE_AC,
// Category_Code, getCategoryAndCode, encode_category), Huffman.hpp (Code,
// SymbolCodeMap, SymbolsPerLength, generateHuffmanCode, huffmanEncode,
// huffmanDecode) and BitstreamGeneric.hpp (Bitstream), built on the C ABI in
// include/jpge.h.  A jpgEnc caller switches by replacing its includes:
//     #include "Image.hpp" / "Coding.hpp" / "Huffman.hpp"  ->  #include "jpge_image.hpp"
// The names are in namespace jpge and, unless JPGE_NO_GLOBAL_NAMES is defined,
// also in the global namespace as the reference declares them, so reference code
// compiles unchanged (ImageTest.cpp / CodingTest.cpp: tests/cpp/test_facade.cpp).
//
// Where the work runs:
//   Image::writeJPEG   the GPU encode path: the fused RGB8 kernels (jpge_encode_rgb8)
//                      while the image is the RGB8 frame loadPPM read, else the
//                      plane kernels on the image's fp64 planes (jpge_encode_planes);
//   convertToColorSpace / applySubsampling / applyDCT / applyQuantization
//                      GPU plane kernels (jpge_color_convert, _subsample_plane,
//                      _dct_plane, _quantize_plane);
//   applyDCdifferenceCoding / doRLEandCategoryCoding / doHuffmanEncoding and the
//                      Coding.hpp functions: per-block host code over the C ABI
//                      (their results are per-block std::vectors, as the
//                      reference's private members are).
// matrix<T> stands in for boost::numeric::ublas::matrix<T> (row-major; operator(),
// size1, size2, data, resize, clear).  Errors surface as std::runtime_error, the
// reference's convention (Image.cpp:428,450).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <istream>
#include <ostream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "jpge.h"

namespace jpge {

typedef unsigned int uint;
typedef uint8_t Byte;
typedef double PixelDataType;

class Image;

namespace detail {
// An Image observes its planes: the first access materialises them from the RGB8
// frame, and a write access retires that frame (the planes are then the truth).
struct PlaneWatch {
    virtual void plane_access(bool write) = 0;

  protected:
    ~PlaneWatch() = default;
};
[[noreturn]] inline void fail(int st, const std::string& what) {
    throw std::runtime_error(what + ": " + jpge_strerror(st));
}
inline void check(int st, const char* what) {
    if (st) fail(st, what);
}
}  // namespace detail

// ---- matrix<T>: the reference's uBLAS matrix, row-major ----
template <typename T>
class matrix {
  public:
    matrix() = default;
    matrix(size_t rows, size_t cols) : r_(rows), c_(cols), v_(rows * cols) {}
    matrix(const matrix& o) : r_(o.r_), c_(o.c_), v_(o.cdata()) {}
    matrix(matrix&& o) noexcept : r_(o.r_), c_(o.c_), v_((o.touch(true), std::move(o.v_))) {}
    template <typename U>
    matrix(const matrix<U>& o) : r_(o.size1()), c_(o.size2()), v_(o.size1() * o.size2()) {
        const auto& src = o.data();
        for (size_t i = 0; i < v_.size(); ++i) v_[i] = static_cast<T>(src[i]);
    }
    matrix& operator=(const matrix& o) {
        if (this != &o) {
            touch(true);
            r_ = o.r_;
            c_ = o.c_;
            v_ = o.cdata();
        }
        return *this;
    }
    matrix& operator=(matrix&& o) noexcept {
        if (this != &o) {
            touch(true);
            o.touch(true);
            r_ = o.r_;
            c_ = o.c_;
            v_ = std::move(o.v_);
        }
        return *this;
    }

    size_t size1() const { return r_; }  // rows
    size_t size2() const { return c_; }  // columns
    T& operator()(size_t i, size_t j) {
        touch(true);
        return v_[i * c_ + j];
    }
    const T& operator()(size_t i, size_t j) const {
        touch(false);
        return v_[i * c_ + j];
    }
    std::vector<T>& data() {
        touch(true);
        return v_;
    }
    const std::vector<T>& data() const { return cdata(); }
    // resize(rows, cols, preserve): the overlapping top-left block is kept
    void resize(size_t rows, size_t cols, bool preserve = true) {
        touch(true);
        std::vector<T> n(rows * cols);
        if (preserve)
            for (size_t i = 0; i < std::min(rows, r_); ++i)
                for (size_t j = 0; j < std::min(cols, c_); ++j) n[i * cols + j] = v_[i * c_ + j];
        r_ = rows;
        c_ = cols;
        v_.swap(n);
    }
    void clear() {  // uBLAS: every element to zero
        touch(true);
        std::fill(v_.begin(), v_.end(), T());
    }
    friend bool operator==(const matrix& a, const matrix& b) {
        return a.r_ == b.r_ && a.c_ == b.c_ && a.cdata() == b.cdata();
    }

  private:
    friend class Image;
    const std::vector<T>& cdata() const {
        touch(false);
        return v_;
    }
    void touch(bool write) const {
        if (watch_) watch_->plane_access(write);
    }
    size_t r_ = 0, c_ = 0;
    std::vector<T> v_;
    detail::PlaneWatch* watch_ = nullptr;  // the Image owning this plane (not copied)
};
using mat = matrix<PixelDataType>;

// ---- Bitstream: BitstreamGeneric.hpp's Bitstream_Generic<uint8_t> ----
// Bit k of the stream is bit (7 - k % 8) of byte k / 8 (MSB first).
class Bitstream {
  public:
    static const unsigned block_size = 8;  // bits per block (Bitstream_Generic<uint8_t>)
    Bitstream() = default;
    Bitstream(std::initializer_list<bool> bits) { *this << bits; }
    Bitstream(uint32_t data, int number_of_bits) { push_back_LSB_mode(data, number_of_bits); }

    Bitstream& operator<<(bool v) {
        if ((sz_ & 7) == 0) b_.push_back(0);
        if (v) b_.back() |= (uint8_t)(0x80u >> (sz_ & 7));
        ++sz_;
        return *this;
    }
    Bitstream& operator<<(std::initializer_list<bool> bits) {
        for (bool v : bits) *this << v;
        return *this;
    }
    Bitstream& operator<<(const Bitstream& s) {
        for (unsigned i = 0; i < s.sz_; ++i) *this << s.bit(i);
        return *this;
    }
    Bitstream& push_back(bool v) { return *this << v; }
    // the number_of_bits highest bits of data, MSB first (BitstreamGeneric.hpp:183-195)
    Bitstream& push_back(uint32_t data, int number_of_bits) {
        for (int i = 0; i < number_of_bits; ++i) *this << (((data << i) & 0x80000000u) != 0);
        return *this;
    }
    // the number_of_bits lowest bits of data, MSB first (BitstreamGeneric.hpp:198-210)
    Bitstream& push_back_LSB_mode(uint32_t data, int number_of_bits) {
        for (int i = number_of_bits - 1; i >= 0; --i) *this << (((data >> i) & 1u) != 0);
        return *this;
    }

    class BitView {
      public:
        operator bool() const { return (b_[i_ >> 3] >> (7 - (i_ & 7))) & 1; }
        void operator=(bool v) {
            const uint8_t m = (uint8_t)(0x80u >> (i_ & 7));
            b_[i_ >> 3] = v ? (uint8_t)(b_[i_ >> 3] | m) : (uint8_t)(b_[i_ >> 3] & ~m);
        }

      private:
        friend class Bitstream;
        BitView(std::vector<uint8_t>& b, unsigned i) : b_(b), i_(i) {}
        std::vector<uint8_t>& b_;
        unsigned i_;
    };
    BitView operator[](unsigned pos) { return BitView(b_, pos); }
    bool operator[](unsigned pos) const { return bit(pos); }

    // number_of_bits bits from from_position, the first one the result's MSB
    // (BitstreamGeneric.hpp:264-305)
    template <typename T>
    T extractT(uint8_t number_of_bits, size_t from_position) const {
        T r = 0;
        for (unsigned i = 0; i < number_of_bits; ++i) r = (T)((r << 1) | (T)bit((unsigned)(from_position + i)));
        return number_of_bits ? (T)(r << (sizeof(T) * 8 - number_of_bits)) : (T)0;
    }
    uint32_t extract(uint8_t number_of_bits, size_t from_position) const {
        return extractT<uint32_t>(number_of_bits, from_position);
    }

    unsigned size() const { return sz_; }
    // 1-bits up to the byte boundary (BitstreamGeneric.hpp:243-248; a stream with no
    // bits yet gets a whole byte of them, as the reference's does)
    void fill() {
        if (sz_ && !(sz_ & 7)) return;  // aligned: nothing to do
        do *this << true;
        while (sz_ & 7);
    }
    const std::vector<uint8_t>& blocks() const { return b_; }  // (extension) the bytes

    friend bool operator==(const Bitstream& a, const Bitstream& b) { return a.sz_ == b.sz_ && a.b_ == b.b_; }
    friend bool operator!=(const Bitstream& a, const Bitstream& b) { return !(a == b); }
    // the bytes with 0x00 after every 0xFF (JPEG byte stuffing, BitstreamGeneric.hpp:213-224)
    friend std::ostream& operator<<(std::ostream& out, const Bitstream& s) {
        if (s.sz_ > 0)
            for (uint8_t v : s.b_) {
                out.put((char)v);
                if (v == 0xFF) out.put(0x00);
            }
        return out;
    }

    // whole blocks appended as read (BitstreamGeneric.hpp:226-234; no unstuffing)
    friend std::istream& operator>>(std::istream& in, Bitstream& s) {
        char c;
        while (in.get(c)) {
            if (s.sz_ & 7) s.sz_ = (s.sz_ | 7) + 1;  // (the reference appends at a block boundary)
            s.b_.push_back((uint8_t)c);
            s.sz_ += 8;
        }
        return in;
    }

  private:
    bool bit(unsigned i) const { return (b_[i >> 3] >> (7 - (i & 7))) & 1; }
    std::vector<uint8_t> b_;
    unsigned sz_ = 0;
};
using Bitstream8 = Bitstream;
typedef std::initializer_list<bool> Bits;

// ---- Coding.hpp ----
template <typename T>
matrix<T> from_vector(const std::vector<T>& v) {  // Coding.hpp:17-28
    if (v.size() != 64) throw std::invalid_argument("from_vector: 64 values expected");
    matrix<T> m(8, 8);
    for (size_t i = 0; i < 64; ++i) m(i / 8, i % 8) = v[i];
    return m;
}

inline int zigzag(int i) {  // Coding.hpp:57-81: natural index of zig-zag position i
    const int n = jpge_zigzag_index(i);
    if (n < 0) throw std::out_of_range("zigzag: position outside 0..63");
    return n;
}

template <typename T>
std::vector<T> zigzag(matrix<T> m) {  // Coding.hpp:30-54: the block in zig-zag order
    if (m.size1() != 8 || m.size2() != 8) throw std::invalid_argument("zigzag: 8x8 block expected");
    std::vector<T> r(64);
    const auto& d = m.data();
    for (int p = 0; p < 64; ++p) r[p] = d[jpge_zigzag_index(p)];
    return r;
}

inline matrix<int> quantize(const mat& m, const mat& table) {  // Coding.hpp:84-97
    if (m.size1() != 8 || m.size2() != 8 || table.size1() != 8 || table.size2() != 8)
        throw std::invalid_argument("quantize: 8x8 blocks expected");
    matrix<int> r(8, 8);
    detail::check(jpge_quantize_block(m.data().data(), table.data().data(), reinterpret_cast<int32_t*>(r.data().data())),
                  "quantize");
    return r;
}

struct RLE_PAIR {  // Coding.hpp:99-109
    unsigned short num_zeros_before : 4;
    int value;

    RLE_PAIR() = default;
    RLE_PAIR(short zeros, int _value) : num_zeros_before(zeros), value(_value) {
        if (zeros < 0 || zeros > 15) throw std::invalid_argument("RLE_PAIR: run outside 0..15");
    }
};
inline bool operator==(const RLE_PAIR& l, const RLE_PAIR& r) {
    return l.num_zeros_before == r.num_zeros_before && l.value == r.value;
}

namespace detail {
inline std::vector<RLE_PAIR> rle(const int32_t* data, size_t n, int zz) {
    uint8_t runs[128];
    int32_t vals[128];
    size_t k = 0;
    std::vector<RLE_PAIR> out;
    int st = jpge_rle_ac(data, n, zz, runs, vals, 128, &k);
    if (st == JPGE_E_NOSPACE) {  // (long vector inputs)
        std::vector<uint8_t> r2(k);
        std::vector<int32_t> v2(k);
        check(jpge_rle_ac(data, n, zz, r2.data(), v2.data(), k, &k), "RLE_AC");
        for (size_t i = 0; i < k; ++i) out.emplace_back((short)r2[i], v2[i]);
        return out;
    }
    check(st, "RLE_AC");
    out.reserve(k);
    for (size_t i = 0; i < k; ++i) out.emplace_back((short)runs[i], vals[i]);
    return out;
}
}  // namespace detail

// RLE of a value list whose first entry is the DC (Coding.hpp:112-144)
inline std::vector<RLE_PAIR> RLE_AC(const std::vector<int>& data) {
    return detail::rle(reinterpret_cast<const int32_t*>(data.data()), data.size(), 0);
}
// RLE of an 8x8 block scanned in zig-zag order (Coding.hpp:148-183)
inline std::vector<RLE_PAIR> RLE_AC(const matrix<int>& data) {
    if (data.size1() != 8 || data.size2() != 8) throw std::invalid_argument("RLE_AC: 8x8 block expected");
    return detail::rle(reinterpret_cast<const int32_t*>(data.data().data()), 64, 1);
}

struct Category_Code {  // Coding.hpp:185-195
    uint8_t symbol;
    Bitstream code;
    Category_Code(uint8_t p, Bitstream b) : symbol(p), code(std::move(b)) {}
};
inline bool operator==(const Category_Code& l, const Category_Code& r) {
    return l.symbol == r.symbol && l.code == r.code;
}

inline void getCategoryAndCode(int value, short& category, Bitstream& code) {  // Coding.hpp:197-230
    uint16_t c = 0;
    uint32_t bits = 0;
    detail::check(jpge_category_code(value, &c, &bits), "getCategoryAndCode");
    category = (short)c;
    code = c ? Bitstream(bits, c) : Bitstream();
}
inline std::pair<short, Bitstream> getCategoryAndCode(int value) {  // Coding.hpp:232-262
    short c = 0;
    Bitstream b;
    getCategoryAndCode(value, c, b);
    return std::make_pair(c, b);
}

inline std::vector<Category_Code> encode_category(const std::vector<RLE_PAIR>& data) {  // Coding.hpp:265-283
    const size_t n = data.size();
    std::vector<uint8_t> runs(n), syms(n), lens(n);
    std::vector<int32_t> vals(n);
    std::vector<uint32_t> codes(n);
    for (size_t i = 0; i < n; ++i) {
        runs[i] = (uint8_t)data[i].num_zeros_before;
        vals[i] = data[i].value;
    }
    detail::check(jpge_encode_category(runs.data(), vals.data(), n, syms.data(), codes.data(), lens.data()),
                  "encode_category");
    std::vector<Category_Code> out;
    out.reserve(n);
    for (size_t i = 0; i < n; ++i) out.emplace_back(syms[i], lens[i] ? Bitstream(codes[i], lens[i]) : Bitstream());
    return out;
}

// ---- Huffman.hpp ----
struct Code {  // Huffman.hpp:21-46: the code MSB-aligned in a 32-bit word
    using CodeType = uint32_t;
    static const auto max_code_length = sizeof(CodeType) * 8;
    Code() : code(0), length(0) {}
    Code(CodeType c, uint8_t len) : code(len ? c << (max_code_length - len) : 0), length(len) {}
    explicit Code(const Bitstream& b) : code(b.extract((uint8_t)b.size(), 0)), length((uint8_t)b.size()) {}
    CodeType code;
    uint8_t length;
};
using SymbolCodeMap = std::unordered_map<int, Code>;
using SymbolsPerLength = std::vector<std::vector<int>>;

// generateHuffmanCode (Huffman.cpp:3-35): the length-limited (16) optimal code of a
// symbol text, with the reference's symbol order per length (libstdc++ container
// order); symbols[len] lists the symbols of each length (17 entries).
inline std::pair<SymbolCodeMap, SymbolsPerLength> generateHuffmanCode(std::vector<int> text) {
    if (text.empty()) throw std::invalid_argument("generateHuffmanCode: empty text");
    std::vector<int> syms(text.size() + 1), lens(text.size() + 1);
    std::vector<uint32_t> codes(text.size() + 1);
    int n = 0;
    detail::check(jpge_huffman_text(text.data(), text.size(), syms.data(), lens.data(), codes.data(), &n),
                  "generateHuffmanCode");
    SymbolCodeMap map;
    SymbolsPerLength per(17);
    for (int i = 0; i < n; ++i) {
        map[syms[i]] = Code(codes[i], (uint8_t)lens[i]);
        per[lens[i]].push_back(syms[i]);
    }
    return std::make_pair(map, per);
}

inline Bitstream huffmanEncode(std::vector<int> text, SymbolCodeMap code_map) {  // Huffman.cpp:69-76
    Bitstream r;
    for (int s : text) {
        const Code& c = code_map[s];
        r.push_back(c.code, c.length);
    }
    return r;
}

inline std::vector<int> huffmanDecode(Bitstream bitstream, SymbolCodeMap code_map) {  // Huffman.cpp:91-146
    std::vector<uint32_t> syms, codes;
    std::vector<uint8_t> lens;
    for (const auto& kv : code_map) {
        syms.push_back((uint32_t)kv.first);
        codes.push_back(kv.second.length ? kv.second.code >> (32 - kv.second.length) : 0);
        lens.push_back(kv.second.length);
    }
    std::vector<uint8_t> bytes = bitstream.blocks();
    bytes.push_back(0);
    size_t n = 0;
    detail::check(jpge_huffman_decode(bytes.data(), bitstream.size(), syms.data(), codes.data(), lens.data(),
                                      (int)syms.size(), nullptr, 0, &n),
                  "huffmanDecode");
    std::vector<int> out(n);
    detail::check(jpge_huffman_decode(bytes.data(), bitstream.size(), syms.data(), codes.data(), lens.data(),
                                      (int)syms.size(), out.data(), n, &n),
                  "huffmanDecode");
    return out;
}

// ---- Image.hpp ----
// fast version of atoi (Image.cpp:326-333): decimal digits, no checks
inline int fast_atoi(const char* str) {
    int val = 0;
    while (*str) val = val * 10 + (*str++ - '0');
    return val;
}

class Image : private detail::PlaneWatch {
  public:
    enum ColorSpace { RGB, YCbCr };
    enum SubsamplingMode { S444, S422, S411, S420, S420_m, S420_lm };  // Image.hpp:44-52
    enum DCTMode { Simple, Matrix, Arai };

    explicit Image(uint w, uint h, ColorSpace color);
    Image(const Image& other);
    Image(Image&& other);
    ~Image() = default;
    Image& operator=(const Image& other);
    Image& operator=(Image&& other);

    // Image.hpp:76-92
    Image convertToColorSpace(ColorSpace target_space) const;
    void applySubsampling(SubsamplingMode mode);
    void applyDCT(DCTMode mode);
    void applyQuantization(const matrix<Byte>& q_table_y, const matrix<Byte>& q_table_c);
    void applyDCdifferenceCoding();
    void doRLEandCategoryCoding();
    void doHuffmanEncoding(SymbolCodeMap& Y_DC, SymbolCodeMap& Y_AC, SymbolCodeMap& C_DC, SymbolCodeMap& C_AC);
    // The whole encode (Image.cpp:831-976) and the file.  Like the reference's, it
    // consumes the image: afterwards the image is YCbCr with empty planes.
    void writeJPEG(std::string file);

    // ---- extensions ----
    // writeJPEG at another quality (IJG scaling of the same tables; 50 = the reference's)
    void writeJPEG(const std::string& file, int quality);
    // the .jpg bytes of the image as writeJPEG would write them (the image is unchanged)
    std::vector<uint8_t> encode(int quality = 50) const;
    // the stage results the reference keeps private (Image.hpp:110-114)
    const matrix<PixelDataType>& dctY() const { return DctY; }
    const matrix<PixelDataType>& dctCb() const { return DctCb; }
    const matrix<PixelDataType>& dctCr() const { return DctCr; }
    const matrix<int>& qY() const { return QY; }
    const matrix<int>& qCb() const { return QCb; }
    const matrix<int>& qCr() const { return QCr; }
    const matrix<std::vector<Category_Code>>& categoryCodeY() const { return CategoryCodeY; }
    const matrix<std::vector<Category_Code>>& categoryCodeCb() const { return CategoryCodeCb; }
    const matrix<std::vector<Category_Code>>& categoryCodeCr() const { return CategoryCodeCr; }
    const matrix<Bitstream>& bitstreamY() const { return BitstreamY; }
    const matrix<Bitstream>& bitstreamCb() const { return BitstreamCb; }
    const matrix<Bitstream>& bitstreamCr() const { return BitstreamCr; }
    ColorSpace colorSpace() const { return color_space_type; }
    // true while the image is still the RGB8 frame loadPPM read (writeJPEG then takes
    // the fused RGB8 kernels; any write through a plane accessor ends this)
    bool isFrame() const { return src_valid_; }

    // Image.hpp:101-105
    uint width, height;
    uint real_width, real_height;
    uint subsample_width, subsample_height;
    matrix<PixelDataType>&R, &G, &B;
    matrix<PixelDataType>&Y, &Cb, &Cr;

  private:
    friend Image loadPPM(std::string path);
    void plane_access(bool write) override;
    void materialize();
    void bind();
    void shape_planes(uint rows, uint cols);  // plane sizes without data (materialised later)
    const double* plane_ptr(int i) const;

    ColorSpace color_space_type;
    matrix<PixelDataType> one, two, three;
    matrix<PixelDataType> DctY, DctCb, DctCr;
    matrix<int> QY, QCb, QCr;
    matrix<std::vector<Category_Code>> CategoryCodeY, CategoryCodeCb, CategoryCodeCr;
    matrix<Bitstream> BitstreamY, BitstreamCb, BitstreamCr;
    // the RGB8 frame of a loaded image (unscaled samples, real size) and its maxval;
    // the planes are materialised from it on first access
    std::shared_ptr<const std::vector<uint8_t>> src_;
    int maxval_ = 255;
    bool src_valid_ = false;
    bool materialized_ = true;
    bool in_watch_ = false;
};

// loadPPM (Image.hpp:28): P3 / P6; throws std::runtime_error on failure.
Image loadPPM(std::string path);

// The process-wide context the facade runs on (device JPGE_DEVICE, default 0).  Its
// calls are serialised by the library, so Images may be used from several threads.
jpge_ctx* default_context();

}  // namespace jpge

#ifndef JPGE_NO_GLOBAL_NAMES
// The reference declares these in the global namespace.
using jpge::Bitstream;
using jpge::Bitstream8;
using jpge::Bits;
using jpge::Byte;
using jpge::Category_Code;
using jpge::Code;
using jpge::Image;
using jpge::PixelDataType;
using jpge::RLE_AC;
using jpge::RLE_PAIR;
using jpge::SymbolCodeMap;
using jpge::SymbolsPerLength;
using jpge::encode_category;
using jpge::fast_atoi;
using jpge::from_vector;
using jpge::generateHuffmanCode;
using jpge::getCategoryAndCode;
using jpge::huffmanDecode;
using jpge::huffmanEncode;
using jpge::loadPPM;
using jpge::mat;
using jpge::matrix;
using jpge::quantize;
using jpge::uint;
using jpge::zigzag;
#endif
