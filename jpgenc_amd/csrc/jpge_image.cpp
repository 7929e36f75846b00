// The drop-in facade's Image (jpge_image.hpp) over the C ABI: loadPPM keeps the RGB8
// frame and materialises the reference's fp64 planes only when they are accessed;
// writeJPEG encodes the frame on the fused GPU path while it is untouched, else the
// planes on the GPU plane path; the plane stages run as GPU kernels; DC/RLE/category
// coding and Huffman emission build the reference's per-block structures on the host.
#include "jpge_image.hpp"

#include <chrono>
#include <cstdlib>
#include <fstream>
#include <future>
#include <iostream>
#include <iterator>
#include <mutex>

namespace jpge {
using detail::check;
using detail::fail;

jpge_ctx* default_context() {
    // opened once; never closed here (a static destructor would run HIP calls during
    // the runtime's own teardown): the library's exit handler closes it (live.hpp)
    static jpge_ctx* ctx = nullptr;
    static int status = 0;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* d = std::getenv("JPGE_DEVICE");
        status = jpge_open(d ? std::atoi(d) : 0, &ctx);
    });
    if (status) fail(status, "jpge_open");
    return ctx;
}

// ---- construction, copies, plane binding ----

Image::Image(uint w, uint h, ColorSpace color)  // Image.cpp:31-41
    : width(w), height(h), real_width(w), real_height(h), subsample_width(w), subsample_height(h),
      R(one), G(two), B(three), Y(one), Cb(two), Cr(three), color_space_type(color), one(h, w), two(h, w),
      three(h, w) {
    bind();
}

Image::Image(const Image& o)
    : width(o.width), height(o.height), real_width(o.real_width), real_height(o.real_height),
      subsample_width(o.subsample_width), subsample_height(o.subsample_height), R(one), G(two), B(three), Y(one),
      Cb(two), Cr(three), color_space_type(o.color_space_type), DctY(o.DctY), DctCb(o.DctCb), DctCr(o.DctCr),
      QY(o.QY), QCb(o.QCb), QCr(o.QCr), CategoryCodeY(o.CategoryCodeY), CategoryCodeCb(o.CategoryCodeCb),
      CategoryCodeCr(o.CategoryCodeCr), BitstreamY(o.BitstreamY), BitstreamCb(o.BitstreamCb),
      BitstreamCr(o.BitstreamCr), src_(o.src_), maxval_(o.maxval_), src_valid_(o.src_valid_),
      materialized_(o.materialized_) {
    // the planes: raw copies (an unmaterialised source stays unmaterialised here too)
    one.r_ = o.one.r_; one.c_ = o.one.c_; one.v_ = o.one.v_;
    two.r_ = o.two.r_; two.c_ = o.two.c_; two.v_ = o.two.v_;
    three.r_ = o.three.r_; three.c_ = o.three.c_; three.v_ = o.three.v_;
    bind();
}

Image::Image(Image&& o)
    : width(o.width), height(o.height), real_width(o.real_width), real_height(o.real_height),
      subsample_width(o.subsample_width), subsample_height(o.subsample_height), R(one), G(two), B(three), Y(one),
      Cb(two), Cr(three), color_space_type(o.color_space_type), DctY(std::move(o.DctY)), DctCb(std::move(o.DctCb)),
      DctCr(std::move(o.DctCr)), QY(std::move(o.QY)), QCb(std::move(o.QCb)), QCr(std::move(o.QCr)),
      CategoryCodeY(std::move(o.CategoryCodeY)), CategoryCodeCb(std::move(o.CategoryCodeCb)),
      CategoryCodeCr(std::move(o.CategoryCodeCr)), BitstreamY(std::move(o.BitstreamY)),
      BitstreamCb(std::move(o.BitstreamCb)), BitstreamCr(std::move(o.BitstreamCr)), src_(std::move(o.src_)),
      maxval_(o.maxval_), src_valid_(o.src_valid_), materialized_(o.materialized_) {
    one.r_ = o.one.r_; one.c_ = o.one.c_; one.v_ = std::move(o.one.v_);
    two.r_ = o.two.r_; two.c_ = o.two.c_; two.v_ = std::move(o.two.v_);
    three.r_ = o.three.r_; three.c_ = o.three.c_; three.v_ = std::move(o.three.v_);
    bind();
}

Image& Image::operator=(const Image& o) {  // Image.cpp:77-92 (plus the stage state)
    if (this != &o) {
        Image t(o);
        *this = std::move(t);
    }
    return *this;
}

Image& Image::operator=(Image&& o) {
    if (this != &o) {
        width = o.width; height = o.height;
        real_width = o.real_width; real_height = o.real_height;
        subsample_width = o.subsample_width; subsample_height = o.subsample_height;
        color_space_type = o.color_space_type;
        one.r_ = o.one.r_; one.c_ = o.one.c_; one.v_ = std::move(o.one.v_);
        two.r_ = o.two.r_; two.c_ = o.two.c_; two.v_ = std::move(o.two.v_);
        three.r_ = o.three.r_; three.c_ = o.three.c_; three.v_ = std::move(o.three.v_);
        DctY = std::move(o.DctY); DctCb = std::move(o.DctCb); DctCr = std::move(o.DctCr);
        QY = std::move(o.QY); QCb = std::move(o.QCb); QCr = std::move(o.QCr);
        CategoryCodeY = std::move(o.CategoryCodeY); CategoryCodeCb = std::move(o.CategoryCodeCb);
        CategoryCodeCr = std::move(o.CategoryCodeCr);
        BitstreamY = std::move(o.BitstreamY); BitstreamCb = std::move(o.BitstreamCb);
        BitstreamCr = std::move(o.BitstreamCr);
        src_ = std::move(o.src_);
        maxval_ = o.maxval_;
        src_valid_ = o.src_valid_;
        materialized_ = o.materialized_;
    }
    return *this;
}

void Image::shape_planes(uint rows, uint cols) {
    for (auto* p : {&one, &two, &three}) {
        p->r_ = rows;
        p->c_ = cols;
        p->v_.clear();
    }
}

void Image::bind() {
    one.watch_ = this;
    two.watch_ = this;
    three.watch_ = this;
}

void Image::plane_access(bool write) {
    if (in_watch_) return;
    if (!materialized_) materialize();
    if (write) src_valid_ = false;
}

// The planes of a loaded image, as loadPPM builds them (Image.cpp:393-531): sample *
// (255. / maxval) in double, padded to the image size by edge replication.
void Image::materialize() {
    materialized_ = true;
    if (!src_) return;
    in_watch_ = true;
    const double scale = 255. / maxval_;
    const auto& s = *src_;
    matrix<PixelDataType>* pl[3] = {&one, &two, &three};
    for (auto* p : pl) p->v_.assign((size_t)p->r_ * p->c_, 0.0);
    for (uint y = 0; y < height; ++y) {
        const uint sy = std::min(y, real_height - 1);
        for (uint x = 0; x < width; ++x) {
            const uint sx = std::min(x, real_width - 1);
            const uint8_t* px = &s[((size_t)sy * real_width + sx) * 3];
            for (int c = 0; c < 3; ++c) pl[c]->v_[(size_t)y * width + x] = px[c] * scale;
        }
    }
    in_watch_ = false;
}

const double* Image::plane_ptr(int i) const {
    const matrix<PixelDataType>& p = i == 0 ? one : i == 1 ? two : three;
    return p.cdata().data();
}

// ---- loadPPM (Image.cpp:421-538) ----

Image loadPPM(std::string path) {
    const auto start = std::chrono::high_resolution_clock::now();
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) throw std::runtime_error("Failed to open \"" + path + "\"");
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    uint32_t w = 0, h = 0;
    int mv = 0;
    int st = jpge_ppm_info(buf.data(), buf.size(), &w, &h, &mv);
    if (st == JPGE_E_FORMAT) throw std::runtime_error("Only P3 and P6 format is supported!");
    if (st) fail(st, "loadPPM(" + path + ")");
    auto rgb = std::make_shared<std::vector<uint8_t>>((size_t)w * h * 3);
    st = jpge_parse_ppm(buf.data(), buf.size(), rgb->data(), rgb->size(), &w, &h, &mv);
    if (st) fail(st, "loadPPM(" + path + ")");
    // the padded size (Image.cpp:480-492); the planes stay unmaterialised
    const uint pw = (w + 15) / 16 * 16, ph = (h + 15) / 16 * 16;
    Image img(0, 0, Image::RGB);
    img.width = pw;
    img.height = ph;
    img.real_width = w;
    img.real_height = h;
    img.subsample_width = pw;
    img.subsample_height = ph;
    img.shape_planes(ph, pw);
    img.src_ = std::move(rgb);
    img.maxval_ = mv;
    img.src_valid_ = true;
    img.materialized_ = false;
    const auto end = std::chrono::high_resolution_clock::now();
    std::cout << "PPM loading took " << std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count()
              << " ms\n";
    return img;
}

// ---- stages ----

Image Image::convertToColorSpace(ColorSpace target) const {  // Image.cpp:112-179
    if (color_space_type == target) return *this;
    Image c(*this);
    const size_t n = (size_t)one.size1() * one.size2();
    if (two.size1() * two.size2() != n || three.size1() * three.size2() != n)
        throw std::logic_error("convertToColorSpace: the planes differ in size (subsampled chroma)");
    std::vector<double> o0(n), o1(n), o2(n);
    check(jpge_color_convert(default_context(), plane_ptr(0), plane_ptr(1), plane_ptr(2), o0.data(), o1.data(),
                             o2.data(), n, target == YCbCr ? JPGE_TO_YCBCR : JPGE_TO_RGB, 0),
          "convertToColorSpace");
    c.in_watch_ = true;
    c.one.v_ = std::move(o0);
    c.two.v_ = std::move(o1);
    c.three.v_ = std::move(o2);
    c.in_watch_ = false;
    c.materialized_ = true;
    c.src_valid_ = false;
    c.color_space_type = target;
    return c;
}

namespace {
int mode_code(Image::SubsamplingMode m) {  // Image::SubsamplingMode -> jpge.h JPGE_S*
    switch (m) {
        case Image::S444: return JPGE_S444;
        case Image::S422: return JPGE_S422;
        case Image::S411: return JPGE_S411;
        case Image::S420: return JPGE_S420;
        case Image::S420_m: return JPGE_S420_M;
        case Image::S420_lm: return JPGE_S420_LM;
    }
    return -1;
}

void subsample_plane(matrix<PixelDataType>& chan, const std::vector<double>& in, int mode) {
    uint32_t orows = 0, ocols = 0;
    check(jpge_subsample_plane(default_context(), in.data(), (uint32_t)chan.size1(), (uint32_t)chan.size2(), mode,
                               nullptr, &orows, &ocols, 0),
          "applySubsampling");
    std::vector<double> out((size_t)orows * ocols);
    check(jpge_subsample_plane(default_context(), in.data(), (uint32_t)chan.size1(), (uint32_t)chan.size2(), mode,
                               out.data(), &orows, &ocols, 0),
          "applySubsampling");
    chan = matrix<PixelDataType>(orows, ocols);  // (keeps the plane's watch)
    chan.data() = std::move(out);
}
}  // namespace

void Image::applySubsampling(SubsamplingMode mode) {  // Image.cpp:237-319
    if (mode == S444) return;
    const int code = mode_code(mode);
    const uint hdiv = mode == S411 ? 4 : 2, vdiv = (mode == S422 || mode == S411) ? 1 : 2;
    subsample_width = width / hdiv;
    subsample_height = height / vdiv;
    const std::vector<double> cr = three.data(), cb = two.data();  // (materialises; a write follows)
    subsample_plane(three, cr, code);
    subsample_plane(two, cb, code);
}

void Image::applyDCT(DCTMode mode) {  // Image.cpp:540-595
    const int m = mode == Simple ? JPGE_DCT_SIMPLE : mode == Matrix ? JPGE_DCT_MATRIX : JPGE_DCT_ARAI;
    auto run = [&](const matrix<PixelDataType>& src, int idx, matrix<PixelDataType>& dst) {
        dst = matrix<PixelDataType>(src.size1(), src.size2());
        check(jpge_dct_plane(default_context(), plane_ptr(idx), (uint32_t)src.size1(), (uint32_t)src.size2(), m,
                             dst.data().data(), 0),
              "applyDCT");
    };
    run(Y, 0, DctY);
    run(Cb, 1, DctCb);
    run(Cr, 2, DctCr);
}

void Image::applyQuantization(const matrix<Byte>& qy, const matrix<Byte>& qc) {  // Image.cpp:597-636
    if (qy.size1() != 8 || qy.size2() != 8 || qc.size1() != 8 || qc.size2() != 8)
        throw std::invalid_argument("applyQuantization: 8x8 tables expected");
    auto run = [&](const matrix<PixelDataType>& src, const matrix<Byte>& t, matrix<int>& dst) {
        dst = matrix<int>(src.size1(), src.size2());
        check(jpge_quantize_plane(default_context(), src.data().data(), (uint32_t)src.size1(), (uint32_t)src.size2(),
                                  t.data().data(), reinterpret_cast<int32_t*>(dst.data().data()), 0),
              "applyQuantization");
    };
    run(DctY, qy, QY);
    run(DctCb, qc, QCb);
    run(DctCr, qc, QCr);
}

void Image::applyDCdifferenceCoding() {  // Image.cpp:638-678
    check(jpge_dc_difference(reinterpret_cast<int32_t*>(QY.data().data()), (uint32_t)QY.size1(), (uint32_t)QY.size2(),
                             reinterpret_cast<int32_t*>(QCb.data().data()),
                             reinterpret_cast<int32_t*>(QCr.data().data()), (uint32_t)QCb.size1(),
                             (uint32_t)QCb.size2()),
          "applyDCdifferenceCoding");
}

namespace {
// RLE + category coding of every block of a plane, raster order (Image.cpp:692-729)
void rle_plane(const matrix<int>& q, matrix<std::vector<Category_Code>>& out) {
    out = matrix<std::vector<Category_Code>>(q.size1() / 8, q.size2() / 8);
    const auto& d = q.data();
    matrix<int> blk(8, 8);
    for (size_t by = 0; by < out.size1(); ++by)
        for (size_t bx = 0; bx < out.size2(); ++bx) {
            for (int r = 0; r < 8; ++r)
                for (int c = 0; c < 8; ++c) blk(r, c) = d[(by * 8 + r) * q.size2() + bx * 8 + c];
            out(by, bx) = encode_category(RLE_AC(blk));
        }
}

// Huffman emission of every block of a plane (Image.cpp:747-823)
void emit_plane(const matrix<std::vector<Category_Code>>& cc, SymbolCodeMap& dc, SymbolCodeMap& ac,
                matrix<Bitstream>& out) {
    out = matrix<Bitstream>(cc.size1(), cc.size2());
    for (size_t i = 0; i < cc.size1(); ++i)
        for (size_t j = 0; j < cc.size2(); ++j) {
            Bitstream s;
            const auto& data = cc(i, j);
            const Code& d = dc[data[0].symbol];
            s.push_back(d.code, d.length);
            s << data[0].code;
            for (size_t k = 1; k < data.size(); ++k) {
                const Code& a = ac[data[k].symbol];
                s.push_back(a.code, a.length);
                s << data[k].code;
            }
            out(i, j) = std::move(s);
        }
}
}  // namespace

void Image::doRLEandCategoryCoding() {  // Image.cpp:680-735, one task per component
    auto f1 = std::async(std::launch::async, [&] { rle_plane(QY, CategoryCodeY); });
    auto f2 = std::async(std::launch::async, [&] { rle_plane(QCb, CategoryCodeCb); });
    rle_plane(QCr, CategoryCodeCr);
    f1.get();
    f2.get();
}

void Image::doHuffmanEncoding(SymbolCodeMap& Y_DC, SymbolCodeMap& Y_AC, SymbolCodeMap& C_DC,
                              SymbolCodeMap& C_AC) {  // Image.cpp:737-829
    emit_plane(CategoryCodeY, Y_DC, Y_AC, BitstreamY);
    emit_plane(CategoryCodeCb, C_DC, C_AC, BitstreamCb);
    emit_plane(CategoryCodeCr, C_DC, C_AC, BitstreamCr);
}

// ---- encode ----

std::vector<uint8_t> Image::encode(int quality) const {
    uint8_t qy[64], qc[64];
    check(jpge_quality_tables(quality, qy, qc), "quality");
    std::vector<uint8_t> out;
    size_t len = 0;
    if (src_valid_ && color_space_type == RGB) {  // the RGB8 frame: the fused kernels
        out.resize(jpge_max_jpeg_bytes(real_width, real_height));
        check(jpge_encode_rgb8(default_context(), src_->data(), real_width, real_height, 0, maxval_, qy, qc,
                               out.data(), out.size(), &len, 0),
              "writeJPEG");
    } else {  // the planes: colour (if RGB), S420_m, DCT, quantisation on the GPU plane kernels
        if (two.size1() != one.size1() || two.size2() != one.size2() || three.size1() != one.size1() ||
            three.size2() != one.size2())
            throw std::logic_error("writeJPEG: the chroma planes are already subsampled");
        out.resize(jpge_max_jpeg_bytes((uint32_t)one.size2(), (uint32_t)one.size1()));
        check(jpge_encode_planes(default_context(), plane_ptr(0), plane_ptr(1), plane_ptr(2), (uint32_t)one.size1(),
                                 (uint32_t)one.size2(), color_space_type == YCbCr ? JPGE_TO_YCBCR : JPGE_TO_RGB,
                                 real_width, real_height, qy, qc, out.data(), out.size(), &len, 0),
              "writeJPEG");
    }
    out.resize(len);
    return out;
}

void Image::writeJPEG(std::string file) { writeJPEG(file, 50); }

void Image::writeJPEG(const std::string& file, int quality) {  // Image.cpp:831-976
    const auto start = std::chrono::high_resolution_clock::now();
    std::cout << "Processing image size: " << real_width << "x" << real_height << std::endl;
    const std::vector<uint8_t> bytes = encode(quality);
    std::ofstream f(file, std::ios::binary);
    if (!f.is_open()) throw std::runtime_error("Failed to open \"" + file + "\"");
    f.write(reinterpret_cast<const char*>(bytes.data()), (std::streamsize)bytes.size());
    // the reference leaves the image converted, subsampled and emptied (Image.cpp:839-885)
    in_watch_ = true;
    for (auto* p : {&one, &two, &three}) {
        p->r_ = p->c_ = 0;
        p->v_.clear();
    }
    in_watch_ = false;
    materialized_ = true;
    src_valid_ = false;
    color_space_type = YCbCr;
    subsample_width = width / 2;
    subsample_height = height / 2;
    const auto end = std::chrono::high_resolution_clock::now();
    std::cout << "Encoding duration: " << std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count()
              << " ms" << std::endl;
}

}  // namespace jpge
