#include "jpge_image.hpp"

#include <chrono>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <iterator>
#include <mutex>

namespace jpge {
namespace {

[[noreturn]] void fail(int st, const std::string& what) {
    throw std::runtime_error(what + ": " + jpge_strerror(st));
}

struct CtxHolder {
    jpge_ctx* ctx = nullptr;
    ~CtxHolder() { if (ctx) jpge_close(ctx); }
};

}  // namespace

jpge_ctx* default_context() {
    static CtxHolder holder;
    static std::once_flag once;
    static int status = 0;
    std::call_once(once, [] {
        const char* d = std::getenv("JPGE_DEVICE");
        status = jpge_open(d ? std::atoi(d) : 0, &holder.ctx);
    });
    if (status) fail(status, "jpge_open");
    return holder.ctx;
}

Image::Image(uint32_t w, uint32_t h, std::vector<uint8_t> rgb, int mv)
    : width((w + 15) / 16 * 16), height((h + 15) / 16 * 16), real_width(w), real_height(h),
      subsample_width(width / 2), subsample_height(height / 2), maxval(mv), rgb_(std::move(rgb)) {}

Image loadPPM(const std::string& path) {
    const auto start = std::chrono::high_resolution_clock::now();
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) throw std::runtime_error("Failed to open \"" + path + "\"");
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    uint32_t w = 0, h = 0;
    int mv = 0;
    int st = jpge_ppm_info(buf.data(), buf.size(), &w, &h, &mv);
    if (st == JPGE_E_FORMAT) throw std::runtime_error("Only P3 and P6 format is supported!");
    if (st) fail(st, "loadPPM(" + path + ")");
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    st = jpge_parse_ppm(buf.data(), buf.size(), rgb.data(), rgb.size(), &w, &h, &mv);
    if (st) fail(st, "loadPPM(" + path + ")");
    const auto end = std::chrono::high_resolution_clock::now();
    std::cout << "PPM loading took "
              << std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count() << " ms\n";
    return Image(w, h, std::move(rgb), mv);
}

std::vector<uint8_t> Image::encode(int quality) const {
    uint8_t qy[64], qc[64];
    int st = jpge_quality_tables(quality, qy, qc);
    if (st) fail(st, "quality");
    std::vector<uint8_t> out(jpge_max_jpeg_bytes(real_width, real_height));
    size_t len = 0;
    st = jpge_encode_rgb8(default_context(), rgb_.data(), real_width, real_height, 0, maxval, qy, qc, out.data(),
                          out.size(), &len, 0);
    if (st) fail(st, "writeJPEG");
    out.resize(len);
    return out;
}

void Image::writeJPEG(const std::string& file, int quality) const {
    const auto start = std::chrono::high_resolution_clock::now();
    std::cout << "Processing image size: " << real_width << "x" << real_height << std::endl;
    const std::vector<uint8_t> bytes = encode(quality);
    std::ofstream f(file, std::ios::binary);
    if (!f.is_open()) throw std::runtime_error("Failed to open \"" + file + "\"");
    f.write(reinterpret_cast<const char*>(bytes.data()), (std::streamsize)bytes.size());
    const auto end = std::chrono::high_resolution_clock::now();
    std::cout << "Encoding duration: "
              << std::chrono::duration_cast<std::chrono::milliseconds>(end - start).count() << " ms" << std::endl;
}

void Image::applyDCTAndQuantization(const uint8_t qy[64], const uint8_t qc[64]) {
    qy_.assign((size_t)width * height, 0);
    qcb_.assign((size_t)subsample_width * subsample_height, 0);
    qcr_.assign((size_t)subsample_width * subsample_height, 0);
    int st = jpge_fdct_quant(default_context(), rgb_.data(), real_width, real_height, 0, maxval, qy, qc,
                             qy_.data(), qcb_.data(), qcr_.data(), 0);
    if (st) fail(st, "applyDCTAndQuantization");
}

}  // namespace jpge
