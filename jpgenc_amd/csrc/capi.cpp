// extern "C" boundary (include/jpge.h) over jpge::Encoder and the host pieces.
#include "jpge.h"

#include <pthread.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "constants.hpp"
#include "encoder.hpp"
#include "host_io.hpp"
#include "huffman.hpp"
#include "ingest.hpp"
#include "kernels.hpp"
#include "live.hpp"

struct jpge_ctx {
    std::unique_ptr<jpge::Encoder> enc;
    std::unique_ptr<jpge::IngestBuffers, jpge::IngestBuffersDeleter> ingest;  // jpge_encode_files' buffers
    // calls in flight, and the exit handler's release (live_release): a call that got in is
    // waited for, every later one returns JPGE_E_ARG
    std::mutex use_mu;
    std::condition_variable use_cv;
    int inflight = 0;
    bool released = false;
};

namespace {
// An entry point's use of a context: false for a null or released handle (or one without
// an encoder); otherwise counted in flight until the call returns.
class CtxUse {
  public:
    explicit CtxUse(jpge_ctx* c) : c_(c) {
        if (!c_) return;
        std::lock_guard<std::mutex> l(c_->use_mu);
        if (c_->released || !c_->enc) { c_ = nullptr; return; }
        ++c_->inflight;
    }
    ~CtxUse() {
        if (!c_) return;
        std::lock_guard<std::mutex> l(c_->use_mu);
        if (--c_->inflight == 0) c_->use_cv.notify_all();
    }
    explicit operator bool() const { return c_ != nullptr; }
    CtxUse(const CtxUse&) = delete;
    CtxUse& operator=(const CtxUse&) = delete;

  private:
    jpge_ctx* c_;
};
jpge::FrameDesc frame(const uint8_t* rgb, uint32_t w, uint32_t h, size_t stride, int maxval) {
    jpge::FrameDesc f;
    f.rgb = rgb;
    f.width = w;
    f.height = h;
    f.stride = stride;
    f.maxval = maxval;
    return f;
}
}  // namespace

namespace jpge {
namespace {
struct LiveSet {
    std::mutex mu;
    std::vector<jpge_ctx*> ctx;
    std::vector<jpge_group*> grp;
    // handles the exit handler released: their resources are gone, the handle stays valid
    // so that a caller's own later jpge_close / jpge_group_close is a no-op
    std::vector<const void*> dead;
};
LiveSet& live() {
    static LiveSet* s = new LiveSet();  // never destroyed: it must outlive every exit handler
    return *s;
}
// (live.hpp) releases every group, then every context, still open at exit
void close_live_at_exit() {
    for (;;) {
        jpge_group* g = nullptr;
        {
            std::lock_guard<std::mutex> l(live().mu);
            if (!live().grp.empty()) g = live().grp.back();
        }
        if (!g) break;
        live_release(g);  // (group.cpp: its RCCL communicators and member contexts too)
    }
    for (;;) {
        jpge_ctx* c = nullptr;
        {
            std::lock_guard<std::mutex> l(live().mu);
            if (!live().ctx.empty()) c = live().ctx.back();
        }
        if (!c) break;
        live_release(c);
    }
}
void forget_in_child() {  // a forked child: the parent's lane threads do not exist here
    live().ctx.clear();
    live().grp.clear();
    new (&live().mu) std::mutex();
}
std::once_flag g_first_open;
template <typename T>
void erase_one(std::vector<T*>& v, T* x) {
    auto it = std::find(v.begin(), v.end(), x);
    if (it != v.end()) v.erase(it);
}
}  // namespace

void live_add(jpge_ctx* c) {
    std::call_once(g_first_open, [] {
        live();
        std::atexit(close_live_at_exit);
        pthread_atfork(nullptr, nullptr, forget_in_child);
    });
    std::lock_guard<std::mutex> l(live().mu);
    live().ctx.push_back(c);
}
void live_remove(jpge_ctx* c) {
    std::lock_guard<std::mutex> l(live().mu);
    erase_one(live().ctx, c);
}
void live_add(jpge_group* g) {
    std::lock_guard<std::mutex> l(live().mu);
    live().grp.push_back(g);
}
void live_remove(jpge_group* g) {
    std::lock_guard<std::mutex> l(live().mu);
    erase_one(live().grp, g);
}
bool live_is_released(const void* h) {
    std::lock_guard<std::mutex> l(live().mu);
    return std::find(live().dead.begin(), live().dead.end(), h) != live().dead.end();
}
void live_mark_released(const void* h) {
    std::lock_guard<std::mutex> l(live().mu);
    live().dead.push_back(h);
}
void live_release(jpge_ctx* c) {
    live_remove(c);
    {  // no call gets in from now on; the ones in flight are waited for, then tear down
        std::unique_lock<std::mutex> l(c->use_mu);
        c->released = true;
        c->use_cv.wait(l, [&] { return c->inflight == 0; });
    }
    c->enc.reset();
    c->ingest.reset();
    live_mark_released(c);
}
void live_handler_after_load() {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(close_live_at_exit); });
}
}  // namespace jpge

extern "C" {

const char* jpge_strerror(int s) {
    switch (s) {
        case JPGE_OK: return "ok";
        case JPGE_E_ARG: return "invalid argument";
        case JPGE_E_NOSPACE: return "output buffer too small";
        case JPGE_E_HIP: return "HIP runtime error";
        case JPGE_E_NODEV: return "no such GPU device";
        case JPGE_E_FORMAT: return "Only P3 and P6 format is supported!";
        case JPGE_E_IO: return "failed to open file";
        case JPGE_E_TRUNC: return "PPM sample data truncated";
        case JPGE_E_RANGE: return "value out of range (maxval must be 1..255)";
        case JPGE_E_TIMEOUT: return "device scan protocol timed out";
        case JPGE_E_RCCL: return "RCCL error";
        default: return "internal error";
    }
}

int jpge_version(void) { return 100; }

int jpge_device_count(int* n) {
    if (!n) return JPGE_E_ARG;
    if (hipGetDeviceCount(n) != hipSuccess) { *n = 0; return JPGE_E_NODEV; }
    return JPGE_OK;
}

int jpge_open(int device, jpge_ctx** ctx) { return jpge_open_ex(device, 0, ctx); }

int jpge_open_ex(int device, int lanes, jpge_ctx** ctx) {
    if (!ctx) return JPGE_E_ARG;
    *ctx = nullptr;
    if (lanes < 0) return JPGE_E_ARG;
    std::unique_ptr<jpge_ctx> c(new (std::nothrow) jpge_ctx());
    if (!c) return JPGE_E_INTERNAL;
    int st = jpge::Encoder::open(device, c->enc, lanes);
    if (st) return st;
    *ctx = c.release();
    jpge::live_add(*ctx);  // (closed at exit if the caller does not: live.hpp)
    return JPGE_OK;
}

int jpge_close(jpge_ctx* ctx) {
    if (!ctx || jpge::live_is_released(ctx)) return JPGE_OK;  // (released at exit: live.hpp)
    jpge::live_remove(ctx);
    delete ctx;
    return JPGE_OK;
}

int jpge_set_timing(jpge_ctx* ctx, int every) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    ctx->enc->set_timing(every);
    return JPGE_OK;
}

int jpge_get_timing(jpge_ctx* ctx, jpge_timing* t) {
    CtxUse use(ctx);
    if (!use || !t) return JPGE_E_ARG;
    const auto& k = ctx->enc->times();
    t->fdct = k.fdct;
    t->dc_stats = k.dc_stats;
    t->entropy = k.entropy;
    t->total = k.total;
    t->fdct_sum = k.fdct_sum;
    t->dc_stats_sum = k.dc_stats_sum;
    t->entropy_sum = k.entropy_sum;
    t->frames = k.frames;
    t->symbols = k.symbols;
    t->code_sum = k.code_sum;
    t->pack_sum = k.pack_sum;
    t->launches = k.launches;
    t->gate_timeouts = ctx->enc->gate_timeouts();
    return JPGE_OK;
}

int jpge_reset_timing(jpge_ctx* ctx) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    ctx->enc->reset_timing();
    return JPGE_OK;
}

int jpge_get_lanes(jpge_ctx* ctx, int* lanes) {
    CtxUse use(ctx);
    if (!use || !lanes) return JPGE_E_ARG;
    *lanes = ctx->enc->lanes();
    return JPGE_OK;
}

int jpge_set_restart_interval(jpge_ctx* ctx, uint32_t mcus) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    return ctx->enc->set_restart(mcus) ? JPGE_E_ARG : JPGE_OK;
}

int jpge_set_subsampling(jpge_ctx* ctx, int mode) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    return ctx->enc->set_subsampling(mode) ? JPGE_E_ARG : JPGE_OK;
}

size_t jpge_max_jpeg_bytes(uint32_t w, uint32_t h) { return jpge::Encoder::max_jpeg_bytes(w, h); }

int jpge_quality_tables(int quality, uint8_t qy[64], uint8_t qc[64]) {
    if (!qy || !qc || quality < 1 || quality > 100) return JPGE_E_ARG;
    jpge::quality_tables(quality, qy, qc);
    return JPGE_OK;
}

int jpge_encode_rgb8(jpge_ctx* ctx, const uint8_t* rgb, uint32_t w, uint32_t h, size_t stride, int maxval,
                     const uint8_t qy[64], const uint8_t qc[64], uint8_t* out, size_t cap, size_t* len,
                     uint32_t flags) {
    CtxUse use(ctx);
    if (!use || !rgb || !qy || !qc || !out || !len) return JPGE_E_ARG;
    jpge::FrameDesc f = frame(rgb, w, h, stride, maxval);
    f.out = out;
    f.cap = cap;
    int st = ctx->enc->encode(f, qy, qc, flags);
    *len = f.len;
    return st;
}

int jpge_encode_batch(jpge_ctx* ctx, jpge_frame* frames, int n, const uint8_t qy[64], const uint8_t qc[64],
                      uint32_t flags) {
    CtxUse use(ctx);
    if (!use || (!frames && n) || n < 0 || !qy || !qc) return JPGE_E_ARG;
    std::vector<jpge::FrameDesc> fd(n);
    for (int i = 0; i < n; ++i) {
        fd[i] = frame(frames[i].rgb, frames[i].width, frames[i].height, frames[i].stride, frames[i].maxval);
        fd[i].out = frames[i].out;
        fd[i].cap = frames[i].cap;
    }
    int st = ctx->enc->encode_batch(fd.data(), n, qy, qc, flags);
    for (int i = 0; i < n; ++i) {
        frames[i].len = fd[i].len;
        frames[i].status = fd[i].status;
    }
    return st;
}

int jpge_fdct_quant(jpge_ctx* ctx, const uint8_t* rgb, uint32_t w, uint32_t h, size_t stride, int maxval,
                    const uint8_t qy[64], const uint8_t qc[64], int16_t* cy, int16_t* ccb, int16_t* ccr,
                    uint32_t flags) {
    CtxUse use(ctx);
    if (!use || !rgb || !qy || !qc || !cy || !ccb || !ccr) return JPGE_E_ARG;
    return ctx->enc->fdct_quant(frame(rgb, w, h, stride, maxval), qy, qc, flags, cy, ccb, ccr);
}

int jpge_symbol_stats(jpge_ctx* ctx, const uint8_t* rgb, uint32_t w, uint32_t h, size_t stride, int maxval,
                      const uint8_t qy[64], const uint8_t qc[64], uint32_t counts[1024], uint64_t first[1024],
                      uint32_t flags) {
    CtxUse use(ctx);
    if (!use || !rgb || !qy || !qc || !counts || !first) return JPGE_E_ARG;
    return ctx->enc->symbol_stats(frame(rgb, w, h, stride, maxval), qy, qc, flags, counts, first);
}

int jpge_concat_segments(int device, void* stream, const uint8_t* const* segs, const size_t* lens, int n,
                         uint8_t* dst, size_t* total) {
    if (n < 0 || (n > 0 && (!segs || !lens || !dst))) return JPGE_E_ARG;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return JPGE_E_HIP;
    if (prev != device && hipSetDevice(device) != hipSuccess) return JPGE_E_NODEV;
    int st = JPGE_OK;
    uint64_t off = 0;
    for (int k0 = 0; k0 < n && st == JPGE_OK; k0 += (int)jpge::kConcatMax) {
        jpge::ConcatArgs a;
        a.dst = dst;
        a.n = (uint32_t)std::min<int>(n - k0, (int)jpge::kConcatMax);
        uint32_t c = 0;
        for (uint32_t k = 0; k < a.n; ++k) {
            if (lens[k0 + k] && !segs[k0 + k]) { st = JPGE_E_ARG; break; }
            a.src[k] = segs[k0 + k];
            a.len[k] = lens[k0 + k];
            a.off[k] = off;
            a.chunk0[k] = c;
            c += jpge::concat_chunks(a.len[k], reinterpret_cast<uintptr_t>(dst + off));
            off += a.len[k];
        }
        a.chunk0[a.n] = c;
        if (st == JPGE_OK && jpge::launch_concat(a, c, static_cast<hipStream_t>(stream)) != hipSuccess)
            st = JPGE_E_HIP;
    }
    if (total) *total = (size_t)off;
    if (prev != device) hipSetDevice(prev);
    return st;
}

int jpge_huffman_table(const uint32_t counts[256], const uint64_t first[256], uint8_t bits[16],
                       uint8_t huffval[256], int* nsym, uint32_t code[256], uint8_t len[256]) {
    if (!counts || !first || !bits || !huffval || !nsym || !code || !len) return JPGE_E_ARG;
    jpge::HuffTable t;
    if (!jpge::build_table(counts, first, t)) return JPGE_E_ARG;
    std::memcpy(bits, t.bits + 1, 16);
    std::memcpy(huffval, t.huffval, 256);
    *nsym = t.nsym;
    std::memcpy(code, t.code, sizeof(t.code));
    std::memcpy(len, t.len, sizeof(t.len));
    return JPGE_OK;
}

int jpge_huffman_text(const int* text, size_t n, int* syms, int* lens, uint32_t* codes, int* nsym) {
    if (!text || !n || !syms || !lens || !codes || !nsym) return JPGE_E_ARG;
    auto r = jpge::generateHuffmanCode(std::vector<int>(text, text + n));
    int k = 0;
    for (const auto& sc : r.first) {
        syms[k] = sc.first;
        lens[k] = sc.second.length;
        codes[k] = sc.second.code;
        ++k;
    }
    *nsym = k;
    return JPGE_OK;
}

int jpge_ppm_info(const uint8_t* buf, size_t n, uint32_t* w, uint32_t* h, int* maxval) {
    if (!buf || !w || !h || !maxval) return JPGE_E_ARG;
    jpge::PpmImage img;
    int st = jpge::parse_ppm(buf, n, img);
    if (st && st != jpge::kErrTruncated && st != jpge::kErrRange) return st;
    if (!img.width) return st ? st : JPGE_E_FORMAT;
    *w = img.width;
    *h = img.height;
    *maxval = img.maxval;
    return JPGE_OK;
}

int jpge_parse_ppm(const uint8_t* buf, size_t n, uint8_t* rgb, size_t cap, uint32_t* w, uint32_t* h, int* maxval) {
    if (!buf || !rgb || !w || !h || !maxval) return JPGE_E_ARG;
    jpge::PpmImage img;
    int st = jpge::parse_ppm(buf, n, img);
    if (st) return st;
    if (img.rgb.size() > cap) return JPGE_E_NOSPACE;
    std::memcpy(rgb, img.rgb.data(), img.rgb.size());
    *w = img.width;
    *h = img.height;
    *maxval = img.maxval;
    return JPGE_OK;
}

int jpge_encode_file(jpge_ctx* ctx, const char* ppm_path, const char* jpg_path, int quality) {
    CtxUse use(ctx);
    if (!use || !ppm_path || !jpg_path) return JPGE_E_ARG;
    jpge::PpmImage img;
    int st = jpge::load_ppm_file(ppm_path, img);
    if (st) return st;
    uint8_t qy[64], qc[64];
    if (quality < 1 || quality > 100) return JPGE_E_ARG;
    jpge::quality_tables(quality, qy, qc);
    std::vector<uint8_t> out(jpge::Encoder::max_jpeg_bytes(img.width, img.height));
    size_t len = 0;
    st = jpge_encode_rgb8(ctx, img.rgb.data(), img.width, img.height, 0, img.maxval, qy, qc, out.data(),
                          out.size(), &len, 0);
    if (st) return st;
    std::ofstream f(jpg_path, std::ios::binary);
    if (!f.is_open()) return JPGE_E_IO;
    f.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)len);
    return f.good() ? JPGE_OK : JPGE_E_IO;
}

int jpge_encode_files(jpge_ctx* ctx, const char* const* ppm_paths, const char* const* jpg_paths, int n, int quality,
                      size_t* lens, int* statuses, int group) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    return jpge::encode_files(*ctx->enc, ctx->ingest, ppm_paths, jpg_paths, n, quality, lens, statuses, group);
}

int jpge_synth_rgb8(uint64_t seed, uint32_t w, uint32_t h, int kind, uint8_t* out, size_t stride) {
    if (!out || !w || !h || kind < 0 || kind > 2) return JPGE_E_ARG;
    jpge::synth_rgb8(seed, w, h, kind, out, stride ? stride : (size_t)w * 3);
    return JPGE_OK;
}

void jpge_arai_constants(double a[5], double s[8]) {
    a[0] = jpge::kA1; a[1] = jpge::kA2; a[2] = jpge::kA3; a[3] = jpge::kA4; a[4] = jpge::kA5;
    s[0] = jpge::kS0; s[1] = jpge::kS1; s[2] = jpge::kS2; s[3] = jpge::kS3;
    s[4] = jpge::kS4; s[5] = jpge::kS5; s[6] = jpge::kS6; s[7] = jpge::kS7;
}

static_assert(sizeof(jpge_stripe_summary) == sizeof(jpge::StripeSummary), "stripe summary layout");

int jpge_stripe_transform(jpge_ctx* ctx, const uint8_t* rgb, size_t stride, uint32_t width, uint32_t height,
                          uint32_t mcu_row0, uint32_t mcu_rows, int maxval, const uint8_t qy[64],
                          const uint8_t qc[64], int32_t last_dc[3]) {
    CtxUse use(ctx);
    if (!use || !rgb || !qy || !qc || !last_dc) return JPGE_E_ARG;
    jpge::Encoder::StripeDesc d;
    d.rgb = rgb;
    d.stride = stride;
    d.width = width;
    d.height = height;
    d.mcu_row0 = mcu_row0;
    d.mcu_rows = mcu_rows;
    d.maxval = maxval;
    return ctx->enc->stripe_transform(d, qy, qc, last_dc);
}

int jpge_stripe_stats(jpge_ctx* ctx, const int32_t seed_dc[3], uint32_t counts[1024], uint64_t first[1024]) {
    CtxUse use(ctx);
    if (!use || !seed_dc || !counts || !first) return JPGE_E_ARG;
    return ctx->enc->stripe_stats(seed_dc, counts, first);
}

int jpge_stripe_code(jpge_ctx* ctx, const uint32_t counts[1024], const uint64_t first[1024],
                     jpge_stripe_summary* summary, size_t* header_len) {
    CtxUse use(ctx);
    if (!use || !counts || !first || !summary) return JPGE_E_ARG;
    return ctx->enc->stripe_code(counts, first, reinterpret_cast<jpge::StripeSummary*>(summary), header_len);
}

int jpge_stripe_place(const jpge_stripe_summary* all, int n, int index, size_t header_len, size_t* seg_off,
                      size_t* total_len) {
    return jpge::Encoder::stripe_place(reinterpret_cast<const jpge::StripeSummary*>(all), n, index, header_len,
                                       nullptr, nullptr, nullptr, seg_off, total_len);
}

int jpge_stripe_pack(jpge_ctx* ctx, const jpge_stripe_summary* all, int n, int index, uint8_t* out, size_t cap,
                     size_t* seg_off, size_t* seg_len, size_t* total_len) {
    CtxUse use(ctx);
    if (!use || !all || !out) return JPGE_E_ARG;
    return ctx->enc->stripe_pack(reinterpret_cast<const jpge::StripeSummary*>(all), n, index, out, cap, seg_off,
                                 seg_len, total_len);
}

}  // extern "C"

// ---- plane stages (the facade's Image stage methods on the GPU) ----
extern "C" {

int jpge_color_convert(jpge_ctx* ctx, const double* in0, const double* in1, const double* in2, double* out0,
                       double* out1, double* out2, size_t n, int target, uint32_t flags) {
    CtxUse use(ctx);
    if (!use || (target != JPGE_TO_RGB && target != JPGE_TO_YCBCR)) return JPGE_E_ARG;
    const double* in[3] = {in0, in1, in2};
    double* out[3] = {out0, out1, out2};
    return ctx->enc->stage_color(in, out, n, target == JPGE_TO_YCBCR, flags);
}

int jpge_subsample_plane(jpge_ctx* ctx, const double* in, uint32_t rows, uint32_t cols, int mode, double* out,
                         uint32_t* out_rows, uint32_t* out_cols, uint32_t flags) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    if (const int e = jpge::Encoder::subsample_shape(mode, rows, cols, out_rows, out_cols)) return e;
    if (!out) return JPGE_OK;
    return ctx->enc->stage_subsample(in, rows, cols, mode, out, flags);
}

int jpge_dct_plane(jpge_ctx* ctx, const double* in, uint32_t rows, uint32_t cols, int dct_mode, double* out,
                   uint32_t flags) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    return ctx->enc->stage_dct(in, rows, cols, dct_mode, out, flags);
}

int jpge_quantize_plane(jpge_ctx* ctx, const double* in, uint32_t rows, uint32_t cols, const uint8_t table[64],
                        int32_t* out, uint32_t flags) {
    CtxUse use(ctx);
    if (!use) return JPGE_E_ARG;
    return ctx->enc->stage_quantize(in, rows, cols, table, out, flags);
}

int jpge_encode_planes(jpge_ctx* ctx, const double* p0, const double* p1, const double* p2, uint32_t rows,
                       uint32_t cols, int colorspace, uint32_t real_width, uint32_t real_height, const uint8_t qy[64],
                       const uint8_t qc[64], uint8_t* out, size_t cap, size_t* len, uint32_t flags) {
    CtxUse use(ctx);
    if (!use || (colorspace != JPGE_TO_RGB && colorspace != JPGE_TO_YCBCR)) return JPGE_E_ARG;
    const double* p[3] = {p0, p1, p2};
    return ctx->enc->encode_planes(p, rows, cols, colorspace == JPGE_TO_YCBCR, real_width, real_height, qy, qc, out,
                                   cap, len, flags);
}

}  // extern "C"
