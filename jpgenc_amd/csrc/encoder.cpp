#include "encoder.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

namespace jpge {

#define JPGE_HIP(expr)                                   \
    do {                                                 \
        if ((expr) != hipSuccess) return kErrHip;        \
    } while (0)

namespace {

inline Geometry geometry(uint32_t w, uint32_t h) {
    Geometry g;
    g.width = w;
    g.height = h;
    g.mw = (w + 15) / 16;
    g.mh = (h + 15) / 16;
    return g;
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Control block zeroed before every frame (Guideline 16: re-initialise every call).
struct CtlLayout {
    size_t cnt, key, ticket, lb_bits, lb_ff, tails, result, total;
    explicit CtlLayout(uint32_t ntiles) {
        size_t o = 0;
        cnt = o; o += align_up((size_t)kHistReplicas * 4 * 256 * 4, 256);
        key = o; o += align_up(4 * 256 * 8, 256);
        ticket = o; o += 256;
        lb_bits = o; o += align_up((size_t)ntiles * 8, 256);
        lb_ff = o; o += align_up((size_t)ntiles * 8, 256);
        tails = o; o += align_up((size_t)ntiles * 4, 256);
        result = o; o += 256;
        total = o;
    }
};

struct HostHist {
    uint32_t cnt[kHistReplicas * 4 * 256];
    uint64_t key[4 * 256];
};

}  // namespace

struct Encoder::Slot {
    hipStream_t stream = nullptr;
    hipEvent_t ev[6] = {};
    Geometry g;
    // device workspace (capacities)
    size_t cap_mcu = 0, cap_in = 0, cap_out = 0, cap_ctl = 0;
    uint8_t* d_in = nullptr;
    int16_t* d_coef = nullptr;
    uint8_t* d_ctl = nullptr;
    uint8_t* d_ubuf = nullptr;  // unstuffed entropy-coded segment (K3 internal)
    size_t cap_ubuf = 0;
    uint8_t* d_out = nullptr;
    uint32_t* d_tab = nullptr;
    // pinned host staging
    HostHist* h_hist = nullptr;
    uint32_t* h_tab = nullptr;
    uint8_t* h_hdr = nullptr;
    uint64_t* h_result = nullptr;
    // per-frame state between phases
    const uint8_t* in_dev = nullptr;
    size_t in_stride = 0;
    uint8_t* out_dev = nullptr;
    size_t out_cap = 0;
    size_t hdr_len = 0;
    uint8_t qy[64], qc[64];

    ~Slot() {
        hipFree(d_in); hipFree(d_coef); hipFree(d_ctl); hipFree(d_ubuf);
        hipFree(d_out); hipFree(d_tab);
        hipHostFree(h_hist); hipHostFree(h_tab); hipHostFree(h_hdr); hipHostFree(h_result);
        for (auto& e : ev) if (e) hipEventDestroy(e);
        if (stream) hipStreamDestroy(stream);
    }
};

size_t Encoder::max_jpeg_bytes(uint32_t w, uint32_t h) {
    // header <= 20 + 2*69 + 19 + 4*(4+17+256) + 14 ; entropy <= 1665 bits/block,
    // doubled for worst-case 0xFF stuffing; + EOI.
    const Geometry g = geometry(w, h);
    return 2048 + (size_t)g.nblocks() * 2 * 209 + 16;
}

int Encoder::open(int device, std::unique_ptr<Encoder>& out) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return kErrNoDevice;
    if (device < 0 || device >= n) return kErrNoDevice;
    JPGE_HIP(hipSetDevice(device));
    std::unique_ptr<Encoder> e(new Encoder());
    e->device_ = device;
    if (const char* ew = std::getenv("JPGE_ENTROPY_WGS")) e->entropy_wgs_ = (uint32_t)std::strtoul(ew, nullptr, 10);
    e->stamps_file_ = std::getenv("JPGE_STAMPS_FILE");
    if (e->stamps_file_) {
        e->dbg_words_ = 3ull * 65536 * kStampSlots;  // up to 64k workgroups per kernel
        JPGE_HIP(hipMalloc((void**)&e->d_dbg_, e->dbg_words_ * 8));
        JPGE_HIP(hipMemset(e->d_dbg_, 0, e->dbg_words_ * 8));
    }
    for (int i = 0; i < 3; ++i) {
        std::unique_ptr<Slot> s(new Slot());
        JPGE_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        for (auto& ev : s->ev) JPGE_HIP(hipEventCreate(&ev));
        JPGE_HIP(hipHostMalloc((void**)&s->h_hist, sizeof(HostHist), hipHostMallocDefault));
        JPGE_HIP(hipHostMalloc((void**)&s->h_tab, 4 * 256 * 4, hipHostMallocDefault));
        JPGE_HIP(hipHostMalloc((void**)&s->h_hdr, 4096, hipHostMallocDefault));
        JPGE_HIP(hipHostMalloc((void**)&s->h_result, 64, hipHostMallocDefault));
        JPGE_HIP(hipMalloc((void**)&s->d_tab, 4 * 256 * 4));
        e->slots_.push_back(std::move(s));
    }
    out = std::move(e);
    return kOk;
}

Encoder::~Encoder() {
    hipSetDevice(device_);
    for (auto& s : slots_) if (s && s->stream) hipStreamSynchronize(s->stream);
    slots_.clear();
    hipFree(d_dbg_);
}

// Diagnostic: raw per-workgroup phase stamps of the last frame, as
// [u64 n_fdct_wg, n_stats_wg, n_entropy_wg] then 3 x 65536 x kStampSlots u64;
// the buffer is cleared afterwards (slots 8-15 accumulate).
void Encoder::dump_stamps(const Slot& s) {
    if (!stamps_file_ || !d_dbg_) return;
    std::vector<uint64_t> h(dbg_words_);
    if (hipMemcpy(h.data(), d_dbg_, dbg_words_ * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    const uint64_t hdr[3] = {fdct_grid(s.g), stats_grid(s.g), entropy_grid(s.g, entropy_wgs_)};
    FILE* f = std::fopen(stamps_file_, "wb");
    if (!f) return;
    std::fwrite(hdr, 8, 3, f);
    std::fwrite(h.data(), 8, h.size(), f);
    std::fclose(f);
    hipMemset(d_dbg_, 0, dbg_words_ * 8);
}

int Encoder::ensure(Slot& s, const Geometry& g, size_t in_bytes, size_t out_cap) {
    const size_t nmcu = g.nmcu();
    if (nmcu > s.cap_mcu) {
        hipFree(s.d_coef);
        s.d_coef = nullptr; s.cap_mcu = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_coef, nmcu * 768));
        s.cap_mcu = nmcu;
    }
    const CtlLayout L(entropy_tiles(g));
    const size_t ubuf = entropy_ubuf_bytes(g, entropy_wgs_);
    if (ubuf > s.cap_ubuf) {
        hipFree(s.d_ubuf); s.d_ubuf = nullptr; s.cap_ubuf = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_ubuf, ubuf));
        s.cap_ubuf = ubuf;
    }
    if (L.total > s.cap_ctl) {
        hipFree(s.d_ctl); s.d_ctl = nullptr; s.cap_ctl = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_ctl, L.total));
        s.cap_ctl = L.total;
    }
    if (in_bytes > s.cap_in) {
        hipFree(s.d_in); s.d_in = nullptr; s.cap_in = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_in, in_bytes));
        s.cap_in = in_bytes;
    }
    if (out_cap > s.cap_out) {
        hipFree(s.d_out); s.d_out = nullptr; s.cap_out = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_out, out_cap));
        s.cap_out = out_cap;
    }
    return kOk;
}

// Phase 1: upload (if host input), statistics kernels, histogram read-back.
int Encoder::phase1(Slot& s, const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags) {
    if (!f.rgb || f.width == 0 || f.height == 0 || f.width > 65535 || f.height > 65535) return kErrArg;
    if (f.maxval < 1 || f.maxval > 255) return kErrRange;
    const Geometry g = geometry(f.width, f.height);
    const size_t row = (size_t)f.width * 3;
    const size_t stride = f.stride ? f.stride : row;
    if (stride < row) return kErrArg;
    const size_t dev_pitch = align_up(row, 16);
    const size_t in_bytes = (flags & kFlagDeviceInput) ? 0 : dev_pitch * f.height;
    const size_t out_cap = (flags & kFlagDeviceOutput) ? 0 : max_jpeg_bytes(f.width, f.height);
    for (int i = 0; i < 64; ++i)
        if (!qy[i] || !qc[i]) return kErrArg;
    const int st = ensure(s, g, in_bytes, out_cap);
    if (st) return st;
    std::memcpy(s.qy, qy, 64);
    std::memcpy(s.qc, qc, 64);
    s.g = g;
    if (flags & kFlagDeviceInput) {
        s.in_dev = f.rgb;
        s.in_stride = stride;
    } else {
        JPGE_HIP(hipMemcpy2DAsync(s.d_in, dev_pitch, f.rgb, stride, row, f.height, hipMemcpyHostToDevice, s.stream));
        s.in_dev = s.d_in;
        s.in_stride = dev_pitch;
    }
    if (flags & kFlagDeviceOutput) {
        s.out_dev = f.out;
        s.out_cap = f.cap;
    } else {
        s.out_dev = s.d_out;
        s.out_cap = s.cap_out;
    }
    const CtlLayout L(entropy_tiles(g));
    JPGE_HIP(hipMemsetAsync(s.d_ctl, 0, L.total, s.stream));

    FdctArgs a;
    a.rgb = s.in_dev;
    a.stride = s.in_stride;
    a.g = g;
    a.maxval = f.maxval;
    for (int i = 0; i < 64; ++i) {
        a.q[i] = (double)qy[i];  // Image.cpp:611-636 divides by the table entry as double
        a.q[64 + i] = (double)qc[i];
    }
    a.coef = s.d_coef;
    a.dbg = d_dbg_;
    StatsArgs st2;
    st2.coef = s.d_coef;
    st2.g = g;
    st2.hist.cnt = reinterpret_cast<uint32_t*>(s.d_ctl + L.cnt);
    st2.hist.key = reinterpret_cast<uint64_t*>(s.d_ctl + L.key);
    st2.dbg = d_dbg_ ? d_dbg_ + 65536 * kStampSlots : nullptr;
    if (timing_) JPGE_HIP(hipEventRecord(s.ev[0], s.stream));
    JPGE_HIP(launch_fdct(a, s.stream));
    if (timing_) JPGE_HIP(hipEventRecord(s.ev[1], s.stream));
    JPGE_HIP(launch_stats(st2, s.stream));
    if (timing_) JPGE_HIP(hipEventRecord(s.ev[2], s.stream));
    JPGE_HIP(hipMemcpyAsync(s.h_hist->cnt, s.d_ctl + L.cnt, sizeof(s.h_hist->cnt), hipMemcpyDeviceToHost, s.stream));
    JPGE_HIP(hipMemcpyAsync(s.h_hist->key, s.d_ctl + L.key, sizeof(s.h_hist->key), hipMemcpyDeviceToHost, s.stream));
    JPGE_HIP(hipEventRecord(s.ev[3], s.stream));
    return kOk;
}

// Phase 2: wait for the histograms, build the four tables on the host
// (generateHuffmanCode semantics), write the headers, launch the entropy kernel.
int Encoder::phase2(Slot& s, const FrameDesc& f, uint32_t flags) {
    (void)flags;
    JPGE_HIP(hipEventSynchronize(s.ev[3]));
    HuffTable tabs[4];
    for (int t = 0; t < 4; ++t) {
        uint32_t cnt[256];
        uint64_t first[256];
        for (int i = 0; i < 256; ++i) {
            uint64_t c = 0;
            for (int r = 0; r < kHistReplicas; ++r) c += s.h_hist->cnt[(r * 4 + t) * 256 + i];
            cnt[i] = (uint32_t)c;
            first[i] = ~s.h_hist->key[t * 256 + i];
        }
        if (!build_table(cnt, first, tabs[t])) return kErrInternal;
        for (int i = 0; i < 256; ++i)
            s.h_tab[t * 256 + i] = ((uint32_t)tabs[t].len[i] << 16) | (tabs[t].code[i] & 0xFFFF);
    }
    const HuffTable* tp[4] = {&tabs[0], &tabs[1], &tabs[2], &tabs[3]};
    const std::vector<uint8_t> hdr = jfif_headers(f.width, f.height, s.qy, s.qc, tp);
    if (hdr.size() > 4096) return kErrInternal;
    std::memcpy(s.h_hdr, hdr.data(), hdr.size());
    s.hdr_len = hdr.size();
    if (s.out_cap < s.hdr_len + 2) return kErrNoSpace;
    JPGE_HIP(hipMemcpyAsync(s.d_tab, s.h_tab, 4 * 256 * 4, hipMemcpyHostToDevice, s.stream));
    JPGE_HIP(hipMemcpyAsync(s.out_dev, s.h_hdr, s.hdr_len, hipMemcpyHostToDevice, s.stream));

    const CtlLayout L(entropy_tiles(s.g));
    EntropyArgs e;
    e.coef = s.d_coef;
    e.g = s.g;
    e.tables = s.d_tab;
    e.out = s.out_dev;
    e.hdr_len = s.hdr_len;
    e.out_cap = s.out_cap;
    e.ticket = reinterpret_cast<uint32_t*>(s.d_ctl + L.ticket);
    e.lb_bits = reinterpret_cast<uint64_t*>(s.d_ctl + L.lb_bits);
    e.lb_ff = reinterpret_cast<uint64_t*>(s.d_ctl + L.lb_ff);
    e.tails = reinterpret_cast<uint32_t*>(s.d_ctl + L.tails);
    e.result = reinterpret_cast<uint64_t*>(s.d_ctl + L.result);
    e.ubuf = s.d_ubuf;
    e.wgs = entropy_wgs_;
    e.dbg = d_dbg_ ? d_dbg_ + 2 * 65536 * kStampSlots : nullptr;
    if (timing_) JPGE_HIP(hipEventRecord(s.ev[4], s.stream));
    JPGE_HIP(launch_entropy(e, s.stream));
    if (timing_) JPGE_HIP(hipEventRecord(s.ev[5], s.stream));
    JPGE_HIP(hipMemcpyAsync(s.h_result, s.d_ctl + L.result, 16, hipMemcpyDeviceToHost, s.stream));
    return kOk;
}

int Encoder::finish(Slot& s, FrameDesc& f, uint32_t flags) {
    JPGE_HIP(hipStreamSynchronize(s.stream));
    if (timing_) {
        hipEventElapsedTime(&times_.fdct, s.ev[0], s.ev[1]);
        hipEventElapsedTime(&times_.dc_stats, s.ev[1], s.ev[2]);
        hipEventElapsedTime(&times_.entropy, s.ev[4], s.ev[5]);
        hipEventElapsedTime(&times_.total, s.ev[0], s.ev[5]);
        times_.fdct_sum += times_.fdct;
        times_.dc_stats_sum += times_.dc_stats;
        times_.entropy_sum += times_.entropy;
        times_.frames += 1;
    }
    dump_stamps(s);
    const uint64_t err = s.h_result[1];
    if (err & 4) { f.len = 0; return kErrNoSpace; }
    if (err) return kErrTimeout;
    const size_t len = (size_t)s.h_result[0];
    f.len = len;
    if (flags & kFlagDeviceOutput) return kOk;
    if (len > f.cap) return kErrNoSpace;
    JPGE_HIP(hipMemcpyAsync(f.out, s.out_dev, len, hipMemcpyDeviceToHost, s.stream));
    JPGE_HIP(hipStreamSynchronize(s.stream));
    return kOk;
}

int Encoder::encode(FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags) {
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *slots_[0];
    int st = phase1(s, f, qy, qc, flags);
    if (!st) st = phase2(s, f, flags);
    if (!st) st = finish(s, f, flags);
    else hipStreamSynchronize(s.stream);
    f.status = st;
    return st;
}

int Encoder::encode_batch(FrameDesc* fr, int n, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags) {
    JPGE_HIP(hipSetDevice(device_));
    const int S = (int)slots_.size();
    int first_err = kOk;
    auto note = [&](int i, int st) {
        if (st && !fr[i].status) fr[i].status = st;
        if (st && !first_err) first_err = st;
    };
    for (int i = 0; i < n; ++i) fr[i].status = 0;
    // software pipeline: phase1(i) || host tables of (i-1) || drain (i-2)
    for (int i = 0; i < n + 2; ++i) {
        if (i < n) note(i, phase1(*slots_[i % S], fr[i], qy, qc, flags));
        if (i - 1 >= 0 && i - 1 < n && !fr[i - 1].status) note(i - 1, phase2(*slots_[(i - 1) % S], fr[i - 1], flags));
        if (i - 2 >= 0 && i - 2 < n) {
            Slot& s = *slots_[(i - 2) % S];
            if (!fr[i - 2].status) note(i - 2, finish(s, fr[i - 2], flags));
            else hipStreamSynchronize(s.stream);
        }
    }
    return first_err;
}

int Encoder::fdct_quant(const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                        int16_t* y, int16_t* cb, int16_t* cr) {
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *slots_[0];
    int st = phase1(s, f, qy, qc, flags | kFlagDeviceOutput);
    if (st) { hipStreamSynchronize(s.stream); return st; }
    JPGE_HIP(hipStreamSynchronize(s.stream));
    const Geometry& g = s.g;
    std::vector<int16_t> coef((size_t)g.nmcu() * 384);
    JPGE_HIP(hipMemcpy(coef.data(), s.d_coef, coef.size() * 2, hipMemcpyDeviceToHost));
    const uint32_t ybw = 2 * g.mw, cbw = g.mw;
    for (uint32_t m = 0; m < g.nmcu(); ++m) {
        const uint32_t mr = m / g.mw, mc = m % g.mw;
        for (int k = 0; k < 6; ++k) {
            const int16_t* src = &coef[((size_t)m * 6 + k) * 64];
            int16_t* dst;
            if (k < 4) dst = y + ((size_t)(2 * mr + (k >> 1)) * ybw + 2 * mc + (k & 1)) * 64;
            else dst = (k == 4 ? cb : cr) + ((size_t)mr * cbw + mc) * 64;
            for (int i = 0; i < 64; ++i) dst[i] = src[i];
        }
    }
    return kOk;
}

int Encoder::symbol_stats(const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                          uint32_t counts[1024], uint64_t first[1024]) {
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *slots_[0];
    int st = phase1(s, f, qy, qc, flags | kFlagDeviceOutput);
    if (st) { hipStreamSynchronize(s.stream); return st; }
    JPGE_HIP(hipEventSynchronize(s.ev[3]));
    for (int t = 0; t < 4; ++t)
        for (int i = 0; i < 256; ++i) {
            uint64_t c = 0;
            for (int r = 0; r < kHistReplicas; ++r) c += s.h_hist->cnt[(r * 4 + t) * 256 + i];
            counts[t * 256 + i] = (uint32_t)c;
            first[t * 256 + i] = c ? ~s.h_hist->key[t * 256 + i] : ~0ull;
        }
    return kOk;
}

}  // namespace jpge
