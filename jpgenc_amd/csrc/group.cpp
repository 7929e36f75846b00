// Device groups (include/jpge.h jpge_group_*): one process driving several MI355X
// devices, one jpge context each, with RCCL communicators over xGMI for the
// exchanges of SURVEY 8(e):
//   frames  (config 4)  jpge_group_encode_batch: frame i on member i mod N, no
//                       collective (every frame has its own tables and DC chain);
//   stripes (config 5)  jpge_group_encode_striped: one image in row stripes of whole
//                       MCU rows, the four jpge_stripe_* phases on every member in
//                       parallel, and between them an RCCL all-gather of the DC seeds,
//                       an all-reduce of the histograms (counts: sum, first-occurrence
//                       keys: min), an all-gather of the stripe summaries, and one
//                       grouped send/recv round moving every stripe's stuffed segment
//                       into member 0's whole-file buffer.
// The output is byte-identical to one device's encode.  RCCL needs distinct devices:
// a group naming a device twice (e.g. a rehearsal of N members on one GPU) does the
// exchanges in host memory and the gather by device copies — the same phases.
// librccl is loaded on first use (dlopen), so the library does not depend on it.
#include <dlfcn.h>

#include <algorithm>
#include <array>
#include <memory>
#include <cstring>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "jpge.h"
#include "live.hpp"

namespace {

// The RCCL entry points the group uses, resolved from librccl.so.1.
struct Rccl {
    decltype(&ncclCommInitAll) commInitAll = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.commInitAll = (decltype(r.commInitAll))dlsym(h, "ncclCommInitAll");
        r.commDestroy = (decltype(r.commDestroy))dlsym(h, "ncclCommDestroy");
        r.groupStart = (decltype(r.groupStart))dlsym(h, "ncclGroupStart");
        r.groupEnd = (decltype(r.groupEnd))dlsym(h, "ncclGroupEnd");
        r.allGather = (decltype(r.allGather))dlsym(h, "ncclAllGather");
        r.allReduce = (decltype(r.allReduce))dlsym(h, "ncclAllReduce");
        r.send = (decltype(r.send))dlsym(h, "ncclSend");
        r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
        r.ok = r.commInitAll && r.commDestroy && r.groupStart && r.groupEnd && r.allGather && r.allReduce && r.send &&
               r.recv;
    });
    return r;
}

#define GRP_HIP(x)                                 \
    do {                                           \
        if ((x) != hipSuccess) return (int)JPGE_E_HIP;  \
    } while (0)
#define GRP_NCCL(x)                                \
    do {                                           \
        if ((x) != ncclSuccess) return (int)JPGE_E_RCCL; \
    } while (0)

// Run f(member) for every member, one host thread each; the first failing status.
template <typename F>
int for_members(int n, F&& f) {
    std::vector<int> st(n, JPGE_OK);
    std::vector<std::thread> th;
    for (int m = 1; m < n; ++m) th.emplace_back([&, m] { st[m] = f(m); });
    st[0] = f(0);
    for (auto& t : th) t.join();
    for (int s : st)
        if (s) return s;
    return (int)JPGE_OK;
}

// Exchange words of one member (device memory): its own contribution and the
// gathered / reduced result, as RCCL sends and receives them.
struct XBuf {
    static constexpr size_t kDc = 0;                 // int32[3]
    static constexpr size_t kDcAll = 64;             // int32[N][3]
    static constexpr size_t kCounts = 1024;          // uint32[1024]
    static constexpr size_t kKeys = kCounts + 4096;  // uint64[1024]
    static constexpr size_t kSum = kKeys + 8192;     // uint64[12]
    static constexpr size_t kSumAll = kSum + 128;    // uint64[N][12]
    static size_t bytes(int n) { return kSumAll + (size_t)n * 96 + 256; }
};

// stripes.stripe_rows: mcu_rows in n contiguous stripes as even as possible, each
// starting at a multiple of `align` rows.
bool stripe_rows(uint32_t mcu_rows, int n, uint32_t align, std::vector<std::pair<uint32_t, uint32_t>>& out) {
    const uint32_t units = (mcu_rows + align - 1) / align;
    if (n < 1 || (uint32_t)n > units) return false;
    const uint32_t base = units / n, extra = units % n;
    uint32_t u0 = 0;
    out.clear();
    for (int r = 0; r < n; ++r) {
        const uint32_t c = base + ((uint32_t)r < extra ? 1 : 0);
        const uint32_t r0 = u0 * align;
        out.emplace_back(r0, std::min(mcu_rows, (u0 + c) * align) - r0);
        u0 += c;
    }
    return true;
}

}  // namespace

struct jpge_group {
    std::vector<int> dev;
    std::vector<jpge_ctx*> ctx;
    bool use_rccl = false;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> xs;  // per member: the stream RCCL runs on
    // per member device buffers, grown on demand: stripe RGB, whole-file output, exchange words
    std::vector<uint8_t*> rgb, out, xb;
    std::vector<size_t> rgb_cap, out_cap;
    uint32_t restart = 0;
    std::mutex mu;  // one call at a time

    int grow(int m, std::vector<uint8_t*>& v, std::vector<size_t>& cap, size_t bytes) {
        if (cap[m] >= bytes) return (int)JPGE_OK;
        GRP_HIP(hipSetDevice(dev[m]));
        hipFree(v[m]);
        v[m] = nullptr;
        cap[m] = 0;
        GRP_HIP(hipMalloc((void**)&v[m], bytes));
        cap[m] = bytes;
        return (int)JPGE_OK;
    }
    int sync_x() {  // RCCL streams of every member
        for (size_t m = 0; m < dev.size(); ++m) {
            GRP_HIP(hipSetDevice(dev[m]));
            GRP_HIP(hipStreamSynchronize(xs[m]));
        }
        return (int)JPGE_OK;
    }
    // Frees everything; the members' contexts are closed, or at exit released (live.hpp).
    void release(bool at_exit) {
        for (size_t m = 0; m < dev.size(); ++m) {
            hipSetDevice(dev[m]);
            if (m < xs.size() && xs[m]) hipStreamSynchronize(xs[m]);
            hipFree(rgb[m]);
            hipFree(out[m]);
            hipFree(xb[m]);
        }
        if (use_rccl)
            for (auto c : comm) rccl().commDestroy(c);
        for (size_t m = 0; m < xs.size(); ++m) {
            hipSetDevice(dev[m]);
            if (xs[m]) hipStreamDestroy(xs[m]);
        }
        for (auto* c : ctx) {
            if (at_exit) jpge::live_release(c);
            else jpge_close(c);
        }
        dev.clear();
        ctx.clear();
        comm.clear();
        xs.clear();
        rgb.clear();
        out.clear();
        xb.clear();
        use_rccl = false;
    }
    ~jpge_group() { release(false); }
};

namespace jpge {
void live_release(jpge_group* g) {  // (the exit handler, capi.cpp)
    live_remove(g);
    { std::lock_guard<std::mutex> wait(g->mu); }  // a call still running on another thread
    g->release(true);
    live_mark_released(g);
}
}  // namespace jpge

extern "C" {

int jpge_group_open(int ndev, const int* devices, int lanes, jpge_group** g) {
    if (!g || ndev < 1 || ndev > 64 || !devices) return (int)JPGE_E_ARG;
    *g = nullptr;
    std::unique_ptr<jpge_group> G(new jpge_group());
    G->dev.assign(devices, devices + ndev);
    const int n = ndev;
    G->rgb.assign(n, nullptr);
    G->out.assign(n, nullptr);
    G->xb.assign(n, nullptr);
    G->rgb_cap.assign(n, 0);
    G->out_cap.assign(n, 0);
    for (int m = 0; m < n; ++m) {
        jpge_ctx* c = nullptr;
        if (const int st = jpge_open_ex(devices[m], lanes, &c)) return st;
        G->ctx.push_back(c);
        if (hipSetDevice(devices[m]) != hipSuccess) return (int)JPGE_E_HIP;
        hipStream_t s = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return (int)JPGE_E_HIP;
        G->xs.push_back(s);
        if (hipMalloc((void**)&G->xb[m], XBuf::bytes(n)) != hipSuccess) return (int)JPGE_E_HIP;
    }
    std::vector<int> sorted(G->dev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct) {  // one RCCL communicator per device (single-process clique)
        if (!rccl().ok) return (int)JPGE_E_RCCL;
        G->comm.assign(n, nullptr);
        if (rccl().commInitAll(G->comm.data(), n, G->dev.data()) != ncclSuccess) return (int)JPGE_E_RCCL;
        G->use_rccl = true;
        jpge::live_handler_after_load();  // (after RCCL's own initialisation: live.hpp)
    }
    *g = G.release();
    jpge::live_add(*g);
    return (int)JPGE_OK;
}

int jpge_group_close(jpge_group* g) {
    if (!g || jpge::live_is_released(g)) return (int)JPGE_OK;  // (released at exit: live.hpp)
    jpge::live_remove(g);
    delete g;
    return (int)JPGE_OK;
}

int jpge_group_size(const jpge_group* g, int* n, int* uses_rccl) {
    if (!g || g->dev.empty() || !n) return (int)JPGE_E_ARG;
    *n = (int)g->dev.size();
    if (uses_rccl) *uses_rccl = g->use_rccl ? 1 : 0;
    return (int)JPGE_OK;
}

int jpge_group_context(jpge_group* g, int member, jpge_ctx** ctx) {
    if (!g || !ctx || member < 0 || member >= (int)g->ctx.size()) return (int)JPGE_E_ARG;
    *ctx = g->ctx[member];
    return (int)JPGE_OK;
}

int jpge_group_set_restart_interval(jpge_group* g, uint32_t mcus) {
    if (!g || g->dev.empty()) return (int)JPGE_E_ARG;
    for (auto* c : g->ctx)
        if (const int st = jpge_set_restart_interval(c, mcus)) return st;
    g->restart = mcus;
    return (int)JPGE_OK;
}

int jpge_group_encode_batch(jpge_group* g, jpge_frame* frames, int n, const uint8_t qy[64], const uint8_t qc[64],
                            uint32_t flags) {
    if (!g || g->dev.empty() || (n > 0 && !frames) || n < 0) return (int)JPGE_E_ARG;
    std::lock_guard<std::mutex> lk(g->mu);
    const int N = (int)g->ctx.size();
    std::vector<std::vector<jpge_frame>> part(N);
    for (int i = 0; i < n; ++i) part[i % N].push_back(frames[i]);
    const int st = for_members(N, [&](int m) {
        return part[m].empty() ? JPGE_OK : jpge_encode_batch(g->ctx[m], part[m].data(), (int)part[m].size(), qy, qc,
                                                             flags);
    });
    for (int i = 0; i < n; ++i) {
        const jpge_frame& f = part[i % N][i / N];
        frames[i].len = f.len;
        frames[i].status = f.status;
    }
    return st;
}

int jpge_group_encode_striped(jpge_group* g, const uint8_t* rgb, uint32_t width, uint32_t height, size_t stride,
                              int maxval, const uint8_t qy[64], const uint8_t qc[64], uint8_t* out, size_t cap,
                              size_t* len) {
    if (!g || g->dev.empty() || !rgb || !out || !len || !qy || !qc || width == 0 || height == 0)
        return (int)JPGE_E_ARG;
    std::lock_guard<std::mutex> lk(g->mu);
    const int N = (int)g->ctx.size();
    const size_t row = (size_t)width * 3, pitch = stride ? stride : row;
    if (pitch < row) return (int)JPGE_E_ARG;
    // stripes of whole MCU rows; with restart intervals every stripe starts one
    const uint32_t mh = (height + 15) / 16, mw = (width + 15) / 16;
    uint32_t align = 1;
    if (g->restart) align = g->restart / std::gcd(g->restart, mw);
    std::vector<std::pair<uint32_t, uint32_t>> rows;
    if (!stripe_rows(mh, N, align, rows)) return (int)JPGE_E_ARG;
    const size_t file_cap = jpge_max_jpeg_bytes(width, height);
    // the stripes' rows to their devices (a dense pitch), whole-file output buffers
    int st = for_members(N, [&](int m) {
        const uint32_t y0 = 16 * rows[m].first, y1 = std::min(height, 16 * (rows[m].first + rows[m].second));
        if (int e = g->grow(m, g->rgb, g->rgb_cap, (size_t)(y1 - y0) * row)) return e;
        if (int e = g->grow(m, g->out, g->out_cap, file_cap)) return e;
        GRP_HIP(hipSetDevice(g->dev[m]));
        // (on the member's stream: the null stream would slow every later launch on the
        // members' lane streams)
        GRP_HIP(hipMemcpy2DAsync(g->rgb[m], row, rgb + (size_t)y0 * pitch, pitch, row, y1 - y0, hipMemcpyHostToDevice,
                                 g->xs[m]));
        GRP_HIP(hipStreamSynchronize(g->xs[m]));
        return (int)JPGE_OK;
    });
    if (st) return st;

    // 1) transform; DC seeds: all-gather of 3 int32 per stripe
    std::vector<std::array<int32_t, 3>> last(N);
    st = for_members(N, [&](int m) {
        return jpge_stripe_transform(g->ctx[m], g->rgb[m], row, width, height, rows[m].first, rows[m].second, maxval,
                                     qy, qc, last[m].data());
    });
    if (st) return st;
    std::vector<std::array<int32_t, 3>> seeds(N, std::array<int32_t, 3>{0, 0, 0});
    if (!g->restart) {  // (restart stripes start their DC chains at 0: nothing to exchange)
        std::vector<int32_t> all(3 * N);
        if (g->use_rccl) {
            for (int m = 0; m < N; ++m) {
                GRP_HIP(hipSetDevice(g->dev[m]));
                GRP_HIP(hipMemcpyAsync(g->xb[m] + XBuf::kDc, last[m].data(), 12, hipMemcpyHostToDevice, g->xs[m]));
            }
            GRP_NCCL(rccl().groupStart());
            for (int m = 0; m < N; ++m)
                GRP_NCCL(rccl().allGather(g->xb[m] + XBuf::kDc, g->xb[m] + XBuf::kDcAll, 3, ncclInt32, g->comm[m],
                                          g->xs[m]));
            GRP_NCCL(rccl().groupEnd());
            GRP_HIP(hipSetDevice(g->dev[0]));
            GRP_HIP(hipMemcpyAsync(all.data(), g->xb[0] + XBuf::kDcAll, 12 * N, hipMemcpyDeviceToHost, g->xs[0]));
            if (int e = g->sync_x()) return e;
        } else {
            for (int m = 0; m < N; ++m) std::memcpy(&all[3 * m], last[m].data(), 12);
        }
        for (int m = 1; m < N; ++m) std::memcpy(seeds[m].data(), &all[3 * (m - 1)], 12);
    }

    // 2) statistics; histograms: all-reduce counts (sum) and first-occurrence keys (min)
    std::vector<std::vector<uint32_t>> cnt(N, std::vector<uint32_t>(1024));
    std::vector<std::vector<uint64_t>> key(N, std::vector<uint64_t>(1024));
    st = for_members(N, [&](int m) { return jpge_stripe_stats(g->ctx[m], seeds[m].data(), cnt[m].data(), key[m].data()); });
    if (st) return st;
    std::vector<uint32_t> counts(1024, 0);
    std::vector<uint64_t> first(1024, ~0ull);
    if (g->use_rccl) {
        for (int m = 0; m < N; ++m) {
            GRP_HIP(hipSetDevice(g->dev[m]));
            GRP_HIP(hipMemcpyAsync(g->xb[m] + XBuf::kCounts, cnt[m].data(), 4096, hipMemcpyHostToDevice, g->xs[m]));
            GRP_HIP(hipMemcpyAsync(g->xb[m] + XBuf::kKeys, key[m].data(), 8192, hipMemcpyHostToDevice, g->xs[m]));
        }
        GRP_NCCL(rccl().groupStart());
        for (int m = 0; m < N; ++m) {
            GRP_NCCL(rccl().allReduce(g->xb[m] + XBuf::kCounts, g->xb[m] + XBuf::kCounts, 1024, ncclUint32, ncclSum,
                                      g->comm[m], g->xs[m]));
            GRP_NCCL(rccl().allReduce(g->xb[m] + XBuf::kKeys, g->xb[m] + XBuf::kKeys, 1024, ncclUint64, ncclMin,
                                      g->comm[m], g->xs[m]));
        }
        GRP_NCCL(rccl().groupEnd());
        GRP_HIP(hipSetDevice(g->dev[0]));
        GRP_HIP(hipMemcpyAsync(counts.data(), g->xb[0] + XBuf::kCounts, 4096, hipMemcpyDeviceToHost, g->xs[0]));
        GRP_HIP(hipMemcpyAsync(first.data(), g->xb[0] + XBuf::kKeys, 8192, hipMemcpyDeviceToHost, g->xs[0]));
        if (int e = g->sync_x()) return e;
    } else {
        for (int m = 0; m < N; ++m)
            for (int i = 0; i < 1024; ++i) {
                counts[i] += cnt[m][i];
                first[i] = std::min(first[i], key[m][i]);
            }
    }

    // 3) tables + code kernel; summaries: all-gather of 12 x uint64 per stripe
    std::vector<jpge_stripe_summary> sum(N);
    std::vector<size_t> hdr(N, 0);
    st = for_members(N, [&](int m) {
        return jpge_stripe_code(g->ctx[m], counts.data(), first.data(), &sum[m], &hdr[m]);
    });
    if (st) return st;
    static_assert(sizeof(jpge_stripe_summary) == 56, "summary layout");
    if (g->use_rccl) {
        for (int m = 0; m < N; ++m) {
            GRP_HIP(hipSetDevice(g->dev[m]));
            GRP_HIP(hipMemcpyAsync(g->xb[m] + XBuf::kSum, &sum[m], sizeof(jpge_stripe_summary), hipMemcpyHostToDevice,
                                   g->xs[m]));
        }
        GRP_NCCL(rccl().groupStart());
        for (int m = 0; m < N; ++m)
            GRP_NCCL(rccl().allGather(g->xb[m] + XBuf::kSum, g->xb[m] + XBuf::kSumAll, sizeof(jpge_stripe_summary),
                                      ncclUint8, g->comm[m], g->xs[m]));
        GRP_NCCL(rccl().groupEnd());
        GRP_HIP(hipSetDevice(g->dev[0]));
        GRP_HIP(hipMemcpyAsync(sum.data(), g->xb[0] + XBuf::kSumAll, sizeof(jpge_stripe_summary) * N,
                               hipMemcpyDeviceToHost, g->xs[0]));
        if (int e = g->sync_x()) return e;
    }

    // 4) pack every stripe at its place in its member's whole-file buffer
    std::vector<size_t> off(N), seg(N), total(N);
    st = for_members(N, [&](int m) {
        return jpge_stripe_pack(g->ctx[m], sum.data(), N, m, g->out[m], g->out_cap[m], &off[m], &seg[m], &total[m]);
    });
    if (st) return st;
    const size_t tot = total[N - 1];
    if (tot > cap) {
        *len = tot;
        return (int)JPGE_E_NOSPACE;
    }
    //    segments to member 0: one grouped send/recv round (every link at once)
    if (g->use_rccl && N > 1) {
        GRP_NCCL(rccl().groupStart());
        for (int m = 1; m < N; ++m) {
            GRP_NCCL(rccl().send(g->out[m] + off[m], seg[m], ncclUint8, 0, g->comm[m], g->xs[m]));
            GRP_NCCL(rccl().recv(g->out[0] + off[m], seg[m], ncclUint8, m, g->comm[0], g->xs[0]));
        }
        GRP_NCCL(rccl().groupEnd());
        if (int e = g->sync_x()) return e;
    } else {
        GRP_HIP(hipSetDevice(g->dev[0]));
        for (int m = 1; m < N; ++m)
            GRP_HIP(hipMemcpyPeerAsync(g->out[0] + off[m], g->dev[0], g->out[m] + off[m], g->dev[m], seg[m], g->xs[0]));
        GRP_HIP(hipStreamSynchronize(g->xs[0]));
    }
    GRP_HIP(hipSetDevice(g->dev[0]));
    GRP_HIP(hipMemcpyAsync(out, g->out[0], tot, hipMemcpyDeviceToHost, g->xs[0]));
    GRP_HIP(hipStreamSynchronize(g->xs[0]));
    *len = tot;
    return (int)JPGE_OK;
}

}  // extern "C"
