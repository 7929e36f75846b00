// PPM files -> .jpg files, pipelined (the PPM ingest + H2D
// pipeline).  Replaces a loop of the reference's main.cpp:8-32 (loadPPM +
// writeJPEG per file, Image.cpp:421-538 / 831-976) over many files.
//
// Three stages run side by side on groups of frames:
//   read   — worker threads read each file straight into pinned host memory and
//            parse it in place (P6: the sample bytes already are the RGB8 frame;
//            P3: the ASCII samples are rewritten as bytes over the text, which
//            they never overtake), with the reference tokenizer (host_io.cpp);
//   encode — the calling thread runs the encoder's batch on the group: the H2D copy
//            of every frame from the pinned buffer is queued on its lane's stream
//            ahead of the kernels; the .jpg bytes stay in device memory;
//   write  — a thread copies each .jpg (its exact length) to the host and writes it.
// Input buffers and device outputs are double-buffered by group, so group g+1 is
// read and group g-1 written while group g encodes.
#include "ingest.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <future>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "host_io.hpp"

namespace jpge {
namespace {

struct PinnedBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    ~PinnedBuf() {
        if (p) hipHostFree(p);
    }
    int reserve(size_t n) {
        if (n <= cap) return kOk;
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc((void**)&p, n, hipHostMallocDefault) != hipSuccess) return kErrHip;
        cap = n;
        return kOk;
    }
};

struct DevBuf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) hipFree(p);
    }
    int reserve(size_t n) {
        if (n <= cap) return kOk;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc((void**)&p, n) != hipSuccess) return kErrHip;
        cap = n;
        return kOk;
    }
};

// Reads `path` whole into pinned memory and parses it in place: desc gets the
// frame (rgb inside buf).  Same statuses as parse_ppm / load_ppm_file.
int read_ppm_pinned(const char* path, PinnedBuf& buf, FrameDesc& desc) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return kErrIo;
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size <= 0) {
        ::close(fd);
        return kErrIo;
    }
    const size_t n = (size_t)st.st_size;
    int rc = buf.reserve(n);
    size_t got = 0;
    while (!rc && got < n) {
        const ssize_t r = ::pread(fd, buf.p + got, n - got, (off_t)got);
        if (r <= 0) rc = kErrIo;
        else got += (size_t)r;
    }
    ::close(fd);
    if (rc) return rc;
    uint32_t w = 0, h = 0;
    int mv = 0;
    size_t off = 0;
    if (const int s = parse_ppm_inplace(buf.p, n, w, h, mv, off)) return s;
    desc = FrameDesc();
    desc.rgb = buf.p + off;
    desc.width = w;
    desc.height = h;
    desc.stride = (size_t)w * 3;
    desc.maxval = mv;
    return kOk;
}

int write_file(const char* path, const uint8_t* p, size_t n) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return kErrIo;
    const size_t w = std::fwrite(p, 1, n, f);
    const int c = std::fclose(f);
    return (w == n && c == 0) ? kOk : kErrIo;
}

}  // namespace

struct IngestBuffers {
    PinnedBuf pin[2][64];   // file bytes (then the frame) of each group's frames
    DevBuf dout[2][64];     // .jpg bytes in device memory
    PinnedBuf hout[2][64];  // .jpg bytes on the way to the file
    // the writers' device-to-host copies, one non-blocking stream per writer thread: never
    // the null stream, whose use slows every later launch on the encoder's lane streams
    hipStream_t copy[64] = {};
    hipStream_t stream(int t) {
        if (!copy[t] && hipStreamCreateWithFlags(&copy[t], hipStreamNonBlocking) != hipSuccess) copy[t] = nullptr;
        return copy[t];
    }
    ~IngestBuffers() {
        for (hipStream_t s : copy)
            if (s) hipStreamDestroy(s);
    }
};
void IngestBuffersDeleter::operator()(IngestBuffers* b) const { delete b; }

int encode_files(Encoder& enc, std::unique_ptr<IngestBuffers, IngestBuffersDeleter>& bufs, const char* const* in,
                 const char* const* out, int n, int quality, size_t* lens, int* statuses, int group) {
    if (n < 0 || (n && (!in || !out)) || quality < 1 || quality > 100) return kErrArg;
    if (n == 0) return kOk;
    const int B = std::max(1, std::min(std::min(group > 0 ? group : 8, 64), n));
    const int ngroups = (n + B - 1) / B;
    uint8_t qy[64], qc[64];
    quality_tables(quality, qy, qc);
    std::vector<int> status(n, kOk);
    std::vector<size_t> length(n, 0);
    if (!bufs) bufs.reset(new IngestBuffers());
    auto& pin = bufs->pin;
    auto& dout = bufs->dout;
    std::vector<FrameDesc> desc[2];
    const int readers = std::max(1, std::min(B, (int)std::max(2u, std::min(8u, std::thread::hardware_concurrency()))));

    // JPGE_INGEST_TRACE=1: per-group stage times on stderr (diagnostic)
    const bool trace = std::getenv("JPGE_INGEST_TRACE") != nullptr;
    const auto t_call = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count(); };
    auto read_group = [&](int g) {
        const double t0 = ms();
        const int s = g & 1, i0 = g * B, cnt = std::min(B, n - i0);
        desc[s].assign(cnt, FrameDesc());
        std::atomic<int> next{0};
        auto work = [&] {
            for (int k; (k = next.fetch_add(1)) < cnt;) status[i0 + k] = read_ppm_pinned(in[i0 + k], pin[s][k], desc[s][k]);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < std::min(readers, cnt); ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
        if (trace) std::fprintf(stderr, "ingest g%d read  %.2f .. %.2f ms\n", g, t0, ms());
    };
    auto& hout = bufs->hout;
    auto write_group = [&](int g, int device) {
        const double t0 = ms();
        const int s = g & 1, i0 = g * B, cnt = std::min(B, n - i0);
        std::atomic<int> next{0};
        const int nw = std::min(readers, cnt);
        for (int t = 0; t < nw; ++t) bufs->stream(t);  // (created here, on one thread)
        auto work = [&](int t) {
            hipSetDevice(device);
            hipStream_t cs = bufs->copy[t];
            for (int k; (k = next.fetch_add(1)) < cnt;) {
                const int i = i0 + k;
                if (status[i]) continue;
                int st = cs ? hout[s][k].reserve(length[i]) : kErrHip;
                if (!st && (hipMemcpyAsync(hout[s][k].p, dout[s][k].p, length[i], hipMemcpyDeviceToHost, cs) != hipSuccess ||
                            hipStreamSynchronize(cs) != hipSuccess))
                    st = kErrHip;
                status[i] = st ? st : write_file(out[i], hout[s][k].p, length[i]);
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nw; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& t : th) t.join();
        if (trace) std::fprintf(stderr, "ingest g%d write %.2f .. %.2f ms\n", g, t0, ms());
    };

    std::future<void> reading = std::async(std::launch::async, read_group, 0);
    std::future<void> writing[2];
    int device = 0;
    hipGetDevice(&device);
    for (int g = 0; g < ngroups; ++g) {
        const int s = g & 1, i0 = g * B, cnt = std::min(B, n - i0);
        reading.get();
        if (writing[s].valid()) writing[s].get();  // group g-2's device outputs are free
        if (g + 1 < ngroups) reading = std::async(std::launch::async, read_group, g + 1);
        // encode the frames that were read: host input (pinned), device output
        std::vector<FrameDesc> batch;
        std::vector<int> idx;
        for (int k = 0; k < cnt; ++k) {
            if (status[i0 + k]) continue;
            FrameDesc f = desc[s][k];
            const size_t cap = Encoder::max_jpeg_bytes(f.width, f.height);
            if (const int r = dout[s][k].reserve(cap)) {
                status[i0 + k] = r;
                continue;
            }
            f.out = dout[s][k].p;
            f.cap = cap;
            batch.push_back(f);
            idx.push_back(k);
        }
        if (!batch.empty()) {
            const double t0 = ms();
            enc.encode_batch(batch.data(), (int)batch.size(), qy, qc, kFlagDeviceOutput);
            if (trace) std::fprintf(stderr, "ingest g%d encode %.2f .. %.2f ms\n", g, t0, ms());
            for (size_t b = 0; b < batch.size(); ++b) {
                status[i0 + idx[b]] = batch[b].status;
                length[i0 + idx[b]] = batch[b].len;
            }
        }
        writing[s] = std::async(std::launch::async, write_group, g, device);
    }
    for (auto& w : writing)
        if (w.valid()) w.get();
    int first = kOk;
    for (int i = 0; i < n; ++i) {
        if (lens) lens[i] = status[i] ? 0 : length[i];
        if (statuses) statuses[i] = status[i];
        if (status[i] && !first) first = status[i];
    }
    return first;
}

}  // namespace jpge
