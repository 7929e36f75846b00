#include "encoder.hpp"
#include "host_par.hpp"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

#include <sys/prctl.h>
#include <vector>

namespace jpge {

#define JPGE_HIP(expr)                                   \
    do {                                                 \
        if ((expr) != hipSuccess) return kErrHip;        \
    } while (0)

namespace {

// MCU shape of a subsampling mode (jpge.h JPGE_S*): Y blocks across, blocks per MCU
// and the 4:2:0 chroma filter; false for an unknown mode.
bool mode_shape(int mode, uint32_t& yh, uint32_t& bpm, uint32_t& cfilt) {
    cfilt = kFiltS420m;
    switch (mode) {
        case 420: yh = 2; bpm = 6; return true;
        case 4201: yh = 2; bpm = 6; cfilt = kFiltS420lm; return true;
        case 4200: yh = 2; bpm = 6; cfilt = kFiltS420; return true;
        case 444: yh = 1; bpm = 3; return true;
        case 422: yh = 2; bpm = 4; return true;
        case 411: yh = 4; bpm = 6; return true;
        default: return false;
    }
}

// The frame in whole MCUs (4:2:0: 16x16 px, the reference's padding, Image.cpp:480-531;
// the other modes pad to their own MCU size: edge replication either way)
inline Geometry geometry(uint32_t w, uint32_t h, int mode = 420) {
    Geometry g;
    g.width = w;
    g.height = h;
    mode_shape(mode, g.yh, g.bpm, g.cfilt);
    g.mw = (w + g.mcu_w() - 1) / g.mcu_w();
    g.mh = (h + g.mcu_h() - 1) / g.mcu_h();
    return g;
}

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Host-side wait with low wake-up latency (the pipeline waits on short intervals).
inline hipError_t wait_event(hipEvent_t e) {
    hipError_t r;
    while ((r = hipEventQuery(e)) == hipErrorNotReady) {
    }
    return r;
}

// Poll a sequence word a kernel writes into mapped host memory after its data
// (release-ordered).  `nap`: sleep ~10 us between polls (pool workers, which have
// slack) instead of spinning (the submitting thread).  Bounded: a stream error or
// ~20 s without progress fails.  The stream is queried only after 2 ms without the
// word (then every ms): a stream query enqueues a marker behind the newest launch,
// which costs the GPU ~6 us of idle each time.  `queued`: set once the kernel that
// writes the word is on the stream (another thread launches it); before that an
// idle stream is no error.
//
// `guess` (napping waits): a running estimate of how long this wait takes at its call
// site.  The first sleep covers most of it in one wake-up, and naps poll the rest, so
// a wait of ~100 us costs two or three wake-ups instead of ten.  The sleep is shortened
// by twice the waits' spread, so irregular waits (16384^2 frames) are polled, not slept
// through.
struct WaitGuess {
    double ema_us = 0;  // smoothed wait duration (0: none yet)
    double dev_us = 0;  // smoothed |wait - ema_us|
    double frac = 0;    // first sleep = frac * ema - 2 * dev (0: off)
    double first_sleep_us() const { return frac * ema_us - 2.0 * dev_us; }
    void add(double us) {
        if (ema_us > 0) {
            dev_us = 0.85 * dev_us + 0.15 * std::fabs(us - ema_us);
            ema_us = 0.85 * ema_us + 0.15 * us;
        } else {
            ema_us = us;
        }
    }
    // statistics (JPGE_CPU_PROF): waits, waits already satisfied on entry, naps, total us
    uint64_t waits = 0, ready = 0, naps = 0;
    double total_us = 0;
};
inline int wait_seq(const uint64_t* word, uint64_t seq, hipStream_t stream, int nap_us = 0,
                    const std::atomic<int>* queued = nullptr, WaitGuess* guess = nullptr,
                    const std::function<bool()>* work = nullptr) {
    const bool nap = nap_us > 0;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto next_query = t0 + std::chrono::milliseconds(2);
    clk::time_point idle_since{};  // the stream was first seen idle without the word
    bool idle = false;
    if (guess) ++guess->waits;
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) {  // (not a wait: the estimate is of waits)
        if (guess) ++guess->ready;
        return kOk;
    }
    // (idle work first: the first sleep only once there is none)
    bool worked = false;
    while (work && __atomic_load_n(word, __ATOMIC_ACQUIRE) != seq && (*work)()) worked = true;
    if (nap && guess && guess->frac > 0 && !worked) {
        const double us = guess->first_sleep_us();
        if (us > 3.0 * nap_us) {
            std::this_thread::sleep_for(std::chrono::microseconds((long)us));
            ++guess->naps;
        }
    }
    for (uint32_t spins = 0;; ++spins) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) {
            if (guess) {
                const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
                guess->add(us);
                guess->total_us += us;
            }
            return kOk;
        }
        if (work && (*work)()) continue;
        if (nap) {
            std::this_thread::sleep_for(std::chrono::microseconds(nap_us));
            if (guess) ++guess->naps;
        }
        if (!nap && (spins & 255) != 255) continue;
        const auto now = clk::now();
        if (now < next_query) continue;
        next_query = now + std::chrono::milliseconds(1);
        const hipError_t q = hipStreamQuery(stream);
        if (q != hipSuccess && q != hipErrorNotReady) return kErrHip;
        // An idle stream without the word: its writer never ran (an error), or the
        // word is still on its way to host memory (seen with several processes on one
        // GPU): an error only once it stays missing for 200 ms.
        if (q == hipSuccess && __atomic_load_n(word, __ATOMIC_ACQUIRE) != seq &&
            (!queued || queued->load(std::memory_order_acquire))) {
            if (!idle) {
                idle = true;
                idle_since = now;
            } else if (now - idle_since > std::chrono::milliseconds(200)) {
                if (std::getenv("JPGE_DEBUG")) std::fprintf(stderr, "jpge: wait_seq: word %llu != %llu, stream idle\n",
                                                          (unsigned long long)__atomic_load_n(word, __ATOMIC_ACQUIRE),
                                                          (unsigned long long)seq);
                return kErrInternal;
            }
        } else {
            idle = false;
        }
        if (now - t0 > std::chrono::seconds(20)) return kErrTimeout;
    }
}

// Pipeline depth limits (defaults in Encoder; the slots in flight = lookahead + drain lag + 1).
constexpr int kMaxLookahead = 8;
constexpr int kMaxDrainLag = 4;
constexpr int kMaxLanes = 8;
constexpr uint64_t kFirstSleepMaxPixels = 16u << 20;   // frames this large poll their results without a first sleep

double abs_us(std::chrono::steady_clock::time_point t) {  // host-trace clock
    return std::chrono::duration<double, std::micro>(t.time_since_epoch()).count();
}

int env_int(const char* name, int dflt, int lo, int hi) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    const long x = std::strtol(v, nullptr, 10);
    return x < lo ? lo : x > hi ? hi : (int)x;
}

constexpr size_t kTabBytes = 4 * 256 * 4;  // code tables as uploaded
constexpr size_t kHdrMax = 4096;           // headers SOI .. SOS (<= 20 + 2*69 + 19 + 4*277 + 14)

// Control block, zeroed at the start of every frame by the first kernel (K1).
struct CtlLayout {
    size_t cnt, key, rec, done, total;  // [0, total): zeroed by K1 every frame
    size_t place, summary, alloc;  // not zeroed (written before they are read)
    explicit CtlLayout(uint32_t ntiles) {  // ntiles: entropy workgroups (records)
        size_t o = 0;
        cnt = o; o += align_up((size_t)kHistReplicas * 4 * 256 * 4, 256);
        key = o; o += align_up(4 * 256 * 8, 256);
        rec = o; o += align_up((size_t)ntiles * kEntropyRecordBytes, 256);
        done = o; o += 256;
        total = o;
        place = o; o += align_up((size_t)ntiles * sizeof(WgPlace), 256);
        summary = o; o += 256;
        alloc = o;
    }
};

constexpr size_t kStatsDoneOff = 64;  // K2's finished-workgroup count: a line of its own in the `done` block
constexpr size_t kPackDoneOff = 128;  // the pack kernel's count, end offset and flag: another line

struct HostHist {  // written by hist_export_kernel into mapped pinned memory
    uint32_t cnt[4 * 256];  // replicas summed
    uint64_t key[4 * 256];  // ~first-occurrence key
    uint64_t seq;           // frame sequence number, written after the data
};

}  // namespace

// A 1-lane encoder's second table thread, for single images (encode()): while the calling
// thread builds the luma AC table (the largest: ~2/3 of a frame's table time), it builds
// the other three.  It is armed when a call starts waiting for its histograms (so its
// wake-up overlaps the two kernels), spins only until the call's tables are built, and
// otherwise sleeps on a condition variable.
class Encoder::TableHelper {
  public:
    TableHelper() {
        th_ = std::thread([this] {
            prctl(PR_SET_NAME, "jpge-tables", 0, 0, 0);
            run();
        });
    }
    ~TableHelper() {
        state_.store(kStop, std::memory_order_release);
        { std::lock_guard<std::mutex> g(mu_); }
        cv_.notify_one();
        th_.join();
    }
    void arm() {
        int idle = kIdle;
        if (state_.compare_exchange_strong(idle, kArmed, std::memory_order_acq_rel)) {
            { std::lock_guard<std::mutex> g(mu_); }
            cv_.notify_one();
        }
    }
    void disarm() {
        int s = state_.load(std::memory_order_acquire);
        while ((s == kArmed || s == kDone) && !state_.compare_exchange_weak(s, kIdle, std::memory_order_acq_rel)) {
        }
    }
    // tables 0, 2 and 3 (DC luma, DC and AC chroma) on the helper; false: not armed (the
    // caller builds them itself)
    bool post(const uint32_t* cnt, const uint64_t* key, bool inverted, HuffTable* tabs, int* ok) {
        if (state_.load(std::memory_order_acquire) != kArmed) return false;
        cnt_ = cnt;
        key_ = key;
        inv_ = inverted;
        tabs_ = tabs;
        ok_ = ok;
        int armed = kArmed;
        return state_.compare_exchange_strong(armed, kJob, std::memory_order_acq_rel);
    }
    void wait() {
        while (state_.load(std::memory_order_acquire) != kDone) __builtin_ia32_pause();
    }

  private:
    enum { kIdle, kArmed, kJob, kDone, kStop };
    void run() {
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return state_.load(std::memory_order_acquire) != kIdle; });
            }
            for (;;) {
                const int s = state_.load(std::memory_order_acquire);
                if (s == kStop) return;
                if (s == kIdle) break;
                if (s == kJob) {
                    for (int t : {0, 2, 3})
                        ok_[t] = inv_ ? build_table_inverted(cnt_ + t * 256, key_ + t * 256, tabs_[t])
                                      : build_table(cnt_ + t * 256, key_ + t * 256, tabs_[t]);
                    state_.store(kDone, std::memory_order_release);
                    continue;
                }
                __builtin_ia32_pause();
            }
        }
    }
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<int> state_{kIdle};
    const uint32_t* cnt_ = nullptr;
    const uint64_t* key_ = nullptr;
    bool inv_ = false;
    HuffTable* tabs_ = nullptr;
    int* ok_ = nullptr;
};

struct Encoder::Slot {
    hipStream_t stream = nullptr;  // the encoder's stream (shared by all slots, not owned)
    // 0-2, 4-5 kernel timing brackets (3, 6, 7 unused)
    hipEvent_t ev[8] = {};
    Geometry g;
    // device workspace (capacities)
    size_t cap_blk = 0, cap_in = 0, cap_out = 0, cap_ctl = 0;
    uint8_t* d_in = nullptr;
    int16_t* d_coef = nullptr;
    uint8_t* d_ctl = nullptr;
    uint8_t* d_ubuf = nullptr;  // unstuffed entropy-coded segment (K3 internal)
    size_t cap_ubuf = 0;
    uint16_t* d_recs = nullptr;    // K2's symbol records, kTileRecords per entropy tile
    uint32_t* d_tcount = nullptr;  // records per tile
    size_t cap_tiles = 0;          // (capacities: records, in words; tiles)
    size_t cap_recs = 0;
    uint8_t* d_out = nullptr;
    uint32_t* d_tab = nullptr;  // [1024] tables, then the header bytes (one upload)
    // pinned host staging
    HostHist* h_hist = nullptr;
    HostHist* d_hist_host = nullptr;  // device view of h_hist
    uint32_t* h_tab = nullptr;     // same layout as d_tab (mapped)
    uint32_t* d_tab_host = nullptr;  // device view of h_tab
    uint64_t* h_result = nullptr;  // mapped: written by the entropy kernel's last workgroup
                                   // ([0, 4)); [6]: encode()'s gate word (gate())
    uint64_t* d_result_host = nullptr;
    // per-frame state between phases
    const uint8_t* in_dev = nullptr;
    size_t in_stride = 0;
    uint8_t* out_dev = nullptr;
    size_t out_cap = 0;
    size_t hdr_len = 0;
    uint64_t symbols = 0;              // Huffman-coded symbols (= K2 symbol records) of the frame
    uint8_t qy[64], qc[64];
    bool timed = false;                // this frame's kernels are bracketed by timing events
    int timed_frames = 1;              // frames those kernels covered (a frame set's launches)
    bool count_symbols = false;        // a member of a timed launch: its symbols go to times_.symbols
    HistPtrs hist{};                   // this frame's device histograms (in d_ctl)
    uint64_t seq = 0;                  // frame sequence number (handshakes via mapped memory)
    std::atomic<int> tables_done{0};   // set by build_tables (any thread)
    std::atomic<int> export_queued{0}; // the kernel exporting this frame's histograms is launched
    std::chrono::steady_clock::time_point t_submit, t_start, t_done;  // table job (host trace)
    // stripe context (a row stripe of a larger image; whole frames: zero seeds and
    // bases, header dimensions = the frame's)
    DcSeed seed;
    Restart rst;  // restart intervals of the frame (stripe: its first MCU in the image's numbering)
    uint64_t key_y0 = 0, key_c0 = 0, key_ncb = 0;
    uint32_t img_w = 0, img_h = 0;
    int tables_status = 0;
    bool inline_tables = false;  // this frame's tables are built inside its lane's pipeline (its waits use the lane's guess)
    // the lane's wait estimates (histograms when its own thread builds the tables; results)
    WaitGuess* guess_hist = nullptr;
    WaitGuess* guess_result = nullptr;

    uint32_t* gate() const { return reinterpret_cast<uint32_t*>(h_result + 6); }

    ~Slot() {
        hipFree(d_in); hipFree(d_coef); hipFree(d_ctl); hipFree(d_ubuf);
        hipFree(d_recs); hipFree(d_tcount);
        hipFree(d_out); hipFree(d_tab);
        hipHostFree(h_hist); hipHostFree(h_tab); hipHostFree(h_result);
        for (auto& e : ev) if (e) hipEventDestroy(e);
    }
};

// An independent pipeline: its own stream and slot ring; lanes other than 0 own a
// host thread that runs the lane's share of a batch.  Between batches the thread
// polls for ~1 ms (back-to-back batches start without a wake-up), then blocks.
struct Encoder::Lane {
    int id = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // end of the lane's batch work on its stream
    std::vector<std::unique_ptr<Slot>> slots;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<int()> job;
    int result = 0;
    std::atomic<uint32_t> posted{0}, finished{0};
    std::atomic<bool> stop{false};
    WaitGuess guess_hist, guess_result;  // (the slots point here)

    void start() {
        th = std::thread([this] {
            prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
            const std::string name = "jpge-lane" + std::to_string(id);
            prctl(PR_SET_NAME, name.c_str(), 0, 0, 0);
            uint32_t seen = 0;
            for (;;) {
                const auto t0 = std::chrono::steady_clock::now();
                while (posted.load(std::memory_order_acquire) == seen && !stop.load(std::memory_order_acquire)) {
                    if (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(1)) {
                        std::this_thread::yield();
                        continue;
                    }
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return posted.load(std::memory_order_acquire) != seen || stop.load(); });
                }
                if (posted.load(std::memory_order_acquire) == seen) return;  // stopped
                seen = posted.load(std::memory_order_acquire);
                result = job();
                finished.store(seen, std::memory_order_release);
            }
        });
    }
    void post(std::function<int()> f) {
        job = std::move(f);
        posted.fetch_add(1, std::memory_order_acq_rel);
        { std::lock_guard<std::mutex> g(mu); }
        cv.notify_one();
    }
    int wait() {
        const uint32_t want = posted.load(std::memory_order_acquire);
        while (finished.load(std::memory_order_acquire) != want) std::this_thread::yield();
        return result;
    }
    void shutdown() {
        if (!th.joinable()) return;
        stop.store(true, std::memory_order_release);
        { std::lock_guard<std::mutex> g(mu); }
        cv.notify_one();
        th.join();
    }
};

int Encoder::set_restart(uint32_t mcus) {
    if (mcus > 65535) return kErrArg;  // DRI carries a 16-bit interval
    restart_mcus_ = mcus;
    return kOk;
}

int Encoder::set_subsampling(int mode) {
    uint32_t yh, bpm, cf;
    if (!mode_shape(mode, yh, bpm, cf)) return kErrArg;
    mode_ = mode;
    return kOk;
}

size_t Encoder::max_jpeg_bytes(uint32_t w, uint32_t h) {
    // header <= 20 + 2*69 + 19 + 4*(4+17+256) + 14 ; entropy <= 1665 bits/block,
    // doubled for worst-case 0xFF stuffing; + EOI.
    // Restart intervals add per MCU at most an RST marker, a fill byte and its stuffing.
    // (The largest bound over the MCU shapes: one capacity serves every mode.)
    size_t cap = 0;
    for (int mode : {420, 444, 422, 411}) {
        const Geometry g = geometry(w, h, mode);
        cap = std::max(cap, 2048 + (size_t)g.nblocks() * 2 * 209 + 16 + (size_t)g.nmcu() * 4);
    }
    return cap;
}

int Encoder::open(int device, std::unique_ptr<Encoder>& out, int lanes) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return kErrNoDevice;
    if (device < 0 || device >= n) return kErrNoDevice;
    JPGE_HIP(hipSetDevice(device));
    std::unique_ptr<Encoder> e(new Encoder());
    e->device_ = device;
    if (const char* ew = std::getenv("JPGE_ENTROPY_WGS")) e->entropy_wgs_ = (uint32_t)std::strtoul(ew, nullptr, 10);
    if (const char* sw = std::getenv("JPGE_STATS_WGS")) e->stats_wgs_ = (uint32_t)std::strtoul(sw, nullptr, 10);
    e->fdct_wgs_ = (uint32_t)env_int("JPGE_FDCT_WGS", 0, 0, 65536);
    e->stamps_file_ = std::getenv("JPGE_STAMPS_FILE");
    e->host_trace_file_ = std::getenv("JPGE_HOST_TRACE");
    e->cpu_prof_ = env_int("JPGE_CPU_PROF", 0, 0, 1) != 0;
    e->lat_prof_ = env_int("JPGE_LAT_PROF", 0, 0, 1) != 0;
    e->table_helper_ = env_int("JPGE_TABLE_HELPER", 1, 0, 1) != 0;
    e->gate_ = env_int("JPGE_GATE", 1, 0, 2);
    // Launch-serialising debug modes block the host in a launch until the kernel (or its
    // predecessor) has finished, so the host could never open the gate behind the gate
    // kernel: every call would run into its time-out.  They get the ungated path.
    if (env_int("AMD_SERIALIZE_KERNEL", 0, 0, 3) != 0 || env_int("HIP_LAUNCH_BLOCKING", 0, 0, 1) != 0) e->gate_ = 0;
    if (const int us = env_int("JPGE_TEST_GATE_TIMEOUT_US", 0, 0, 1000000)) e->gate_ticks_ = 100ull * (uint64_t)us;
    e->gate_delay_us_ = env_int("JPGE_TEST_GATE_DELAY_US", 0, 0, 1000000);
    if (e->gate_ == 2) {  // (the runtime's stream wait needs device support)
        int wv = 0;
        if (hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, device) != hipSuccess || !wv) e->gate_ = 0;
        (void)hipGetLastError();
    }
    e->hist_nap_us_ = env_int("JPGE_HIST_NAP_US", e->hist_nap_us_, 0, 1000);
    e->lookahead_ = env_int("JPGE_LOOKAHEAD", e->lookahead_, 1, kMaxLookahead);
    e->drain_lag_ = env_int("JPGE_DRAIN_LAG", e->drain_lag_, 0, kMaxDrainLag);
    e->set_ = env_int("JPGE_SET", 0, 0, kMaxSet);
    e->nap_us_ = env_int("JPGE_NAP_US", e->nap_us_, 1, 1000);
    e->first_sleep_ = env_int("JPGE_FIRST_SLEEP", (int)(e->first_sleep_ * 100 + 0.5), 0, 95) / 100.0;
    const int nap = env_int("JPGE_NAP", -1, -1, 1);
    e->ext_place_ = env_int("JPGE_EXT_PLACE", -1, -1, 1);
    e->place_in_code_ = env_int("JPGE_PLACE_IN_CODE", 1, 0, 1) != 0;
    if (e->stamps_file_) {
        e->dbg_words_ = 4ull * 65536 * kStampSlots;  // up to 64k workgroups per kernel, 4 kernels
        JPGE_HIP(hipMalloc((void**)&e->d_dbg_, e->dbg_words_ * 8));
        JPGE_HIP(hipMemset(e->d_dbg_, 0, e->dbg_words_ * 8));  // (diagnostic stamps only: the null stream)
    }
    // Lanes: each an in-order stream whose frame i+1.. transform and statistics
    // kernels are queued ahead of frame i's entropy kernels, so the host builds frame
    // i's tables while the GPU works on later frames.  Lanes run frames side by side,
    // so one lane's kernels fill another's launch tails and latency-bound phases
    // (4 lanes = the hardware queues HIP opens per process; measured best).
    const int nlanes = e->stamps_file_ ? 1
                       : lanes > 0   ? std::min(lanes, kMaxLanes)
                                     : env_int("JPGE_LANES", 4, 1, kMaxLanes);
    // Lane threads nap between polls when several lanes share the GPU: the same
    // throughput at 2.6 instead of 5.8 host CPUs per GPU (4 lanes, 4K bench); a single
    // lane spins for its latency.
    e->nap_ = nap < 0 ? nlanes > 1 : nap != 0;
    const int nslots = e->lookahead_ + e->drain_lag_ + 1;  // a slot is reused after its drain
    // Several lanes: each lane's stream is created with a full CU mask, which gives it a
    // hardware queue of its own (ROCclr hands such a stream a dedicated queue instead of
    // one from the process's shared pool of GPU_MAX_HW_QUEUES).  From the pool, two lanes
    // could land on one in-order queue and serialise: the 1080p batch (config 4) ran
    // 107.8-109.9 vs 88.6-90.8 GPix/s, the same as with GPU_MAX_HW_QUEUES=6 (110.2-110.3);
    // 4K unchanged (185.2 vs 185.4).  JPGE_CU_MASK_STREAMS=0: pool streams.
    const bool cumask = env_int("JPGE_CU_MASK_STREAMS", nlanes > 1 ? 1 : 0, 0, 1) != 0;
    std::vector<uint32_t> mask;
    if (cumask) {
        int ncu = 0;
        JPGE_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
        mask.assign((size_t)(ncu + 31) / 32, 0xFFFFFFFFu);
        if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
    }
    for (int l = 0; l < nlanes; ++l) {
        std::unique_ptr<Lane> ln(new Lane());
        ln->id = l;
        // (a runtime that refuses CU masks gets a pool stream: correct, possibly shared)
        if (!cumask || hipExtStreamCreateWithCUMask(&ln->stream, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
            (void)hipGetLastError();
            JPGE_HIP(hipStreamCreateWithFlags(&ln->stream, hipStreamNonBlocking));
        }
        JPGE_HIP(hipEventCreateWithFlags(&ln->done, hipEventDisableTiming));
        ln->guess_hist.frac = ln->guess_result.frac = e->first_sleep_;
        if (const int st = e->add_slots(*ln, nslots)) return st;
        if (l > 0) ln->start();
        e->lanes_.push_back(std::move(ln));
    }
    out = std::move(e);
    return kOk;
}

int Encoder::add_slots(Lane& ln, int count) {
    while ((int)ln.slots.size() < count) {
        std::unique_ptr<Slot> s(new Slot());
        s->stream = ln.stream;
        s->guess_hist = &ln.guess_hist;
        s->guess_result = &ln.guess_result;
        for (int k = 0; k < 8; ++k)
            JPGE_HIP(hipEventCreateWithFlags(&s->ev[k], hipEventDefault));
        JPGE_HIP(hipHostMalloc((void**)&s->h_hist, sizeof(HostHist), hipHostMallocMapped));
        JPGE_HIP(hipHostGetDevicePointer((void**)&s->d_hist_host, s->h_hist, 0));
        JPGE_HIP(hipHostMalloc((void**)&s->h_tab, kTabBytes + kHdrMax, hipHostMallocMapped));
        JPGE_HIP(hipHostGetDevicePointer((void**)&s->d_tab_host, s->h_tab, 0));
        // (zeroed: a code kernel behind encode()'s gate reads whatever tables are here when
        // a table build fails, and zero lengths keep it within its bounds)
        std::memset(s->h_tab, 0, kTabBytes + kHdrMax);
        JPGE_HIP(hipHostMalloc((void**)&s->h_result, 64, hipHostMallocMapped));
        std::memset(s->h_result, 0, 64);
        JPGE_HIP(hipHostGetDevicePointer((void**)&s->d_result_host, s->h_result, 0));
        JPGE_HIP(hipMalloc((void**)&s->d_tab, kTabBytes + kHdrMax));
        // (zeroed too: a gate that times out leaves the code kernel these tables, ADVICE r5;
        // on the lane's stream: an operation on the null stream made every later launch on
        // the lanes' streams slower, the 4K pipeline -3%)
        JPGE_HIP(hipMemsetAsync(s->d_tab, 0, kTabBytes + kHdrMax, ln.stream));
        ln.slots.push_back(std::move(s));
    }
    return kOk;
}

Encoder::~Encoder() {
    if (lat_prof_ && lat_calls_)
        std::fprintf(stderr, "jpge encode() phases per call (us, wall): launch-1 %.2f histogram-wait %.2f tables %.2f "
                             "launch-entropy %.2f result-wait %.2f end %.2f (%lld calls)\n",
                     lat_ns_[0] / 1e3 / lat_calls_, lat_ns_[1] / 1e3 / lat_calls_, lat_ns_[2] / 1e3 / lat_calls_,
                     lat_ns_[3] / 1e3 / lat_calls_, lat_ns_[4] / 1e3 / lat_calls_, lat_ns_[5] / 1e3 / lat_calls_,
                     (long long)lat_calls_);
    if (lat_prof_ && lat_calls_)
        std::fprintf(stderr, "jpge   of launch-1: argument preparation %.2f, K1 launch %.2f\n", lat_ns_[6] / 1e3 / lat_calls_,
                     lat_ns_[7] / 1e3 / lat_calls_);
    if (cpu_prof_ && cpu_frames_.load()) {
        const double f = (double)cpu_frames_.load();
        std::fprintf(stderr, "jpge cpu per frame (us): tables %.2f launch-1 %.2f launch-entropy %.2f finish %.2f "
                             "loop-top %.2f end %.2f\n",
                     cpu_ns_[1] / f / 1e3, cpu_ns_[2] / f / 1e3, cpu_ns_[3] / f / 1e3, cpu_ns_[4] / f / 1e3,
                     cpu_ns_[0] / f / 1e3, cpu_ns_[5] / f / 1e3);
        if (cpu_builds_.load())
            std::fprintf(stderr, "jpge table builds: %lld, histogram read %.2f us, tables + headers %.2f us each\n",
                         (long long)cpu_builds_.load(), cpu_read_ns_.load() / 1e3 / cpu_builds_.load(),
                         cpu_build_ns_.load() / 1e3 / cpu_builds_.load());
        if (cpu_builds_.load())
            std::fprintf(stderr, "jpge   of which: 4 tables %.2f us, code words to mapped memory %.2f us, headers %.2f us\n",
                         cpu_part_ns_[0].load() / 1e3 / cpu_builds_.load(), cpu_part_ns_[1].load() / 1e3 / cpu_builds_.load(),
                         cpu_part_ns_[2].load() / 1e3 / cpu_builds_.load());
        for (auto& ln : lanes_)
            for (const WaitGuess* g : {&ln->guess_hist, &ln->guess_result})
                std::fprintf(stderr, "jpge lane %d %s waits: %llu (%llu ready on entry), %.2f naps and %.1f us per wait, ema %.1f\n",
                             ln->id, g == &ln->guess_hist ? "histogram" : "result", (unsigned long long)g->waits,
                             (unsigned long long)g->ready, g->waits ? (double)g->naps / g->waits : 0.0,
                             g->waits ? g->total_us / g->waits : 0.0, g->ema_us);
    }
    helper_.reset();
    for (auto& ln : lanes_) ln->shutdown();
    for (auto& b : scratch_) hipFree(b.first);
    hipSetDevice(device_);
    for (auto& ln : lanes_) {
        if (ln->stream) hipStreamSynchronize(ln->stream);
        ln->slots.clear();
        if (ln->done) hipEventDestroy(ln->done);
        if (ln->stream) hipStreamDestroy(ln->stream);
    }
    hipFree(d_dbg_);
}

// Diagnostic: raw per-workgroup phase stamps of the last frame, as
// [u64 n_fdct_wg, n_stats_wg, n_code_wg, n_pack_wg] then 4 x 65536 x kStampSlots u64;
// the buffer is cleared afterwards (slots 8-15 accumulate).
void Encoder::dump_stamps(const Slot& s) {
    if (!stamps_file_ || !d_dbg_) return;
    std::vector<uint64_t> h(dbg_words_);
    if (hipMemcpy(h.data(), d_dbg_, dbg_words_ * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    const uint64_t hdr[4] = {fdct_grid(s.g, lanes_.size() == 1, fdct_wgs_), stats_grid(layout(s.g), stats_wgs()), layout(s.g).grid(),
                             layout(s.g).grid()};
    FILE* f = std::fopen(stamps_file_, "wb");
    if (!f) return;
    std::fwrite(hdr, 8, 4, f);
    std::fwrite(h.data(), 8, h.size(), f);
    std::fclose(f);
    hipMemset(d_dbg_, 0, dbg_words_ * 8);
}

int Encoder::ensure(Slot& s, const Geometry& g, size_t in_bytes, size_t out_cap) {
    const size_t nblk = g.nblocks();
    if (nblk > s.cap_blk) {
        hipFree(s.d_coef);
        s.d_coef = nullptr; s.cap_blk = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_coef, nblk * 128));
        s.cap_blk = nblk;
    }
    const CtlLayout L(layout(g).grid());
    const size_t ntiles = seg_tiles(layout(g));
    const size_t nrecs = (size_t)seg_tiles(layout(g)) * kTileRecords;
    if (ntiles > s.cap_tiles || nrecs > s.cap_recs) {
        hipFree(s.d_recs); hipFree(s.d_tcount);
        s.d_recs = nullptr; s.d_tcount = nullptr; s.cap_tiles = s.cap_recs = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_recs, nrecs * sizeof(*s.d_recs)));
        JPGE_HIP(hipMalloc((void**)&s.d_tcount, ntiles * kRecSub * 4));
        s.cap_tiles = ntiles;
        s.cap_recs = nrecs;
    }
    const size_t ubuf = entropy_ubuf_bytes(layout(g));
    if (ubuf > s.cap_ubuf) {
        hipFree(s.d_ubuf); s.d_ubuf = nullptr; s.cap_ubuf = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_ubuf, ubuf));
        s.cap_ubuf = ubuf;
    }
    if (L.alloc > s.cap_ctl) {
        hipFree(s.d_ctl); s.d_ctl = nullptr; s.cap_ctl = 0;
        JPGE_HIP(hipMalloc((void**)&s.d_ctl, L.alloc));
        s.cap_ctl = L.alloc;
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

SegLayout Encoder::slot_layout(const Slot& s) const {
    return seg_layout(s.g, s.rst.mcus, entropy_wgs());
}

// Kernel parameter blocks of a slot's frame (or stripe).
FdctArgs Encoder::fdct_args(Slot& s, int maxval, Slot* imp) {
    const CtlLayout L(slot_layout(s).grid());
    FdctArgs a;
    a.rgb = s.in_dev;
    a.stride = s.in_stride;
    a.g = s.g;
    a.maxval = maxval;
    a.solo = lanes_.size() == 1;  // (several lanes: K1 runs beside other frames' kernels)
    a.wgs = fdct_wgs_;
    for (int i = 0; i < 64; ++i) {
        a.q[i] = s.qy[i];
        a.q[64 + i] = s.qc[i];
    }
    a.coef = s.d_coef;
    a.zero = reinterpret_cast<uint32_t*>(s.d_ctl);
    a.zero_words = (uint32_t)(L.total / 4);
    a.imp_src = imp ? reinterpret_cast<const uint4*>(imp->d_tab_host) : nullptr;
    a.imp_dst = imp ? reinterpret_cast<uint4*>(imp->d_tab) : nullptr;
    a.imp_n16 = imp ? (uint32_t)((kTabBytes + imp->hdr_len + 15) / 16) : 0u;
    a.dbg = d_dbg_;
    return a;
}

StatsArgs Encoder::stats_args(Slot& s) {
    const CtlLayout L(slot_layout(s).grid());
    StatsArgs st;
    st.coef = s.d_coef;
    st.g = s.g;
    st.hist.cnt = reinterpret_cast<uint32_t*>(s.d_ctl + L.cnt);
    st.hist.key = reinterpret_cast<uint64_t*>(s.d_ctl + L.key);
    st.seed = s.seed;
    st.rst = s.rst;
    st.key_y0 = s.key_y0;
    st.key_c0 = s.key_c0;
    st.key_ncb = s.key_ncb;
    st.seg = seg_layout(s.g, s.rst.mcus, entropy_wgs());
    st.recs = s.d_recs;
    st.tcount = s.d_tcount;
    st.wgs = stats_wgs();
    if (!stats_wgs_ && lanes_.size() > 1) {
        // frames under ~3 MPix (fewer than 3 tiles per workgroup at 384): about 3 tiles per
        // workgroup, not one each (a workgroup's fixed costs, its first load not overlapped:
        // 1080p batch +9%); 4K and larger keep one workgroup per CU (stats_wgs)
        const uint32_t t = seg_tiles(st.seg);
        if (t < 3u * 384u) st.wgs = std::max(1u, (t + 2) / 3);
    }
    st.dbg = d_dbg_ ? d_dbg_ + 65536 * kStampSlots : nullptr;
    return st;
}

EntropyArgs Encoder::entropy_args(Slot& s) {
    const CtlLayout L(slot_layout(s).grid());
    EntropyArgs e;
    e.coef = s.d_coef;
    e.recs = s.d_recs;
    e.tcount = s.d_tcount;
    e.g = s.g;
    e.tables = s.d_tab;
    e.out = s.out_dev;
    e.hdr_len = s.hdr_len;
    e.out_cap = s.out_cap;
    e.rec = s.d_ctl + L.rec;
    e.place = reinterpret_cast<WgPlace*>(s.d_ctl + L.place);
    e.summary = reinterpret_cast<StripeSummary*>(s.d_ctl + L.summary);
    if (ext_place_ > 0 || (ext_place_ < 0 && lanes_.size() > 1)) {
        e.flags |= kExtPlace;
        // the last code workgroup places every workgroup (no placement launch); the
        // counter is in the block K1 zeroes
        if (place_in_code_ && !s.rst.mcus && slot_layout(s).grid() <= kPlaceInCodeMaxWgs)
            e.done = reinterpret_cast<uint32_t*>(s.d_ctl + L.done);
    }
    e.host_result = s.d_result_host;
    e.seq = s.seq;
    e.ubuf = s.d_ubuf;
    e.wgs = entropy_wgs_;
    e.seed = s.seed;
    e.rst = s.rst;
    e.seg = slot_layout(s);
    if (s.rst.mcus) {  // a stripe's first interval follows the previous stripes' ones
        e.seg_index0 = s.rst.mcu0 / s.rst.mcus;
        e.seg_markers0 = e.seg_index0 > 0 ? 1u : 0u;
    }
    e.exp_hist = HistPtrs{};
    e.exp_cnt = nullptr;
    e.exp_key = nullptr;
    e.exp_seq = nullptr;
    e.exp_seqv = 0;
    e.dbg = d_dbg_ ? d_dbg_ + 2 * 65536 * kStampSlots : nullptr;
    return e;
}

// Phase 1: upload (if host input), statistics kernels, histogram read-back.
int Encoder::prep1(Slot& s, const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                   Slot* imp, FdctArgs& a, StatsArgs& st) {
    if (!f.rgb || f.width == 0 || f.height == 0 || f.width > 65535 || f.height > 65535) return kErrArg;
    if (f.maxval < 1 || f.maxval > 255) return kErrRange;
    const Geometry g = geometry(f.width, f.height, mode_);
    const size_t row = (size_t)f.width * 3;
    const size_t stride = f.stride ? f.stride : row;
    if (stride < row) return kErrArg;
    const size_t dev_pitch = align_up(row, 16);
    const size_t in_bytes = (flags & kFlagDeviceInput) ? 0 : dev_pitch * f.height;
    const size_t out_cap = (flags & kFlagDeviceOutput) ? 0 : max_jpeg_bytes(f.width, f.height);
    for (int i = 0; i < 64; ++i)
        if (!qy[i] || !qc[i]) return kErrArg;
    const int st0 = ensure(s, g, in_bytes, out_cap);
    if (st0) return st0;
    std::memcpy(s.qy, qy, 64);
    std::memcpy(s.qc, qc, 64);
    s.g = g;
    if (flags & kFlagDeviceInput) {
        s.in_dev = f.rgb;
        s.in_stride = stride;
    } else {
        if (stride == dev_pitch)  // one linear copy (a 2D copy can fall back to a slower engine path)
            JPGE_HIP(hipMemcpyAsync(s.d_in, f.rgb, dev_pitch * f.height, hipMemcpyHostToDevice, s.stream));
        else
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
    s.seed = DcSeed();
    s.rst = Restart();
    s.rst.mcus = restart_mcus_;
    s.key_y0 = s.key_c0 = s.key_ncb = 0;
    s.img_w = f.width;
    s.img_h = f.height;
    a = fdct_args(s, f.maxval, imp);
    st = stats_args(s);
    s.tables_done.store(0, std::memory_order_relaxed);
    s.export_queued.store(0, std::memory_order_relaxed);
    return kOk;
}

int Encoder::phase1(Slot& s, const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                    Slot* imp, bool export_hist) {
    FdctArgs a;
    StatsArgs st2;
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = lat_prof_ ? clk::now() : clk::time_point{};
    if (const int st = prep1(s, f, qy, qc, flags, imp, a, st2)) return st;
    const clk::time_point t1 = lat_prof_ ? clk::now() : clk::time_point{};
    s.timed = timing_every_ && (frame_counter_++ % (uint64_t)timing_every_) == 0;
    s.timed_frames = 1;
    s.count_symbols = s.timed;
    // sampled frames: each kernel launched with its own events (KTimer, kernels.hpp)
    const KTimer t1k{s.ev[0], s.ev[1]}, t2k{s.ev[2], s.ev[3]};
    s.seq = ++seq_counter_;
    s.hist = st2.hist;
    if (export_hist) {  // (by K2's last workgroup: no launch of its own)
        st2.done = reinterpret_cast<uint32_t*>(s.d_ctl + CtlLayout(slot_layout(s).grid()).done + kStatsDoneOff);
        st2.host_cnt = s.d_hist_host->cnt;
        st2.host_key = s.d_hist_host->key;
        st2.host_seq = &s.d_hist_host->seq;
        st2.seq = s.seq;
    }
    JPGE_HIP(launch_fdct(a, s.stream, s.timed ? &t1k : nullptr));
    const clk::time_point t2 = lat_prof_ ? clk::now() : clk::time_point{};
    JPGE_HIP(launch_stats(st2, s.stream, s.timed ? &t2k : nullptr));
    if (export_hist) s.export_queued.store(1, std::memory_order_release);
    if (lat_prof_) {
        lat_ns_[6] += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        lat_ns_[7] += std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
    }
    return kOk;
}

// A frame set's phase 1: the members' arguments come from prep1 (members it refused
// are not in the set).  Their histograms leave through a later code kernel or
// launch_hist_export.
// K1 workgroups per frame of a set (unless JPGE_FDCT_WGS is given): a set's launch has
// n times the tiles, so fewer, longer-lived workgroups per frame (4K, 4 lanes: 214.6 vs
// 212.4 GPix/s with the single-frame cap of 512; alone, a set of 4 in 48 instead of 52 us)
constexpr uint32_t kSetFdctWgs = 256;
int Encoder::phase1_set(Slot* const* s, int n, const FdctArgs* a_in, const StatsArgs* st) {
    FdctArgs a[kMaxSet];
    for (int m = 0; m < n; ++m) {
        a[m] = a_in[m];
        if (!fdct_wgs_ && n > 1) a[m].wgs = kSetFdctWgs;
    }
    // a sampled set: its launches timed with the first member's events, as n frames' work
    for (int m = 0; m < n; ++m) s[m]->timed = false;
    const uint64_t c = frame_counter_.fetch_add((uint64_t)n);
    Slot& t = *s[0];
    const uint64_t E = (uint64_t)timing_every_;
    t.timed = E && (c + E - 1) / E * E <= c + (uint64_t)n - 1;  // (a sampled frame number in the set)
    t.timed_frames = n;
    for (int m = 0; m < n; ++m) s[m]->count_symbols = t.timed;
    const KTimer t1{t.ev[0], t.ev[1]}, t2{t.ev[2], t.ev[3]};
    JPGE_HIP(launch_fdct_set(a, n, t.stream, t.timed ? &t1 : nullptr));
    JPGE_HIP(launch_stats_set(st, n, t.stream, t.timed ? &t2 : nullptr));
    for (int m = 0; m < n; ++m) {
        s[m]->seq = ++seq_counter_;
        s[m]->hist = st[m].hist;
    }
    return kOk;
}

// Phase 2a (host; the calling thread or a lane's thread): wait for the histograms,
// build the four tables (generateHuffmanCode semantics, Huffman.cpp:3-35) and the
// headers into the slot's pinned staging buffer.
int Encoder::build_tables(Slot& s, bool parallel, TableHelper* helper) {
    // (frames above kFirstSleepMaxPixels nap even on a single lane: their kernels take
    // milliseconds, and a spinning thread would burn a core for them)
    const bool big = (uint64_t)s.g.width * s.g.height > kFirstSleepMaxPixels;
    if (const int w = wait_seq(&s.h_hist->seq, s.seq, s.stream, nap_ || big ? nap_us_ : (parallel ? 0 : hist_nap_us_), &s.export_queued,
                               s.inline_tables ? s.guess_hist : nullptr))
        return w;
    if (lat_prof_) lat_hist_seen_ = std::chrono::steady_clock::now();
    auto thread_ns = [] {
        timespec t;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
        return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
    };
    const int64_t t0 = cpu_prof_ ? thread_ns() : 0;
    // (the tables read the mapped export in place: the keys stay inverted, and only the
    // present symbols' keys are read)
    const int64_t t1 = cpu_prof_ ? thread_ns() : 0;
    const int r = build_tables_from(s, s.h_hist->cnt, s.h_hist->key, parallel, /*inverted=*/true, helper);
    if (cpu_prof_) {
        cpu_read_ns_.fetch_add(t1 - t0, std::memory_order_relaxed);
        cpu_build_ns_.fetch_add(thread_ns() - t1, std::memory_order_relaxed);
        cpu_builds_.fetch_add(1, std::memory_order_relaxed);
    }
    return r;
}

// The four tables from counts and first-occurrence keys, and the headers (the
// image's real dimensions in SOF0), into the slot's pinned staging buffer.
int Encoder::build_tables_from(Slot& s, const uint32_t* cnt_all, const uint64_t* first_all, bool parallel,
                               bool inverted, TableHelper* helper) {
    auto thread_ns = [] {
        timespec t;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
        return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
    };
    const int64_t t0 = cpu_prof_ ? thread_ns() : 0;
    HuffTable tabs[4];
    int ok[4] = {0, 0, 0, 0};
    // the four tables are independent; the AC tables dominate
    auto one = [&](long t) {
        ok[t] = inverted ? build_table_inverted(cnt_all + t * 256, first_all + t * 256, tabs[t])
                         : build_table(cnt_all + t * 256, first_all + t * 256, tabs[t]);
    };
    if (helper && helper->post(cnt_all, first_all, inverted, tabs, ok)) {
        one(1);  // (the luma AC table here, the other three on the helper)
        helper->wait();
    } else {
        parallel_for(4, parallel ? 4 : 1, one);
    }
    const int64_t t1 = cpu_prof_ ? thread_ns() : 0;
    for (int t = 0; t < 4; ++t)
        if (ok[t])
            for (int i = 0; i < 256; ++i)
                s.h_tab[t * 256 + i] = ((uint32_t)tabs[t].len[i] << 16) | (tabs[t].code[i] & 0xFFFF);
    const int64_t t2 = cpu_prof_ ? thread_ns() : 0;
    const int bad = !(ok[0] & ok[1] & ok[2] & ok[3]);
    uint64_t nsym = 0;
    for (int i = 0; i < 1024; ++i) nsym += cnt_all[i];
    s.symbols = nsym;
    if (bad) {
        if (std::getenv("JPGE_DEBUG")) {
            std::fprintf(stderr, "jpge: table build failed (seq %llu):", (unsigned long long)s.seq);
            for (int t = 0; t < 4; ++t) {
                uint64_t n = 0;
                for (int i = 0; i < 256; ++i) n += cnt_all[t * 256 + i];
                std::fprintf(stderr, " t%d ok=%d n=%llu", t, ok[t], (unsigned long long)n);
            }
            std::fprintf(stderr, "\n");
        }
        return kErrInternal;
    }
    const HuffTable* tp[4] = {&tabs[0], &tabs[1], &tabs[2], &tabs[3]};
    const std::vector<uint8_t> hdr = jfif_headers(s.img_w, s.img_h, s.qy, s.qc, tp, restart_mcus_,
                                                    (uint8_t)((s.g.yh << 4) | s.g.yv()));
    if (hdr.size() > kHdrMax) return kErrInternal;
    std::memcpy(reinterpret_cast<uint8_t*>(s.h_tab) + kTabBytes, hdr.data(), hdr.size());
    s.hdr_len = hdr.size();
    if (cpu_prof_) {
        cpu_part_ns_[0].fetch_add(t1 - t0, std::memory_order_relaxed);
        cpu_part_ns_[1].fetch_add(t2 - t1, std::memory_order_relaxed);
        cpu_part_ns_[2].fetch_add(thread_ns() - t2, std::memory_order_relaxed);
    }
    if (s.out_cap && s.out_cap < s.hdr_len + 2) return kErrNoSpace;
    return kOk;
}

// Tables + headers to the device by a copy (when no transform kernel carries them).
int Encoder::import_tables_copy(Slot& s) {
    JPGE_HIP(hipMemcpyAsync(s.d_tab, s.h_tab, kTabBytes + s.hdr_len, hipMemcpyHostToDevice, s.stream));
    return kOk;
}

// Phase 2b (GPU): the entropy kernels (tables already on the device); `exp`: a
// later frame whose histograms the code kernel exports on the way.
int Encoder::launch_entropy_phase(Slot& s, Slot* exp, bool lone, int parts) {
    EntropyArgs e = entropy_args(s);
    // A single image on a 1-lane encoder (encode()): the result is handed over once every
    // pack workgroup's write-through stores have completed, so the call need not wait for
    // the kernel's formal end (9 us per 4K call).  The pipeline streams its stores
    // instead (write-through cost it 1.3%) and awaits its stream at the batch's end.
    if (lone && lanes_.size() == 1)
        e.pack_done = reinterpret_cast<uint32_t*>(s.d_ctl + CtlLayout(slot_layout(s).grid()).done + kPackDoneOff);
    if (parts == 3) s.h_result[2] = 0;  // (the slot's previous entropy kernel finished before phase1; gated: encode())
    e.exp_hist = exp ? exp->hist : HistPtrs{};
    e.exp_cnt = exp ? exp->d_hist_host->cnt : nullptr;
    e.exp_key = exp ? exp->d_hist_host->key : nullptr;
    e.exp_seq = exp ? &exp->d_hist_host->seq : nullptr;
    e.exp_seqv = exp ? exp->seq : 0;
    const KTimer tc{s.ev[4], s.ev[5]}, tp{s.ev[6], s.ev[7]};
    if (parts & 1) JPGE_HIP(launch_entropy_code(e, s.stream, s.timed ? &tc : nullptr));
    if (parts & 2) JPGE_HIP(launch_entropy_pack(e, s.stream, s.timed ? &tp : nullptr));
    return kOk;
}

int Encoder::finish(Slot& s, FrameDesc& f, uint32_t flags, bool guess_wait, const std::function<bool()>* idle) {
    // (a first sleep only up to kFirstSleepMaxPixels: 16384^2 frames, few per lane and
    // irregular, lost 3.7% to it)
    // (a set's later members: their results follow the first one's within microseconds,
    // and their short waits would blur the estimate of the real one)
    WaitGuess* const guess =
        guess_wait && (uint64_t)s.g.width * s.g.height <= kFirstSleepMaxPixels ? s.guess_result : nullptr;
    const bool big = (uint64_t)s.g.width * s.g.height > kFirstSleepMaxPixels;  // (as build_tables)
    if (const int w = wait_seq(&s.h_result[3], s.seq, s.stream, nap_ || big ? nap_us_ : 0, nullptr, guess, idle)) return w;
    if (s.timed) {
        JPGE_HIP(wait_event(s.ev[7]));
        std::lock_guard<std::mutex> g(times_mu_);
        float code = 0, pack = 0;
        hipEventElapsedTime(&times_.fdct, s.ev[0], s.ev[1]);
        hipEventElapsedTime(&times_.dc_stats, s.ev[2], s.ev[3]);
        hipEventElapsedTime(&code, s.ev[4], s.ev[5]);
        hipEventElapsedTime(&pack, s.ev[6], s.ev[7]);
        hipEventElapsedTime(&times_.entropy, s.ev[4], s.ev[7]);
        hipEventElapsedTime(&times_.total, s.ev[0], s.ev[7]);
        times_.fdct_sum += times_.fdct;
        times_.dc_stats_sum += times_.dc_stats;
        times_.entropy_sum += times_.entropy;
        times_.code_sum += code;
        times_.pack_sum += pack;
        times_.frames += s.timed_frames;                       // (the launches' frames)
        times_.launches += 1;
    }
    if (s.count_symbols) {  // (every member of a timed set: the launches' record bytes are the sum over them)
        std::lock_guard<std::mutex> g(times_mu_);
        times_.symbols += s.symbols;
    }
    if (stamps_file_) hipStreamSynchronize(s.stream);
    dump_stamps(s);
    const uint64_t err = s.h_result[1] | s.h_result[2];
    if (err & 4) { f.len = 0; return kErrNoSpace; }
    if (err) return kErrTimeout;
    const size_t len = (size_t)s.h_result[0];
    f.len = len;
    if (flags & kFlagDeviceOutput) return kOk;
    if (len > f.cap) return kErrNoSpace;
    // Queued on the lane's stream and not awaited here: every caller synchronises the
    // stream afterwards (a batch at its end), and the slot's next pack kernel is behind
    // the copy in stream order.  (Waiting here held the lane's host thread for the
    // stream's queued kernels too: 77 GPix/s with host outputs.)
    JPGE_HIP(hipMemcpyAsync(f.out, s.out_dev, len, hipMemcpyDeviceToHost, s.stream));
    return kOk;
}

int Encoder::encode(FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *lanes_[0]->slots[0];
    using clk = std::chrono::steady_clock;
    clk::time_point T[6];
    if (lat_prof_) T[0] = clk::now();
    int st = phase1(s, f, qy, qc, flags, nullptr, true);
    // The gate: the tables' copy and the code kernel are queued now, behind a stream wait
    // on a mapped word the host sets once the tables are in h_tab, so their launches
    // overlap K1 and K2 instead of following the tables (the pack kernel's arguments
    // carry the header length, so it is launched after them, while the code kernel
    // runs).  Every path below opens the gate.  (A failed table build: the code kernel
    // reads the tables h_tab holds, valid ones or zeros, and its output is discarded.)
    struct Gate {  // (opened at the latest when the call unwinds)
        uint32_t* word;
        uint32_t value;  // (the word holds the previous gated call's value, one less)
        bool shut = false;
        void open() {
            if (shut) __atomic_store_n(word, value, __ATOMIC_RELEASE);
            shut = false;
        }
        ~Gate() { open(); }
    } gate{s.gate(), gate_count_ + 1};
    if (!st && gate_) ++gate_count_;
    if (!st && gate_ == 1) {  // a workgroup of ours waits and copies (entropy.hip gate_copy_kernel)
        s.h_result[2] = 0;  // (its time-out flag)
        if (launch_gate_copy(reinterpret_cast<const uint32_t*>(s.d_result_host + 6), gate.value, s.d_tab_host, s.d_tab,
                             (uint32_t)((kTabBytes + kHdrMax) / 16), s.d_result_host + 2, gate_ticks_,
                             s.stream) == hipSuccess) {
            gate.shut = true;
            st = launch_entropy_phase(s, nullptr, /*lone=*/true, /*parts=*/1);
            if (st) gate.open();
        } else {
            st = kErrHip;
        }
    } else if (!st && gate_ == 2) {  // the runtime's stream wait, then a copy
        if (hipStreamWaitValue32(s.stream, gate.word, gate.value, hipStreamWaitValueEq, 0xFFFFFFFFu) == hipSuccess) {
            gate.shut = true;
            s.h_result[2] = 0;
            if (hipMemcpyAsync(s.d_tab, s.h_tab, kTabBytes + kHdrMax, hipMemcpyHostToDevice, s.stream) != hipSuccess)
                st = kErrHip;
            if (!st) st = launch_entropy_phase(s, nullptr, /*lone=*/true, /*parts=*/1);
            if (st) gate.open();
        } else {
            (void)hipGetLastError();
        }
    }
    if (lat_prof_) T[1] = clk::now();
    // The tables: on this thread, with the helper thread of a 1-lane encoder for frames
    // of 1 MPix and up (armed now, so its wake-up overlaps the kernels; spawning threads
    // per call would cost more than the tables it overlaps).  Not above
    // kFirstSleepMaxPixels: the helper spins from here to the histograms, which take
    // milliseconds there, for tables that are a small part of such a call.
    TableHelper* helper = nullptr;
    const uint64_t npx = (uint64_t)f.width * f.height;
    if (!st && table_helper_ && lanes_.size() == 1 && npx >= (1u << 20) && npx <= kFirstSleepMaxPixels) {
        if (!helper_) helper_.reset(new TableHelper());
        helper = helper_.get();
        helper->arm();
    }
    if (!st) st = build_tables(s, false, helper);
    if (helper) helper->disarm();
    if (lat_prof_) T[2] = clk::now();
    const bool gated = gate.shut;
    if (gate.shut) {
        if (gate_delay_us_) std::this_thread::sleep_for(std::chrono::microseconds(gate_delay_us_));  // (tests)
        gate.open();
        if (!st) st = launch_entropy_phase(s, nullptr, /*lone=*/true, /*parts=*/2);
    } else {
        if (!st) st = import_tables_copy(s);
        if (!st) st = launch_entropy_phase(s, nullptr, /*lone=*/true);
    }
    if (lat_prof_) T[3] = clk::now();
    if (!st) st = finish(s, f, flags);
    if (st == kErrTimeout && gated && s.h_result[2] == 1) {
        // The gate kernel timed out before the host opened it (a host thread stalled for
        // longer than the time-out): the code kernel ran on stale tables, so the frame is
        // coded again behind a plain copy of the tables now in h_tab.
        gate_timeouts_.fetch_add(1, std::memory_order_relaxed);
        s.h_result[2] = 0;
        s.seq = ++seq_counter_;
        st = import_tables_copy(s);
        if (!st) st = launch_entropy_phase(s, nullptr, /*lone=*/true);
        if (!st) st = finish(s, f, flags);
    }
    if (lat_prof_) T[4] = clk::now();
    // Every output byte is in place.  Device output on a 1-lane encoder: the result word is
    // written once every pack workgroup's (write-through) stores have completed, so the
    // kernel's formal end is not awaited (the stream orders the context's next work after
    // it; ~9 us).  Host
    // output: the copy queued by finish(), awaited by spinning as a batch lane's end (a
    // blocking stream synchronisation adds tens of us of wake-up).
    const bool await_end = st || !(flags & kFlagDeviceOutput) || lanes_.size() != 1;
    if (await_end) {
        if (hipEventRecord(lanes_[0]->done, s.stream) != hipSuccess) {
            hipStreamSynchronize(s.stream);
        } else {
            const hipError_t w = wait_event(lanes_[0]->done);
            if (w != hipSuccess && !st) st = kErrHip;
        }
    }
    if (lat_prof_ && !st) {
        T[5] = clk::now();
        auto ns = [](clk::time_point a, clk::time_point b) {
            return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
        };
        lat_ns_[0] += ns(T[0], T[1]);
        lat_ns_[1] += ns(T[1], lat_hist_seen_);
        lat_ns_[2] += ns(lat_hist_seen_, T[2]);
        lat_ns_[3] += ns(T[2], T[3]);
        lat_ns_[4] += ns(T[3], T[4]);
        lat_ns_[5] += ns(T[4], T[5]);
        ++lat_calls_;
    }
    f.status = st;
    return st;
}

int Encoder::encode_batch(FrameDesc* fr, int n, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    const auto t_enter = std::chrono::steady_clock::now();
    JPGE_HIP(hipSetDevice(device_));
    for (int i = 0; i < n; ++i) fr[i].status = 0;
    if (n <= 0) return kOk;
    // Frames are dealt dynamically: a lane takes the batch's next frame (or frame set)
    // when its pipeline has room, so lanes finish together.  Lane 0 runs on the calling
    // thread.
    const int set = batch_set_size(fr, n);
    const int nl = std::min<int>((int)lanes_.size(), (n + set - 1) / set);
    for (int l = 0; l < nl; ++l)
        if (const int st = add_slots(*lanes_[l], (lookahead_ + drain_lag_ + 1) * set)) return st;
    std::atomic<int> next{0};
    for (int l = 1; l < nl; ++l)
        lanes_[l]->post([this, l, fr, n, &next, set, qy, qc, flags] {
            hipSetDevice(device_);
            return run_lane(*lanes_[l], fr, n, &next, set, qy, qc, flags);
        });
    // (napping on the calling thread: ~1 us timer slack for the call, restored after)
    const long slack = nap_ ? prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0) : -1;
    if (slack > 0) prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
    int st = run_lane(*lanes_[0], fr, n, &next, set, qy, qc, flags);
    if (slack > 0) prctl(PR_SET_TIMERSLACK, (unsigned long)slack, 0, 0, 0);
    const auto t_lane0 = std::chrono::steady_clock::now();
    for (int l = 1; l < nl; ++l) {
        const int e = lanes_[l]->wait();
        if (!st) st = e;
    }
    if (host_trace_file_) {
        std::lock_guard<std::mutex> g(trace_mu_);
        if (FILE* f = std::fopen(host_trace_file_, "a")) {
            std::fprintf(f, "-2 -2 0 -1 %.2f %.2f %.2f\n", abs_us(t_enter), abs_us(t_lane0),
                         abs_us(std::chrono::steady_clock::now()));
            std::fclose(f);
        }
    }
    int bad = st;
    for (int i = 0; i < n && !bad; ++i) bad = fr[i].status;
    if (bad)  // an error exit (run_lane's early returns included) may leave device-to-host
              // copies into the caller's buffers queued: drain every lane before returning
        for (int l = 0; l < nl; ++l) hipStreamSynchronize(lanes_[l]->stream);
    for (int i = 0; i < n; ++i)  // the first failing frame's status
        if (fr[i].status) return fr[i].status;
    return st;
}

// Frames per launch: sets of frames of one geometry (kernels.hpp FrameSet), up to
// kMaxSet and about four 4K frames' pixels per launch (4K: 192 -> 208 GPix/s with sets
// of 4, 203 with 2; 1080p batch: 111 -> 143).  A set's entropy launch needs every member
// placed by its own last code workgroup (the pipeline's placement mode, no restart
// intervals).
constexpr uint64_t kSetPixels = 4ull * 3840ull * 2160ull;
int Encoder::batch_set_size(const FrameDesc* fr, int n) const {
    if (n < 2 || set_ == 1) return 1;
    const FrameDesc& f0 = fr[0];
    if (!f0.width || !f0.height || f0.width > 65535 || f0.height > 65535) return 1;
    for (int i = 1; i < n; ++i)
        if (fr[i].width != f0.width || fr[i].height != f0.height || (fr[i].maxval == 255) != (f0.maxval == 255))
            return 1;
    const bool placed_in_code = (ext_place_ > 0 || (ext_place_ < 0 && lanes_.size() > 1)) && place_in_code_;
    if (!placed_in_code || restart_mcus_ || layout(geometry(f0.width, f0.height, mode_)).grid() > kPlaceInCodeMaxWgs)
        return 1;
    if (set_) return set_;
    const uint64_t k = kSetPixels / ((uint64_t)f0.width * f0.height);
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(kMaxSet, k));
}

int Encoder::run_lane(Lane& ln, FrameDesc* frames, int total, std::atomic<int>* next, int set, const uint8_t qy[64],
                      const uint8_t qc[64], uint32_t flags) {
    const int S = (int)ln.slots.size() / set;  // slot sets (add_slots: >= lookahead + drain lag + 1)
    // Pipeline step t handles frame set t of this lane: frames mine[t*set ..], each in
    // slot (t mod S) * set + member.  Only the lane's last set may be short.
    std::vector<int> mine;  // batch indices of the frames this lane took, in its order
    mine.reserve(total);
    auto members = [&](int t) { return std::min(set, (int)mine.size() - t * set); };
    auto frame = [&](int t, int m) -> FrameDesc& { return frames[mine[t * set + m]]; };
    auto slot = [&](int t, int m) -> Slot& { return *ln.slots[(t % S) * set + m]; };
    int first_err = kOk;
    auto note = [&](int t, int m, int st) {
        if (st && !frame(t, m).status) frame(t, m).status = st;
        if (st && !first_err) first_err = st;
    };
    // Software pipeline on the lane's stream (steps are lane-local).  Step i queues
    //   K1(i) [carrying set j = i-L's tables + headers to the device], K2(i),
    //   then set j's entropy kernels [the code kernel carrying set i's histograms to
    //   the host for a table worker],
    // so the host builds a set's tables while the GPU works through the L sets queued
    // ahead of its entropy launch; set i-L-D is drained D steps after that launch (about
    // D sets of queued GPU work while the host waits).  Member m of one set pairs with
    // member m of the other for the carried duties.  The pipeline's edges fall back to a
    // standalone export kernel and a table copy.
    const int L = lookahead_, D = drain_lag_;
    // This lane's frames whose tables are not built yet: the lane's waits build any whose
    // histograms are in (the ~25 us of a 1080p frame's tables fill a wait instead of a
    // worker's polling and hand-off), and a frame's entropy launch builds its own if they
    // are still missing.
    std::vector<Slot*> pend;
    pend.reserve((size_t)(L + D + 2) * set);
    const std::function<bool()> build_ready = [&]() -> bool {
        for (size_t q = 0; q < pend.size(); ++q) {
            Slot& s = *pend[q];
            if (s.tables_done.load(std::memory_order_relaxed)) {
                pend.erase(pend.begin() + (long)q);
                return true;
            }
            if (__atomic_load_n(&s.h_hist->seq, __ATOMIC_ACQUIRE) != s.seq) continue;
            pend.erase(pend.begin() + (long)q);
            s.tables_status = build_tables(s, false);
            s.tables_done.store(1, std::memory_order_release);
            return true;
        }
        return false;
    };
    auto submit_tables = [&](Slot& s) {
        s.tables_done.store(0, std::memory_order_relaxed);
        s.inline_tables = true;
        pend.push_back(&s);
    };
    // diagnostic host trace: (step, point, us since the call, and at point 1 the
    // awaited table job's submit / start / done times)
    std::vector<std::array<double, 6>> trace;
    const auto t_call = std::chrono::steady_clock::now();
    auto us = [&](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::micro>(t - t_call).count();
    };
    // diagnostic (JPGE_CPU_PROF): this thread's CPU time per loop segment, summed per encoder
    int64_t cpu_last = 0;
    int64_t cpu_acc[6] = {0, 0, 0, 0, 0, 0};
    auto thread_ns = [] {
        timespec t;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
        return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
    };
    if (cpu_prof_) cpu_last = thread_ns();
    auto mark = [&](int i, int point, const Slot* job = nullptr) {
        if (cpu_prof_) {
            const int64_t t = thread_ns();
            cpu_acc[point] += t - cpu_last;
            cpu_last = t;
        }
        if (host_trace_file_)
            trace.push_back({(double)i, (double)point, us(std::chrono::steady_clock::now()),
                             job ? us(job->t_submit) : 0.0, job ? us(job->t_start) : 0.0,
                             job ? us(job->t_done) : 0.0});
    };
    int n = 0;         // sets taken so far
    bool open = true;  // the batch may still have frames
    for (int i = 0;; ++i) {
        if (open && i == n) {  // room for a new set: take the batch's next frames
            const int g = next->fetch_add(set, std::memory_order_relaxed);
            if (g < total) {
                for (int m = 0; m < set && g + m < total; ++m) mine.push_back(g + m);
                ++n;
            } else {
                open = false;
            }
        }
        if (!open && i >= n + L + D) break;
        const int j = i - L, k = i - L - D;
        mark(i, 0);
        Slot* sj[kMaxSet] = {};  // set j's members, tables built, ready for their entropy kernels
        if (j >= 0 && j < n) {
            for (int m = 0; m < members(j); ++m) {
                if (frame(j, m).status) continue;
                Slot& s = slot(j, m);
                if (!s.tables_done.load(std::memory_order_acquire)) {
                    s.tables_status = build_tables(s, /*parallel=*/false);
                    s.tables_done.store(1, std::memory_order_release);
                }
                if (s.tables_status) note(j, m, s.tables_status);
                else sj[m] = &s;
            }
            mark(i, 1, sj[0]);
        } else {
            mark(i, 1);
        }
        Slot* si[kMaxSet] = {};  // set i's members whose histograms set j's code kernels export
        bool imported[kMaxSet] = {};
        if (i < n) {
            const int mi = members(i);
            if (set == 1) {
                Slot& s = slot(i, 0);
                note(i, 0, phase1(s, frame(i, 0), qy, qc, flags, sj[0], /*export_hist=*/sj[0] == nullptr));
                if (!frame(i, 0).status) {
                    imported[0] = sj[0] != nullptr;
                    si[0] = sj[0] ? &s : nullptr;
                    submit_tables(s);
                }
            } else {
                Slot* ss[kMaxSet];
                FdctArgs fa[kMaxSet];
                StatsArgs sa[kMaxSet];
                int ms[kMaxSet], ok = 0;
                for (int m = 0; m < mi; ++m) {
                    Slot& s = slot(i, m);
                    const int st = prep1(s, frame(i, m), qy, qc, flags, sj[m], fa[ok], sa[ok]);
                    note(i, m, st);
                    if (st) continue;
                    ss[ok] = &s;
                    ms[ok++] = m;
                }
                if (ok) {
                    const int st = phase1_set(ss, ok, fa, sa);
                    for (int q = 0; q < ok; ++q) {
                        const int m = ms[q];
                        note(i, m, st);
                        if (st) continue;
                        Slot& s = slot(i, m);
                        imported[m] = sj[m] != nullptr;
                        if (sj[m]) {
                            si[m] = &s;
                        } else {  // (no code kernel of set j to carry the export)
                            const hipError_t e = launch_hist_export(s.hist, s.d_hist_host->cnt, s.d_hist_host->key,
                                                                    &s.d_hist_host->seq, s.seq, s.stream);
                            note(i, m, e == hipSuccess ? kOk : kErrHip);
                            if (e == hipSuccess) s.export_queued.store(1, std::memory_order_release);
                        }
                        if (!frame(i, m).status) submit_tables(s);
                    }
                }
            }
        }
        mark(i, 2);
        if (j >= 0 && j < n) {
            // set j's entropy kernels: one launch per kernel for the set, or frame by frame
            // (a single frame; a member its code kernel does not place)
            EntropyArgs ea[kMaxSet];
            int ms[kMaxSet], ne = 0;
            bool as_set = set > 1;
            for (int m = 0; m < members(j); ++m) {
                if (!sj[m]) continue;
                const int st = imported[m] ? kOk : import_tables_copy(*sj[m]);
                note(j, m, st);
                if (st) {
                    sj[m] = nullptr;
                    continue;
                }
                ea[ne] = entropy_args(*sj[m]);
                if (Slot* ex = si[m] && !frame(i, m).status ? si[m] : nullptr) {  // (carried export)
                    ea[ne].exp_hist = ex->hist;
                    ea[ne].exp_cnt = ex->d_hist_host->cnt;
                    ea[ne].exp_key = ex->d_hist_host->key;
                    ea[ne].exp_seq = &ex->d_hist_host->seq;
                    ea[ne].exp_seqv = ex->seq;
                }
                as_set = as_set && ea[ne].done;
                ms[ne++] = m;
            }
            if (ne) {
                if (as_set) {
                    Slot* tm = nullptr;  // (a sampled set's member: its events time the launches)
                    for (int q = 0; q < ne; ++q) {
                        sj[ms[q]]->h_result[2] = 0;
                        if (sj[ms[q]]->timed && !tm) tm = sj[ms[q]];
                    }
                    const KTimer tc{tm ? tm->ev[4] : nullptr, tm ? tm->ev[5] : nullptr};
                    const KTimer tp{tm ? tm->ev[6] : nullptr, tm ? tm->ev[7] : nullptr};
                    const hipError_t e = launch_entropy_set(ea, ne, sj[ms[0]]->stream, tm ? &tc : nullptr,
                                                            tm ? &tp : nullptr);
                    for (int q = 0; q < ne; ++q) note(j, ms[q], e == hipSuccess ? kOk : kErrHip);
                    if (e != hipSuccess) ne = 0;
                } else {
                    for (int q = 0; q < ne; ++q) {
                        const int m = ms[q];
                        const int st = launch_entropy_phase(*sj[m], si[m] && !frame(i, m).status ? si[m] : nullptr);
                        note(j, m, st);
                        if (st) sj[m] = nullptr;
                    }
                }
                for (int q = 0; q < ne; ++q) {  // exported by member m of set j's code kernel
                    const int m = ms[q];
                    if (sj[m] && si[m] && !frame(i, m).status) {
                        si[m]->export_queued.store(1, std::memory_order_release);
                        si[m] = nullptr;
                    }
                }
            }
        }
        mark(i, 3);
        for (int m = 0; m < kMaxSet; ++m) {  // (no carrier: export set i's histograms on their own)
            Slot* s = si[m];
            if (!s) continue;
            const hipError_t e = launch_hist_export(s->hist, s->d_hist_host->cnt, s->d_hist_host->key,
                                                    &s->d_hist_host->seq, s->seq, s->stream);
            note(i, m, e == hipSuccess ? kOk : kErrHip);
            if (e == hipSuccess) s->export_queued.store(1, std::memory_order_release);
        }
        if (k >= 0 && k < n) {
            for (int m = 0; m < members(k); ++m) {
                Slot& s = slot(k, m);
                if (!frame(k, m).status)
                    note(k, m, finish(s, frame(k, m), flags, /*guess_wait=*/m == 0, pend.empty() ? nullptr : &build_ready));
                else hipStreamSynchronize(s.stream);
            }
        }
        mark(i, 4);
    }
    // every output byte is in place: the stream's tail, awaited by spinning (a
    // blocking stream synchronisation adds tens of us of wake-up latency)
    JPGE_HIP(hipEventRecord(ln.done, ln.stream));
    JPGE_HIP(wait_event(ln.done));
    mark(n + L + D, 5);  // (n: this lane's set count)
    if (cpu_prof_) {
        for (int q = 0; q < 6; ++q) cpu_ns_[q].fetch_add(cpu_acc[q], std::memory_order_relaxed);
        cpu_frames_.fetch_add((int64_t)mine.size(), std::memory_order_relaxed);
    }
    if (host_trace_file_) {
        std::lock_guard<std::mutex> g(trace_mu_);
        if (FILE* f = std::fopen(host_trace_file_, "a")) {
            for (const auto& t : trace)
                std::fprintf(f, "%d %d %.2f %d %.2f %.2f %.2f\n", (int)t[0], (int)t[1], t[2], ln.id, t[3], t[4], t[5]);
            std::fprintf(f, "-1 -1 0 %d %.2f %.2f 0\n", ln.id, abs_us(t_call),
                         abs_us(std::chrono::steady_clock::now()));
            std::fclose(f);
        }
    }
    return first_err;
}

int Encoder::fdct_quant(const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                        int16_t* y, int16_t* cb, int16_t* cr) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *lanes_[0]->slots[0];
    int st = phase1(s, f, qy, qc, flags | kFlagDeviceOutput | kFlagCoefficients, nullptr, true);
    if (st) { hipStreamSynchronize(s.stream); return st; }
    JPGE_HIP(hipStreamSynchronize(s.stream));
    const Geometry& g = s.g;
    std::vector<int16_t> coef((size_t)g.nblocks() * 64);
    JPGE_HIP(hipMemcpyAsync(coef.data(), s.d_coef, coef.size() * 2, hipMemcpyDeviceToHost, s.stream));  // (not the null stream)
    JPGE_HIP(hipStreamSynchronize(s.stream));
    const uint32_t ybw = g.yh * g.mw, cbw = g.mw;
    for (uint32_t m = 0; m < g.nmcu(); ++m) {
        const uint32_t mr = m / g.mw, mc = m % g.mw;
        for (int k = 0; k < (int)g.bpm; ++k) {
            const int16_t* src = &coef[((size_t)m * g.bpm + k) * 64];
            const int comp = block_comp(k, g.bpm);
            int16_t* dst;
            if (comp == 0) dst = y + ((size_t)(mr * g.yv() + k / g.yh) * ybw + mc * g.yh + k % g.yh) * 64;
            else dst = (comp == 1 ? cb : cr) + ((size_t)mr * cbw + mc) * 64;
            for (int i = 0; i < 64; ++i) dst[i] = src[i];
        }
    }
    return kOk;
}

int Encoder::symbol_stats(const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                          uint32_t counts[1024], uint64_t first[1024]) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *lanes_[0]->slots[0];
    int st = phase1(s, f, qy, qc, flags | kFlagDeviceOutput, nullptr, true);
    if (st) { hipStreamSynchronize(s.stream); return st; }
    JPGE_HIP(hipStreamSynchronize(s.stream));
    for (int t = 0; t < 4; ++t)
        for (int i = 0; i < 256; ++i) {
            const uint32_t c = s.h_hist->cnt[t * 256 + i];
            counts[t * 256 + i] = c;
            first[t * 256 + i] = c ? ~s.h_hist->key[t * 256 + i] : ~0ull;
        }
    return kOk;
}


// ---- stripes ----
// A stripe is the MCU rows [mcu_row0, mcu_row0 + mcu_rows) of a width x height
// image; its own geometry has the stripe's real pixel rows (the last stripe's bottom
// padding replicates the image's last row, Image.cpp:511-519).  Every phase runs on
// lane 0's first slot and returns when its results are on the host.
int Encoder::stripe_transform(const StripeDesc& d, const uint8_t qy[64], const uint8_t qc[64], int32_t last_dc[3]) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    if (!d.rgb || !last_dc || d.width == 0 || d.height == 0 || d.width > 65535 || d.height > 65535) return kErrArg;
    if (mode_ != 420) return kErrArg;  // stripes are S420_m (the reference's subsampling)
    if (d.maxval < 1 || d.maxval > 255) return kErrRange;
    const uint32_t mh_img = (d.height + 15) / 16;
    if (d.mcu_rows == 0 || d.mcu_row0 >= mh_img || d.mcu_rows > mh_img - d.mcu_row0) return kErrArg;
    const size_t row = (size_t)d.width * 3, stride = d.stride ? d.stride : row;
    if (stride < row) return kErrArg;
    for (int i = 0; i < 64; ++i)
        if (!qy[i] || !qc[i]) return kErrArg;
    const uint32_t hs = std::min(16 * d.mcu_rows, d.height - 16 * d.mcu_row0);
    const Geometry g = geometry(d.width, hs);
    // restart intervals: the stripe must start one (its bytes are then its own)
    if (restart_mcus_ && ((uint64_t)d.mcu_row0 * g.mw) % restart_mcus_ != 0) return kErrArg;
    Slot& s = *lanes_[0]->slots[0];
    if (const int st = ensure(s, g, 0, 0)) return st;
    std::memcpy(s.qy, qy, 64);
    std::memcpy(s.qc, qc, 64);
    s.g = g;
    s.in_dev = d.rgb;
    s.in_stride = stride;
    s.img_w = d.width;
    s.img_h = d.height;
    s.seed = DcSeed();
    s.rst = Restart();
    s.rst.mcus = restart_mcus_;
    s.rst.mcu0 = d.mcu_row0 * g.mw;
    s.key_y0 = 2ull * d.mcu_row0 * (2ull * g.mw);  // Y blocks above the stripe (raster)
    s.key_c0 = (uint64_t)d.mcu_row0 * g.mw;         // Cb blocks above it
    s.key_ncb = (uint64_t)mh_img * g.mw;            // Cb blocks of the image
    JPGE_HIP(launch_fdct(fdct_args(s, d.maxval, nullptr), s.stream));
    int16_t lastmcu[6 * 64];  // the stripe's last MCU: its Y11, Cb and Cr DCs seed the next stripe
    JPGE_HIP(hipMemcpyAsync(lastmcu, s.d_coef + ((size_t)g.nmcu() - 1) * 384, sizeof lastmcu, hipMemcpyDeviceToHost,
                            s.stream));
    JPGE_HIP(hipStreamSynchronize(s.stream));
    last_dc[0] = lastmcu[3 * 64];
    last_dc[1] = lastmcu[4 * 64];
    last_dc[2] = lastmcu[5 * 64];
    return kOk;
}

int Encoder::stripe_stats(const int32_t seed[3], uint32_t counts[1024], uint64_t first[1024]) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *lanes_[0]->slots[0];
    if (!s.in_dev || !seed || !counts || !first) return kErrArg;
    for (int c = 0; c < 3; ++c) s.seed.v[c] = seed[c];
    const StatsArgs st = stats_args(s);
    JPGE_HIP(launch_stats(st, s.stream));
    s.seq = ++seq_counter_;
    s.hist = st.hist;
    JPGE_HIP(launch_hist_export(st.hist, s.d_hist_host->cnt, s.d_hist_host->key, &s.d_hist_host->seq, s.seq, s.stream));
    JPGE_HIP(hipStreamSynchronize(s.stream));
    for (int i = 0; i < 1024; ++i) {
        const uint32_t c = s.h_hist->cnt[i];
        counts[i] = c;
        first[i] = c ? ~s.h_hist->key[i] : ~0ull;
    }
    return kOk;
}

int Encoder::stripe_code(const uint32_t counts[1024], const uint64_t first[1024], StripeSummary* sum,
                         size_t* hdr_len) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *lanes_[0]->slots[0];
    if (!s.in_dev || !counts || !first || !sum) return kErrArg;
    s.out_dev = nullptr;
    s.out_cap = 0;
    if (const int st = build_tables_from(s, counts, first, true)) return st;
    if (const int st = import_tables_copy(s)) return st;
    EntropyArgs e = entropy_args(s);
    e.done = nullptr;  // (stripes: placed by the stripe phases)
    JPGE_HIP(launch_entropy_code_summary(e, s.stream));
    JPGE_HIP(hipMemcpyAsync(sum, e.summary, sizeof(StripeSummary), hipMemcpyDeviceToHost, s.stream));
    JPGE_HIP(hipStreamSynchronize(s.stream));
    if (hdr_len) *hdr_len = s.hdr_len;
    return kOk;
}

namespace {
uint32_t split_bits(uint32_t ptail, uint32_t head, uint32_t b) {  // 0 < b < 8 (entropy.hip)
    return (((ptail & ((1u << b) - 1)) << (8 - b)) | ((head & 0xFF) >> b)) & 0xFF;
}
uint32_t fill_bits(uint32_t eb, uint32_t tail) {  // Bitstream::fill, BitstreamGeneric.hpp:243-248
    return (((tail & ((1u << eb) - 1)) << (8 - eb)) | (0xFFu >> eb)) & 0xFF;
}
}  // namespace

int Encoder::stripe_place(const StripeSummary* all, int n, int index, size_t hdr_len, uint64_t* p_ext,
                          uint64_t* q_ext, uint32_t* head_split, size_t* seg_off, size_t* total_len) {
    if (!all || n <= 0 || index < 0 || index >= n) return kErrArg;
    if (all[0].restart) {  // restart stripes: self-contained byte runs, one after another
        uint64_t base = 0;
        for (int r = 0; r < n; ++r) {
            if (!all[r].restart) return kErrArg;
            if (r == index) {
                if (p_ext) *p_ext = 0;
                if (q_ext) *q_ext = base;  // (the byte base of the stripe after the header)
                if (head_split) *head_split = 0;
                if (seg_off) *seg_off = r == 0 ? 0 : hdr_len + (size_t)base;
            }
            base += all[r].bits;
        }
        if (total_len) *total_len = hdr_len + (size_t)base + 2;
        return kOk;
    }
    uint64_t p = 0, q = 0;
    for (int r = 0; r < n; ++r) {
        if (all[r].bits < 8) return kErrArg;  // (a stripe codes >= 2 bits per block, 6 blocks per MCU)
        const uint32_t b = (uint32_t)(p & 7);
        const uint32_t split = (b && r > 0) ? split_bits(all[r - 1].tail, all[r].head, b) : 0u;
        if (r == index) {
            if (p_ext) *p_ext = p;
            if (q_ext) *q_ext = q;
            if (head_split) *head_split = split;
            if (seg_off) *seg_off = r == 0 ? 0 : hdr_len + (size_t)(p >> 3) + (size_t)q;
        }
        // 0xFF bytes stripe r owns: its inside bytes at its alignment, the byte it
        // shares with its predecessor, the image's 1-filled final byte
        q += all[r].ff[b] + ((b && r > 0 && split == 0xFF) ? 1u : 0u);
        p += all[r].bits;
        if (r == n - 1 && (p & 7) && fill_bits((uint32_t)(p & 7), all[r].tail) == 0xFF) q += 1;
    }
    if (total_len) *total_len = hdr_len + (size_t)((p + 7) >> 3) + (size_t)q + 2;
    return kOk;
}

int Encoder::stripe_pack(const StripeSummary* all, int n, int index, uint8_t* out_dev, size_t cap, size_t* seg_off,
                         size_t* seg_len, size_t* total_len) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    Slot& s = *lanes_[0]->slots[0];
    if (!s.in_dev || !out_dev || !s.hdr_len) return kErrArg;
    uint64_t p_ext = 0, q_ext = 0;
    uint32_t head = 0;
    size_t off = 0, total = 0;
    if (const int st = stripe_place(all, n, index, s.hdr_len, &p_ext, &q_ext, &head, &off, &total)) return st;
    if (total > cap) return kErrNoSpace;
    s.out_dev = out_dev;
    s.out_cap = cap;
    s.seq = ++seq_counter_;
    s.h_result[2] = 0;
    EntropyArgs e = entropy_args(s);
    e.done = nullptr;  // (stripes: placed by the stripe phases)
    if (s.rst.mcus) {
        e.out_base = q_ext;  // (placed in phase 3, relative to the stripe's start)
    } else {
        e.p_ext = p_ext;
        e.q_ext = q_ext;
        e.head_split = head;
    }
    e.flags = (index == 0 ? kStripeFirst : 0u) | (index == n - 1 ? kStripeLast : 0u) | kExtPlace;
    JPGE_HIP(launch_entropy_place_pack(e, s.stream));
    if (const int w = wait_seq(&s.h_result[3], s.seq, s.stream)) return w;
    JPGE_HIP(hipStreamSynchronize(s.stream));
    if (s.h_result[1] & 4) return kErrNoSpace;
    const size_t end = (size_t)s.h_result[0];
    if (seg_off) *seg_off = off;
    if (seg_len) *seg_len = end - off;
    if (total_len) *total_len = total;
    return (index == n - 1 && end != total) ? kErrInternal : kOk;
}

// ---- plane stages (the facade's Image stage methods; planes.hip) ----

void* Encoder::scratch(int i, size_t bytes) {
    if ((int)scratch_.size() <= i) scratch_.resize(i + 1, {nullptr, 0});
    auto& b = scratch_[i];
    if (b.second < bytes) {
        hipFree(b.first);
        b = {nullptr, 0};
        if (hipMalloc(&b.first, bytes) != hipSuccess) return nullptr;
        b.second = bytes;
    }
    return b.first;
}

#define JPGE_SCRATCH(var, idx, bytes)                     \
    void* var = scratch((idx), (bytes));                  \
    if (!var) return kErrHip

int Encoder::stage_color(const double* const in[3], double* const out[3], size_t n, int to_ycc, uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    for (int c = 0; c < 3; ++c)
        if (!in[c] || !out[c]) return kErrArg;
    if (n == 0) return kOk;
    hipStream_t st = lanes_[0]->stream;
    const size_t bytes = n * 8;
    PlaneColorArgs a;
    const double* din[3];
    double* dout[3];
    for (int c = 0; c < 3; ++c) {
        if (flags & kFlagDeviceInput) {
            din[c] = in[c];
        } else {
            JPGE_SCRATCH(b, c, bytes);
            JPGE_HIP(hipMemcpyAsync(b, in[c], bytes, hipMemcpyHostToDevice, st));
            din[c] = static_cast<const double*>(b);
        }
        if (flags & kFlagDeviceOutput) {
            dout[c] = out[c];
        } else {
            JPGE_SCRATCH(b, 3 + c, bytes);
            dout[c] = static_cast<double*>(b);
        }
    }
    a.in0 = din[0]; a.in1 = din[1]; a.in2 = din[2];
    a.out0 = dout[0]; a.out1 = dout[1]; a.out2 = dout[2];
    a.n = n;
    a.to_ycc = to_ycc;
    JPGE_HIP(launch_plane_color(a, st));
    if (!(flags & kFlagDeviceOutput))
        for (int c = 0; c < 3; ++c) JPGE_HIP(hipMemcpyAsync(out[c], dout[c], bytes, hipMemcpyDeviceToHost, st));
    JPGE_HIP(hipStreamSynchronize(st));
    return kOk;
}

// applySubsampling's masks (Image.cpp:256-309) as PlaneSubsampleArgs; S444 leaves
// the plane as it is.
static bool subsample_mask(int mode, PlaneSubsampleArgs& a, uint32_t& vdiv) {
    a.mask[0] = 1; a.mask[1] = 0; a.mask[2] = 0; a.mask[3] = 0;
    a.m = 2; a.row_step = 2; a.avg_div = 0; vdiv = 2;
    switch (mode) {
        case 444: a.m = 1; a.row_step = 1; vdiv = 1; return true;
        case 422: a.row_step = 1; vdiv = 1; return true;               // {1, 0}
        case 411: a.m = 4; a.row_step = 1; vdiv = 1; return true;      // {1, 0, 0, 0}
        case 4200: return true;                                         // {1, 0}, scanline jump
        case 420: a.mask[1] = 1; a.avg_div = 4; return true;           // {1, 1}, averaging / 4
        case 4201: a.avg_div = 2; return true;                         // {1, 0}, averaging / 2
        default: return false;
    }
}

int Encoder::subsample_shape(int mode, uint32_t rows, uint32_t cols, uint32_t* out_rows, uint32_t* out_cols) {
    PlaneSubsampleArgs a;
    uint32_t vdiv;
    if (!subsample_mask(mode, a, vdiv)) return kErrArg;
    // the reference's loop reads whole mask runs and, in pairs, the next scanline
    if (rows == 0 || cols == 0 || cols % a.m || (a.row_step == 2 && rows % 2)) return kErrArg;
    if (out_rows) *out_rows = rows / vdiv;
    if (out_cols) *out_cols = cols / a.m;
    return kOk;
}

int Encoder::stage_subsample(const double* in, uint32_t rows, uint32_t cols, int mode, double* out, uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    PlaneSubsampleArgs a;
    uint32_t vdiv, orows, ocols;
    if (!in || !out || !subsample_mask(mode, a, vdiv)) return kErrArg;
    if (const int e = subsample_shape(mode, rows, cols, &orows, &ocols)) return e;
    hipStream_t st = lanes_[0]->stream;
    const size_t ib = (size_t)rows * cols * 8, ob = (size_t)orows * ocols * 8;
    const double* din = in;
    if (!(flags & kFlagDeviceInput)) {
        JPGE_SCRATCH(b, 0, ib);
        JPGE_HIP(hipMemcpyAsync(b, in, ib, hipMemcpyHostToDevice, st));
        din = static_cast<const double*>(b);
    }
    double* dout = out;
    if (!(flags & kFlagDeviceOutput)) {
        JPGE_SCRATCH(b, 1, ob);
        dout = static_cast<double*>(b);
    }
    if (mode == 444) {
        JPGE_HIP(hipMemcpyAsync(dout, din, ib, hipMemcpyDeviceToDevice, st));
    } else {
        a.in = din;
        a.out = dout;
        a.cols = cols;
        a.out_rows = orows;
        a.out_cols = ocols;
        JPGE_HIP(launch_plane_subsample(a, st));
    }
    if (!(flags & kFlagDeviceOutput)) JPGE_HIP(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, st));
    JPGE_HIP(hipStreamSynchronize(st));
    return kOk;
}

// Dct.hpp:220-235: A(k, n) = C0(k) sqrt(2/8) cos((2n+1) (k pi / 16)), glibc cos on the host
static void dct_matrix_a(double A[64]) {
    const double pi = 0x1.921fb54442d18p+1, root_two = 0x1.6a09e667f3bcdp+0;
    const double scale = std::sqrt(2. / 8);
    for (int k = 0; k < 8; ++k)
        for (int n = 0; n < 8; ++n) {
            const double cos_term = (2. * n + 1.) * ((k * pi) / (2. * 8));
            A[k * 8 + n] = (k == 0 ? 1. / root_two : 1.) * scale * std::cos(cos_term);
        }
}

int Encoder::stage_dct(const double* in, uint32_t rows, uint32_t cols, int dct_mode, double* out, uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    if (!in || !out || rows % 8 || cols % 8 || dct_mode < kDctSimple || dct_mode > kDctArai) return kErrArg;
    if (rows == 0 || cols == 0) return kOk;
    hipStream_t st = lanes_[0]->stream;
    const size_t bytes = (size_t)rows * cols * 8;
    const double* din = in;
    if (!(flags & kFlagDeviceInput)) {
        JPGE_SCRATCH(b, 0, bytes);
        JPGE_HIP(hipMemcpyAsync(b, in, bytes, hipMemcpyHostToDevice, st));
        din = static_cast<const double*>(b);
    }
    double* dout = out;
    if (!(flags & kFlagDeviceOutput)) {
        JPGE_SCRATCH(b, 1, bytes);
        dout = static_cast<double*>(b);
    }
    PlaneBlockArgs a{};
    a.in0 = din;
    a.cols = cols;
    a.nblocks = (uint64_t)(rows / 8) * (cols / 8);
    a.sink = kSinkDouble;
    dct_matrix_a(a.A);
    a.out_d = dout;
    JPGE_HIP(launch_plane_block(a, dct_mode, st));
    if (!(flags & kFlagDeviceOutput)) JPGE_HIP(hipMemcpyAsync(out, dout, bytes, hipMemcpyDeviceToHost, st));
    JPGE_HIP(hipStreamSynchronize(st));
    return kOk;
}

int Encoder::stage_quantize(const double* in, uint32_t rows, uint32_t cols, const uint8_t table[64], int32_t* out,
                            uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    if (!in || !out || !table || rows % 8 || cols % 8) return kErrArg;
    if (rows == 0 || cols == 0) return kOk;
    hipStream_t st = lanes_[0]->stream;
    const size_t n = (size_t)rows * cols;
    const double* din = in;
    if (!(flags & kFlagDeviceInput)) {
        JPGE_SCRATCH(b, 0, n * 8);
        JPGE_HIP(hipMemcpyAsync(b, in, n * 8, hipMemcpyHostToDevice, st));
        din = static_cast<const double*>(b);
    }
    int32_t* dout = out;
    if (!(flags & kFlagDeviceOutput)) {
        JPGE_SCRATCH(b, 1, n * 4);
        dout = static_cast<int32_t*>(b);
    }
    PlaneQuantArgs a;
    a.in = din;
    a.out = dout;
    a.rows = rows;
    a.cols = cols;
    for (int i = 0; i < 64; ++i) a.q[i] = table[i];
    JPGE_HIP(launch_plane_quant(a, st));
    if (!(flags & kFlagDeviceOutput)) JPGE_HIP(hipMemcpyAsync(out, dout, n * 4, hipMemcpyDeviceToHost, st));
    JPGE_HIP(hipStreamSynchronize(st));
    return kOk;
}

int Encoder::encode_planes(const double* const planes[3], uint32_t rows, uint32_t cols, int ycc, uint32_t real_w,
                           uint32_t real_h, const uint8_t qy[64], const uint8_t qc[64], uint8_t* out, size_t cap,
                           size_t* len, uint32_t flags) {
    std::lock_guard<std::recursive_mutex> call_lock(call_mu_);
    JPGE_HIP(hipSetDevice(device_));
    for (int c = 0; c < 3; ++c)
        if (!planes[c]) return kErrArg;
    if (!out || !len || !qy || !qc || rows == 0 || cols == 0 || rows % 16 || cols % 16 || rows > 65536 ||
        cols > 65536 || real_w == 0 || real_h == 0 || real_w > 65535 || real_h > 65535)
        return kErrArg;
    for (int i = 0; i < 64; ++i)
        if (!qy[i] || !qc[i]) return kErrArg;
    Slot& s = *lanes_[0]->slots[0];
    hipStream_t st = s.stream;
    // the frame as writeJPEG sees it: S420_m MCUs over the planes (rows, cols already
    // whole MCUs: loadPPM pads to 16, Image.cpp:480-531); SOF0 carries the real size
    Geometry g = geometry(cols, rows, 420);
    const size_t out_cap = (flags & kFlagDeviceOutput) ? 0 : max_jpeg_bytes(cols, rows);
    if (const int e = ensure(s, g, 0, out_cap)) return e;
    const size_t n = (size_t)rows * cols, bytes = n * 8;
    const double* p[3];
    for (int c = 0; c < 3; ++c) {
        if (flags & kFlagDeviceInput) {
            p[c] = planes[c];
        } else {
            JPGE_SCRATCH(b, c, bytes);
            JPGE_HIP(hipMemcpyAsync(b, planes[c], bytes, hipMemcpyHostToDevice, st));
            p[c] = static_cast<const double*>(b);
        }
    }
    if (!ycc) {  // *this = convertToColorSpace(YCbCr), Image.cpp:839
        double* q[3];
        for (int c = 0; c < 3; ++c) {
            JPGE_SCRATCH(b, 3 + c, bytes);
            q[c] = static_cast<double*>(b);
        }
        PlaneColorArgs a;
        a.in0 = p[0]; a.in1 = p[1]; a.in2 = p[2];
        a.out0 = q[0]; a.out1 = q[1]; a.out2 = q[2];
        a.n = n;
        a.to_ycc = 1;
        JPGE_HIP(launch_plane_color(a, st));
        for (int c = 0; c < 3; ++c) p[c] = q[c];
    }
    // applySubsampling(S420_m), Image.cpp:842 (Cr, then Cb: independent planes)
    const double* sub[2];
    for (int c = 0; c < 2; ++c) {
        PlaneSubsampleArgs a;
        uint32_t vdiv;
        subsample_mask(420, a, vdiv);
        JPGE_SCRATCH(b, 6 + c, bytes / 4);
        a.in = p[1 + c];
        a.out = static_cast<double*>(b);
        a.cols = cols;
        a.out_rows = rows / 2;
        a.out_cols = cols / 2;
        JPGE_HIP(launch_plane_subsample(a, st));
        sub[c] = a.out;
    }
    std::memcpy(s.qy, qy, 64);
    std::memcpy(s.qc, qc, 64);
    s.g = g;
    s.in_dev = reinterpret_cast<const uint8_t*>(p[0]);  // (marks the slot in use; K1 is not run)
    s.in_stride = 0;
    if (flags & kFlagDeviceOutput) {
        s.out_dev = out;
        s.out_cap = cap;
    } else {
        s.out_dev = s.d_out;
        s.out_cap = s.cap_out;
    }
    s.seed = DcSeed();
    s.rst = Restart();
    s.rst.mcus = restart_mcus_;
    s.key_y0 = s.key_c0 = s.key_ncb = 0;
    s.img_w = real_w;
    s.img_h = real_h;
    s.timed = false;
    s.count_symbols = false;
    s.tables_done.store(0, std::memory_order_relaxed);
    s.export_queued.store(0, std::memory_order_relaxed);
    // applyDCT(Arai) + applyQuantization (Image.cpp:844-871) into the MCU layout; the
    // control block is zeroed here (K1 does it on the RGB8 path)
    const CtlLayout L(layout(g).grid());
    JPGE_HIP(hipMemsetAsync(s.d_ctl, 0, L.total, st));
    PlaneBlockArgs b{};
    b.in0 = p[0];
    b.in1 = sub[0];
    b.in2 = sub[1];
    b.cols = cols;
    b.nblocks = (uint64_t)g.nblocks();
    b.mcu = 1;
    b.sink = kSinkMcu16;
    for (int i = 0; i < 64; ++i) {
        b.q[i] = qy[i];
        b.q[64 + i] = qc[i];
    }
    b.out_h = s.d_coef;
    JPGE_HIP(launch_plane_block(b, kDctArai, st));
    const StatsArgs st2 = stats_args(s);
    JPGE_HIP(launch_stats(st2, st));
    s.seq = ++seq_counter_;
    s.hist = st2.hist;
    JPGE_HIP(launch_hist_export(st2.hist, s.d_hist_host->cnt, s.d_hist_host->key, &s.d_hist_host->seq, s.seq, st));
    s.export_queued.store(1, std::memory_order_release);
    FrameDesc f;
    f.out = out;
    f.cap = cap;
    int e = build_tables(s, false);
    if (!e) e = import_tables_copy(s);
    if (!e) e = launch_entropy_phase(s, nullptr);
    if (!e) e = finish(s, f, flags);
    hipStreamSynchronize(st);
    *len = f.len;
    return e;
}

}  // namespace jpge
