// Host orchestration of the GPU encode path: one Encoder = one HIP device and a few
// independent pipelines ("lanes"), each a stream with a small ring of frame slots
// (each slot its own workspace), plus the per-image Huffman-table build between the
// statistics kernels and the entropy kernels.  This is the engine behind the C ABI
// (include/jpge.h).
#pragma once
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <functional>
#include <mutex>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "host_io.hpp"
#include "huffman.hpp"
#include "kernels.hpp"
#include "planes.hpp"

namespace jpge {

constexpr uint32_t kFlagDeviceInput = 1u;
constexpr uint32_t kFlagDeviceOutput = 2u;
constexpr uint32_t kFlagCoefficients = 1u << 30;  // (internal) the frame's coefficients are read back

struct FrameDesc {
    const uint8_t* rgb = nullptr;
    uint32_t width = 0, height = 0;
    size_t stride = 0;  // bytes per input row (0 = width*3)
    int maxval = 255;
    uint8_t* out = nullptr;
    size_t cap = 0;
    size_t len = 0;
    int status = 0;
};

struct KernelTimes {  // milliseconds of the last timed frame (each kernel's own events, KTimer)
    float fdct = 0, dc_stats = 0, entropy = 0, total = 0;
    double fdct_sum = 0, dc_stats_sum = 0, entropy_sum = 0;  // accumulated since reset
    uint64_t frames = 0;
    uint64_t symbols = 0;  // Huffman-coded symbols of the timed frames
    double code_sum = 0, pack_sum = 0;  // the entropy stage's code and pack kernels alone
    uint64_t launches = 0;  // timed launches of each kernel (a frame set's launch covers its frames)
};

class Encoder {
  public:
    // lanes <= 0: JPGE_LANES or the default (4)
    static int open(int device, std::unique_ptr<Encoder>& out, int lanes = 0);
    ~Encoder();

    int encode(FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags);
    int encode_batch(FrameDesc* frames, int n, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags);

    // Stage entry: quantised coefficients (before DC differencing), per component
    // in block raster order, 64 natural-order values per block (host buffers).
    int fdct_quant(const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                   int16_t* y, int16_t* cb, int16_t* cr);
    // Stage entry: the four symbol histograms and first-occurrence keys.
    int symbol_stats(const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags,
                     uint32_t counts[1024], uint64_t first[1024]);

    // ---- plane stages: the reference's Image stage methods on fp64 planes (planes.hip).
    // Host or device buffers (kFlagDeviceInput / kFlagDeviceOutput); each call returns
    // with its results in place.
    // convertToColorSpace (Image.cpp:112-179): to_ycc 1 = RGB -> YCbCr, 0 = back
    int stage_color(const double* const in[3], double* const out[3], size_t n, int to_ycc, uint32_t flags);
    // Image::subsample with applySubsampling's mask for `mode` (jpge.h JPGE_S*)
    static int subsample_shape(int mode, uint32_t rows, uint32_t cols, uint32_t* out_rows, uint32_t* out_cols);
    int stage_subsample(const double* in, uint32_t rows, uint32_t cols, int mode, double* out, uint32_t flags);
    // applyDCT(mode) (Image.cpp:540-595) over one plane of 8x8 blocks
    int stage_dct(const double* in, uint32_t rows, uint32_t cols, int dct_mode, double* out, uint32_t flags);
    // quantize (Coding.hpp:84-97) of every 8x8 block of a plane (applyQuantization)
    int stage_quantize(const double* in, uint32_t rows, uint32_t cols, const uint8_t table[64], int32_t* out,
                       uint32_t flags);
    // writeJPEG (Image.cpp:831-976) on three fp64 planes of rows x cols (multiples of
    // 16) in colour space `ycc` (0 RGB, 1 YCbCr with full-size chroma): convert,
    // S420_m, Arai, quantise on the GPU, then the statistics and entropy kernels.
    int encode_planes(const double* const planes[3], uint32_t rows, uint32_t cols, int ycc, uint32_t real_w,
                      uint32_t real_h, const uint8_t qy[64], const uint8_t qc[64], uint8_t* out, size_t cap,
                      size_t* len, uint32_t flags);

    // ---- row stripes of a larger image (one stripe per device) ----
    // Phases, with the exchanges between them done by the caller (RCCL or a test):
    //   transform -> all-gather last DCs -> stats(seed = previous stripe's last DCs)
    //   -> all-reduce counts (sum) / keys (min) -> code -> all-gather summaries -> pack.
    struct StripeDesc {
        const uint8_t* rgb = nullptr;  // device: first pixel row of the stripe (row 16*mcu_row0)
        size_t stride = 0;
        uint32_t width = 0, height = 0;   // whole image
        uint32_t mcu_row0 = 0, mcu_rows = 0;
        int maxval = 255;
    };
    int stripe_transform(const StripeDesc& d, const uint8_t qy[64], const uint8_t qc[64], int32_t last_dc[3]);
    int stripe_stats(const int32_t seed[3], uint32_t counts[1024], uint64_t first[1024]);
    int stripe_code(const uint32_t counts[1024], const uint64_t first[1024], StripeSummary* sum, size_t* hdr_len);
    int stripe_pack(const StripeSummary* all, int n, int index, uint8_t* out_dev, size_t cap, size_t* seg_off,
                    size_t* seg_len, size_t* total_len);
    // Host arithmetic: where stripe `index` starts (global bit p_ext, stuffing bytes
    // q_ext before it, the byte it shares with its predecessor), its first output
    // byte and the whole file's length.
    static int stripe_place(const StripeSummary* all, int n, int index, size_t hdr_len, uint64_t* p_ext,
                            uint64_t* q_ext, uint32_t* head_split, size_t* seg_off, size_t* total_len);

    // Kernel timing with HIP events: 0 off, N >= 1 brackets the kernels of every
    // N-th frame (events cost GPU time; sampling keeps the pipeline's shape).
    void set_timing(int every) { timing_every_ = every > 0 ? every : 0; }
    void reset_timing() { times_ = KernelTimes(); }
    const KernelTimes& times() const { return times_; }
    int device() const { return device_; }
    static size_t max_jpeg_bytes(uint32_t w, uint32_t h);
    // restart interval in MCUs for the following encodes (0 = none, the reference's
    // stream); not for the stripe phases
    int set_restart(uint32_t mcus);
    uint32_t restart() const { return restart_mcus_; }
    // chroma subsampling of the following encodes (jpge.h JPGE_S*): 420 (S420_m, the
    // reference's writeJPEG), 444, 422, 411, 4200 (S420), 4201 (S420_lm); stripes are 420 only
    int set_subsampling(int mode);
    int subsampling() const { return mode_; }

    int lanes() const { return (int)lanes_.size(); }

  private:
    struct Slot;
    struct Lane;
    class TableHelper;
    Encoder() = default;
    int ensure(Slot& s, const Geometry& g, size_t in_bytes, size_t out_cap);
    // phase 1 (GPU): upload, transform + statistics kernels, histogram download
    // (carries `imp`'s tables to the device; exports its own histograms if asked)
    int phase1(Slot& s, const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags, Slot* imp,
               bool export_hist);
    // phase 1's host half: validate, size the slot, record the frame's state, the kernels' arguments
    int prep1(Slot& s, const FrameDesc& f, const uint8_t qy[64], const uint8_t qc[64], uint32_t flags, Slot* imp,
              FdctArgs& a, StatsArgs& st);
    // phase 1 of a frame set (kernels.hpp FrameSet: one transform and one statistics
    // launch for n frames of one geometry, prepared by prep1)
    int phase1_set(Slot* const* s, int n, const FdctArgs* a, const StatsArgs* st);
    // frames per launch for a batch: kMaxSet when every frame has one small geometry
    // (JPGE_SET: 1..kMaxSet forces a size), else 1
    int batch_set_size(const FrameDesc* fr, int n) const;
    // a lane's slots: at least `count`
    int add_slots(Lane& ln, int count);
    // phase 2a (host, any thread): Huffman tables + headers from the histograms
    int build_tables(Slot& s, bool parallel, TableHelper* helper = nullptr);
    int build_tables_from(Slot& s, const uint32_t* cnt, const uint64_t* first, bool parallel,
                          bool inverted = false,  // inverted: first holds ~keys (the device export)
                          TableHelper* helper = nullptr);  // (builds three of the four tables)
    FdctArgs fdct_args(Slot& s, int maxval, Slot* imp);
    StatsArgs stats_args(Slot& s);
    EntropyArgs entropy_args(Slot& s);
    // phase 2b (GPU): table upload (when not carried) + entropy kernels
    int import_tables_copy(Slot& s);
    // lone: encode()'s single image; parts: 1 the code kernel, 2 the pack kernel, 3 both
    int launch_entropy_phase(Slot& s, Slot* exp, bool lone = false, int parts = 3);
    // idle: work the wait may do between its polls (returns whether it did any)
    int finish(Slot& s, FrameDesc& f, uint32_t flags, bool guess_wait = true, const std::function<bool()>* idle = nullptr);
    // one lane's software pipeline over the frames it takes from fr[0..total) through `next`
    // (frames go in sets of `set` when set > 1: a pipeline step is a set, one launch per kernel)
    int run_lane(Lane& ln, FrameDesc* fr, int total, std::atomic<int>* next, int set, const uint8_t qy[64],
                 const uint8_t qc[64], uint32_t flags);

    int device_ = 0;
    int timing_every_ = 0;
    std::atomic<uint64_t> frame_counter_{0};
    std::atomic<uint64_t> seq_counter_{0};
    std::unique_ptr<TableHelper> helper_;  // single images on a 1-lane encoder: a second table thread
    bool table_helper_ = true;             // JPGE_TABLE_HELPER=0: none
    int gate_ = 1;  // encode()'s gate: 1 our wait-and-copy kernel, 2 the runtime's stream wait (JPGE_GATE), 0 none
    uint32_t gate_count_ = 0;  // gated calls (their gate values: 1, 2, ...)
    uint64_t gate_ticks_ = 100000000ull;  // the gate kernel's time-out (1 s; JPGE_TEST_GATE_TIMEOUT_US, tests)
    int gate_delay_us_ = 0;               // JPGE_TEST_GATE_DELAY_US (tests): the host opens the gate this late
    std::atomic<uint64_t> gate_timeouts_{0};  // calls re-coded after a gate time-out
  public:
    uint64_t gate_timeouts() const { return gate_timeouts_.load(std::memory_order_relaxed); }
  private:
    uint32_t entropy_wgs_ = 0;  // JPGE_ENTROPY_WGS: entropy workgroup count (tests; clamped)
    uint32_t stats_wgs_ = 0;    // JPGE_STATS_WGS: statistics workgroup count (diagnostics; clamped)
    uint32_t restart_mcus_ = 0; // restart interval (jpge_set_restart_interval)
    int mode_ = 420;            // subsampling mode (jpge_set_subsampling)
    // entropy workgroups: the override, else 512 for a single lane's lone frames (their
    // latency: -5 us at 4K) and seg_layout's default (384, or 2 tiles per workgroup under
    // 768 tiles) beside other lanes (+3% throughput) and for a single lane's frame sets
    // (JPGE_SET: four 1080p frames per launch 49 -> 36 us for the code + pack kernels
    // alone, 4K equal)
    uint32_t entropy_wgs() const {
        return entropy_wgs_ ? entropy_wgs_ : (lanes_.size() == 1 && set_ <= 1 ? 512u : 0u);
    }
    // statistics workgroups: 2 per CU alone (4K: 29.1 us vs 30.8 at 3 per CU, 37-40 at
    // 1.5 or 1), 1 per CU beside other lanes (6 tiles per workgroup at 4K: its fixed
    // costs, the prologue, first load and flush, amortised; 256 vs 512: +1.6% in the
    // pipeline, 1.25, 1.5 and 0.75 per CU slower)
    // (statistics workgroups of 8 waves: 3 per CU alone, 1.5 per CU beside other lanes)
    uint32_t stats_wgs() const { return stats_wgs_ ? stats_wgs_ : (lanes_.size() == 1 ? 768u : 384u); }
    SegLayout layout(const Geometry& g) const { return seg_layout(g, restart_mcus_, entropy_wgs()); }
    // the entropy partition a slot's current frame runs on
    SegLayout slot_layout(const Slot& s) const;
    uint32_t fdct_wgs_ = 0;     // JPGE_FDCT_WGS: pipeline transform grid (0: fdct_grid's cap)
    int lookahead_ = 2;         // JPGE_LOOKAHEAD: frames transformed ahead of an entropy launch
    int drain_lag_ = 1;         // JPGE_DRAIN_LAG: iterations between an entropy launch and its drain
    int set_ = 0;               // JPGE_SET: frames per launch (0: batch_set_size decides)
    int nap_us_ = 40;           // JPGE_NAP_US: a napping thread's sleep between polls (10: equal throughput, more wake-ups)
    // JPGE_FIRST_SLEEP (percent): a lane's first sleep in a result wait, of its usual length
    // less twice its spread (WaitGuess).  At 80%: 4K host CPU 1.45 -> 1.22 at equal
    // throughput; frames above kFirstSleepMaxPixels (16384^2: -3.7%) poll without it.
    double first_sleep_ = 0.8;
    // JPGE_EXT_PLACE: 1 = entropy placement by the scan kernel at every size, 0 = by each
    // pack workgroup up to kInlineScanMaxWgs; default (-1): the scan kernel beside other
    // lanes (one small launch instead of every pack workgroup scanning all records:
    // +0.8% in the pipeline), inline alone (one launch less per frame)
    int ext_place_ = -1;
    bool place_in_code_ = true;  // JPGE_PLACE_IN_CODE: the last code workgroup places (pipeline)
    bool nap_ = false;          // lane threads sleep ~10 us between polls instead of spinning (default: >1 lane; JPGE_NAP)
    const char* host_trace_file_ = nullptr;  // JPGE_HOST_TRACE: append per-iteration host timestamps
    bool cpu_prof_ = false;                  // JPGE_CPU_PROF: lane threads' CPU per loop segment (printed at close)
    std::atomic<int64_t> cpu_ns_[6] = {};
    std::atomic<int64_t> cpu_frames_{0};
    std::atomic<int64_t> cpu_read_ns_{0}, cpu_build_ns_{0}, cpu_builds_{0}, cpu_part_ns_[3] = {};
    int hist_nap_us_ = 0;    // a single lane's histogram wait: nap between polls (0: spin, for latency)
    bool lat_prof_ = false;  // JPGE_LAT_PROF: single-frame encode() phases, wall time (printed at close)
    int64_t lat_ns_[8] = {}, lat_calls_ = 0;  // (6, 7: phase1's argument preparation, K1 launch)
    std::chrono::steady_clock::time_point lat_hist_seen_{};
    const char* stamps_file_ = nullptr;  // JPGE_STAMPS_FILE: dump diagnostic phase stamps (diag builds)
    uint64_t* d_dbg_ = nullptr;
    size_t dbg_words_ = 0;
    void dump_stamps(const Slot& s);
    KernelTimes times_;
    std::mutex times_mu_;  // finish() of several lanes
    // Serialises the context's public calls: single-frame calls share lane 0's first
    // slot, and a batch uses every lane (jpge.h: a context is safe to share between
    // threads; calls on it run one at a time).
    std::recursive_mutex call_mu_;
    // device scratch of the plane stages, grown on demand (index -> buffer)
    std::vector<std::pair<void*, size_t>> scratch_;
    void* scratch(int i, size_t bytes);
  public:
    std::recursive_mutex& call_mutex() { return call_mu_; }
  private:
    std::mutex trace_mu_;
    std::vector<std::unique_ptr<Lane>> lanes_;  // JPGE_LANES (default 4: the device's hardware queues); lane 0 serves single-frame calls
};

}  // namespace jpge
