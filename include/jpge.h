/*
 * jpge — MI355X-native JPEG baseline encoder, C ABI (the drop-in boundary).
 *
 * The reference (Nuos/jpgEnc) has no FFI: its encode path is the C++ API of the
 * static library jpgEncLib (src/CMakeLists.txt:6-11) consumed by src/main.cpp.
 * Each entry point below replaces one piece of that API; the C++ facade in
 * jpgenc_amd/csrc/jpge_image.hpp re-exposes them under the reference's names.
 *
 * Conventions: every function returns a jpge_status (0 = ok); no exceptions or
 * C++ types cross this boundary; all buffers are owned by the caller; a context
 * (one HIP device + its streams and workspace) may be shared between threads: its
 * calls run one at a time (each call holds the context).  Output bytes are
 * bit-identical to the reference encoder.
 */
#ifndef JPGE_H_
#define JPGE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    JPGE_OK = 0,
    JPGE_E_ARG = 1,       /* invalid argument */
    JPGE_E_NOSPACE = 2,   /* output buffer too small; *len receives the size needed */
    JPGE_E_HIP = 3,       /* HIP runtime failure */
    JPGE_E_NODEV = 4,     /* no GPU / bad device index */
    JPGE_E_FORMAT = 5,    /* not a P3/P6 PPM (reference: std::runtime_error, Image.cpp:449-450) */
    JPGE_E_IO = 6,        /* cannot open/read/write a file (Image.cpp:427-428) */
    JPGE_E_TRUNC = 7,     /* PPM sample data shorter than width*height*3 */
    JPGE_E_RANGE = 8,     /* maxval outside 1..255 (Image.cpp:462) or sample > 255 */
    JPGE_E_TIMEOUT = 9,   /* device-side scan protocol did not complete */
    JPGE_E_RCCL = 10,     /* RCCL failure (multi-GPU paths) */
    JPGE_E_INTERNAL = 11
} jpge_status;

#define JPGE_DEVICE_INPUT 1u  /* rgb points to device memory */
#define JPGE_DEVICE_OUTPUT 2u /* out points to device memory */

typedef struct jpge_ctx jpge_ctx;

/* One frame of a batch (jpge_encode_batch). */
typedef struct {
    const uint8_t* rgb; /* interleaved RGB8 (host, or device with JPGE_DEVICE_INPUT) */
    uint32_t width, height;
    size_t stride;      /* bytes per row, 0 = width*3 */
    int maxval;         /* PPM maxval, 1..255; samples are scaled by 255./maxval (Image.cpp:465) */
    uint8_t* out;       /* .jpg destination */
    size_t cap;         /* capacity of out */
    size_t len;         /* [out] bytes written */
    int status;         /* [out] jpge_status of this frame */
} jpge_frame;

/* Per-kernel device times of the last timed frame (ms; see jpge_set_timing for
 * sampling).  Each kernel of a timed frame is launched with its own pair of HIP
 * events bound to its dispatch (hipExtLaunchKernel), so a kernel's figure is its
 * execution time as rocprofv3 reports it, without launch gaps. */
typedef struct {
    float fdct;     /* K1: colour + 4:2:0 + FDCT + quantise */
    float dc_stats; /* K2: DC chain + RLE/category symbol histograms + first-occurrence keys */
    float entropy;  /* K3: code kernel start .. pack kernel end (Huffman emission, MCU interleave, fill, stuffing) */
    float total;    /* K1 start .. K3 end of that frame (includes the queued work of other frames) */
    double fdct_sum, dc_stats_sum, entropy_sum; /* accumulated since jpge_reset_timing (ms) */
    uint64_t frames;                            /* frames accumulated */
    uint64_t symbols; /* Huffman-coded symbols of those frames (= K2's 4-byte symbol records) */
    double code_sum, pack_sum; /* K3's entropy_code_kernel and entropy_pack_kernel alone (ms, accumulated) */
    uint64_t launches;         /* timed launches of each kernel (batches of small frames launch frame sets:
                                  one launch per kernel for up to 4 frames; the sums are per launch) */
    uint64_t gate_timeouts;    /* single-frame calls whose table gate timed out on the device and were
                                  re-coded ungated (jpge_encode_rgb8; not reset by jpge_reset_timing) */
} jpge_timing;

const char* jpge_strerror(int status);
int jpge_version(void);
int jpge_device_count(int* n);

/* Context lifetime (replaces nothing in the reference: its encoder is stateless). */
int jpge_open(int device, jpge_ctx** ctx);
/* jpge_open with an explicit lane count (0 = JPGE_LANES or the default 4; at most 8;
 * 1 = a single pipeline, e.g. to time kernels without other frames beside them). */
int jpge_open_ex(int device, int lanes, jpge_ctx** ctx);
/* Contexts and groups still open when the process exits are released by the library
 * itself (an std::atexit handler registered at the first jpge_open): their threads,
 * streams and memory are freed, but the handle stays valid, so a jpge_close or
 * jpge_group_close the caller makes later (e.g. from its own exit handler) is a no-op,
 * and any other call on it returns JPGE_E_ARG. */
int jpge_close(jpge_ctx* ctx);
/* Kernel timing with HIP events on the encoder's stream: every = 0 off, N >= 1
 * times the kernels of every N-th frame (1 = all; events cost GPU time). */
int jpge_set_timing(jpge_ctx* ctx, int every);
int jpge_get_timing(jpge_ctx* ctx, jpge_timing* t);
int jpge_reset_timing(jpge_ctx* ctx);
/* Pipelines ("lanes") the context runs a batch on: each lane is a HIP stream with
 * its own frame slots and host thread; a batch's frames are dealt round-robin to
 * them (env JPGE_LANES at jpge_open, default 4). */
int jpge_get_lanes(jpge_ctx* ctx, int* lanes);

/* Restart intervals for the context's following encodes (jpge_encode_rgb8, _batch,
 * _file): every `mcus` MCUs the DC predictions restart and the entropy stream is
 * 1-filled and followed by an RSTn marker, announced by a DRI segment before SOS
 * (ITU T.81 B.2.4.4, F.1.2.3).  0 (the default) = none: the reference's stream,
 * bit-identical to it.  Replaces nothing in the reference (writeJPEG never emits
 * DRI/RSTn, Image.cpp:931-972); its decoded pixels equal the mcus = 0 output's.
 * 1..65535, else JPGE_E_ARG; the stripe phases (jpge_stripe_*) need mcus = 0. */
int jpge_set_restart_interval(jpge_ctx* ctx, uint32_t mcus);

/* Subsampling modes: the SubsamplingMode enum of Image.hpp:44-52, as passed to
 * Image::applySubsampling (Image.cpp:237-319). */
#define JPGE_S420_M 420  /* mean of 2x2 (writeJPEG's mode; the default)        MCU 16x16, Y 2x2 */
#define JPGE_S444 444    /* no subsampling                                    MCU  8x8,  Y 1x1 */
#define JPGE_S422 422    /* every second pixel of a row                       MCU 16x8,  Y 2x1 */
#define JPGE_S411 411    /* every fourth pixel of a row                       MCU 32x8,  Y 4x1 */
#define JPGE_S420 4200   /* every second pixel of every second row            MCU 16x16, Y 2x2 */
#define JPGE_S420_LM 4201 /* mean of the two rows' left pixels                MCU 16x16, Y 2x2 */

/* Chroma subsampling for the context's following encodes.  JPGE_S420_M (the
 * default) is applySubsampling(S420_m) as writeJPEG hard-codes it (Image.cpp:842),
 * bit-identical to the reference.  The other modes follow Image::subsample
 * (Image.cpp:198-235) for the masks of applySubsampling; writeJPEG cannot emit
 * them, so the oracle's composition of the pinned stages defines their bytes: the
 * frame edge-replicated to whole MCUs, MCU = the Y blocks row by row + Cb + Cr,
 * SOF0 declaring Y as H x V.  Unknown modes: JPGE_E_ARG.  jpge_fdct_quant then
 * returns the mode's planes; the stripe phases (jpge_stripe_*) need JPGE_S420_M. */
int jpge_set_subsampling(jpge_ctx* ctx, int mode);

/* Worst-case .jpg size for a frame, in any subsampling mode (header + 2x
 * worst-case entropy + RST markers + EOI). */
size_t jpge_max_jpeg_bytes(uint32_t width, uint32_t height);

/* Quantisation tables for quality 1..100: the reference's Annex-K tables
 * (Image.cpp:850-869) scaled by the IJG rule; quality 50 returns them unchanged,
 * which is the only table pair the reference itself uses. Natural order. */
int jpge_quality_tables(int quality, uint8_t qy[64], uint8_t qc[64]);

/* Full encode — replaces Image::writeJPEG (Image.hpp:92, Image.cpp:831-976) for an
 * image as produced by loadPPM: SOI APP0 DQT DQT SOF0 DHTx4 SOS <entropy> EOI.
 * Returns once every output byte is in place: in host memory (host output), or in
 * device memory (JPGE_DEVICE_OUTPUT), readable from any stream.  On a 1-lane context
 * with device output the call returns as soon as the bytes are written, while the
 * context's stream may still be retiring the last kernel (later work on the context
 * is ordered after it). */
int jpge_encode_rgb8(jpge_ctx* ctx, const uint8_t* rgb, uint32_t width, uint32_t height, size_t stride,
                     int maxval, const uint8_t qy[64], const uint8_t qc[64], uint8_t* out, size_t cap,
                     size_t* len, uint32_t flags);

/* Many independent frames, pipelined on the context's stream (configs 3/4): the
 * transform of later frames is queued ahead of each frame's entropy kernel while
 * host threads build that frame's tables. */
int jpge_encode_batch(jpge_ctx* ctx, jpge_frame* frames, int n, const uint8_t qy[64], const uint8_t qc[64],
                      uint32_t flags);

/* Stage entry — convertToColorSpace + applySubsampling(S420_m) + applyDCT(Arai) +
 * applyQuantization (Image.cpp:839-871) on the GPU: quantised coefficients before
 * DC differencing, per component, blocks in raster order, 64 natural-order values
 * per block (host buffers of (W'/8)(H'/8)*64 and 2 x (W'/16)(H'/16)*64 int16; at
 * 4:4:4 three buffers of ceil(W/8)*ceil(H/8)*64 int16). */
int jpge_fdct_quant(jpge_ctx* ctx, const uint8_t* rgb, uint32_t width, uint32_t height, size_t stride,
                    int maxval, const uint8_t qy[64], const uint8_t qc[64], int16_t* coef_y, int16_t* coef_cb,
                    int16_t* coef_cr, uint32_t flags);

/* Stage entry — the symbol "texts" of writeJPEG (Image.cpp:888-906) as histograms:
 * counts[t*256+s] and first[t*256+s] = position key of the first occurrence
 * (~0 if absent); t = 0 Y-DC, 1 Y-AC, 2 C-DC, 3 C-AC. */
int jpge_symbol_stats(jpge_ctx* ctx, const uint8_t* rgb, uint32_t width, uint32_t height, size_t stride,
                      int maxval, const uint8_t qy[64], const uint8_t qc[64], uint32_t counts[1024],
                      uint64_t first[1024], uint32_t flags);

/* Host table build — replaces generateHuffmanCode (Huffman.hpp:53, Huffman.cpp:3-66)
 * for byte symbols given counts and first-occurrence keys.  bits[0..15] = number
 * of codes of length 1..16, huffval = DHT symbol order, code/len per symbol. */
int jpge_huffman_table(const uint32_t counts[256], const uint64_t first[256], uint8_t bits[16],
                       uint8_t huffval[256], int* nsym, uint32_t code[256], uint8_t len[256]);

/* Same for an arbitrary int symbol text (the reference signature, for tests and
 * tools): writes n distinct symbols as (symbol, length, code) in DHT order. */
int jpge_huffman_text(const int* text, size_t n, int* syms, int* lens, uint32_t* codes, int* nsym);

/* Concatenate n device byte segments (segs[k], lens[k] bytes) back to back into the
 * device buffer dst, in one kernel launch per 96 segments on `stream` (a hipStream_t;
 * NULL = the null stream), without waiting for it; *total (optional) = the sum of the
 * lengths.  device: the GPU the buffers live on (the caller's current device is kept).
 * Config 4's gather packs a rank's .jpg bytes with it (jpgenc_amd/gather.py) before
 * the one transfer to rank 0.  Replaces nothing in the reference (its encoder is one
 * process); an addition of this library.  Any alignments; segments below 2 GB. */
int jpge_concat_segments(int device, void* stream, const uint8_t* const* segs, const size_t* lens, int n,
                         uint8_t* dst, size_t* total);

/* ---- Decode-side verification utilities (host) ---- */

/* huffmanDecode (Huffman.hpp:62, Huffman.cpp:91-146): the symbol text coded in the
 * first nbits bits (MSB-first bytes) by the table of nsym (symbol, code, length)
 * entries, codes right-aligned as jpge_huffman_text returns them.  `bits` must hold
 * at least ceil(nbits / 8) bytes.  text = NULL: count only.  JPGE_E_FORMAT where no
 * code matches (the reference asserts). */
int jpge_huffman_decode(const uint8_t* bits, uint64_t nbits, const uint32_t* table_syms, const uint32_t* table_codes,
                        const uint8_t* table_lens, int nsym, int* text, size_t cap, size_t* n);

/* inverseDctMat (Dct.hpp:278-306) of one 8x8 block, row-major doubles:
 * (A^T X) A with A(k, n) = C(k) sqrt(2/8) cos((2n+1) k pi / 16). */
void jpge_idct8x8(const double in[64], double out[64]);

/* A decoded jpge stream's frame (jpge_decode_coeffs). */
typedef struct {
    uint32_t width, height;  /* SOF0: the real size */
    uint32_t yh, yv;         /* Y sampling factors (chroma is 1x1) */
    uint32_t restart;        /* DRI interval in MCUs, 0 = none */
    size_t y_blocks, c_blocks; /* coefficient blocks per plane */
    uint8_t qy[64], qc[64];  /* DQT tables, natural order */
} jpge_decoded;

/* Baseline entropy decode of a .jpg written by this library (SOF0, three
 * components, chroma 1x1, Y 1x1 / 2x1 / 4x1 / 2x2, optional DRI/RSTn): the
 * quantised coefficients with the DC differences undone (Image.cpp:638-678
 * inverted), natural order, blocks in raster order per component — the planes
 * jpge_fdct_quant returns.  y = NULL: fill *info only (sizes).  Verification
 * utility, not on the encode path. */
int jpge_decode_coeffs(const uint8_t* jpg, size_t len, jpge_decoded* info, int16_t* y, int16_t* cb, int16_t* cr,
                       size_t cap_y_blocks, size_t cap_c_blocks);

/* PPM front end — replaces loadPPM (Image.hpp:28, Image.cpp:421-538) up to the
 * padding, which the GPU path performs by clamped addressing.  parse: rgb gets
 * width*height*3 unscaled samples (cap bytes available). */
int jpge_parse_ppm(const uint8_t* buf, size_t n, uint8_t* rgb, size_t cap, uint32_t* width, uint32_t* height,
                   int* maxval);
int jpge_ppm_info(const uint8_t* buf, size_t n, uint32_t* width, uint32_t* height, int* maxval);

/* Convenience: PPM file -> .jpg file at the given quality (the CLI path, main.cpp:8-32). */
int jpge_encode_file(jpge_ctx* ctx, const char* ppm_path, const char* jpg_path, int quality);

/* Many PPM files -> .jpg files (the CLI path over a list), pipelined: worker threads
 * read and parse each file into pinned memory while the previous group of frames is
 * encoded (H2D queued ahead of the kernels on each lane) and the one before is copied
 * back and written.  lens/statuses (optional, n entries) get each file's .jpg length
 * and jpge_status; returns the first failing status.  group = frames per stage
 * (0 = 8, at most 64).  Bytes equal jpge_encode_file's for every file. */
int jpge_encode_files(jpge_ctx* ctx, const char* const* ppm_paths, const char* const* jpg_paths, int n, int quality,
                      size_t* lens, int* statuses, int group);

/* Deterministic synthetic frame (kind 0 photo-like, 1 random bytes, 2 flat). */
int jpge_synth_rgb8(uint64_t seed, uint32_t width, uint32_t height, int kind, uint8_t* out, size_t stride);

/* The Arai constants compiled into the kernels (Dct.hpp:21-43), for verification:
 * a[0..4] = a1..a5, s[0..7] = s0..s7. */
void jpge_arai_constants(double a[5], double s[8]);

/* ---- Coding.hpp primitives (host; per block, as the reference's free functions) ----
 * The GPU path computes all of these inside its kernels; these entries serve the
 * facade's Coding.hpp functions (jpge_image.hpp) and their known-answer tests. */

/* zigzag(int) (Coding.hpp:57-81): the natural (row-major) index of zig-zag position
 * i (0..63); -1 for i outside 0..63 (the reference asserts). */
int jpge_zigzag_index(int i);
/* zigzag(matrix) (Coding.hpp:30-54): out[zig-zag position of (r, c)] = in[r * 8 + c]. */
int jpge_zigzag_block(const int32_t in[64], int32_t out[64]);
/* quantize (Coding.hpp:84-97): out[i] = (int)round(block[i] / table[i]), row-major. */
int jpge_quantize_block(const double block[64], const double table[64], int32_t out[64]);
/* RLE_AC (Coding.hpp:112-183): (run, value) pairs; pair 0 is (0, DC); a value after
 * more than 15 zeros is preceded by (15, 0) pairs; a trailing zero run ends with the
 * EOB pair (0, 0).  zigzag_scan = 0: the vector version over data[0..n) as given
 * (n >= 2); 1: the matrix version over a natural-order 8x8 block (n = 64) scanned in
 * zig-zag order.  *npairs receives the count (JPGE_E_NOSPACE if cap is smaller). */
int jpge_rle_ac(const int32_t* data, size_t n, int zigzag_scan, uint8_t* runs, int32_t* values, size_t cap,
                size_t* npairs);
/* getCategoryAndCode (Coding.hpp:197-262): category = bit length of |value| (0 for
 * 0), bits = value if > 0 else (2^category - 1) - |value| (the low `category` bits,
 * written MSB-first).  JPGE_E_RANGE for |value| >= 2^15 (the reference asserts). */
int jpge_category_code(int32_t value, uint16_t* category, uint32_t* bits);
/* encode_category (Coding.hpp:265-283): per pair, symbol = (run << 4) | category and
 * its extra bits (code, code_lens[i] = category). */
int jpge_encode_category(const uint8_t* runs, const int32_t* values, size_t n, uint8_t* symbols, uint32_t* codes,
                         uint8_t* code_lens);
/* applyDCdifferenceCoding (Image.cpp:638-678), in place on quantised int planes:
 * the Y DCs in MCU order (2x2 blocks of 8x8 per 16x16 MCU), each chroma plane's DCs
 * in block raster order; every chain starts at 0.  Y is rows x cols (multiples of
 * 16), the chroma planes crows x ccols (multiples of 8). */
int jpge_dc_difference(int32_t* y, uint32_t rows, uint32_t cols, int32_t* cb, int32_t* cr, uint32_t crows,
                       uint32_t ccols);

/* ---- Plane stages: the reference's Image stage methods on fp64 planes (GPU) ----
 * Row-major planes of doubles (Image's matrix<PixelDataType>); host buffers, or
 * device buffers with JPGE_DEVICE_INPUT / JPGE_DEVICE_OUTPUT.  Each call returns with
 * its results in place.  Bit-identical to the reference's loops. */
#define JPGE_TO_RGB 0
#define JPGE_TO_YCBCR 1
/* convertToColorSpace (Image.cpp:112-179) of n pixels: JPGE_TO_YCBCR takes R,G,B
 * planes to Y,Cb,Cr; JPGE_TO_RGB the reverse. */
int jpge_color_convert(jpge_ctx* ctx, const double* in0, const double* in1, const double* in2, double* out0,
                       double* out1, double* out2, size_t n, int target, uint32_t flags);
/* Image::subsample with applySubsampling's mask for `mode` (JPGE_S*; Image.cpp:
 * 198-319) on one rows x cols plane; out gets out_rows x out_cols (S444: a copy).
 * out = NULL: only the output size. */
int jpge_subsample_plane(jpge_ctx* ctx, const double* in, uint32_t rows, uint32_t cols, int mode, double* out,
                         uint32_t* out_rows, uint32_t* out_cols, uint32_t flags);
#define JPGE_DCT_SIMPLE 0 /* dctDirect (Dct.hpp:238-262) */
#define JPGE_DCT_MATRIX 1 /* dctMat (Dct.hpp:264-276) */
#define JPGE_DCT_ARAI 2   /* dctArai (Dct.hpp:47-215), writeJPEG's */
/* applyDCT(mode) (Image.cpp:540-595) on one plane of 8x8 blocks (rows, cols
 * multiples of 8). */
int jpge_dct_plane(jpge_ctx* ctx, const double* in, uint32_t rows, uint32_t cols, int dct_mode, double* out,
                   uint32_t flags);
/* applyQuantization's per-block quantize (Image.cpp:597-636, Coding.hpp:84-97) on
 * one plane of 8x8 blocks with one natural-order table. */
int jpge_quantize_plane(jpge_ctx* ctx, const double* in, uint32_t rows, uint32_t cols, const uint8_t table[64],
                        int32_t* out, uint32_t flags);
/* writeJPEG (Image.cpp:831-976) on an Image's three planes (rows x cols, multiples of
 * 16): colorspace JPGE_TO_RGB = the planes are R,G,B (converted first), JPGE_TO_YCBCR
 * = they are Y,Cb,Cr with full-size chroma; then S420_m, Arai, quantisation, DC/RLE/
 * category, per-image tables and emission, all on the GPU.  SOF0 carries
 * real_width x real_height.  The context's restart interval applies. */
int jpge_encode_planes(jpge_ctx* ctx, const double* p0, const double* p1, const double* p2, uint32_t rows,
                       uint32_t cols, int colorspace, uint32_t real_width, uint32_t real_height, const uint8_t qy[64],
                       const uint8_t qc[64], uint8_t* out, size_t cap, size_t* len, uint32_t flags);

/* ---- Row stripes of one large image across devices ----
 * The image (width x height, 4:2:0) is cut into stripes of whole MCU rows (16 px);
 * each stripe is encoded by its own context (one per GPU) in four phases, with
 * three small exchanges between them that the caller performs (RCCL all-gather /
 * all-reduce, or plain copies in one process).  The result is byte-identical to
 * encoding the whole image at once: the reference never emits restart markers, so
 * its DC chain (Image.cpp:638-678), its histograms (Image.cpp:888-906) and its
 * single bit stream (Image.cpp:957-972) run across stripe boundaries.
 *   1 jpge_stripe_transform  -> last_dc; exchange: all-gather, stripe r's seed = r-1's last_dc
 *   2 jpge_stripe_stats      -> counts/first; exchange: all-reduce counts (sum), first (min)
 *   3 jpge_stripe_code       -> summary; exchange: all-gather summaries
 *   4 jpge_stripe_pack       -> the stripe's bytes at their place in a whole-file device
 *                               buffer; then gather every [seg_off, seg_off + seg_len) to one rank.
 * With a restart interval set (jpge_set_restart_interval on every context) whose
 * boundaries include every stripe start, the stripes are independent but for the
 * shared tables: no DC seed is needed (phase 1's exchange can be skipped), and the
 * summaries only carry byte lengths — the output equals the whole-image restart
 * encode.  Replaces nothing in the reference (single-process, single-image encoder). */
typedef struct {
    uint64_t bits;    /* length of the stripe's bit stream (restart intervals: its byte length) */
    uint32_t ff[8];   /* 0xFF bytes wholly inside it when it starts at bit a (mod 8) */
    uint32_t head;    /* its first 8 bits */
    uint32_t tail;    /* its last 8 bits */
    uint32_t restart; /* 1: restart-interval stripe (every stripe starts an interval: its bytes
                         are self-contained, so placement is a prefix sum of byte lengths) */
    uint32_t pad;
} jpge_stripe_summary;

/* K1 on MCU rows [mcu_row0, mcu_row0 + mcu_rows) of the image; rgb = device pointer
 * to the stripe's first pixel row (image row 16*mcu_row0), stride bytes per row. */
int jpge_stripe_transform(jpge_ctx* ctx, const uint8_t* rgb, size_t stride, uint32_t width, uint32_t height,
                          uint32_t mcu_row0, uint32_t mcu_rows, int maxval, const uint8_t qy[64],
                          const uint8_t qc[64], int32_t last_dc[3]);
/* K2 with the DC chain seeded by the previous stripe's last Y/Cb/Cr DC (0,0,0 for
 * the first stripe); counts/first as jpge_symbol_stats, keys in the image's texts. */
int jpge_stripe_stats(jpge_ctx* ctx, const int32_t seed_dc[3], uint32_t counts[1024], uint64_t first[1024]);
/* Tables from the image's (summed) counts and (minimum) first keys, then the code
 * kernel; returns the stripe's summary and the header length. */
int jpge_stripe_code(jpge_ctx* ctx, const uint32_t counts[1024], const uint64_t first[1024],
                     jpge_stripe_summary* summary, size_t* header_len);
/* Host only: stripe `index`'s first output byte and the whole file's length. */
int jpge_stripe_place(const jpge_stripe_summary* all, int n, int index, size_t header_len, size_t* seg_off,
                      size_t* total_len);
/* Stuffed bytes of stripe `index` into out (device, whole-file capacity cap) at
 * [seg_off, seg_off + seg_len); stripe 0 includes the headers, the last one the
 * 1-fill and EOI. */
int jpge_stripe_pack(jpge_ctx* ctx, const jpge_stripe_summary* all, int n, int index, uint8_t* out, size_t cap,
                     size_t* seg_off, size_t* seg_len, size_t* total_len);

/* ---- Device groups: one process, several devices ----
 * A group owns one context per listed device and, when the devices are distinct, a
 * single-process RCCL clique (ncclCommInitAll) over xGMI.  A device listed more than
 * once (a rehearsal of N members on one GPU) makes the group exchange through host
 * memory and device copies instead; the bytes are the same.  Replaces nothing in
 * the reference (a single-threaded CPU encoder). */
typedef struct jpge_group jpge_group;
/* lanes: per member context, as jpge_open_ex.  JPGE_E_RCCL if librccl cannot be
 * loaded or the communicators cannot be created. */
int jpge_group_open(int ndev, const int* devices, int lanes, jpge_group** g);
int jpge_group_close(jpge_group* g);
/* members, and whether the exchanges ride RCCL (1) or host memory (0) */
int jpge_group_size(const jpge_group* g, int* n, int* uses_rccl);
/* member i's context (for per-member settings; owned by the group) */
int jpge_group_context(jpge_group* g, int member, jpge_ctx** ctx);
/* restart interval of every member (jpge_set_restart_interval) */
int jpge_group_set_restart_interval(jpge_group* g, uint32_t mcus);
/* Config 4: independent frames, frame i encoded by member i mod N (no collective);
 * with JPGE_DEVICE_INPUT / _OUTPUT frame i's buffers live on that member's device.
 * Per-frame len/status as jpge_encode_batch. */
int jpge_group_encode_batch(jpge_group* g, jpge_frame* frames, int n, const uint8_t qy[64], const uint8_t qc[64],
                            uint32_t flags);
/* Config 5: one 4:2:0 image (host RGB8) in row stripes of whole MCU rows over the
 * members — the jpge_stripe_* phases on every member at once, with an RCCL all-gather
 * of the DC seeds, all-reduce of the histograms (sum) and first-occurrence keys
 * (min), all-gather of the stripe summaries, and a grouped send/recv of the stuffed
 * segments to member 0 — then the whole .jpg to host memory.  Byte-identical to
 * jpge_encode_rgb8 on one device (with the group's restart interval, every stripe
 * starts an interval and the DC seed exchange drops out). */
int jpge_group_encode_striped(jpge_group* g, const uint8_t* rgb, uint32_t width, uint32_t height, size_t stride,
                              int maxval, const uint8_t qy[64], const uint8_t qc[64], uint8_t* out, size_t cap,
                              size_t* len);

#ifdef __cplusplus
}
#endif
#endif /* JPGE_H_ */
