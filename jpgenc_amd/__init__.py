"""jpge — MI355X-native JPEG baseline encoder (Python side of the C ABI).

This module is a thin ctypes binding over ``jpgenc_amd/lib/libjpge.so`` (the
HIP kernels + host C++; see ``include/jpge.h``).  It mirrors the reference's
entry points — ``load_ppm`` (Image.hpp:28 ``loadPPM``) and
``Encoder.encode`` / ``write_jpeg`` (Image.hpp:92 ``Image::writeJPEG``) — and
raises ``JpgeError`` (a ``RuntimeError``, the reference's ``std::runtime_error``
convention, Image.cpp:428/450) on failure.  There is no CPU fallback: if the
library or a GPU is missing, calls fail loudly.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import weakref
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JPGE_LIB") or os.path.join(_HERE, "lib", "libjpge.so")

JPGE_DEVICE_INPUT = 1
JPGE_DEVICE_OUTPUT = 2

#: subsampling modes (jpge.h JPGE_S*) -> (Y blocks across, Y blocks down) an MCU
SUBSAMPLING = {420: (2, 2), 4200: (2, 2), 4201: (2, 2), 444: (1, 1), 422: (2, 1), 411: (4, 1)}

STATUS = {
    0: "JPGE_OK", 1: "JPGE_E_ARG", 2: "JPGE_E_NOSPACE", 3: "JPGE_E_HIP", 4: "JPGE_E_NODEV",
    5: "JPGE_E_FORMAT", 6: "JPGE_E_IO", 7: "JPGE_E_TRUNC", 8: "JPGE_E_RANGE", 9: "JPGE_E_TIMEOUT",
    10: "JPGE_E_RCCL", 11: "JPGE_E_INTERNAL",
}

# every symbol include/jpge.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "jpge_strerror", "jpge_version", "jpge_device_count", "jpge_open", "jpge_open_ex", "jpge_close", "jpge_set_timing",
    "jpge_get_timing", "jpge_reset_timing", "jpge_get_lanes", "jpge_set_restart_interval", "jpge_set_subsampling",
    "jpge_max_jpeg_bytes", "jpge_quality_tables", "jpge_encode_rgb8", "jpge_encode_batch",
    "jpge_fdct_quant", "jpge_symbol_stats", "jpge_huffman_table", "jpge_huffman_text", "jpge_parse_ppm",
    "jpge_ppm_info", "jpge_encode_file", "jpge_encode_files", "jpge_synth_rgb8", "jpge_arai_constants",
    "jpge_stripe_transform", "jpge_stripe_stats", "jpge_stripe_code", "jpge_stripe_place", "jpge_stripe_pack",
    "jpge_huffman_decode", "jpge_idct8x8", "jpge_decode_coeffs",
    "jpge_zigzag_index", "jpge_zigzag_block", "jpge_quantize_block", "jpge_rle_ac", "jpge_category_code",
    "jpge_encode_category", "jpge_dc_difference", "jpge_color_convert", "jpge_subsample_plane", "jpge_dct_plane",
    "jpge_quantize_plane", "jpge_encode_planes",
    "jpge_group_open", "jpge_group_close", "jpge_group_size", "jpge_group_context", "jpge_group_set_restart_interval",
    "jpge_group_encode_batch", "jpge_group_encode_striped", "jpge_concat_segments",
)

JPGE_TO_RGB, JPGE_TO_YCBCR = 0, 1
DCT_SIMPLE, DCT_MATRIX, DCT_ARAI = 0, 1, 2


class JpgeError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = lib().jpge_strerror(status).decode() if _LIB is not None else STATUS.get(status, str(status))
        super().__init__(f"{what}: {STATUS.get(status, status)} ({msg})" if what else msg)


class Frame(ctypes.Structure):
    _fields_ = [
        ("rgb", ctypes.c_void_p), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
        ("stride", ctypes.c_size_t), ("maxval", ctypes.c_int), ("out", ctypes.c_void_p),
        ("cap", ctypes.c_size_t), ("len", ctypes.c_size_t), ("status", ctypes.c_int),
    ]


class StripeSummary(ctypes.Structure):
    """jpge_stripe_summary: a stripe's bit count, inside-0xFF count per start
    alignment, first and last 8 bits."""
    _fields_ = [("bits", ctypes.c_uint64), ("ff", ctypes.c_uint32 * 8), ("head", ctypes.c_uint32),
                ("tail", ctypes.c_uint32), ("restart", ctypes.c_uint32), ("pad", ctypes.c_uint32)]

    def as_tuple(self):
        return (int(self.bits), tuple(int(x) for x in self.ff), int(self.head), int(self.tail), int(self.restart))

    @classmethod
    def from_tuple(cls, t):
        s = cls()
        s.bits, s.head, s.tail = t[0], t[2], t[3]
        s.restart = t[4] if len(t) > 4 else 0
        for i in range(8):
            s.ff[i] = t[1][i]
        return s


class Decoded(ctypes.Structure):
    """jpge_decoded: the frame header of a decoded jpge stream."""
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("yh", ctypes.c_uint32),
                ("yv", ctypes.c_uint32), ("restart", ctypes.c_uint32), ("y_blocks", ctypes.c_size_t),
                ("c_blocks", ctypes.c_size_t), ("qy", ctypes.c_uint8 * 64), ("qc", ctypes.c_uint8 * 64)]


class Timing(ctypes.Structure):
    _fields_ = [("fdct", ctypes.c_float), ("dc_stats", ctypes.c_float), ("entropy", ctypes.c_float),
                ("total", ctypes.c_float), ("fdct_sum", ctypes.c_double), ("dc_stats_sum", ctypes.c_double),
                ("entropy_sum", ctypes.c_double), ("frames", ctypes.c_uint64),
                ("symbols", ctypes.c_uint64), ("code_sum", ctypes.c_double), ("pack_sum", ctypes.c_double),
                ("launches", ctypes.c_uint64), ("gate_timeouts", ctypes.c_uint64)]


_LIB = None


def lib() -> ctypes.CDLL:
    """Load libjpge.so (raises if it has not been built).  A process that also uses
    torch on the GPU must import torch first: torch ships its own HIP runtime, and
    loaded after libjpge's (ROCm's) it finds no GPU."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, sz, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int
        L.jpge_strerror.restype = ctypes.c_char_p
        L.jpge_strerror.argtypes = [i32]
        L.jpge_open.argtypes = [i32, ctypes.POINTER(vp)]
        L.jpge_open_ex.argtypes = [i32, i32, ctypes.POINTER(vp)]
        L.jpge_close.argtypes = [vp]
        L.jpge_set_timing.argtypes = [vp, i32]
        L.jpge_get_timing.argtypes = [vp, ctypes.POINTER(Timing)]
        L.jpge_reset_timing.argtypes = [vp]
        L.jpge_get_lanes.argtypes = [vp, ctypes.POINTER(i32)]
        L.jpge_set_restart_interval.argtypes = [vp, u32]
        L.jpge_set_subsampling.argtypes = [vp, i32]
        L.jpge_device_count.argtypes = [ctypes.POINTER(i32)]
        L.jpge_max_jpeg_bytes.restype = sz
        L.jpge_max_jpeg_bytes.argtypes = [u32, u32]
        L.jpge_quality_tables.argtypes = [i32, vp, vp]
        L.jpge_encode_rgb8.argtypes = [vp, vp, u32, u32, sz, i32, vp, vp, vp, sz, ctypes.POINTER(sz), u32]
        L.jpge_encode_batch.argtypes = [vp, ctypes.POINTER(Frame), i32, vp, vp, u32]
        L.jpge_fdct_quant.argtypes = [vp, vp, u32, u32, sz, i32, vp, vp, vp, vp, vp, u32]
        L.jpge_symbol_stats.argtypes = [vp, vp, u32, u32, sz, i32, vp, vp, vp, vp, u32]
        L.jpge_stripe_transform.argtypes = [vp, vp, sz, u32, u32, u32, u32, i32, vp, vp, vp]
        L.jpge_stripe_stats.argtypes = [vp, vp, vp, vp]
        L.jpge_stripe_code.argtypes = [vp, vp, vp, ctypes.POINTER(StripeSummary), ctypes.POINTER(sz)]
        L.jpge_stripe_place.argtypes = [ctypes.POINTER(StripeSummary), i32, i32, sz, ctypes.POINTER(sz),
                                        ctypes.POINTER(sz)]
        L.jpge_stripe_pack.argtypes = [vp, ctypes.POINTER(StripeSummary), i32, i32, vp, sz, ctypes.POINTER(sz),
                                       ctypes.POINTER(sz), ctypes.POINTER(sz)]
        L.jpge_huffman_table.argtypes = [vp, vp, vp, vp, ctypes.POINTER(i32), vp, vp]
        L.jpge_concat_segments.argtypes = [i32, vp, vp, vp, i32, vp, ctypes.POINTER(sz)]
        L.jpge_huffman_text.argtypes = [vp, sz, vp, vp, vp, ctypes.POINTER(i32)]
        L.jpge_parse_ppm.argtypes = [vp, sz, vp, sz, ctypes.POINTER(u32), ctypes.POINTER(u32),
                                     ctypes.POINTER(i32)]
        L.jpge_ppm_info.argtypes = [vp, sz, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(i32)]
        L.jpge_encode_file.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, i32]
        L.jpge_encode_files.argtypes = [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p), i32,
                                        i32, vp, vp, i32]
        L.jpge_synth_rgb8.argtypes = [ctypes.c_uint64, u32, u32, i32, vp, sz]
        L.jpge_arai_constants.argtypes = [vp, vp]
        L.jpge_arai_constants.restype = None
        L.jpge_huffman_decode.argtypes = [vp, ctypes.c_uint64, vp, vp, vp, i32, vp, sz, ctypes.POINTER(sz)]
        L.jpge_idct8x8.argtypes = [vp, vp]
        L.jpge_idct8x8.restype = None
        L.jpge_decode_coeffs.argtypes = [vp, sz, ctypes.POINTER(Decoded), vp, vp, vp, sz, sz]
        L.jpge_zigzag_index.argtypes = [i32]
        L.jpge_zigzag_block.argtypes = [vp, vp]
        L.jpge_quantize_block.argtypes = [vp, vp, vp]
        L.jpge_rle_ac.argtypes = [vp, sz, i32, vp, vp, sz, ctypes.POINTER(sz)]
        L.jpge_category_code.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(u32)]
        L.jpge_encode_category.argtypes = [vp, vp, sz, vp, vp, vp]
        L.jpge_dc_difference.argtypes = [vp, u32, u32, vp, vp, u32, u32]
        L.jpge_color_convert.argtypes = [vp, vp, vp, vp, vp, vp, vp, sz, i32, u32]
        L.jpge_subsample_plane.argtypes = [vp, vp, u32, u32, i32, vp, ctypes.POINTER(u32), ctypes.POINTER(u32), u32]
        L.jpge_dct_plane.argtypes = [vp, vp, u32, u32, i32, vp, u32]
        L.jpge_quantize_plane.argtypes = [vp, vp, u32, u32, vp, vp, u32]
        L.jpge_encode_planes.argtypes = [vp, vp, vp, vp, u32, u32, i32, u32, u32, vp, vp, vp, sz, ctypes.POINTER(sz),
                                         u32]
        L.jpge_group_open.argtypes = [i32, vp, i32, ctypes.POINTER(vp)]
        L.jpge_group_close.argtypes = [vp]
        L.jpge_group_size.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.jpge_group_context.argtypes = [vp, i32, ctypes.POINTER(vp)]
        L.jpge_group_set_restart_interval.argtypes = [vp, u32]
        L.jpge_group_encode_batch.argtypes = [vp, ctypes.POINTER(Frame), i32, vp, vp, u32]
        L.jpge_group_encode_striped.argtypes = [vp, vp, u32, u32, sz, i32, vp, vp, vp, sz, ctypes.POINTER(sz)]
        _LIB = L
    return _LIB


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def _check(st: int, what: str) -> None:
    if st != 0:
        raise JpgeError(st, what)


def quality_tables(quality: int = 50) -> tuple[np.ndarray, np.ndarray]:
    """Annex-K tables scaled for `quality` (50 = the reference's tables, Image.cpp:850-869)."""
    qy = np.zeros(64, np.uint8)
    qc = np.zeros(64, np.uint8)
    _check(lib().jpge_quality_tables(int(quality), _p(qy), _p(qc)), "quality_tables")
    return qy, qc


def synth_rgb8(seed: int, width: int, height: int, kind: int = 0) -> np.ndarray:
    """Deterministic synthetic frame (H, W, 3) uint8: 0 photo-like, 1 random bytes, 2 flat."""
    out = np.empty((height, width, 3), np.uint8)
    _check(lib().jpge_synth_rgb8(seed, width, height, kind, _p(out), width * 3), "synth_rgb8")
    return out


@dataclass
class PPM:
    rgb: np.ndarray  # (H, W, 3) uint8, unscaled samples
    maxval: int

    @property
    def width(self) -> int:
        return self.rgb.shape[1]

    @property
    def height(self) -> int:
        return self.rgb.shape[0]


def parse_ppm(data: bytes) -> PPM:
    """P3/P6 parser with the reference's tokenizer semantics (Image.cpp:334-474)."""
    buf = np.frombuffer(data, np.uint8)
    w, h, mv = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
    _check(lib().jpge_ppm_info(_p(buf), buf.size, ctypes.byref(w), ctypes.byref(h), ctypes.byref(mv)),
           "parse_ppm")
    rgb = np.empty((h.value, w.value, 3), np.uint8)
    _check(lib().jpge_parse_ppm(_p(buf), buf.size, _p(rgb), rgb.size, ctypes.byref(w), ctypes.byref(h),
                                ctypes.byref(mv)), "parse_ppm")
    return PPM(rgb, mv.value)


def load_ppm(path: str) -> PPM:
    """loadPPM (Image.hpp:28)."""
    with open(path, "rb") as f:
        return parse_ppm(f.read())


def huffman_text(text) -> list[tuple[int, int, int]]:
    """generateHuffmanCode (Huffman.hpp:53) on an int text -> [(symbol, length, code)] in DHT order."""
    t = np.ascontiguousarray(np.asarray(text, dtype=np.int32))
    n = max(1, len(set(t.tolist())))
    syms = np.zeros(n + 1, np.int32)
    lens = np.zeros(n + 1, np.int32)
    codes = np.zeros(n + 1, np.uint32)
    k = ctypes.c_int()
    _check(lib().jpge_huffman_text(_p(t), t.size, _p(syms), _p(lens), _p(codes), ctypes.byref(k)), "huffman_text")
    return list(zip(syms[:k.value].tolist(), lens[:k.value].tolist(), codes[:k.value].tolist()))


def huffman_decode(data: bytes, nbits: int, table) -> list[int]:
    """huffmanDecode (Huffman.cpp:91-146): the symbols coded in the first nbits bits of
    data by table = [(symbol, length, code)] (as huffman_text returns it)."""
    buf = np.frombuffer(bytes(data) + b"\0", np.uint8)
    syms = np.ascontiguousarray([t[0] for t in table], np.uint32)
    lens = np.ascontiguousarray([t[1] for t in table], np.uint8)
    codes = np.ascontiguousarray([t[2] for t in table], np.uint32)
    n = ctypes.c_size_t()
    _check(lib().jpge_huffman_decode(_p(buf), nbits, _p(syms), _p(codes), _p(lens), len(table), None, 0,
                                     ctypes.byref(n)), "huffman_decode")
    out = np.zeros(max(1, n.value), np.int32)
    _check(lib().jpge_huffman_decode(_p(buf), nbits, _p(syms), _p(codes), _p(lens), len(table), _p(out), out.size,
                                     ctypes.byref(n)), "huffman_decode")
    return out[:n.value].tolist()


def idct8x8(block) -> np.ndarray:
    """inverseDctMat (Dct.hpp:278-306) of an 8x8 block."""
    x = np.ascontiguousarray(block, np.float64).reshape(64)
    out = np.zeros(64, np.float64)
    lib().jpge_idct8x8(_p(x), _p(out))
    return out.reshape(8, 8)


def decode_coeffs(data: bytes):
    """Entropy-decode a jpge .jpg -> (Decoded header, Y, Cb, Cr) quantised coefficient
    planes of shape (blocks, 64), raster block order, natural order (jpge_decode_coeffs)."""
    buf = np.frombuffer(bytes(data), np.uint8)
    info = Decoded()
    _check(lib().jpge_decode_coeffs(_p(buf), buf.size, ctypes.byref(info), None, None, None, 0, 0), "decode_coeffs")
    y = np.zeros((info.y_blocks, 64), np.int16)
    cb = np.zeros((info.c_blocks, 64), np.int16)
    cr = np.zeros_like(cb)
    _check(lib().jpge_decode_coeffs(_p(buf), buf.size, ctypes.byref(info), _p(y), _p(cb), _p(cr), y.shape[0],
                                    cb.shape[0]), "decode_coeffs")
    return info, y, cb, cr


def concat_segments(device: int, stream: int, ptrs, lens, dst: int) -> int:
    """jpge_concat_segments: device byte runs (pointers ptrs[k], lens[k] bytes) back to
    back into the device buffer dst, queued on `stream` (a hipStream_t as an int, 0 =
    the null stream).  ptrs/lens may be ctypes arrays (reused) or sequences.  Returns
    the total length."""
    n = len(ptrs)
    if not isinstance(ptrs, ctypes.Array):
        ptrs = (ctypes.c_void_p * n)(*ptrs)
    if not isinstance(lens, ctypes.Array):
        lens = (ctypes.c_size_t * n)(*lens)
    tot = ctypes.c_size_t()
    _check(lib().jpge_concat_segments(int(device), stream or None, ptrs, lens, n, dst, ctypes.byref(tot)),
           "concat_segments")
    return tot.value


def huffman_table(counts, first):
    """Byte-symbol table from counts/first-occurrence keys -> (bits[16], huffval list, code[256], len[256])."""
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    f = np.ascontiguousarray(first, dtype=np.uint64)
    bits = np.zeros(16, np.uint8)
    hv = np.zeros(256, np.uint8)
    code = np.zeros(256, np.uint32)
    ln = np.zeros(256, np.uint8)
    n = ctypes.c_int()
    _check(lib().jpge_huffman_table(_p(c), _p(f), _p(bits), _p(hv), ctypes.byref(n), _p(code), _p(ln)),
           "huffman_table")
    return bits, hv[:n.value].tolist(), code, ln


# ---- Coding.hpp primitives (host, C ABI) ----
def zigzag_index(i: int) -> int:
    """zigzag(int) (Coding.hpp:57-81): natural index of zig-zag position i (-1 outside 0..63)."""
    return int(lib().jpge_zigzag_index(int(i)))


def zigzag_block(block) -> np.ndarray:
    """zigzag(matrix) (Coding.hpp:30-54) of a natural-order 8x8 block."""
    a = np.ascontiguousarray(block, np.int32).reshape(64)
    out = np.zeros(64, np.int32)
    _check(lib().jpge_zigzag_block(_p(a), _p(out)), "zigzag_block")
    return out


def quantize_block(block, table) -> np.ndarray:
    """quantize (Coding.hpp:84-97): round-half-away of block / table, natural order."""
    b = np.ascontiguousarray(block, np.float64).reshape(64)
    t = np.ascontiguousarray(table, np.float64).reshape(64)
    out = np.zeros(64, np.int32)
    _check(lib().jpge_quantize_block(_p(b), _p(t), _p(out)), "quantize_block")
    return out.reshape(8, 8)


def rle_ac(data, zigzag_scan: bool = False) -> list[tuple[int, int]]:
    """RLE_AC (Coding.hpp:112-183): [(run, value)]; zigzag_scan: the 8x8 matrix version."""
    d = np.ascontiguousarray(data, np.int32).reshape(-1)
    runs = np.zeros(d.size + 64, np.uint8)
    vals = np.zeros(d.size + 64, np.int32)
    n = ctypes.c_size_t()
    _check(lib().jpge_rle_ac(_p(d), d.size, int(zigzag_scan), _p(runs), _p(vals), runs.size, ctypes.byref(n)),
           "rle_ac")
    return list(zip(runs[:n.value].tolist(), vals[:n.value].tolist()))


def category_code(value: int) -> tuple[int, int]:
    """getCategoryAndCode (Coding.hpp:197-262): (category, extra bits)."""
    c, b = ctypes.c_uint16(), ctypes.c_uint32()
    _check(lib().jpge_category_code(int(value), ctypes.byref(c), ctypes.byref(b)), "category_code")
    return c.value, b.value


def encode_category(pairs) -> list[tuple[int, int, int]]:
    """encode_category (Coding.hpp:265-283): [(symbol, extra bits, bit count)]."""
    n = len(pairs)
    runs = np.ascontiguousarray([p[0] for p in pairs] or [0], np.uint8)
    vals = np.ascontiguousarray([p[1] for p in pairs] or [0], np.int32)
    syms, lens = np.zeros(max(1, n), np.uint8), np.zeros(max(1, n), np.uint8)
    codes = np.zeros(max(1, n), np.uint32)
    _check(lib().jpge_encode_category(_p(runs), _p(vals), n, _p(syms), _p(codes), _p(lens)), "encode_category")
    return list(zip(syms[:n].tolist(), codes[:n].tolist(), lens[:n].tolist()))


def dc_difference(qy: np.ndarray, qcb: np.ndarray, qcr: np.ndarray) -> None:
    """applyDCdifferenceCoding (Image.cpp:638-678) in place on int32 planes."""
    for a in (qy, qcb, qcr):
        if a.dtype != np.int32 or not a.flags.c_contiguous:
            raise ValueError("int32 C-contiguous planes expected")
    _check(lib().jpge_dc_difference(_p(qy), qy.shape[0], qy.shape[1], _p(qcb), _p(qcr), qcb.shape[0], qcb.shape[1]),
           "dc_difference")


def arai_constants() -> tuple[np.ndarray, np.ndarray]:
    a = np.zeros(5)
    s = np.zeros(8)
    lib().jpge_arai_constants(_p(a), _p(s))
    return a, s


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().jpge_device_count(ctypes.byref(n))
    return n.value


def max_jpeg_bytes(width: int, height: int) -> int:
    return int(lib().jpge_max_jpeg_bytes(width, height))


# Encoders (and device groups) still open at interpreter exit are closed by an atexit hook, ahead of the
# HIP runtime's own teardown in the C++ static destructors (a lane stream destroyed
# after that, e.g. once a profiler's tool library has finalised, can fault the process).
_live_encoders = weakref.WeakSet()


@atexit.register
def _close_live_encoders() -> None:
    for e in list(_live_encoders):
        try:
            e.close()
        except Exception:
            pass


class Encoder:
    """One GPU context (jpge_open).  Host-array methods copy in/out; the `*_dev`
    variants take device pointers (ints) for HBM-resident frames."""

    def __init__(self, device: int = 0, lanes: int = 0):
        """lanes: concurrent pipelines on the device (0 = JPGE_LANES or the default 4)."""
        self._ctx = ctypes.c_void_p()
        _check(lib().jpge_open_ex(int(device), int(lanes), ctypes.byref(self._ctx)), f"jpge_open({device})")
        _live_encoders.add(self)
        self.device = device
        self._qcache = {}     # quality -> (qy, qc) byte tables
        self._desc = None     # (key, Frame array) of the last device batch

    def close(self) -> None:
        if self._ctx:
            lib().jpge_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self) -> ctypes.c_void_p:
        return self._ctx

    def set_timing(self, every: int = 1) -> None:
        """HIP-event kernel timing of every `every`-th frame (0/False = off, True = all)."""
        _check(lib().jpge_set_timing(self._ctx, int(every)), "set_timing")

    def timing(self) -> dict:
        t = Timing()
        _check(lib().jpge_get_timing(self._ctx, ctypes.byref(t)), "get_timing")
        return {"fdct": t.fdct, "dc_stats": t.dc_stats, "entropy": t.entropy, "total": t.total,
                "fdct_sum": t.fdct_sum, "dc_stats_sum": t.dc_stats_sum, "entropy_sum": t.entropy_sum,
                "frames": t.frames, "symbols": t.symbols, "code_sum": t.code_sum, "pack_sum": t.pack_sum,
                "launches": t.launches, "gate_timeouts": t.gate_timeouts}

    def reset_timing(self) -> None:
        _check(lib().jpge_reset_timing(self._ctx), "reset_timing")

    def set_restart(self, mcus: int) -> None:
        """Restart interval in MCUs for the following encodes (0 = none: the reference's stream)."""
        _check(lib().jpge_set_restart_interval(self._ctx, int(mcus)), "set_restart_interval")

    def set_subsampling(self, mode: int) -> None:
        """Chroma subsampling for the following encodes (applySubsampling's modes,
        Image.hpp:44-52): 420 (S420_m, the reference's writeJPEG, the default), 444
        (S444), 422 (S422), 411 (S411), 4200 (S420) or 4201 (S420_lm); see SUBSAMPLING."""
        _check(lib().jpge_set_subsampling(self._ctx, int(mode)), "set_subsampling")
        self._sub = int(mode)

    def lanes(self) -> int:
        n = ctypes.c_int32()
        _check(lib().jpge_get_lanes(self._ctx, ctypes.byref(n)), "get_lanes")
        return n.value

    @staticmethod
    def _tables(quality, qy, qc):
        if qy is None or qc is None:
            qy, qc = quality_tables(quality)
        return np.ascontiguousarray(qy, np.uint8), np.ascontiguousarray(qc, np.uint8)

    def encode(self, rgb: np.ndarray, quality: int = 50, maxval: int = 255, qy=None, qc=None) -> bytes:
        """Image::writeJPEG (Image.cpp:831-976) on an (H, W, 3) uint8 frame -> .jpg bytes."""
        rgb = np.ascontiguousarray(rgb, np.uint8)
        h, w = rgb.shape[:2]
        qy, qc = self._tables(quality, qy, qc)
        out = np.empty(max_jpeg_bytes(w, h), np.uint8)
        n = ctypes.c_size_t()
        _check(lib().jpge_encode_rgb8(self._ctx, _p(rgb), w, h, w * 3, int(maxval), _p(qy), _p(qc), _p(out),
                                      out.size, ctypes.byref(n), 0), "encode")
        return out[:n.value].tobytes()

    def encode_ptr(self, rgb_ptr: int, w: int, h: int, stride: int, out_ptr: int, cap: int, quality: int = 50,
                   maxval: int = 255, flags: int = JPGE_DEVICE_INPUT | JPGE_DEVICE_OUTPUT) -> int:
        """One frame through jpge_encode_rgb8 on raw pointers (device or host per `flags`;
        host pointers may be pinned memory); returns the .jpg length."""
        q = self._qcache.get(quality)
        if q is None:
            qy, qc = self._tables(quality, None, None)
            q = self._qcache[quality] = (qy, qc, _p(qy), _p(qc))
        n = ctypes.c_size_t()
        _check(lib().jpge_encode_rgb8(self._ctx, rgb_ptr, w, h, stride, int(maxval), q[2], q[3], out_ptr, cap,
                                      ctypes.byref(n), int(flags)), "encode_rgb8")
        return n.value

    def encode_batch_dev(self, frames: list[tuple[int, int, int, int]], outs: list[tuple[int, int]],
                         quality: int = 50, maxval: int = 255,
                         flags: int = JPGE_DEVICE_INPUT | JPGE_DEVICE_OUTPUT) -> list[int]:
        """Pipelined batch on device memory: frames = [(ptr, w, h, stride)], outs = [(ptr, cap)].
        Returns the .jpg length of each frame (bytes stay in device memory; without
        JPGE_DEVICE_OUTPUT in `flags` the outs are host pointers, e.g. pinned memory).
        The quality tables and the descriptor array of a repeated batch are reused."""
        q = self._qcache.get(quality)
        if q is None:
            qy, qc = self._tables(quality, None, None)
            q = self._qcache[quality] = (qy, qc, _p(qy), _p(qc))
        key = (tuple(frames), tuple(outs), maxval)
        if self._desc is None or self._desc[0] != key:
            arr = (Frame * len(frames))()
            for i, ((p, w, h, s), (o, cap)) in enumerate(zip(frames, outs)):
                arr[i].rgb, arr[i].width, arr[i].height, arr[i].stride, arr[i].maxval = p, w, h, s, maxval
                arr[i].out, arr[i].cap = o, cap
            self._desc = (key, arr)
        arr = self._desc[1]
        st = lib().jpge_encode_batch(self._ctx, arr, len(frames), q[2], q[3], int(flags))
        _check(st, "encode_batch")
        return [f.len for f in arr]

    def encode_batch(self, frames: list[np.ndarray], quality: int = 50, maxval: int = 255) -> list[bytes]:
        qy, qc = self._tables(quality, None, None)
        frames = [np.ascontiguousarray(f, np.uint8) for f in frames]
        outs = [np.empty(max_jpeg_bytes(f.shape[1], f.shape[0]), np.uint8) for f in frames]
        arr = (Frame * len(frames))()
        for i, (f, o) in enumerate(zip(frames, outs)):
            arr[i].rgb, arr[i].width, arr[i].height = _p(f), f.shape[1], f.shape[0]
            arr[i].stride, arr[i].maxval, arr[i].out, arr[i].cap = f.shape[1] * 3, maxval, _p(o), o.size
        _check(lib().jpge_encode_batch(self._ctx, arr, len(frames), _p(qy), _p(qc), 0), "encode_batch")
        return [outs[i][:arr[i].len].tobytes() for i in range(len(frames))]

    def fdct_quant(self, rgb: np.ndarray, quality: int = 50, maxval: int = 255, qy=None, qc=None):
        """Stage dump: quantised coefficients (before DC diff) -> (Y, Cb, Cr) arrays of shape
        (nblocks, 64), blocks in raster order, natural order within a block."""
        rgb = np.ascontiguousarray(rgb, np.uint8)
        h, w = rgb.shape[:2]
        yh, yv = SUBSAMPLING[getattr(self, "_sub", 420)]
        mw, mh = -(-w // (8 * yh)), -(-h // (8 * yv))  # MCUs across / down
        y = np.zeros((mw * yh * mh * yv, 64), np.int16)
        cb = np.zeros((mw * mh, 64), np.int16)
        cr = np.zeros_like(cb)
        qy, qc = self._tables(quality, qy, qc)
        _check(lib().jpge_fdct_quant(self._ctx, _p(rgb), w, h, w * 3, int(maxval), _p(qy), _p(qc), _p(y), _p(cb),
                                     _p(cr), 0), "fdct_quant")
        return y, cb, cr

    # ---- row stripes (jpge_stripe_*; orchestration in jpgenc_amd.stripes) ----
    def stripe_transform(self, rgb_ptr: int, stride: int, width: int, height: int, mcu_row0: int, mcu_rows: int,
                         quality: int = 50, maxval: int = 255) -> np.ndarray:
        """K1 on a stripe (device RGB of its rows); returns its last Y/Cb/Cr DC (int32[3])."""
        qy, qc = self._tables(quality, None, None)
        last = np.zeros(3, np.int32)
        _check(lib().jpge_stripe_transform(self._ctx, rgb_ptr, stride, width, height, mcu_row0, mcu_rows,
                                           int(maxval), _p(qy), _p(qc), _p(last)), "stripe_transform")
        return last

    def stripe_stats(self, seed_dc) -> tuple[np.ndarray, np.ndarray]:
        seed = np.ascontiguousarray(seed_dc, np.int32)
        counts = np.zeros(1024, np.uint32)
        first = np.zeros(1024, np.uint64)
        _check(lib().jpge_stripe_stats(self._ctx, _p(seed), _p(counts), _p(first)), "stripe_stats")
        return counts, first

    def stripe_code(self, counts: np.ndarray, first: np.ndarray) -> tuple[tuple, int]:
        counts = np.ascontiguousarray(counts, np.uint32)
        first = np.ascontiguousarray(first, np.uint64)
        sm = StripeSummary()
        hl = ctypes.c_size_t()
        _check(lib().jpge_stripe_code(self._ctx, _p(counts), _p(first), ctypes.byref(sm), ctypes.byref(hl)),
               "stripe_code")
        return sm.as_tuple(), hl.value

    def stripe_pack(self, summaries: list, index: int, out_ptr: int, cap: int) -> tuple[int, int, int]:
        arr = (StripeSummary * len(summaries))(*[StripeSummary.from_tuple(t) for t in summaries])
        off, ln, tot = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        _check(lib().jpge_stripe_pack(self._ctx, arr, len(summaries), index, out_ptr, cap, ctypes.byref(off),
                                      ctypes.byref(ln), ctypes.byref(tot)), "stripe_pack")
        return off.value, ln.value, tot.value

    # ---- plane stages: the reference's Image stage methods on fp64 planes (GPU) ----
    def color_convert(self, p0, p1, p2, target: int = JPGE_TO_YCBCR):
        """convertToColorSpace (Image.cpp:112-179) of three equal-size planes."""
        ins = [np.ascontiguousarray(p, np.float64) for p in (p0, p1, p2)]
        outs = [np.empty_like(ins[0]) for _ in range(3)]
        _check(lib().jpge_color_convert(self._ctx, *[_p(a) for a in ins], *[_p(a) for a in outs], ins[0].size,
                                        int(target), 0), "color_convert")
        return outs

    def subsample_plane(self, plane, mode: int) -> np.ndarray:
        """Image::subsample with applySubsampling's mask for `mode` (jpge.h JPGE_S*)."""
        a = np.ascontiguousarray(plane, np.float64)
        r, c = ctypes.c_uint32(), ctypes.c_uint32()
        _check(lib().jpge_subsample_plane(self._ctx, _p(a), a.shape[0], a.shape[1], int(mode), None, ctypes.byref(r),
                                          ctypes.byref(c), 0), "subsample_plane")
        out = np.empty((r.value, c.value), np.float64)
        _check(lib().jpge_subsample_plane(self._ctx, _p(a), a.shape[0], a.shape[1], int(mode), _p(out),
                                          ctypes.byref(r), ctypes.byref(c), 0), "subsample_plane")
        return out

    def dct_plane(self, plane, mode: int = DCT_ARAI) -> np.ndarray:
        """applyDCT(mode) (Image.cpp:540-595) on one plane of 8x8 blocks."""
        a = np.ascontiguousarray(plane, np.float64)
        out = np.empty_like(a)
        _check(lib().jpge_dct_plane(self._ctx, _p(a), a.shape[0], a.shape[1], int(mode), _p(out), 0), "dct_plane")
        return out

    def quantize_plane(self, plane, table) -> np.ndarray:
        """applyQuantization's per-block quantize (Coding.hpp:84-97) with one table."""
        a = np.ascontiguousarray(plane, np.float64)
        t = np.ascontiguousarray(table, np.uint8).reshape(64)
        out = np.empty(a.shape, np.int32)
        _check(lib().jpge_quantize_plane(self._ctx, _p(a), a.shape[0], a.shape[1], _p(t), _p(out), 0),
               "quantize_plane")
        return out

    def encode_planes(self, p0, p1, p2, real_width: int, real_height: int, colorspace: int = JPGE_TO_RGB,
                      quality: int = 50) -> bytes:
        """writeJPEG (Image.cpp:831-976) on an Image's three fp64 planes (rows x cols,
        multiples of 16): R,G,B (colorspace JPGE_TO_RGB) or Y,Cb,Cr (JPGE_TO_YCBCR)."""
        ins = [np.ascontiguousarray(p, np.float64) for p in (p0, p1, p2)]
        rows, cols = ins[0].shape
        qy, qc = self._tables(quality, None, None)
        out = np.empty(max_jpeg_bytes(cols, rows), np.uint8)
        n = ctypes.c_size_t()
        _check(lib().jpge_encode_planes(self._ctx, *[_p(a) for a in ins], rows, cols, int(colorspace), real_width,
                                        real_height, _p(qy), _p(qc), _p(out), out.size, ctypes.byref(n), 0),
               "encode_planes")
        return out[:n.value].tobytes()

    def encode_file(self, ppm_path: str, jpg_path: str, quality: int = 50) -> None:
        """main.cpp: loadPPM(ppm_path) + writeJPEG(jpg_path)."""
        _check(lib().jpge_encode_file(self._ctx, ppm_path.encode(), jpg_path.encode(), int(quality)), "encode_file")

    def encode_files(self, ppm_paths: list[str], jpg_paths: list[str], quality: int = 50, group: int = 0):
        """Many PPM files -> .jpg files through the ingest pipeline; returns the .jpg lengths."""
        n = len(ppm_paths)
        if len(jpg_paths) != n:
            raise ValueError("ppm_paths and jpg_paths differ in length")
        ins = (ctypes.c_char_p * n)(*[p.encode() for p in ppm_paths])
        outs = (ctypes.c_char_p * n)(*[p.encode() for p in jpg_paths])
        lens = np.zeros(n, np.uint64)
        sts = np.zeros(n, np.int32)
        st = lib().jpge_encode_files(self._ctx, ins, outs, n, int(quality), _p(lens), _p(sts), int(group))
        _check(st, f"encode_files (statuses {sts.tolist()})" if st else "encode_files")
        return [int(x) for x in lens]

    def symbol_stats(self, rgb: np.ndarray, quality: int = 50, maxval: int = 255):
        rgb = np.ascontiguousarray(rgb, np.uint8)
        h, w = rgb.shape[:2]
        qy, qc = self._tables(quality, None, None)
        counts = np.zeros(1024, np.uint32)
        first = np.zeros(1024, np.uint64)
        _check(lib().jpge_symbol_stats(self._ctx, _p(rgb), w, h, w * 3, int(maxval), _p(qy), _p(qc), _p(counts),
                                       _p(first), 0), "symbol_stats")
        return counts.reshape(4, 256), first.reshape(4, 256)


class Group:
    """A device group (jpge_group_open): one process, one context per listed device,
    RCCL over xGMI between distinct devices (a device listed twice: host exchanges)."""

    def __init__(self, devices, lanes: int = 0):
        devs = (ctypes.c_int * len(devices))(*devices)
        self._g = ctypes.c_void_p()
        _check(lib().jpge_group_open(len(devices), devs, int(lanes), ctypes.byref(self._g)), "group_open")
        _live_encoders.add(self)

    def close(self) -> None:
        if self._g:
            lib().jpge_group_close(self._g)
            self._g = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def size(self) -> tuple[int, bool]:
        """(members, whether the exchanges ride RCCL)"""
        n, r = ctypes.c_int(), ctypes.c_int()
        _check(lib().jpge_group_size(self._g, ctypes.byref(n), ctypes.byref(r)), "group_size")
        return n.value, bool(r.value)

    def set_restart(self, mcus: int) -> None:
        _check(lib().jpge_group_set_restart_interval(self._g, int(mcus)), "group_set_restart_interval")

    def encode_batch(self, frames: list[np.ndarray], quality: int = 50, maxval: int = 255) -> list[bytes]:
        """Config 4: frame i on member i mod N."""
        qy, qc = quality_tables(quality)
        frames = [np.ascontiguousarray(f, np.uint8) for f in frames]
        outs = [np.empty(max_jpeg_bytes(f.shape[1], f.shape[0]), np.uint8) for f in frames]
        arr = (Frame * len(frames))()
        for i, (f, o) in enumerate(zip(frames, outs)):
            arr[i].rgb, arr[i].width, arr[i].height = _p(f), f.shape[1], f.shape[0]
            arr[i].stride, arr[i].maxval, arr[i].out, arr[i].cap = f.shape[1] * 3, maxval, _p(o), o.size
        _check(lib().jpge_group_encode_batch(self._g, arr, len(frames), _p(qy), _p(qc), 0), "group_encode_batch")
        return [outs[i][:arr[i].len].tobytes() for i in range(len(frames))]

    def encode_striped(self, rgb: np.ndarray, quality: int = 50, maxval: int = 255) -> bytes:
        """Config 5: one image in row stripes over the members."""
        rgb = np.ascontiguousarray(rgb, np.uint8)
        h, w = rgb.shape[:2]
        qy, qc = quality_tables(quality)
        out = np.empty(max_jpeg_bytes(w, h), np.uint8)
        n = ctypes.c_size_t()
        _check(lib().jpge_group_encode_striped(self._g, _p(rgb), w, h, w * 3, int(maxval), _p(qy), _p(qc), _p(out),
                                               out.size, ctypes.byref(n)), "group_encode_striped")
        return out[:n.value].tobytes()


def stripe_place(summaries: list, index: int, header_len: int) -> tuple[int, int]:
    """Host-only placement of stripe `index`: (first output byte, whole file length)."""
    arr = (StripeSummary * len(summaries))(*[StripeSummary.from_tuple(t) for t in summaries])
    off, tot = ctypes.c_size_t(), ctypes.c_size_t()
    _check(lib().jpge_stripe_place(arr, len(summaries), index, header_len, ctypes.byref(off), ctypes.byref(tot)),
           "stripe_place")
    return off.value, tot.value


def write_jpeg(path: str, ppm: PPM, quality: int = 50, device: int = 0) -> int:
    """loadPPM + writeJPEG convenience; returns bytes written."""
    with Encoder(device) as enc:
        data = enc.encode(ppm.rgb, quality=quality, maxval=ppm.maxval)
    with open(path, "wb") as f:
        f.write(data)
    return len(data)
