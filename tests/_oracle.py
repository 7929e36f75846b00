"""ctypes access to the TEST-ONLY oracle (oracle/build/liborc.so) and, when it was
built in this container, the reference's own Huffman/Bitstream code
(oracle/_ref/libref.so).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this module."""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORC_PATH = os.path.join(ROOT, "oracle", "build", "liborc.so")
REF_PATH = os.path.join(ROOT, "oracle", "_ref", "libref.so")

_orc = None
_ref = None


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def orc() -> ctypes.CDLL:
    global _orc
    if _orc is None:
        if not os.path.exists(ORC_PATH):
            raise ImportError(f"{ORC_PATH} missing: run `make oracle`")
        L = ctypes.CDLL(ORC_PATH)
        vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
        L.orc_quality_tables.argtypes = [i32, vp, vp]
        L.orc_arai_constants.argtypes = [vp, vp, vp]
        L.orc_dct_arai.argtypes = [vp, vp]
        L.orc_quantize.argtypes = [vp, vp, vp]
        L.orc_ycc.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, vp]
        L.orc_zigzag_to_natural.argtypes = [i32]
        L.orc_subsample420m.argtypes = [vp, i32, i32, vp]
        L.orc_category.argtypes = [i32, vp]
        L.orc_rle_block.argtypes = [vp, vp, vp, vp, vp, vp]
        L.orc_huffman.argtypes = [vp, i32, vp, vp, vp]
        L.orc_pack_bits.restype = i64
        L.orc_pack_bits.argtypes = [vp, vp, i32, i32, vp, i64, vp]
        L.orc_parse_ppm.argtypes = [vp, sz, vp, vp, vp, vp, sz]
        L.orc_stage_coeffs.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, vp]
        L.orc_stage_ycc.argtypes = [vp, i32, i32, i32, vp, vp, vp]
        L.orc_stage_hist.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp]
        L.orc_encode_rgb.restype = i64
        L.orc_encode_rgb.argtypes = [vp, i32, i32, i32, vp, vp, vp, i64]
        L.orc_encode_rgb_restart.restype = i64
        L.orc_encode_rgb_restart.argtypes = [vp, i32, i32, i32, vp, vp, i32, vp, i64]
        L.orc_encode_rgb_ex.restype = i64
        L.orc_encode_rgb_ex.argtypes = [vp, i32, i32, i32, vp, vp, i32, i32, vp, i64]
        L.orc_stage_coeffs444.argtypes = [vp, i32, i32, i32, vp, vp, vp, vp, vp]
        L.orc_encode_rgb_mode.restype = i64
        L.orc_encode_rgb_mode.argtypes = [vp, i32, i32, i32, vp, vp, i32, i32, i32, vp, i64]
        L.orc_stage_coeffs_mode.argtypes = [vp, i32, i32, i32, vp, vp, i32, vp, vp, vp]
        L.orc_subsample_mode.argtypes = [vp, i32, i32, i32, vp]
        L.orc_set_threads.argtypes = [i32]
        _orc = L
    return _orc


def ref() -> ctypes.CDLL | None:
    """The reference's own code, or None when it could not be built here."""
    global _ref
    if _ref is None and os.path.exists(REF_PATH):
        L = ctypes.CDLL(REF_PATH)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        L.ref_huffman.argtypes = [vp, i32, vp, vp, vp]
        L.ref_package_merge.argtypes = [vp, vp, i32, i32, vp, vp]
        L.ref_pack_bits.restype = i64
        L.ref_pack_bits.argtypes = [vp, vp, vp, i32, i32, vp, i64, vp]
        _ref = L
    return _ref


def quality_tables(q: int):
    qy = np.zeros(64, np.uint8)
    qc = np.zeros(64, np.uint8)
    orc().orc_quality_tables(q, _p(qy), _p(qc))
    return qy, qc


def huffman(text, lib=None, fn="orc_huffman"):
    t = np.ascontiguousarray(np.asarray(text, np.int32))
    n = len(t) + 1
    s = np.zeros(n, np.int32)
    ln = np.zeros(n, np.int32)
    c = np.zeros(n, np.uint32)
    L = lib if lib is not None else orc()
    k = getattr(L, fn)(_p(t), t.size, _p(s), _p(ln), _p(c))
    return list(zip(s[:k].tolist(), ln[:k].tolist(), c[:k].tolist()))


#: subsampling mode -> (Y blocks across, Y blocks down) an MCU (jpge.h JPGE_S*)
SHAPES = {420: (2, 2), 4200: (2, 2), 4201: (2, 2), 444: (1, 1), 422: (2, 1), 411: (4, 1)}


def encode(rgb: np.ndarray, quality: int = 50, maxval: int = 255, qy=None, qc=None, restart: int = 0,
           subsampling: int = 420, generic: bool = False) -> bytes:
    """writeJPEG; restart > 0: the restart-interval variant (DRI + RSTn every `restart` MCUs);
    subsampling 444 / 422 / 411 / 4200 (S420) / 4201 (S420_lm): the subsampling variants;
    generic: force the generic subsampling path (consistency checks at 420 / 444)."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    if qy is None:
        qy, qc = quality_tables(quality)
    cap = 4096 + ((w + 31) // 8) * ((h + 15) // 8) * (3 * 420 + 4)
    out = np.empty(cap, np.uint8)
    qy8, qc8 = np.ascontiguousarray(qy, np.uint8), np.ascontiguousarray(qc, np.uint8)
    if subsampling != 420 or generic:
        n = orc().orc_encode_rgb_mode(_p(rgb), w, h, maxval, _p(qy8), _p(qc8), int(restart), int(subsampling),
                                      int(generic), _p(out), cap)
    elif restart:
        n = orc().orc_encode_rgb_restart(_p(rgb), w, h, maxval, _p(qy8), _p(qc8), int(restart), _p(out), cap)
    else:
        n = orc().orc_encode_rgb(_p(rgb), w, h, maxval, _p(qy8), _p(qc8), _p(out), cap)
    if n < 0:
        raise RuntimeError(f"oracle encode failed: {n}")
    return out[:n].tobytes()


def stage_coeffs(rgb: np.ndarray, quality: int = 50, maxval: int = 255):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    W, H = (w + 15) // 16 * 16, (h + 15) // 16 * 16
    qy, qc = quality_tables(quality)
    y = np.zeros(((W // 8) * (H // 8), 64), np.int16)
    cb = np.zeros(((W // 16) * (H // 16), 64), np.int16)
    cr = np.zeros_like(cb)
    orc().orc_stage_coeffs(_p(rgb), w, h, maxval, _p(qy), _p(qc), _p(y), _p(cb), _p(cr))
    return y, cb, cr


def stage_coeffs444(rgb: np.ndarray, quality: int = 50, maxval: int = 255):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    qy, qc = quality_tables(quality)
    planes = [np.zeros((((w + 7) // 8) * ((h + 7) // 8), 64), np.int16) for _ in range(3)]
    orc().orc_stage_coeffs444(_p(rgb), w, h, maxval, _p(qy), _p(qc), *(_p(p) for p in planes))
    return tuple(planes)


def stage_coeffs_mode(rgb: np.ndarray, mode: int, quality: int = 50, maxval: int = 255):
    """Quantised coefficients of the generic subsampling path (before DC differencing)."""
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    yh, yv = SHAPES[mode]
    mw, mh = -(-w // (8 * yh)), -(-h // (8 * yv))
    qy, qc = quality_tables(quality)
    y = np.zeros((mw * yh * mh * yv, 64), np.int16)
    cb = np.zeros((mw * mh, 64), np.int16)
    cr = np.zeros_like(cb)
    orc().orc_stage_coeffs_mode(_p(rgb), w, h, maxval, _p(qy), _p(qc), int(mode), _p(y), _p(cb), _p(cr))
    return y, cb, cr


def subsample_mode(plane: np.ndarray, mode: int) -> np.ndarray:
    p = np.ascontiguousarray(plane, np.float64)
    H, W = p.shape
    yh, yv = SHAPES[mode]
    out = np.zeros((H // yv) * (W // yh) if mode != 444 else H * W, np.float64)
    orc().orc_subsample_mode(_p(p), W, H, int(mode), _p(out))
    return out.reshape(H // yv, W // yh) if mode != 444 else out.reshape(H, W)


def stage_hist(rgb: np.ndarray, quality: int = 50, maxval: int = 255):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w = rgb.shape[:2]
    qy, qc = quality_tables(quality)
    counts = np.zeros(1024, np.uint32)
    first = np.zeros(1024, np.int64)
    orc().orc_stage_hist(_p(rgb), w, h, maxval, _p(qy), _p(qc), _p(counts), _p(first))
    return counts.reshape(4, 256), first.reshape(4, 256)


def parse_ppm(data: bytes):
    buf = np.frombuffer(data, np.uint8)
    w, h, mv = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    st = orc().orc_parse_ppm(_p(buf), buf.size, ctypes.byref(w), ctypes.byref(h), ctypes.byref(mv), None, 0)
    if st:
        return st, None, None
    samples = np.zeros(w.value * h.value * 3, np.int32)
    st = orc().orc_parse_ppm(_p(buf), buf.size, ctypes.byref(w), ctypes.byref(h), ctypes.byref(mv), _p(samples),
                             samples.size)
    return st, samples.reshape(h.value, w.value, 3), mv.value


def pack_bits(vals, nbits, do_fill=True, modes=None, lib=None):
    v = np.ascontiguousarray(vals, np.uint32)
    nb = np.ascontiguousarray(nbits, np.int32)
    cap = int(nb.sum()) // 4 + 64
    out = np.empty(cap, np.uint8)
    raw = ctypes.c_int64()
    if lib is None:
        n = orc().orc_pack_bits(_p(v), _p(nb), v.size, int(do_fill), _p(out), cap, ctypes.byref(raw))
    else:
        m = np.ascontiguousarray(modes if modes is not None else np.zeros(v.size), np.int32)
        n = lib.ref_pack_bits(_p(v), _p(nb), _p(m), v.size, int(do_fill), _p(out), cap, ctypes.byref(raw))
    return out[:n].tobytes(), raw.value
