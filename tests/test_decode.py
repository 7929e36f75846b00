"""Decode-side verification utilities (include/jpge.h):
jpge_huffman_decode (huffmanDecode, Huffman.cpp:91-146), jpge_idct8x8
(inverseDctMat, Dct.hpp:278-306) and jpge_decode_coeffs (the baseline entropy
decode of a jpge stream back to its quantised coefficients).

Pinning: huffmanDecode against the reference's own huffmanEncode/huffmanDecode
round trip (oracle/_ref, HuffmanTest.cpp:65-85) when it is built here, and its
texts; inverseDctMat against DctTest.cpp:50-84's matrix; the entropy decoder
against the oracle's stage coefficients of its own streams in every subsampling
mode, with and without restart intervals."""
import ctypes

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

# HuffmanTest.cpp:66 and :77
TEXTS = [[4, 4, 4, 4, 2, 2, 1, 5, 5, 5, 5, 5],
         [4, 4, 4, 4, 2, 2, 1, 5, 5, 5, 5, 5, 3, 5, 6, 5, 3, 4, 5, 6, 1010, 203, 4, 0, 111111]]


def _pack(text, table):
    code = {s: (ln, c) for s, ln, c in table}
    bits = "".join(format(code[s][1], f"0{code[s][0]}b") for s in text)
    pad = (8 - len(bits) % 8) % 8
    data = (int(bits, 2) << pad).to_bytes((len(bits) + 7) // 8, "big") if bits else b""
    return data, len(bits)


@pytest.mark.parametrize("text", TEXTS)
def test_huffman_decode_reference_texts(text):
    table = J.huffman_text(text)
    data, nbits = _pack(text, table)
    assert J.huffman_decode(data, nbits, table) == text


def test_huffman_decode_random_texts():
    rng = np.random.default_rng(7)
    for n, k in [(1, 1), (50, 1), (200, 3), (1000, 40), (5000, 256)]:
        text = rng.integers(0, k, n).tolist()
        table = J.huffman_text(text)
        data, nbits = _pack(text, table)
        assert J.huffman_decode(data, nbits, table) == text


def test_huffman_decode_matches_reference_library():
    ref = _oracle.ref()
    if ref is None or not hasattr(ref, "ref_huffman_roundtrip"):
        pytest.skip("oracle/_ref/libref.so not built (needs /root/reference)")
    ref.ref_huffman_roundtrip.restype = ctypes.c_int64
    ref.ref_huffman_roundtrip.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p]
    rng = np.random.default_rng(3)
    texts = TEXTS + [rng.integers(0, 30, 400).tolist(), (rng.geometric(0.2, 2000) % 200).tolist()]
    for text in texts:
        t = np.ascontiguousarray(text, np.int32)
        bits = np.zeros(len(text) * 4 + 8, np.uint8)
        dec = np.zeros(len(text), np.int32)
        nb = ref.ref_huffman_roundtrip(t.ctypes.data, t.size, bits.ctypes.data, bits.size, dec.ctypes.data)
        assert nb >= 0 and dec.tolist() == text
        # the same bits through jpge_huffman_decode with jpge's table (= the reference's)
        table = J.huffman_text(text)
        assert J.huffman_decode(bits[:(nb + 7) // 8].tobytes(), nb, table) == text


def test_idct_reference_kat():
    # DctTest.cpp:50-84: inverseDctMat(dctMat(m)) == m for m = 1..64
    true_dct = np.zeros((8, 8))
    true_dct[0] = [260, -18.2216411837961, 7.69085915161152e-15, -1.90481782616726, 0, -0.568239222367164,
                   1.85673764701218e-14, -0.143407824981022]
    true_dct[1:, 0] = [-145.773129470369, 0, -15.2385426093380, 0, -4.54591377893732, 0, -1.14726259984816]
    m = np.arange(1, 65, dtype=np.float64).reshape(8, 8)
    assert np.allclose(J.idct8x8(true_dct), m, atol=1e-9)


def test_idct_inverts_the_arai_dct():
    # the Arai FDCT (Dct.hpp:47-215) is orthonormal-scaled: inverseDctMat recovers the block
    rng = np.random.default_rng(1)
    for _ in range(20):
        x = rng.uniform(-128, 127, 64)
        y = np.zeros(64)
        _oracle.orc().orc_dct_arai(x.ctypes.data, y.ctypes.data)
        assert np.allclose(J.idct8x8(y.reshape(8, 8)).reshape(64), x, atol=1e-9)


def _expected(rgb, quality, mode):
    if mode == 420:
        return _oracle.stage_coeffs(rgb, quality)
    if mode == 444:
        return _oracle.stage_coeffs444(rgb, quality)
    return _oracle.stage_coeffs_mode(rgb, mode, quality)


@pytest.mark.parametrize("mode", [420, 444, 422, 411, 4200, 4201])
@pytest.mark.parametrize("w,h,r", [(1, 1, 0), (37, 23, 0), (130, 75, 0), (130, 75, 4), (64, 64, 1)])
def test_decode_coeffs_of_oracle_streams(mode, w, h, r):
    rgb = J.synth_rgb8(w * 5 + h + r, w, h)
    data = _oracle.encode(rgb, 90, restart=r, subsampling=mode)
    info, y, cb, cr = J.decode_coeffs(data)
    yh, yv = J.SUBSAMPLING[mode]
    assert (info.width, info.height, info.yh, info.yv, info.restart) == (w, h, yh, yv, r)
    qy, qc = _oracle.quality_tables(90)
    assert bytes(info.qy) == qy.tobytes() and bytes(info.qc) == qc.tobytes()
    for got, want in zip((y, cb, cr), _expected(rgb, 90, mode)):
        assert np.array_equal(got, want)


@pytest.mark.parametrize("kind,quality", [(1, 100), (2, 50)])
def test_decode_coeffs_stress(kind, quality):
    # random bytes (long codes, many stuffed 0xFF) and flat frames (one-symbol tables)
    rgb = J.synth_rgb8(40 + kind, 96, 80, kind=kind)
    info, y, cb, cr = J.decode_coeffs(_oracle.encode(rgb, quality))
    for got, want in zip((y, cb, cr), _oracle.stage_coeffs(rgb, quality)):
        assert np.array_equal(got, want)


def test_decode_coeffs_rejects_garbage():
    with pytest.raises(J.JpgeError):
        J.decode_coeffs(b"\xff\xd8\xff\xd9")
    data = bytearray(_oracle.encode(J.synth_rgb8(1, 40, 40), 90))
    with pytest.raises(J.JpgeError):  # truncated entropy data
        J.decode_coeffs(bytes(data[: len(data) // 2]))


def _segment(data, marker):
    """Offset of the first marker segment `marker` (0xFF <marker>) in a header."""
    pos = 2
    while pos + 4 <= len(data):
        assert data[pos] == 0xFF
        if data[pos + 1] == marker:
            return pos
        pos += 2 + (data[pos + 2] << 8 | data[pos + 3])
    raise AssertionError("segment not found")


def test_decode_coeffs_rejects_short_segments():
    # DRI / SOS segments whose declared length is too short, and table selectors past
    # the four table slots, are format errors (no read past the segment)
    data = _oracle.encode(J.synth_rgb8(3, 48, 32), 90, restart=2)
    assert J.decode_coeffs(data)[0].restart == 2
    bad = bytearray(data)
    p = _segment(bad, 0xDD)
    bad[p + 2:p + 4] = b"\x00\x02"  # DRI length 2: no interval field
    bad[p + 4:p + 6] = b"\xff\xfe"  # (the old field now reads as the next segment's marker: COM)
    with pytest.raises(J.JpgeError):
        J.decode_coeffs(bytes(bad))
    bad = bytearray(data)
    p = _segment(bad, 0xDA)
    bad[p + 2:p + 4] = b"\x00\x08"  # SOS length 8 < 12
    with pytest.raises(J.JpgeError):
        J.decode_coeffs(bytes(bad))
    bad = bytearray(data)
    p = _segment(bad, 0xDA)
    bad[p + 4 + 2] = 0x07  # Y: DC table 0, AC table 7
    with pytest.raises(J.JpgeError):
        J.decode_coeffs(bytes(bad))
