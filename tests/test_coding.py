"""Coding.hpp primitives of the C ABI (jpge_zigzag_*, jpge_quantize_block, jpge_rle_ac,
jpge_category_code, jpge_encode_category, jpge_dc_difference) on the host, against
the test-only oracle and against plain restatements of the reference's loops
(Coding.hpp:30-283, Image.cpp:638-678); and the drop-in facade compiled against the
reference's own unit-test values (tests/cpp/test_facade.cpp, cpu part)."""
import os
import subprocess

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FACADE = os.path.join(ROOT, "tests", "cpp", "bin", "test_facade")
PPM = os.path.join(ROOT, "tests", "golden", "ppm")


def test_zigzag_index_and_block():
    for i in range(64):
        assert J.zigzag_index(i) == _oracle.orc().orc_zigzag_to_natural(i)
    assert J.zigzag_index(-1) == -1 and J.zigzag_index(64) == -1
    blk = np.arange(64, dtype=np.int32) * 3 - 50
    zz = J.zigzag_block(blk)
    assert [int(zz[p]) for p in range(64)] == [int(blk[J.zigzag_index(p)]) for p in range(64)]


def test_quantize_block_matches_oracle():
    rng = np.random.default_rng(1)
    q = rng.integers(1, 256, 64).astype(np.int32)
    for _ in range(200):
        # include exact half-integers: round half away from zero (std::round)
        b = np.where(rng.random(64) < 0.3, (rng.integers(-2000, 2000, 64) + 0.5) * q, rng.normal(0, 400, 64))
        want = np.zeros(64, np.int32)
        _oracle.orc().orc_quantize(_oracle._p(np.ascontiguousarray(b)), _oracle._p(q), _oracle._p(want))
        assert np.array_equal(J.quantize_block(b, q).reshape(64), want)


def _rle_vector_restated(data):
    """RLE_AC(const std::vector<int>&), Coding.hpp:112-144."""
    out = [(0, int(data[0]))]
    zeros = 0
    for v in data[1:]:
        if v == 0:
            zeros += 1
            continue
        while zeros > 15:
            out.append((15, 0))
            zeros -= 16
        out.append((zeros, int(v)))
        zeros = 0
    if zeros > 0:
        out.append((0, 0))
    return out


def _sparse(rng, n, p):
    return np.where(rng.random(n) < p, rng.integers(-300, 300, n), 0).astype(np.int32)


@pytest.mark.parametrize("p", [0.02, 0.1, 0.5, 1.0])
def test_rle_block_matches_oracle(p):
    rng = np.random.default_rng(int(p * 100))
    runs, vals, syms, nbits = (np.zeros(80, np.int32) for _ in range(4))
    bits = np.zeros(80, np.uint32)
    for _ in range(300):
        blk = _sparse(rng, 64, p)
        if rng.random() < 0.3:
            blk[63] = 5  # no EOB
        n = _oracle.orc().orc_rle_block(_oracle._p(blk), _oracle._p(runs), _oracle._p(vals), _oracle._p(syms),
                                        _oracle._p(nbits), _oracle._p(bits))
        pairs = J.rle_ac(blk, zigzag_scan=True)
        assert pairs == list(zip(runs[:n].tolist(), vals[:n].tolist()))
        coded = J.encode_category(pairs)
        assert coded == list(zip(syms[:n].tolist(), bits[:n].tolist(), nbits[:n].tolist()))


def test_rle_vector_matches_restatement():
    rng = np.random.default_rng(7)
    for n in (2, 3, 17, 64, 100, 300):
        for _ in range(30):
            d = _sparse(rng, n, 0.08)
            assert J.rle_ac(d) == _rle_vector_restated(d.tolist())


def test_category_code_matches_oracle():
    b = np.zeros(1, np.uint32)
    for v in list(range(-2100, 2100)) + [-32767, -16384, -16383, 16383, 16384, 32767]:
        c = _oracle.orc().orc_category(v, _oracle._p(b))
        assert J.category_code(v) == (c, int(b[0])), v
    with pytest.raises(J.JpgeError):
        J.category_code(32768)


def test_dc_difference_matches_restatement():
    rng = np.random.default_rng(3)
    H, W = 48, 64
    qy = rng.integers(-500, 500, (H, W)).astype(np.int32)
    qcb = rng.integers(-500, 500, (H // 2, W // 2)).astype(np.int32)
    qcr = rng.integers(-500, 500, (H // 2, W // 2)).astype(np.int32)
    wy, wcb, wcr = qy.copy(), qcb.copy(), qcr.copy()
    b = 0
    for h in range(0, H, 16):  # Image.cpp:640-659
        for w in range(0, W, 16):
            for (r, c) in ((h, w), (h, w + 8), (h + 8, w), (h + 8, w + 8)):
                t = int(wy[r, c])
                wy[r, c] = t - b
                b = t
    for p in (wcb, wcr):  # Image.cpp:661-677
        b = 0
        for h in range(0, H // 2, 8):
            for w in range(0, W // 2, 8):
                t = int(p[h, w])
                p[h, w] = t - b
                b = t
    J.dc_difference(qy, qcb, qcr)
    assert np.array_equal(qy, wy) and np.array_equal(qcb, wcb) and np.array_equal(qcr, wcr)


def test_facade_cpp_reference_unit_tests_cpu():
    """CodingTest.cpp:5-162, BitstreamGenericTest.cpp:11-221, DctTest.cpp:86-158 and
    ImageTest.cpp:7-45 through the facade header, as reference code calls them."""
    assert os.path.exists(FACADE), "run make"
    r = subprocess.run([FACADE, "cpu", PPM], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert ", 0 failed" in r.stdout
