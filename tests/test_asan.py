"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer ("run the
host under -fsanitize=address,undefined in CI here").  `make asan` rebuilds every
host .cpp of libjpge sanitized (the HIP device objects are linked unsanitized; no GPU
is touched) and the host tests; these tests run them and fail on any sanitizer report:

- tests/cpp/test_host_asan.cpp: PPM tokenizer on the reference's test images, every
  prefix and random corruptions; the per-frame Huffman builder on 3000 histograms of
  1..256 symbols with heavy ties and 15-bit-limited depths (heap_pop's look-ahead at
  every heap size, the hash-order emulation); huffman text/decode round trips; the
  .jpg decode utility on oracle streams, truncations and corruptions; stripe
  placement on random summaries; coding primitives;
- tests/cpp/test_facade.cpp (cpu mode): the reference's own unit tests through the
  C++ facade;
- tests/cpp/test_huffman_fast.cpp, tests/cpp/test_quant_fast.cpp: the fast table
  builder against the standard containers, K1's quantiser against the reference's
  roundings.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import _oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "bin", "asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def asan_bins():
    if not shutil.which("g++"):
        pytest.skip("no host compiler")
    r = subprocess.run(["make", "-s", "-j8", "asan"], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return BIN


def _run(args, timeout=300):
    r = subprocess.run(args, cwd=ROOT, env=ENV, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_host_entry_points_sanitized(asan_bins, golden_dir, tmp_path):
    jpgs = []
    rng = np.random.default_rng(7)
    for i, (w, h, q, rst) in enumerate([(64, 48, 90, 0), (33, 17, 50, 2), (200, 136, 100, 0), (96, 64, 10, 5)]):
        rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        p = tmp_path / f"s{i}.jpg"
        p.write_bytes(_oracle.encode(rgb, q, restart=rst))
        jpgs.append(str(p))
    out = _run([os.path.join(asan_bins, "test_host_asan"), os.path.join(golden_dir, "ppm")] + jpgs)
    assert ", 0 failed" in out


def test_facade_cpu_sanitized(asan_bins, golden_dir):
    out = _run([os.path.join(asan_bins, "test_facade"), "cpu", os.path.join(golden_dir, "ppm")])
    assert ", 0 failed" in out


def test_huffman_fast_sanitized(asan_bins):
    out = _run([os.path.join(asan_bins, "test_huffman_fast"), "1500"])
    assert "0 mismatches" in out


def test_quant_fast_sanitized(asan_bins):
    out = _run([os.path.join(asan_bins, "test_quant_fast"), "300"])
    assert "0 mismatches" in out
