"""Regenerates the golden fixtures under tests/golden/ (run in the build container,
where /root/reference and oracle/_ref/libref.so exist):

  reference_kats.json   known-answer data transcribed from the reference's own
                        unit tests (file:line cited per entry) — data only
  huffman_ref.json.gz   generateHuffmanCode outputs of the reference's own
                        src/Huffman.cpp (oracle/_ref) on seeded random texts
  bitpack_ref.json.gz   Bitstream push/fill/stuffing outputs of the reference's
                        own BitstreamGeneric.hpp (oracle/_ref)
  ppm/*.ppm             the reference's test images (src/test/res), data files

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle  # noqa: E402

REF = "/root/reference"

RAMP = list(range(1, 65))
KATS = {
    "dct_ramp": {
        "src": "src/test/DctTest.cpp:9-48 (dctArai of the ramp 1..64 vs true_dct, tolerance 1e-5 per unittest.hpp:12)",
        "input": RAMP,
        "expected": [
            260, -18.2216411837961, 7.69085915161152e-15, -1.90481782616726, 0, -0.568239222367164,
            1.85673764701218e-14, -0.143407824981022,
            -145.773129470369, 0, 0, 0, 0, 0, 0, 0,
            0, 0, 0, 0, 0, 0, 0, 0,
            -15.2385426093380, 0, 0, 0, 0, 0, 0, 0,
            0, 0, 0, 0, 0, 0, 0, 0,
            -4.54591377893732, 0, 0, 0, 0, 0, 0, 0,
            0, 0, 0, 0, 0, 0, 0, 0,
            -1.14726259984816, 0, 0, 0, 0, 0, 0, 0],
        "tol": 1e-5,
    },
    "zigzag": {
        "src": "src/test/DctTest.cpp:86-109 (zigzag of the ramp)",
        "input": RAMP,
        "expected": [1, 2, 9, 17, 10, 3, 4, 11, 18, 25, 33, 26, 19, 12, 5, 6, 13, 20, 27, 34, 41, 49, 42, 35, 28, 21,
                     14, 7, 8, 15, 22, 29, 36, 43, 50, 57, 58, 51, 44, 37, 30, 23, 16, 24, 31, 38, 45, 52, 59, 60, 53,
                     46, 39, 32, 40, 47, 54, 61, 62, 55, 48, 56, 63, 64],
    },
    "quantize": {
        "src": "src/test/DctTest.cpp:112-158 (quantize with the Annex K luma table)",
        "table": [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
                  14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                  49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99],
        "chroma_table": [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99,
                         99, 47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32,
        "input": [581, -144, 56, 17, 15, -7, 25, -9, -242, 133, -48, 42, -2, -7, 13, -4, 108, -18, -40, 71, -33, 12,
                  6, -10, -56, -93, 48, 19, -8, 7, 6, -2, -17, 9, 7, -23, -3, -10, 5, 3, 4, 9, -4, -5, 2, 2, -7, 3,
                  -9, 7, 8, -6, 5, 12, 2, -5, -9, -4, -2, -3, 6, 1, -1, -1],
        "expected": [36, -13, 6, 1, 1, 0, 0, 0, -20, 11, -3, 2, 0, 0, 0, 0, 8, -1, -3, 3, -1, 0, 0, 0,
                     -4, -5, 2, 1, 0, 0, 0, 0, -1, 0, 0, 0, 0, 0, 0, 0] + [0] * 24,
    },
    "rle_vector": {
        "src": "src/test/CodingTest.cpp:5-68 (RLE_AC(vector) on already zig-zag-ordered data + encode_category)",
        "cases": [
            {"input": [-111, 57] + [0] * 18 + [3] + [0] * 4 + [-2] + [0] * 37 + [-2],
             "pairs": [[0, -111], [0, 57], [15, 0], [2, 3], [4, -2], [15, 0], [15, 0], [5, -2]],
             "coding": [[7, 16, 7], [6, 57, 6], [240, 0, 0], [34, 3, 2], [66, 1, 2], [240, 0, 0], [240, 0, 0],
                        [82, 1, 2]]},
            {"input": [-111, 57] + [0] * 18 + [3] + [0] * 4 + [-2] + [0] * 38,
             "pairs": [[0, -111], [0, 57], [15, 0], [2, 3], [4, -2], [0, 0]]},
        ],
    },
    "rle_matrix": {
        "src": "src/test/CodingTest.cpp:70-131 (RLE_AC(matrix): natural-order block, zig-zag scan)",
        "cases": [
            {"input": [-111, 57] + [0] * 18 + [3] + [0] * 4 + [-2] + [0] * 37 + [-2],
             "pairs": [[0, -111], [0, 57], [9, -2], [13, 3], [15, 0], [15, 0], [5, -2]]},
            {"input": [-111, 57] + [0] * 18 + [3] + [0] * 4 + [-2] + [0] * 38,
             "pairs": [[0, -111], [0, 57], [9, -2], [13, 3], [0, 0]]},
        ],
    },
    "category": {
        "src": "src/test/CodingTest.cpp:133-162 (getCategoryAndCode: value -> (category, offset bits))",
        "cases": [[0, 0, 0], [-1, 1, 0], [1, 1, 1], [-3, 2, 0], [-2, 2, 1], [2, 2, 2], [3, 2, 3], [-7, 3, 0],
                  [-6, 3, 1], [-4, 3, 3], [4, 3, 4], [6, 3, 6], [7, 3, 7], [-1023, 10, 0], [-1022, 10, 1],
                  [-512, 10, 511], [512, 10, 512], [1022, 10, 1022], [1023, 10, 1023]],
    },
    "ppm_load": {
        "src": "src/test/ImageTest.cpp:7-45 (tester_p3.ppm, maxval 15, padded to 16x16 by edge replication)",
        "file": "tester_p3.ppm",
        "checks": [[0, 0, 0, 0, 0], [0, 3, 255, 0, 255], [2, 2, 0, 255, 119], [15, 0, 255, 0, 255],
                   [0, 15, 255, 0, 255], [1, 15, 0, 0, 0], [15, 1, 0, 0, 0], [15, 15, 0, 0, 0]],
    },
    "color": {
        "src": "src/test/ImageTest.cpp:47-73 (convertToColorSpace(YCbCr) of tester_p3, tolerance 1e-5)",
        "file": "tester_p3.ppm",
        "checks": [[0, 3, -22.685, 84.4815, 106.7685], [1, 1, 35.251, -24.956, -116.417698]],
        "tol": 1e-5,
    },
    "s420m": {
        "src": "src/test/ImageTest.cpp:154-175 (S420_m of the RGB planes of tester_p3: exact 2x2 means)",
        "file": "tester_p3.ppm",
        "B": [[0, 0, 29.75], [1, 0, 63.75], [0, 1, 63.75], [1, 1, 29.75]],
        "G": [[0, 0, 63.75], [1, 0, 0], [0, 1, 0], [1, 1, 63.75]],
    },
    "segments": {
        "src": "src/test/ImageTest.cpp:302,319 (sizeof(sAPP0)==18, sizeof(sSOF0)==19)",
        "app0_bytes": 18, "sof0_bytes": 19,
    },
    "bitstream": {
        "src": "src/test/BitstreamGenericTest.cpp:52-68,104-127",
        "push_back_0x34000000_6": [0, 0, 1, 1, 0, 1],
        "append_101100_001100_u16": 0xB0C0,
        "fill_1001": [1, 0, 0, 1, 1, 1, 1, 1],
        "fill_aligned_size": 8,
    },
    "huffman_libstdcxx": {
        "src": "HuffmanTest.cpp:13-48 texts; expected values = the reference built here with libstdc++ "
               "(SURVEY.md Appendix C.2; the file's own expectations are MSVC hash order)",
        "cases": [
            {"text": [5, 5, 5, 5, 5, 4, 4, 4, 4, 2, 2, 1],
             "codes": {"5": "0", "4": "10", "2": "110", "1": "1110"}},
            {"text": [2, 2, 22, 22, 5, 5, 5, 5, 5, 3, 3, 3, 33, 33, 33, 7, 7, 7, 7, 7, 7, 7],
             "codes": {"5": "00", "7": "01", "33": "100", "3": "101", "22": "110", "2": "1110"}},
            {"text": [123], "codes": {"123": "0"}},
        ],
    },
}


def rand_text(rng, kind):
    nsym = int(rng.integers(1, 180))
    n = int(rng.integers(nsym, 6000))
    alpha = rng.choice(256, size=nsym, replace=False)
    if kind == 0:
        p = rng.dirichlet(np.ones(nsym) * rng.uniform(0.05, 3))
    else:  # heavy-tailed, JPEG-like
        p = 1.0 / (np.arange(1, nsym + 1) ** rng.uniform(0.5, 2.5))
        p /= p.sum()
    text = rng.choice(alpha, size=n, p=p)
    return text.astype(np.int32)


def main():
    ref = _oracle.ref()
    if ref is None:
        sys.exit("oracle/_ref/libref.so is missing: run `make oracle` here (needs /root/reference)")
    with open(os.path.join(HERE, "reference_kats.json"), "w") as f:
        json.dump(KATS, f, indent=1)

    # Huffman: store each text as its first-occurrence (symbol, count) list (the
    # table depends on nothing else), plus the reference output.
    rng = np.random.default_rng(20261015)
    cases = []
    for i in range(600):
        text = rand_text(rng, i % 2)
        order = []
        seen = {}
        for s in text.tolist():
            if s not in seen:
                seen[s] = 0
                order.append(s)
            seen[s] += 1
        fc = [[s, seen[s]] for s in order]
        # canonical text that has the same first-occurrence order and counts
        canon = [s for s in order] + [s for s in order for _ in range(seen[s] - 1)]
        out = _oracle.huffman(canon, lib=ref, fn="ref_huffman")
        cases.append({"first_counts": fc, "table": out})
    with gzip.open(os.path.join(HERE, "huffman_ref.json.gz"), "wt") as f:
        json.dump(cases, f)

    # package_merge directly (PackageMergeTest.cpp:15-44 inputs)
    import ctypes
    syms = np.array([0, 4, 1, 9, 7], np.int32)
    freqs = np.array([6, 20, 3, 24, 1], np.int32)
    pm = {}
    for limit in (5, 3):
        os_ = np.zeros(64, np.int32)
        ol = np.zeros(64, np.int32)
        k = ref.ref_package_merge(syms.ctypes.data, freqs.ctypes.data, 5, limit, os_.ctypes.data, ol.ctypes.data)
        pm[str(limit)] = list(zip(os_[:k].tolist(), ol[:k].tolist()))
    with open(os.path.join(HERE, "package_merge_ref.json"), "w") as f:
        json.dump({"src": "PackageMergeTest.cpp:15-44 inputs; outputs from the reference built here",
                   "symbols": syms.tolist(), "freqs": freqs.tolist(), "result": pm}, f)

    # Bitstream: random pushes in both modes, with fill, through the reference class
    bp = []
    for i in range(300):
        n = int(rng.integers(1, 400))
        nb = rng.integers(1, 17, size=n).astype(np.int32)
        if i % 5 == 0:
            vals = ((1 << nb) - 1).astype(np.uint32)  # all ones: lots of 0xFF stuffing
        else:
            vals = (rng.integers(0, 1 << 16, size=n) & ((1 << nb) - 1)).astype(np.uint32)
        modes = rng.integers(0, 2, size=n).astype(np.int32)
        data, raw = _oracle.pack_bits(vals, nb, True, modes, lib=ref)
        bp.append({"vals": vals.tolist(), "nbits": nb.tolist(), "modes": modes.tolist(), "raw_bits": raw,
                   "bytes": data.hex()})
    with gzip.open(os.path.join(HERE, "bitpack_ref.json.gz"), "wt") as f:
        json.dump(bp, f)

    # reference test images
    dst = os.path.join(HERE, "ppm")
    os.makedirs(dst, exist_ok=True)
    res = os.path.join(REF, "src", "test", "res")
    for fn in sorted(os.listdir(res)):
        if fn.endswith(".ppm"):
            shutil.copyfile(os.path.join(res, fn), os.path.join(dst, fn))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
