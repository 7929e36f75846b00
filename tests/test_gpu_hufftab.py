"""Huffman tables on the GPU (hufftab.hip) against the host builder (huffman.cpp,
pinned to the reference's own Huffman.cpp by tests/test_host.py's golden cases):
every code, length, bits[] and huffval of every table, on the reference's golden
histograms, tie-heavy and skewed random histograms of 1..162 symbols, and the
histograms of real frames from the oracle."""
import gzip
import json
import os

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu


def _host_table(counts, first):
    bits, huffval, code, ln = J.huffman_table(counts, first)
    tab = np.where(ln > 0, (ln.astype(np.uint32) << 16) | (code & 0xFFFF), 0).astype(np.uint32)
    return bits, huffval, tab


def _check(cs, fs):
    cs = np.asarray(cs, np.uint32).reshape(-1, 4, 256)
    fs = np.asarray(fs, np.uint64).reshape(-1, 4, 256)
    tab, dht, ns = J.huffman_tables_device(cs, fs)
    bad = []
    for i in range(cs.shape[0]):
        for t in range(4):
            if not cs[i, t].any():
                assert ns[i, t] == 0
                continue
            bits, huffval, htab = _host_table(cs[i, t], fs[i, t])
            n = len(huffval)
            ok = (ns[i, t] == n and dht[i, t, 0] == [0x00, 0x10, 0x01, 0x11][t]
                  and dht[i, t, 1:17].tolist() == list(bits) and dht[i, t, 17:17 + n].tolist() == huffval
                  and np.array_equal(tab[i, t], htab))
            if not ok:
                bad.append((i, t, n))
    assert not bad, f"{len(bad)} tables differ, first {bad[:5]}"


def _random_sets(rng, nsets, alphabet=None):
    cs = np.zeros((nsets, 4, 256), np.uint32)
    fs = np.full((nsets, 4, 256), np.iinfo(np.uint64).max, np.uint64)
    for i in range(nsets):
        for t in range(4):
            n = int(rng.integers(1, 13 if t % 2 == 0 else 163))
            syms = rng.choice(alphabet if alphabet is not None else 256, n, replace=False)
            mode = int(rng.integers(5))
            for s in syms:
                cs[i, t, s] = [1 + rng.integers(3), 1 + rng.integers(1000), 2 ** int(rng.integers(22)),
                               1 + rng.integers(50), 1 + rng.integers(2)][mode]
                fs[i, t, s] = rng.integers(1 << 40)
    return cs, fs


def test_device_tables_equal_host_on_golden_cases(golden_dir):
    with gzip.open(os.path.join(golden_dir, "huffman_ref.json.gz"), "rt") as f:
        cases = json.load(f)
    rng = np.random.default_rng(11)
    cs = np.zeros((len(cases), 4, 256), np.uint32)
    fs = np.full((len(cases), 4, 256), np.iinfo(np.uint64).max, np.uint64)
    for i, c in enumerate(cases):
        fc = c["first_counts"]
        if any(s < 0 or s > 255 for s, _ in fc):
            continue
        keys = np.sort(rng.choice(1 << 40, size=len(fc), replace=False))
        t = 1 if len(fc) > 12 else 0
        for (s, n), k in zip(fc, keys):
            cs[i, t, s] = n
            fs[i, t, s] = k
    _check(cs, fs)


@pytest.mark.parametrize("seed", range(4))
def test_device_tables_equal_host_on_random_histograms(seed):
    cs, fs = _random_sets(np.random.default_rng(seed), 300)
    _check(cs, fs)


def test_device_tables_equal_host_on_jpeg_alphabets():
    # AC symbols run << 4 | size (sizes 1..10), EOB and ZRL; DC categories 0..11
    ac = np.array([0x00, 0xF0] + [(r << 4) | c for r in range(16) for c in range(1, 11)])
    cs, fs = _random_sets(np.random.default_rng(99), 200, alphabet=ac)
    _check(cs, fs)


def test_device_tables_equal_host_on_frame_histograms():
    sets_c, sets_f = [], []
    for seed, (w, h), q in [(3, (1920, 1080), 90), (4, (640, 480), 50), (5, (512, 512), 100), (6, (333, 211), 10)]:
        c, f = _oracle.stage_hist(J.synth_rgb8(seed, w, h), q)
        sets_c.append(c)
        sets_f.append(f)
    _check(np.stack(sets_c), np.stack(sets_f))
