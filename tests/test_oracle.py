"""Pins the TEST-ONLY oracle to the reference: its own unit-test known answers
(tests/golden/reference_kats.json) and the outputs of its own Huffman/Bitstream
code (tests/golden/*_ref.json*, and live oracle/_ref when built here)."""
import gzip
import json
import os

import numpy as np
import pytest

import _oracle
from _oracle import _p


@pytest.fixture(scope="module")
def kats(golden_dir):
    with open(os.path.join(golden_dir, "reference_kats.json")) as f:
        return json.load(f)


def test_arai_constants_match_glibc_cos():
    c = np.zeros(8)
    a = np.zeros(5)
    s = np.zeros(8)
    _oracle.orc().orc_arai_constants(_p(c), _p(a), _p(s))
    # SURVEY.md Appendix A.3 bit patterns (glibc cos at static init)
    assert c[1].hex() == "0x1.f6297cff75cb0p-1"
    assert a[1].hex() == "0x1.1517a7bdb3894p-1"
    assert a[3].hex() == "0x1.4e7ae9144f0fcp+0"
    assert s[0].hex() == "0x1.6a09e667f3bccp-2"
    assert s[7].hex() == "0x1.480d9d073b426p+0"


def test_dct_ramp_kat(kats):
    k = kats["dct_ramp"]
    x = np.array(k["input"], np.float64)
    y = np.zeros(64)
    _oracle.orc().orc_dct_arai(_p(x), _p(y))
    np.testing.assert_allclose(y, np.array(k["expected"]), atol=k["tol"], rtol=0)


def test_zigzag_kat(kats):
    k = kats["zigzag"]
    nat = [_oracle.orc().orc_zigzag_to_natural(i) for i in range(64)]
    assert [k["input"][n] for n in nat] == k["expected"]


def test_quantize_kat(kats):
    k = kats["quantize"]
    x = np.array(k["input"], np.float64)
    q = np.array(k["table"], np.int32)
    out = np.zeros(64, np.int32)
    _oracle.orc().orc_quantize(_p(x), _p(q), _p(out))
    assert out.tolist() == k["expected"]


def _rle(block_natural):
    b = np.array(block_natural, np.int32)
    runs, vals, syms, nb = (np.zeros(80, np.int32) for _ in range(4))
    bits = np.zeros(80, np.uint32)
    n = _oracle.orc().orc_rle_block(_p(b), _p(runs), _p(vals), _p(syms), _p(nb), _p(bits))
    return [[int(r), int(v)] for r, v in zip(runs[:n], vals[:n])], list(zip(syms[:n], bits[:n], nb[:n]))


def test_rle_matrix_kat(kats):
    for case in kats["rle_matrix"]["cases"]:
        pairs, _ = _rle(case["input"])
        assert pairs == case["pairs"]


def test_rle_vector_kat(kats):
    # RLE_AC(vector) takes already-zig-zag-ordered data: place it at natural positions.
    nat = [_oracle.orc().orc_zigzag_to_natural(i) for i in range(64)]
    for case in kats["rle_vector"]["cases"]:
        blk = [0] * 64
        for i, v in enumerate(case["input"]):
            blk[nat[i]] = v
        pairs, coding = _rle(blk)
        assert pairs == case["pairs"]
        if "coding" in case:
            assert [[int(s), int(b), int(n)] for s, b, n in coding] == case["coding"]


def test_category_kat(kats):
    for v, cat, off in kats["category"]["cases"]:
        b = np.zeros(1, np.uint32)
        c = _oracle.orc().orc_category(v, _p(b))
        assert (c, int(b[0]) if c else 0) == (cat, off), v


def _load_padded(golden_dir, name):
    with open(os.path.join(golden_dir, "ppm", name), "rb") as f:
        st, samples, mv = _oracle.parse_ppm(f.read())
    assert st == 0
    h, w = samples.shape[:2]
    H, W = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    yy = np.minimum(np.arange(H), h - 1)
    xx = np.minimum(np.arange(W), w - 1)
    return samples[yy][:, xx] * (255.0 / mv), samples, mv


def test_ppm_load_and_pad_kat(kats, golden_dir):
    k = kats["ppm_load"]
    img, _, _ = _load_padded(golden_dir, k["file"])
    for y, x, r, g, b in k["checks"]:
        assert img[y, x].tolist() == [r, g, b], (y, x)


def test_color_kat(kats, golden_dir):
    k = kats["color"]
    img, samples, mv = _load_padded(golden_dir, k["file"])
    for y, x, Y, Cb, Cr in k["checks"]:
        out = np.zeros(3)
        _oracle.orc().orc_ycc(*img[y, x].tolist(), _p(out))
        np.testing.assert_allclose(out, [Y, Cb, Cr], atol=k["tol"], rtol=0)


def test_s420m_kat(kats, golden_dir):
    # The oracle's S420_m routine is exercised on the RGB planes exactly as the
    # reference test does (applySubsampling averages whatever Cb/Cr hold).
    k = kats["s420m"]
    img, _, _ = _load_padded(golden_dir, k["file"])
    H, W = img.shape[:2]
    for ch, key in ((2, "B"), (1, "G")):
        p = np.ascontiguousarray(img[:, :, ch])
        sub = np.zeros((H // 2, W // 2))
        _oracle.orc().orc_subsample420m(_p(p), W, H, _p(sub))
        for y, x, v in k[key]:
            assert sub[y, x] == v


def test_oracle_stage_ycc_matches_reference_colour(golden_dir):
    # the whole-frame colour stage equals the per-pixel KAT routine
    img, samples, mv = _load_padded(golden_dir, "tester_p3.ppm")
    h, w = samples.shape[:2]
    Y = np.zeros(16 * 16)
    Cb = np.zeros(64)
    Cr = np.zeros(64)
    rgb = np.ascontiguousarray(samples, np.uint8)
    _oracle.orc().orc_stage_ycc(_p(rgb), w, h, mv, _p(Y), _p(Cb), _p(Cr))
    out = np.zeros(3)
    _oracle.orc().orc_ycc(*img[0, 3].tolist(), _p(out))
    assert Y.reshape(16, 16)[0, 3] == out[0]


def test_huffman_libstdcxx_kat(kats):
    for case in kats["huffman_libstdcxx"]["cases"]:
        got = {str(s): format(c, f"0{l}b") for s, l, c in _oracle.huffman(case["text"])}
        assert got == case["codes"]


def test_huffman_matches_reference_goldens(golden_dir):
    with gzip.open(os.path.join(golden_dir, "huffman_ref.json.gz"), "rt") as f:
        cases = json.load(f)
    for c in cases:
        order = [s for s, _ in c["first_counts"]]
        text = order + [s for s, n in c["first_counts"] for _ in range(n - 1)]
        assert [list(t) for t in _oracle.huffman(text)] == c["table"]


def test_bitpack_matches_reference_goldens(golden_dir):
    with gzip.open(os.path.join(golden_dir, "bitpack_ref.json.gz"), "rt") as f:
        cases = json.load(f)
    for c in cases:
        data, raw = _oracle.pack_bits(c["vals"], c["nbits"], True)
        assert raw == c["raw_bits"]
        assert data.hex() == c["bytes"]


def test_bitstream_kat(kats):
    k = kats["bitstream"]
    data, raw = _oracle.pack_bits([0x34000000 >> 26], [6], False)
    bits = [(data[0] >> (7 - i)) & 1 for i in range(6)]
    assert bits == k["push_back_0x34000000_6"]
    data, raw = _oracle.pack_bits([0b101100, 0b001100], [6, 6], False)
    assert raw == 12 and ((data[0] << 8) | data[1]) == k["append_101100_001100_u16"]
    data, raw = _oracle.pack_bits([0b1001], [4], True)
    assert [(data[0] >> (7 - i)) & 1 for i in range(8)] == k["fill_1001"]
    data, raw = _oracle.pack_bits([0], [8], True)
    assert raw == k["fill_aligned_size"]


@pytest.mark.skipif(_oracle.ref() is None, reason="reference not built in this container")
def test_huffman_live_reference_random():
    rng = np.random.default_rng(7)
    for _ in range(300):
        nsym = int(rng.integers(1, 120))
        text = rng.choice(rng.choice(256, nsym, replace=False), size=int(rng.integers(1, 2000)),
                          p=rng.dirichlet(np.ones(nsym) * 0.3))
        assert _oracle.huffman(text) == _oracle.huffman(text, lib=_oracle.ref(), fn="ref_huffman")


def test_oracle_encode_is_thread_count_invariant():
    import jpgenc_amd  # synth generator only (host code, no GPU)
    rgb = jpgenc_amd.synth_rgb8(3, 200, 136)
    _oracle.orc().orc_set_threads(1)
    a = _oracle.encode(rgb, 90)
    _oracle.orc().orc_set_threads(4)
    b = _oracle.encode(rgb, 90)
    assert a == b and a[:2] == b"\xff\xd8" and a[-2:] == b"\xff\xd9"


def test_oracle_output_decodes_with_pil():
    PIL = pytest.importorskip("PIL.Image")
    import io

    import jpgenc_amd
    rgb = jpgenc_amd.synth_rgb8(11, 96, 80)
    data = _oracle.encode(rgb, 90)
    im = PIL.open(io.BytesIO(data))
    im.load()
    assert im.size == (96, 80)
    dec = np.asarray(im.convert("RGB"), np.float64)
    psnr = 10 * np.log10(255 ** 2 / np.mean((dec - rgb) ** 2))
    assert psnr > 25


@pytest.mark.parametrize("w,h,r", [(64, 48, 1), (200, 136, 3), (333, 211, 7), (512, 512, 32), (100, 60, 1000)])
def test_oracle_restart_variant_decodes_to_reference_pixels(w, h, r):
    # The restart-interval variant changes the DC prediction and
    # the byte alignment only: DRI present, RSTn markers cycling 0..7 between the
    # intervals, and the decoded pixels identical to the reference-mode stream's.
    Image = pytest.importorskip("PIL.Image")
    import io

    import jpgenc_amd as J
    rgb = J.synth_rgb8(w * 7 + h, w, h)
    plain = _oracle.encode(rgb, 90)
    rst = _oracle.encode(rgb, 90, restart=r)
    nmcu = ((w + 15) // 16) * ((h + 15) // 16)
    nint = (nmcu + r - 1) // r
    assert rst.count(b"\xff\xdd\x00\x04") == 1
    body = rst[rst.index(b"\xff\xda"):]
    markers = [body[i + 1] for i in range(len(body) - 1) if body[i] == 0xFF and 0xD0 <= body[i + 1] <= 0xD7]
    assert markers == [0xD0 + (k & 7) for k in range(nint - 1)]
    a = np.asarray(Image.open(io.BytesIO(plain)).convert("RGB"))
    b = np.asarray(Image.open(io.BytesIO(rst)).convert("RGB"))
    assert np.array_equal(a, b)


@pytest.mark.parametrize("w,h", [(8, 8), (17, 9), (96, 80), (333, 211)])
def test_oracle_s444_luma_equals_s420_luma(w, h):
    # S444 changes only the chroma: the Y plane's coefficients are the S420_m path's
    # (pinned to the reference), cropped to whole 8x8 blocks.
    import jpgenc_amd as J
    rgb = J.synth_rgb8(w + 5 * h, w, h, kind=1)
    y420, _, _ = _oracle.stage_coeffs(rgb, 90)
    y444, cb, cr = _oracle.stage_coeffs444(rgb, 90)
    bw16, bw8, bh8 = (w + 15) // 16 * 2, (w + 7) // 8, (h + 7) // 8
    crop = y420.reshape(-1, bw16, 64)[:bh8, :bw8].reshape(-1, 64)
    assert np.array_equal(y444, crop)
    assert cb.shape == cr.shape == y444.shape


def test_oracle_s444_flat_chroma():
    # a flat frame: every chroma block is DC-only, DC = round(8 * c / q0) with c the
    # exact colour value (8 * c is the Arai DC of a constant block)
    rgb = np.zeros((24, 40, 3), np.uint8)
    rgb[...] = (200, 30, 90)
    _, cb, cr = _oracle.stage_coeffs444(rgb, 50)
    qy, qc = _oracle.quality_tables(50)
    c = {"cb": -.1687 * 200 - .3312 * 30 + .5 * 90, "cr": .5 * 200 - .4186 * 30 - .0813 * 90}
    for name, plane in (("cb", cb), ("cr", cr)):
        assert np.all(plane[:, 1:] == 0)
        assert np.all(plane[:, 0] == int(np.round(8 * c[name] / qc[0])))


@pytest.mark.parametrize("w,h,r", [(8, 8, 0), (17, 33, 0), (96, 80, 0), (333, 211, 0), (64, 48, 1), (200, 136, 7)])
def test_oracle_s444_decodes(w, h, r):
    # The S444 variant is a valid baseline JPEG with 1x1 sampling everywhere: it
    # decodes at full chroma resolution, closer to the input than the 4:2:0 stream.
    Image = pytest.importorskip("PIL.Image")
    import io

    import jpgenc_amd as J
    rgb = J.synth_rgb8(w * 3 + h, w, h)
    data = _oracle.encode(rgb, 90, restart=r, subsampling=444)
    sof = data.index(b"\xff\xc0")
    assert data[sof + 10:sof + 19] == bytes([1, 0x11, 0, 2, 0x11, 1, 3, 0x11, 1])
    assert (b"\xff\xdd" in data) == bool(r)
    im = Image.open(io.BytesIO(data))
    im.load()
    assert im.size == (w, h)
    dec = np.asarray(im.convert("RGB"), np.float64)
    d420 = np.asarray(Image.open(io.BytesIO(_oracle.encode(rgb, 90))).convert("RGB"), np.float64)
    mse444, mse420 = np.mean((dec - rgb) ** 2), np.mean((d420 - rgb) ** 2)
    assert 10 * np.log10(255 ** 2 / mse444) > 30
    assert mse444 <= mse420 * 1.05
