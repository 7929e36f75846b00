"""GPU parity of the 4:4:4 mode (applySubsampling(S444)).  The
reference's writeJPEG hard-codes S420_m, so the bytes are pinned to the oracle's
S444 variant (oracle/jpge_oracle.cpp run_to_quant444 / dc_diff444), whose luma is
the pinned 4:2:0 luma (tests/test_oracle.py)."""
import io

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc444():
    e = J.Encoder(0)
    e.set_subsampling(444)
    yield e
    e.close()


# one MCU, ragged edges in both directions, exact multiples, a 16-MCU tile plus one,
# a single MCU row / column, frames over several K2/K3 tiles
SIZES = [(8, 8), (1, 1), (9, 7), (17, 33), (64, 48), (100, 60), (128, 8), (136, 16), (8, 1040), (1040, 8),
         (333, 211), (640, 480), (1920, 1080)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("quality", [50, 90])
def test_s444_bit_exact(enc444, w, h, quality):
    rgb = J.synth_rgb8(w * 13 + h, w, h)
    assert enc444.encode(rgb, quality=quality) == _oracle.encode(rgb, quality, subsampling=444)


@pytest.mark.parametrize("kind,quality", [(1, 100), (1, 50), (2, 90), (2, 10)])
def test_s444_stress_kinds(enc444, kind, quality):
    # random bytes: long codes, many 0xFF; flat: one-symbol tables
    rgb = J.synth_rgb8(77 + kind, 248, 152, kind=kind)
    assert enc444.encode(rgb, quality=quality) == _oracle.encode(rgb, quality, subsampling=444)


@pytest.mark.parametrize("maxval", [1, 15, 100, 254])
def test_s444_maxval(enc444, maxval):
    rgb = (J.synth_rgb8(5 + maxval, 120, 72).astype(np.uint32) * maxval // 255).astype(np.uint8)
    assert enc444.encode(rgb, quality=75, maxval=maxval) == _oracle.encode(rgb, 75, maxval=maxval, subsampling=444)


def test_s444_coefficients(enc444):
    rgb = J.synth_rgb8(9, 203, 117, kind=1)
    got = enc444.fdct_quant(rgb, quality=90)
    want = _oracle.stage_coeffs444(rgb, 90)
    for g, w in zip(got, want):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("w,h,r", [(8, 8, 1), (64, 48, 1), (100, 60, 7), (333, 211, 42), (640, 480, 80),
                                   (1920, 1080, 240), (130, 70, 5000)])
def test_s444_restart(enc444, w, h, r):
    rgb = J.synth_rgb8(w + 3 * r, w, h)
    enc444.set_restart(r)
    try:
        got = enc444.encode(rgb, quality=90)
    finally:
        enc444.set_restart(0)
    assert got == _oracle.encode(rgb, 90, restart=r, subsampling=444)


def test_s444_batch_and_mode_switch(enc444):
    frames = [J.synth_rgb8(300 + i, 160 + 8 * i, 96 + 24 * (i % 2)) for i in range(6)]
    outs = enc444.encode_batch(frames, quality=80)
    for f, o in zip(frames, outs):
        assert o == _oracle.encode(f, 80, subsampling=444)
    enc444.set_subsampling(420)
    try:
        assert enc444.encode(frames[0], quality=80) == _oracle.encode(frames[0], 80)
    finally:
        enc444.set_subsampling(444)
    assert enc444.encode(frames[1], quality=80) == outs[1]


def test_s444_decodes(enc444):
    Image = pytest.importorskip("PIL.Image")
    rgb = J.synth_rgb8(21, 320, 240)
    im = Image.open(io.BytesIO(enc444.encode(rgb, quality=95)))
    assert im.size == (320, 240)
    dec = np.asarray(im.convert("RGB"), np.float64)
    assert 10 * np.log10(255 ** 2 / np.mean((dec - rgb) ** 2)) > 32


def test_s444_rejects_bad_mode_and_stripes(enc444):
    with pytest.raises(J.JpgeError):
        enc444.set_subsampling(421)
    with pytest.raises(J.JpgeError):  # (rejected before the pointer is used)
        enc444.stripe_transform(16, 64 * 3, 64, 64, 0, 4)


# a single-lane encoder with one tile per entropy workgroup (the 512-group
# override and JPGE_ENTROPY_WGS), on flat 4:4:4 frames of 129 MCUs (387 blocks: a
# ragged last tile), where a workgroup's stream is shortest.  Balanced tiles keep
# every tile >= 64 blocks, so every workgroup codes >= 128 bits.
@pytest.mark.parametrize("wgs", [0, 4, 512])
@pytest.mark.parametrize("w,h", [(344, 24), (1032, 8), (8, 1032)])
def test_s444_single_lane_one_tile_per_workgroup(w, h, wgs):
    import os
    old = os.environ.get("JPGE_ENTROPY_WGS")
    if wgs:
        os.environ["JPGE_ENTROPY_WGS"] = str(wgs)
    try:
        e = J.Encoder(0, lanes=1)
    finally:
        if old is None:
            os.environ.pop("JPGE_ENTROPY_WGS", None)
        else:
            os.environ["JPGE_ENTROPY_WGS"] = old
    try:
        e.set_subsampling(444)
        for kind, q in [(2, 50), (2, 90), (0, 90)]:
            rgb = J.synth_rgb8(3 + w, w, h, kind=kind)
            assert e.encode(rgb, quality=q) == _oracle.encode(rgb, q, subsampling=444)
            frames = [rgb, J.synth_rgb8(4 + w, w, h, kind=kind)]
            assert e.encode_batch(frames, quality=q) == [_oracle.encode(f, q, subsampling=444) for f in frames]
    finally:
        e.close()
