"""GPU parity of the subsampling modes beyond 4:2:0 S420_m and 4:4:4 (SURVEY 8(f)
rank 3): S422, S411 (MCUs one block row high, fdct_row8_kernel) and the S420 /
S420_lm chroma filters of the 4:2:0 kernel.  writeJPEG hard-codes S420_m
(Image.cpp:842), so the bytes are pinned to the oracle's generic subsampling path
(oracle/jpge_oracle.cpp encode_frame_mode), which tests/test_oracle_subsampling.py
checks against the pinned 4:2:0 / 4:4:4 paths and Image::subsample's arithmetic."""
import io

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu

MODES = [422, 411, 4200, 4201]


@pytest.fixture(scope="module")
def enc():
    e = J.Encoder(0)
    yield e
    e.close()


def encode(enc, mode, rgb, **kw):
    enc.set_subsampling(mode)
    try:
        return enc.encode(rgb, **kw)
    finally:
        enc.set_subsampling(420)


# one MCU, ragged edges, a tile (128 px across) plus one MCU, a single MCU row or
# column, frames over several K2/K3 tiles
SIZES = [(1, 1), (8, 8), (9, 7), (17, 33), (32, 8), (100, 60), (128, 16), (160, 8), (8, 1040), (1040, 8),
         (333, 211), (1920, 1080)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("mode", MODES)
def test_modes_bit_exact(enc, mode, w, h):
    rgb = J.synth_rgb8(w * 13 + h + mode, w, h)
    assert encode(enc, mode, rgb, quality=90) == _oracle.encode(rgb, 90, subsampling=mode)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("kind,quality", [(1, 100), (1, 50), (2, 90), (0, 10)])
def test_modes_stress(enc, mode, kind, quality):
    rgb = J.synth_rgb8(77 + kind, 248, 152, kind=kind)
    assert encode(enc, mode, rgb, quality=quality) == _oracle.encode(rgb, quality, subsampling=mode)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("maxval", [1, 100, 254])
def test_modes_maxval(enc, mode, maxval):
    rgb = (J.synth_rgb8(5 + maxval, 120, 72).astype(np.uint32) * maxval // 255).astype(np.uint8)
    got = encode(enc, mode, rgb, quality=75, maxval=maxval)
    assert got == _oracle.encode(rgb, 75, maxval=maxval, subsampling=mode)


@pytest.mark.parametrize("mode", MODES)
def test_modes_coefficients(enc, mode):
    rgb = J.synth_rgb8(9, 203, 117, kind=1)
    enc.set_subsampling(mode)
    try:
        got = enc.fdct_quant(rgb, quality=90)
    finally:
        enc.set_subsampling(420)
    for g, w in zip(got, _oracle.stage_coeffs_mode(rgb, mode, 90)):
        assert np.array_equal(g, w)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("w,h,r", [(64, 48, 1), (333, 211, 42), (1920, 1080, 120)])
def test_modes_restart(enc, mode, w, h, r):
    rgb = J.synth_rgb8(w + 3 * r, w, h)
    enc.set_restart(r)
    try:
        got = encode(enc, mode, rgb, quality=90)
    finally:
        enc.set_restart(0)
    assert got == _oracle.encode(rgb, 90, restart=r, subsampling=mode)


@pytest.mark.parametrize("mode", MODES)
def test_modes_batch(enc, mode):
    frames = [J.synth_rgb8(300 + i, 160 + 8 * i, 96 + 24 * (i % 2)) for i in range(6)]
    enc.set_subsampling(mode)
    try:
        outs = enc.encode_batch(frames, quality=80)
    finally:
        enc.set_subsampling(420)
    for f, o in zip(frames, outs):
        assert o == _oracle.encode(f, 80, subsampling=mode)


@pytest.mark.parametrize("mode", MODES)
def test_modes_decode(enc, mode):
    Image = pytest.importorskip("PIL.Image")
    rgb = J.synth_rgb8(21, 320, 240)
    im = Image.open(io.BytesIO(encode(enc, mode, rgb, quality=95)))
    assert im.size == (320, 240)
    dec = np.asarray(im.convert("RGB"), np.float64)
    assert 10 * np.log10(255 ** 2 / np.mean((dec - rgb) ** 2)) > 28


def test_modes_4k(enc):
    rgb = J.synth_rgb8(3, 3840, 2160)
    for mode in MODES:
        assert encode(enc, mode, rgb, quality=90) == _oracle.encode(rgb, 90, subsampling=mode)


def test_unknown_mode_and_stripes_rejected(enc):
    with pytest.raises(J.JpgeError):
        enc.set_subsampling(421)
    enc.set_subsampling(422)
    try:
        with pytest.raises(J.JpgeError):
            enc.stripe_transform(16, 64 * 3, 64, 64, 0, 4)
    finally:
        enc.set_subsampling(420)
