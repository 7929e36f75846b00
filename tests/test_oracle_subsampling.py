"""CPU checks of the oracle's subsampling variants.

The reference's writeJPEG hard-codes S420_m (Image.cpp:842), so the other modes of
applySubsampling (Image.cpp:237-319: S444, S422, S411, S420, S420_lm) have no
reference bytes: the oracle composes them from the pinned stages plus
`subsample_mode`, a restatement of Image::subsample (Image.cpp:198-235).  These
tests pin that composition:
  * the generic path reproduces the pinned 4:2:0 and 4:4:4 paths byte for byte;
  * subsample_mode matches the reference's mask arithmetic, written out per mode;
  * the luma of every 4:2:0 filter is the pinned luma;
  * every mode's file decodes (PIL) to the input, and restart intervals leave the
    decoded pixels unchanged.
"""
import io

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

MODES = [422, 411, 4200, 4201]


def synth(seed, w, h, kind=0):
    return J.synth_rgb8(seed, w, h, kind)


@pytest.mark.parametrize("mode", [420, 444])
@pytest.mark.parametrize("w,h,r", [(1, 1, 0), (37, 23, 0), (64, 48, 3), (250, 130, 0), (250, 130, 17)])
def test_generic_path_equals_pinned(mode, w, h, r):
    rgb = synth(w * 7 + h, w, h)
    assert _oracle.encode(rgb, 90, restart=r, subsampling=mode, generic=True) == \
        _oracle.encode(rgb, 90, restart=r, subsampling=mode)


def _mask_reference(p, mode):
    """Image::subsample's sums for each mask of applySubsampling, op by op."""
    if mode == 422:
        return (0.0 + 1 * p[:, 0::2]) + 0 * p[:, 1::2]
    if mode == 411:
        return (((0.0 + 1 * p[:, 0::4]) + 0 * p[:, 1::4]) + 0 * p[:, 2::4]) + 0 * p[:, 3::4]
    top = lambda r, a, b: (0.0 + a * r[:, 0::2]) + b * r[:, 1::2]
    if mode == 4200:  # scanline jump: even rows only
        return top(p[0::2], 1, 0)
    if mode == 4201:
        return (top(p[0::2], 1, 0) + top(p[1::2], 1, 0)) / 2
    return (top(p[0::2], 1, 1) + top(p[1::2], 1, 1)) / 4  # S420_m


@pytest.mark.parametrize("mode", MODES + [420])
def test_subsample_mode_matches_mask_arithmetic(mode):
    rng = np.random.default_rng(mode)
    p = rng.normal(0, 40, (16, 32))
    assert np.array_equal(_oracle.subsample_mode(p, mode), _mask_reference(p, mode))


@pytest.mark.parametrize("mode", [4200, 4201])
def test_420_filters_share_the_pinned_luma(mode):
    rgb = synth(11, 90, 70)
    y, cb, _ = _oracle.stage_coeffs_mode(rgb, mode, 90)
    y0, cb0, _ = _oracle.stage_coeffs(rgb, 90)
    assert np.array_equal(y, y0)
    assert cb.shape == cb0.shape and not np.array_equal(cb, cb0)


@pytest.mark.parametrize("mode", MODES)
def test_modes_decode(mode):
    Image = pytest.importorskip("PIL.Image")
    rgb = synth(21, 200, 120)
    data = _oracle.encode(rgb, 95, subsampling=mode)
    im = Image.open(io.BytesIO(data))
    assert im.size == (200, 120)
    dec = np.asarray(im.convert("RGB"), np.float64)
    assert 10 * np.log10(255 ** 2 / np.mean((dec - rgb) ** 2)) > 28
    # SOF0 declares Y as yh x yv
    sof = data.index(b"\xff\xc0")
    yh, yv = _oracle.SHAPES[mode]
    assert data[sof + 11] == (yh << 4) | yv


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("w,h,r", [(33, 17, 1), (200, 120, 7)])
def test_modes_restart_decode_equivalent(mode, w, h, r):
    Image = pytest.importorskip("PIL.Image")
    rgb = synth(w + r, w, h)
    a = np.asarray(Image.open(io.BytesIO(_oracle.encode(rgb, 90, subsampling=mode))).convert("RGB"))
    b = np.asarray(Image.open(io.BytesIO(_oracle.encode(rgb, 90, restart=r, subsampling=mode))).convert("RGB"))
    assert np.array_equal(a, b)
