"""Round trips of GPU streams through the decode-side utilities (SURVEY 8(f) rank
4): the entropy decode (jpge_decode_coeffs) of a GPU-encoded .jpg must give back
exactly the quantised coefficients K1 produced (jpge_fdct_quant) — a
size-independent property, checked here at sizes the CPU oracle is too slow for
(4K in every subsampling mode, 16384^2, restart intervals)."""
import numpy as np
import pytest

import jpgenc_amd as J

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    e = J.Encoder(0)
    yield e
    e.close()


def roundtrip(enc, rgb, quality, mode=420, restart=0):
    enc.set_subsampling(mode)
    enc.set_restart(restart)
    try:
        data = enc.encode(rgb, quality=quality)
        planes = enc.fdct_quant(rgb, quality=quality)
    finally:
        enc.set_subsampling(420)
        enc.set_restart(0)
    info, y, cb, cr = J.decode_coeffs(data)
    h, w = rgb.shape[:2]
    assert (info.width, info.height, info.restart) == (w, h, restart)
    assert (info.yh, info.yv) == J.SUBSAMPLING[mode]
    for got, want in zip((y, cb, cr), planes):
        assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", [420, 444, 422, 411, 4200, 4201])
def test_roundtrip_4k_modes(enc, mode):
    roundtrip(enc, J.synth_rgb8(3, 3840, 2160), 90, mode)


@pytest.mark.parametrize("kind,quality", [(1, 100), (2, 50), (0, 10)])
def test_roundtrip_1080p_stress(enc, kind, quality):
    roundtrip(enc, J.synth_rgb8(11 + kind, 1920, 1080, kind=kind), quality)


@pytest.mark.parametrize("mode,restart", [(420, 240), (444, 7), (422, 480), (411, 1)])
def test_roundtrip_restart(enc, mode, restart):
    roundtrip(enc, J.synth_rgb8(17, 1920, 1080), 90, mode, restart)


def test_roundtrip_16k(enc):
    roundtrip(enc, J.synth_rgb8(5, 16384, 16384), 90)
