"""GPU parity of the restart-interval mode (DRI + RSTn every R MCUs; SURVEY 8(f)
rank 2).  The reference never emits restart markers, so the bytes are pinned to
the oracle's restart variant (oracle/jpge_oracle.cpp encode_frame, restart > 0),
and the decoded pixels to those of the reference-mode stream (restart intervals
change only the DC prediction and the byte alignment, never a coefficient)."""
import io
import os

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu


def _encoder(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return J.Encoder(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def renc():
    e = J.Encoder(0)
    yield e
    e.close()


# (w, h, restart MCUs): intervals of one MCU, ragged last intervals, whole MCU
# rows, one interval larger than the frame (DRI but no marker)
CASES = [(16, 16, 1), (17, 33, 1), (64, 48, 2), (100, 60, 7), (200, 136, 13), (333, 211, 21), (512, 512, 32),
         (512, 512, 33), (640, 480, 40), (1040, 16, 65), (16, 1040, 1), (130, 70, 1000)]


@pytest.mark.parametrize("w,h,r", CASES)
@pytest.mark.parametrize("quality", [50, 90])
def test_restart_bit_exact(renc, w, h, r, quality):
    rgb = J.synth_rgb8(w * 31 + h + r, w, h)
    renc.set_restart(r)
    try:
        got = renc.encode(rgb, quality=quality)
    finally:
        renc.set_restart(0)
    assert got == _oracle.encode(rgb, quality, restart=r)


@pytest.mark.parametrize("kind,quality", [(1, 100), (1, 50), (2, 90)])
@pytest.mark.parametrize("r", [1, 5, 30])
def test_restart_stress_kinds(renc, kind, quality, r):
    # random bytes: long codes and many 0xFF (stuffed fill bytes); flat: one-symbol tables
    rgb = J.synth_rgb8(91 + kind, 240, 160, kind=kind)
    renc.set_restart(r)
    try:
        got = renc.encode(rgb, quality=quality)
    finally:
        renc.set_restart(0)
    assert got == _oracle.encode(rgb, quality, restart=r)


# Workgroups per interval from one to one per tile, and placement across many
# segments: every partition must give the same bytes.
@pytest.mark.parametrize("wgs", [1, 7, 100000])
@pytest.mark.parametrize("w,h,r,kind", [(1920, 1080, 120, 0), (1920, 1080, 37, 1), (500, 300, 3, 0)])
def test_restart_partitions(wgs, w, h, r, kind):
    enc = _encoder(JPGE_ENTROPY_WGS=wgs)
    try:
        enc.set_restart(r)
        rgb = J.synth_rgb8(7 + w + r, w, h, kind=kind)
        assert enc.encode(rgb, quality=90) == _oracle.encode(rgb, 90, restart=r)
    finally:
        enc.close()


def test_restart_4k_rows(renc):
    # one interval per MCU row of a 4K frame (240 MCUs): 135 intervals
    rgb = J.synth_rgb8(3, 3840, 2160)
    renc.set_restart(240)
    try:
        got = renc.encode(rgb, quality=90)
    finally:
        renc.set_restart(0)
    assert got == _oracle.encode(rgb, 90, restart=240)


def test_restart_batch_matches_single(renc):
    frames = [J.synth_rgb8(500 + i, 320 + 16 * (i % 3), 200 + 8 * i) for i in range(5)]
    renc.set_restart(9)
    try:
        outs = renc.encode_batch(frames, quality=90)
        for f, o in zip(frames, outs):
            assert o == _oracle.encode(f, 90, restart=9)
    finally:
        renc.set_restart(0)


def test_restart_decodes_to_reference_pixels(renc):
    Image = pytest.importorskip("PIL.Image")
    rgb = J.synth_rgb8(42, 640, 480, kind=1)
    plain = renc.encode(rgb, quality=75)
    renc.set_restart(4)
    try:
        rst = renc.encode(rgb, quality=75)
    finally:
        renc.set_restart(0)
    assert rst != plain and rst.count(b"\xff\xdd") == 1
    a = np.asarray(Image.open(io.BytesIO(plain)).convert("RGB"))
    b = np.asarray(Image.open(io.BytesIO(rst)).convert("RGB"))
    assert np.array_equal(a, b)


def test_restart_rejects_bad_interval(renc):
    with pytest.raises(J.JpgeError):
        renc.set_restart(65536)
