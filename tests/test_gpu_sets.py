"""Frame sets (kernels.hpp FrameSet): a batch of small frames of one geometry runs
up to 4 frames per launch of each kernel; every frame's bytes must equal its own
encode and the oracle's, whatever the set size, the lane count, a short last set or
the frames' colour paths (maxval)."""
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


@pytest.mark.parametrize("lanes", [2, 4])
@pytest.mark.parametrize("nframes", [2, 5, 9])
def test_default_sets_bit_exact(lanes, nframes):
    enc = _encoder(JPGE_LANES=lanes)
    try:
        frames = [J.synth_rgb8(5000 + i, 320, 200, kind=i % 3) for i in range(nframes)]
        outs = enc.encode_batch(frames, quality=90)
        assert outs == [_oracle.encode(f, 90) for f in frames]
    finally:
        enc.close()


@pytest.mark.parametrize("set_size", [1, 2, 3, 4])
def test_forced_set_sizes_bit_exact(set_size):
    enc = _encoder(JPGE_LANES=3, JPGE_SET=set_size)
    try:
        frames = [J.synth_rgb8(6000 + i, 136, 72) for i in range(11)]
        for q in (50, 100):
            assert enc.encode_batch(frames, quality=q) == [_oracle.encode(f, q) for f in frames]
    finally:
        enc.close()


def test_set_members_with_own_maxval():
    # one colour path per set (maxval < 255: the scaled path), each frame its own maxval
    enc = _encoder(JPGE_LANES=2, JPGE_SET=4)
    try:
        frames = [J.synth_rgb8(7000 + i, 96, 64) for i in range(6)]
        for maxval in (255, 100):
            scaled = [(f.astype(np.uint32) * maxval // 255).astype(np.uint8) for f in frames]
            got = enc.encode_batch(scaled, quality=75, maxval=maxval)
            assert got == [_oracle.encode(f, 75, maxval) for f in scaled]
    finally:
        enc.close()


def test_sets_then_mixed_then_large():
    # set batches, a mixed-size batch (frame by frame) and a larger frame on the same
    # context: the slots resize and regroup between batches
    enc = _encoder(JPGE_LANES=4)
    try:
        small = [J.synth_rgb8(8000 + i, 200, 120) for i in range(8)]
        assert enc.encode_batch(small, quality=90) == [_oracle.encode(f, 90) for f in small]
        mixed = [J.synth_rgb8(8100 + i, 120 + 16 * i, 80) for i in range(5)]
        assert enc.encode_batch(mixed, quality=90) == [_oracle.encode(f, 90) for f in mixed]
        big = [J.synth_rgb8(8200 + i, 640, 480) for i in range(3)]
        assert enc.encode_batch(big, quality=90) == [_oracle.encode(f, 90) for f in big]
        assert enc.encode_batch(small, quality=50) == [_oracle.encode(f, 50) for f in small]
    finally:
        enc.close()


def test_1080p_sets_match_single_frames():
    # config 4's frame size in sets of 4 (a short last set) against frame-by-frame encodes
    enc = _encoder(JPGE_LANES=4)
    ref = _encoder(JPGE_LANES=4, JPGE_SET=1)
    try:
        frames = [J.synth_rgb8(9000 + i, 1920, 1080, kind=i % 3) for i in range(10)]
        assert enc.encode_batch(frames, quality=90) == ref.encode_batch(frames, quality=90)
    finally:
        enc.close()
        ref.close()


def test_sets_fall_back_with_restart_then_scaled_path():
    # restart intervals (no placement in the code kernel) launch frame by frame with the
    # same bytes as single encodes; then sets again, on both colour paths
    enc = _encoder(JPGE_LANES=4)
    try:
        frames = [J.synth_rgb8(9500 + i, 200, 136) for i in range(6)]
        enc.set_restart(4)
        got = enc.encode_batch(frames, quality=90)
        assert got == [enc.encode(f, quality=90) for f in frames]
        enc.set_restart(0)
        scaled = [f if i % 2 else (f.astype(np.uint32) * 200 // 255).astype(np.uint8) for i, f in enumerate(frames)]
        for maxval in (255, 200):
            got = enc.encode_batch(scaled, quality=75, maxval=maxval)
            assert got == [_oracle.encode(f, 75, maxval) for f in scaled]
    finally:
        enc.close()


def test_set_member_errors_stay_with_their_frame():
    # one member of a set with too small an output buffer: that frame reports
    # JPGE_E_NOSPACE, every other frame of the batch (its set included) is unaffected
    import ctypes

    enc = _encoder(JPGE_LANES=2)
    try:
        frames = [np.ascontiguousarray(J.synth_rgb8(9700 + i, 240, 160)) for i in range(7)]
        outs = [np.zeros(J.max_jpeg_bytes(240, 160), np.uint8) for _ in frames]
        arr = (J.Frame * len(frames))()
        for i, (f, o) in enumerate(zip(frames, outs)):
            arr[i].rgb, arr[i].width, arr[i].height = f.ctypes.data, 240, 160
            arr[i].stride, arr[i].maxval = 240 * 3, 255
            arr[i].out, arr[i].cap = o.ctypes.data, (100 if i == 2 else o.size)
        qy, qc = J.quality_tables(90)
        st = J.lib().jpge_encode_batch(enc._ctx, arr, len(frames), qy.ctypes.data_as(ctypes.c_void_p),
                                       qc.ctypes.data_as(ctypes.c_void_p), 0)
        assert st == 2 and arr[2].status == 2  # JPGE_E_NOSPACE
        for i, f in enumerate(frames):
            if i != 2:
                assert arr[i].status == 0
                assert outs[i][:arr[i].len].tobytes() == _oracle.encode(f, 90)
    finally:
        enc.close()
