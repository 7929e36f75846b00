"""The encoder's tuning switches (read from the environment when a context opens,
encoder.cpp Encoder::open): every setting other than the default selects a different
host pipeline shape or kernel grid, never different bytes.  Each one runs a batch in
frame sets and single images (1-lane context, the table helper's size class) against
the oracle (no switch selects a product path that no test runs)."""
import os

import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu


def _encoder(lanes=0, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return J.Encoder(0, lanes=lanes) if lanes else J.Encoder(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


MODES = [
    {"JPGE_LOOKAHEAD": 1}, {"JPGE_LOOKAHEAD": 3}, {"JPGE_LOOKAHEAD": 8},
    {"JPGE_DRAIN_LAG": 0}, {"JPGE_DRAIN_LAG": 2}, {"JPGE_DRAIN_LAG": 4},
    {"JPGE_FDCT_WGS": 64}, {"JPGE_STATS_WGS": 16}, {"JPGE_ENTROPY_WGS": 24},
    {"JPGE_NAP_US": 200}, {"JPGE_NAP": 0}, {"JPGE_NAP": 1}, {"JPGE_FIRST_SLEEP": 0},
    {"JPGE_HIST_NAP_US": 50}, {"JPGE_CU_MASK_STREAMS": 0},
]


@pytest.mark.parametrize("env", MODES, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_batch_under_switch_bit_exact(env):
    frames = [J.synth_rgb8(9100 + i, 320 + 16 * (i // 7), 176, kind=i % 3) for i in range(11)]
    want = [_oracle.encode(f, 90) for f in frames]
    enc = _encoder(**env)
    try:
        assert enc.encode_batch(frames, quality=90) == want
    finally:
        enc.close()


@pytest.mark.parametrize("env", [{"JPGE_TABLE_HELPER": 0}, {"JPGE_TABLE_HELPER": 1}, {"JPGE_HIST_NAP_US": 30},
                                 {"JPGE_GATE": 0}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_single_images_under_switch_bit_exact(env):
    # 1280x832 (>= 1 MPix: the table helper's class) and a small frame, on a 1-lane context
    frames = [J.synth_rgb8(9200, 1280, 832), J.synth_rgb8(9201, 200, 136, kind=1), J.synth_rgb8(9202, 1280, 832, kind=2)]
    enc = _encoder(lanes=1, **env)
    try:
        for f in frames:
            assert enc.encode(f, quality=90) == _oracle.encode(f, 90)
    finally:
        enc.close()
