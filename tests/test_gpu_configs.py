"""BASELINE.json's configs on the GPU against the oracle, and the quality sweep.

- config 1: 512x512 4:4:4 Q90 (seed 1), and the reference's own 4:2:0 at 512^2;
- config 4: the batch of 256 distinct 1920x1080 Q90 frames (seeds 1000+i) through
  the device batch path, every frame's SHA-256 against tests/golden/batch1080.json
  (tests/golden/make_batch.py, the oracle in the survey container);
- config 5 as the north star words it ("tiled with restart intervals"): 16384^2 Q90
  with one restart interval per MCU row, whole-frame and in 8 row stripes, against
  the oracle restart variant's hash (tests/golden/large_frames.json);
- quality: every Q from 1 to 100 on a 200x136 frame, and Q 1/5/97/100 at 1080p —
  the IJG scaling and the [1, 255] clamp (Image.cpp:850-871 tables, SURVEY 8(c)
  quality variant) change the tables' shape at the low and high ends.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_config1_512_s444_q90():
    rgb = J.synth_rgb8(1, 512, 512)  # 512^2 seed 1
    with J.Encoder(0) as enc:
        enc.set_subsampling(444)
        got = enc.encode(rgb, quality=90)
    assert got == _oracle.encode(rgb, 90, subsampling=444)


@pytest.mark.parametrize("quality", [50, 90, 100])
def test_config1_512_reference_420(encoder, quality):
    rgb = J.synth_rgb8(1, 512, 512)
    assert encoder.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)


@pytest.mark.timeout(240)
def test_config4_batch_256x1080p_matches_oracle_hashes():
    torch = pytest.importorskip("torch")
    with open(os.path.join(GOLDEN, "batch1080.json")) as f:
        g = json.load(f)
    W, H, Q, S0 = g["width"], g["height"], g["quality"], g["seed0"]
    B = len(g["frames"])
    assert (W, H, Q, B, S0) == (1920, 1080, 90, 256, 1000)
    ins = torch.empty((B, H * W * 3), dtype=torch.uint8, device="cuda")
    for i in range(B):
        ins[i].copy_(torch.from_numpy(J.synth_rgb8(S0 + i, W, H).reshape(-1)))
    cap = 4 << 20
    out = torch.empty(B * cap, dtype=torch.uint8, device="cuda")
    with J.Encoder(0) as enc:
        lens = enc.encode_batch_dev([(ins[i].data_ptr(), W, H, W * 3) for i in range(B)],
                                    [(out.data_ptr() + i * cap, cap) for i in range(B)], quality=Q)
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    bad = [i for i in range(B)
           if [lens[i], hashlib.sha256(host[i * cap:i * cap + lens[i]].tobytes()).hexdigest()] != g["frames"][i]]
    assert not bad, f"{len(bad)} frames differ, first {bad[:8]}"


def _golden_16k(quality, restart):
    with open(os.path.join(GOLDEN, "large_frames.json")) as f:
        return next(fr for fr in json.load(f)["frames"]
                    if fr["width"] == 16384 and fr["quality"] == quality and fr.get("restart", 0) == restart)


@pytest.mark.timeout(240)
def test_config5_16k_restart_whole_frame_matches_oracle_hash():
    torch = pytest.importorskip("torch")
    g = _golden_16k(90, 1024)
    src = torch.from_numpy(J.synth_rgb8(g["seed"], 16384, 16384).reshape(-1)).cuda()
    cap = J.max_jpeg_bytes(16384, 16384)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    with J.Encoder(0) as enc:
        enc.set_restart(1024)
        n = enc.encode_batch_dev([(src.data_ptr(), 16384, 16384, 16384 * 3)], [(out.data_ptr(), cap)], quality=90)[0]
    torch.cuda.synchronize()
    assert n == g["len"]
    assert hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest() == g["sha256"]


@pytest.mark.timeout(240)
def test_config5_16k_restart_in_8_stripes_matches_oracle_hash():
    from test_gpu_stripes import _encode_striped

    g = _golden_16k(90, 1024)
    jpg = _encode_striped(J.synth_rgb8(g["seed"], 16384, 16384), 8, 90, restart=1024)
    assert len(jpg) == g["len"]
    assert hashlib.sha256(jpg).hexdigest() == g["sha256"]


@pytest.mark.parametrize("quality", range(1, 101))
def test_quality_sweep_200x136(encoder, quality):
    rgb = J.synth_rgb8(200 + quality, 200, 136)
    assert encoder.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)


@pytest.mark.parametrize("quality", [1, 5, 97, 100])
def test_quality_extremes_1080p(encoder, quality):
    rgb = J.synth_rgb8(2, 1920, 1080)  # 1080p seed 2
    assert encoder.encode(rgb, quality=quality) == _oracle.encode(rgb, quality)
