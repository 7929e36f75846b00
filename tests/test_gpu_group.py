"""Device groups (jpge_group_*, group.cpp): the C-ABI multi-device path of SURVEY
8(e).  On this one-GPU box a group is either one member (a real single-process RCCL
clique: every collective and the init run, with one rank) or N members on the same
device (the exchanges through host memory and device copies).  Both must give the
single-device bytes — the oracle's."""
import os
import subprocess

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_one_member_group_uses_rccl():
    with J.Group([0]) as g:
        assert g.size() == (1, True)
        rgb = J.synth_rgb8(12, 640, 480)
        assert g.encode_striped(rgb, quality=90) == _oracle.encode(rgb, 90)


@pytest.mark.parametrize("n,w,h,quality,kind", [(2, 640, 480, 90, 0), (3, 1920, 1080, 75, 0), (4, 333, 211, 100, 1),
                                                (5, 512, 512, 50, 2), (8, 1920, 1080, 90, 1)])
def test_striped_group_matches_oracle(n, w, h, quality, kind):
    rgb = J.synth_rgb8(40 + n, w, h, kind=kind)
    with J.Group([0] * n, lanes=1) as g:
        assert g.size() == (n, False)
        assert g.encode_striped(rgb, quality=quality) == _oracle.encode(rgb, quality)


@pytest.mark.parametrize("n,restart", [(1, 120), (3, 120), (2, 37), (4, 60)])
def test_striped_group_restart_matches_oracle(n, restart):
    rgb = J.synth_rgb8(9, 1920, 1080)
    with J.Group([0] * n, lanes=1) as g:
        g.set_restart(restart)
        assert g.encode_striped(rgb, quality=90) == _oracle.encode(rgb, 90, restart=restart)


def test_group_batch_matches_oracle():
    frames = [J.synth_rgb8(1000 + i, 1920 if i % 3 else 640, 1080 if i % 3 else 480) for i in range(7)]
    with J.Group([0, 0, 0]) as g:
        outs = g.encode_batch(frames, quality=90)
    for f, o in zip(frames, outs):
        assert o == _oracle.encode(f, 90)


def test_group_rejects_more_stripes_than_rows():
    with J.Group([0] * 3, lanes=1) as g:
        with pytest.raises(J.JpgeError):
            g.encode_striped(J.synth_rgb8(1, 64, 32), quality=50)  # 2 MCU rows, 3 stripes


def test_cli_stripes_over_a_group(tmp_path):
    """jpgenc --devices 0,0,0: the CLI row-stripes one image over a device group."""
    rgb = J.synth_rgb8(77, 700, 500)
    ppm = tmp_path / "in.ppm"
    with open(ppm, "wb") as f:
        f.write(b"P6\n700 500\n255\n" + rgb.tobytes())
    out = tmp_path / "out.jpg"
    r = subprocess.run([os.path.join(ROOT, "jpgenc_amd", "bin", "jpgenc"), "--devices", "0,0,0", "-q", "90", str(ppm),
                        str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == _oracle.encode(rgb, 90)
