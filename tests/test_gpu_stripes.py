"""Row stripes: several contexts, each encoding a stripe of whole MCU
rows with the exchanges done in-process (jpgenc_amd.stripes.encode_stripes_local),
must produce the single-device bytes — the oracle's."""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle
import jpgenc_amd as J
from jpgenc_amd import stripes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _encode_striped(rgb: np.ndarray, n: int, quality: int, restart: int = 0) -> bytes:
    h, w = rgb.shape[:2]
    dev = torch.from_numpy(rgb.reshape(-1)).cuda()
    stride = w * 3
    rows = stripes.stripe_rows((h + 15) // 16, n, stripes.restart_align(w, restart))
    ptrs = [(dev.data_ptr() + r0 * 16 * stride, stride) for r0, _ in rows]
    cap = J.max_jpeg_bytes(w, h)
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    encs = [J.Encoder(0, lanes=1) for _ in range(n)]
    try:
        for e in encs:
            e.set_restart(restart)
        total = stripes.encode_stripes_local(encs, ptrs, w, h, quality, out.data_ptr(), cap, rows=rows)
    finally:
        for e in encs:
            e.close()
    torch.cuda.synchronize()
    return out[:total].cpu().numpy().tobytes()


@pytest.mark.parametrize("w,h,n,kind,quality", [
    (512, 512, 2, 0, 90), (512, 512, 3, 0, 50), (512, 512, 5, 1, 100), (512, 512, 4, 2, 50),
    (1920, 1080, 4, 0, 90), (1920, 1080, 8, 1, 90), (300, 200, 5, 0, 75), (640, 48, 3, 1, 100),
    (33, 17, 2, 0, 90), (1000, 1000, 7, 0, 95),
])
def test_stripes_match_single_device(w, h, n, kind, quality):
    rgb = J.synth_rgb8(77 + n + kind, w, h, kind=kind)
    assert _encode_striped(rgb, n, quality) == _oracle.encode(rgb, quality)


# Restart intervals whose boundaries include every stripe start (SURVEY 8(e) "tiled
# with restart intervals"): the stripes share only the tables; the output equals the
# whole-frame restart encode, i.e. the oracle's restart variant.
@pytest.mark.parametrize("w,h,n,r,kind,quality", [
    (512, 512, 2, 32, 0, 90), (512, 512, 4, 16, 1, 100), (1920, 1080, 4, 120, 0, 90), (1920, 1080, 8, 240, 1, 90),
    (1000, 1000, 3, 63, 0, 75), (300, 200, 5, 19, 2, 50), (640, 48, 3, 40, 0, 90),
])
def test_restart_stripes_match_oracle(w, h, n, r, kind, quality):
    rgb = J.synth_rgb8(55 + n + kind, w, h, kind=kind)
    assert _encode_striped(rgb, n, quality, restart=r) == _oracle.encode(rgb, quality, restart=r)


def test_restart_stripe_must_start_an_interval():
    enc = J.Encoder(0, lanes=1)
    try:
        enc.set_restart(7)  # 1920 px: 120 MCUs per row, so row 1 is no interval start
        rgb = torch.zeros(1920 * 3 * 32, dtype=torch.uint8, device="cuda")
        with pytest.raises(J.JpgeError):
            enc.stripe_transform(rgb.data_ptr(), 1920 * 3, 1920, 1080, 1, 2, 90)
    finally:
        enc.close()


def test_16k_in_8_stripes_matches_oracle_hash():
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large_frames.json")) as f:
        g = next(fr for fr in json.load(f)["frames"] if fr["width"] == 16384 and fr["quality"] == 90 and not fr.get("restart"))
    rgb = J.synth_rgb8(g["seed"], 16384, 16384, kind=g["kind"])
    jpg = _encode_striped(rgb, 8, 90)
    assert len(jpg) == g["len"]
    assert hashlib.sha256(jpg).hexdigest() == g["sha256"]


def _gpu_rank(rank, world, port, w, h, quality, q, restart=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch as T
    import torch.distributed as dist

    import jpgenc_amd as JJ
    from jpgenc_amd import stripes as S

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rgb = JJ.synth_rgb8(91, w, h)
    r0, nr = S.stripe_rows((h + 15) // 16, world, S.restart_align(w, restart))[rank]
    part = np.ascontiguousarray(rgb[16 * r0:min(h, 16 * (r0 + nr))])
    dev = T.from_numpy(part.reshape(-1)).cuda()
    out = T.zeros(JJ.max_jpeg_bytes(w, h), dtype=T.uint8, device="cuda")
    enc = JJ.Encoder(0, lanes=1)
    enc.set_restart(restart)
    total = S.encode_stripe_dist(enc, dev.data_ptr(), w * 3, w, h, quality, out, restart=restart)
    T.cuda.synchronize()
    q.put((rank, out[:total].cpu().numpy().tobytes() if rank == 0 else b""))
    enc.close()
    dist.destroy_process_group()


# The torch.distributed driver end to end on the real kernels: 3 ranks sharing this
# box's GPU (gloo for the exchanges; RCCL needs one GPU per rank), each holding only
# its own stripe's rows.
@pytest.mark.timeout(300)
@pytest.mark.parametrize("restart", [0, 80])
def test_three_rank_striped_encode_matches_oracle(restart):
    import socket

    mp = pytest.importorskip("torch.multiprocessing")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    w, h, quality = 1280, 720, 90
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_rank, args=(r, 3, port, w, h, quality, q, restart)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert res[0] == _oracle.encode(J.synth_rgb8(91, w, h), quality, restart=restart)
