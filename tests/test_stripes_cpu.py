"""Row-stripe host logic on CPU (no GPU): the placement arithmetic of
jpge_stripe_place against a bit-level model of the reference's stream
(concatenate, 1-fill, 0xFF -> 0xFF 0x00; BitstreamGeneric.hpp:213-248), and the
torch.distributed orchestration of jpgenc_amd.stripes with two gloo ranks and a
stand-in engine whose stripes are random bit strings."""
import ctypes
import os
import random
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import jpgenc_amd as J  # noqa: E402
from jpgenc_amd import stripes  # noqa: E402


def _bits(rng, n, p1):
    return [1 if rng.random() < p1 else 0 for _ in range(n)]


def _byte(bits):
    v = 0
    for b in bits:
        v = (v << 1) | b
    return v


def _summary(bits):
    """(bits, ff[a], head, tail, restart=0) as the GPU computes it: 0xFF bytes wholly
    inside the stripe when it starts at bit a (mod 8)."""
    L = len(bits)
    ff = []
    for a in range(8):
        s = (-a) % 8
        c = 0
        while s + 8 <= L:
            c += all(bits[s:s + 8])
            s += 8
        ff.append(c)
    return (L, tuple(ff), _byte(bits[:8]), _byte(bits[-8:]), 0)


def _file(streams, hdr):
    allbits = [b for s in streams for b in s]
    allbits += [1] * ((-len(allbits)) % 8)
    raw = [_byte(allbits[i:i + 8]) for i in range(0, len(allbits), 8)]
    out = bytearray(hdr)
    for v in raw:
        out.append(v)
        if v == 0xFF:
            out.append(0)
    return bytes(out) + b"\xff\xd9", raw


def _expected_offsets(streams, hdr_len):
    _, raw = _file(streams, b"")
    offs, p = [], 0
    for r, s in enumerate(streams):
        j = p >> 3
        offs.append(0 if r == 0 else hdr_len + j + sum(1 for v in raw[:j] if v == 0xFF))
        p += len(s)
    return offs


def _random_streams(rng, n):
    p1 = rng.choice([0.5, 0.9, 0.97])
    return [_bits(rng, rng.randint(8, 200), p1) for _ in range(n)]


def test_stripe_rows_partition():
    assert stripes.stripe_rows(10, 3) == [(0, 4), (4, 3), (7, 3)]
    assert stripes.stripe_rows(1024, 8) == [(128 * i, 128) for i in range(8)]
    with pytest.raises(ValueError):
        stripes.stripe_rows(2, 3)


@pytest.mark.parametrize("seed", range(40))
def test_stripe_place_matches_bit_model(seed):
    rng = random.Random(seed)
    n = rng.randint(1, 6)
    streams = _random_streams(rng, n)
    hdr_len = rng.randint(20, 400)
    want_file, _ = _file(streams, b"\0" * hdr_len)
    want_off = _expected_offsets(streams, hdr_len)
    summaries = [_summary(s) for s in streams]
    for r in range(n):
        off, total = J.stripe_place(summaries, r, hdr_len)
        assert off == want_off[r]
        assert total == len(want_file)


def test_combine_stats_sum_and_min():
    c = [np.array([1, 0, 3], np.uint32), np.array([2, 5, 0], np.uint32)]
    f = [np.array([7, 2**64 - 1, 4], np.uint64), np.array([3, 9, 2**64 - 1], np.uint64)]
    counts, first = stripes.combine_stats(c, f)
    assert counts.tolist() == [3, 5, 3] and first.tolist() == [3, 9, 4]


class _FakeStripeEngine:
    """Stands in for a GPU context: its 'stripe' is a random bit string shared by
    every rank through a common seed, and pack writes this stripe's slice of the
    model file where the real kernels would."""

    def __init__(self, rank, n, seed):
        rng = random.Random(seed)
        self.streams = _random_streams(rng, n)
        self.rank, self.n = rank, n
        self.hdr = bytes(range(40))
        self.file, _ = _file(self.streams, self.hdr)
        self.counts = [np.arange(1024, dtype=np.uint32) * (r + 1) for r in range(n)]
        self.first = [np.full(1024, 1000 - r, np.uint64) for r in range(n)]
        self.log = {}

    def stripe_transform(self, rgb_ptr, stride, width, height, row0, rows, quality, maxval):
        self.log["rows"] = (row0, rows)
        return np.array([10 * self.rank + 1, 10 * self.rank + 2, 10 * self.rank + 3], np.int32)

    def stripe_stats(self, seed):
        self.log["seed"] = list(seed)
        return self.counts[self.rank], self.first[self.rank]

    def stripe_code(self, counts, first):
        self.log["counts_ok"] = bool((counts == sum(self.counts)).all())
        present = counts > 0  # (absent symbols: key ~0)
        self.log["first_ok"] = bool((first[present] == np.minimum.reduce(self.first)[present]).all())
        return _summary(self.streams[self.rank]), len(self.hdr)

    def stripe_pack(self, summaries, index, out_ptr, cap):
        offs = [J.stripe_place(summaries, r, len(self.hdr))[0] for r in range(self.n)]
        end = offs[index + 1] if index + 1 < self.n else len(self.file)
        seg = self.file[offs[index]:end]
        ctypes.memmove(out_ptr + offs[index], seg, len(seg))
        return offs[index], len(seg), len(self.file)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dist_worker(rank, world, port, seed, q, members=None):
    """members: the global ranks of a subgroup that encodes the image (the others
    only take part in creating the group); None = the whole world."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from jpgenc_amd import stripes as S

    dist.init_process_group("gloo", rank=rank, world_size=world)
    group = dist.new_group(members) if members else None
    if members and rank not in members:
        q.put((rank, None, None, {}))
        dist.destroy_process_group()
        return
    grank = members.index(rank) if members else rank
    n = len(members) if members else world
    eng = _FakeStripeEngine(grank, n, seed)
    out = torch.zeros(len(eng.file) + 64, dtype=torch.uint8)
    total = S.encode_stripe_dist(eng, 0, 0, 64, 16 * 4 * n, 90, out, group=group)
    ok_file = grank != 0 or bytes(out[:total].numpy().tobytes()) == eng.file
    q.put((rank, total == len(eng.file), ok_file, eng.log))
    dist.destroy_process_group()


def _run_ranks(world, seed, members=None):
    mp = pytest.importorskip("torch.multiprocessing")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_worker, args=(r, world, port, seed, q, members)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(240)
@pytest.mark.parametrize("seed", [1, 2])
def test_two_rank_stripe_orchestration(seed):
    for rank, ok_total, ok_file, log in _run_ranks(2, seed):
        assert ok_total and ok_file
        assert log["counts_ok"] and log["first_ok"]
        assert log["rows"] == stripes.stripe_rows(8, 2)[rank]
        assert log["seed"] == ([0, 0, 0] if rank == 0 else [1, 2, 3])


@pytest.mark.timeout(240)
def test_stripes_on_a_subgroup():
    """the image encoded by ranks [1, 2] of a 3-rank world.  The group's
    rank 0 (global rank 1) must end up with the whole file; peers of the segment
    gather are global ranks."""
    res = _run_ranks(3, 3, members=[1, 2])
    assert res[0][1] is None  # rank 0 is not in the group
    for rank, ok_total, ok_file, log in res[1:]:
        g = rank - 1
        assert ok_total and ok_file
        assert log["counts_ok"] and log["first_ok"]
        assert log["rows"] == stripes.stripe_rows(8, 2)[g]
        assert log["seed"] == ([0, 0, 0] if g == 0 else [1, 2, 3])
