"""One image in row stripes across devices.

The image is cut into stripes of whole MCU rows (16 px); each stripe runs on its
own encoder context (one per GPU) through the four jpge_stripe_* phases, with the
three small exchanges of 8(e) between them and a gather of the stuffed segments:

    transform  -> all-gather last DCs      (stripe r's DC chain starts at r-1's last DC)
    stats      -> all-reduce counts (sum), first-occurrence keys (min)
    code       -> all-gather stripe summaries (bits, 0xFF counts per alignment, edge bits)
    pack       -> every stripe's bytes at their global offsets; segments to rank 0

The result is byte-identical to the single-device encode (no restart markers, as
in the reference: Image.cpp:638-678 DC chain, :888-906 texts, :957-972 stream).

Two drivers: `encode_stripes_local` (all stripes in one process, e.g. several
contexts on one GPU; the exchanges are plain array operations) and
`encode_stripe_dist` (one rank per GPU; the exchanges are torch.distributed
collectives: RCCL over xGMI with the "nccl" backend, gloo on CPU).
"""
from __future__ import annotations

import numpy as np

import jpgenc_amd as J


def stripe_rows(mcu_rows: int, n: int, align: int = 1) -> list[tuple[int, int]]:
    """Split mcu_rows MCU rows into n contiguous stripes (first rows0, count), as even as
    possible, every stripe starting at a multiple of `align` rows."""
    units = (mcu_rows + align - 1) // align
    if n < 1 or n > units:
        raise ValueError(f"cannot cut {mcu_rows} MCU rows into {n} stripes of whole {align}-row units")
    base, extra = divmod(units, n)
    out, u0 = [], 0
    for r in range(n):
        c = base + (1 if r < extra else 0)
        r0 = u0 * align
        out.append((r0, min(mcu_rows, (u0 + c) * align) - r0))
        u0 += c
    return out


def restart_align(width: int, restart: int) -> int:
    """MCU rows between possible stripe starts when every stripe must begin a restart
    interval of `restart` MCUs (1 without restart intervals)."""
    import math
    if not restart:
        return 1
    mw = (width + 15) // 16
    return restart // math.gcd(restart, mw)


def combine_stats(all_counts: list[np.ndarray], all_first: list[np.ndarray]) -> tuple[np.ndarray, np.ndarray]:
    """Whole-image histograms from the stripes': counts add, first-occurrence keys take the minimum."""
    counts = np.sum(np.stack(all_counts).astype(np.uint64), axis=0).astype(np.uint32)
    first = np.min(np.stack(all_first), axis=0).astype(np.uint64)
    return counts, first


def seeds_from(last_dcs: list[np.ndarray], r: int) -> np.ndarray:
    """DC chain seed of stripe r: the previous stripe's last Y/Cb/Cr DC (zeros for the first)."""
    return np.zeros(3, np.int32) if r == 0 else np.asarray(last_dcs[r - 1], np.int32)


def encode_stripes_local(encoders: list, stripes_rgb: list[tuple[int, int]], width: int, height: int,
                         quality: int, out_ptr: int, cap: int, maxval: int = 255, rows=None) -> int:
    """All stripes in one process: encoders[r] encodes stripe r (device RGB pointer, stride);
    every stripe writes into the same whole-file device buffer out_ptr.  Returns the length."""
    n = len(encoders)
    rows = rows or stripe_rows((height + 15) // 16, n)
    last = [encoders[r].stripe_transform(stripes_rgb[r][0], stripes_rgb[r][1], width, height, rows[r][0],
                                         rows[r][1], quality, maxval) for r in range(n)]
    stats = [encoders[r].stripe_stats(seeds_from(last, r)) for r in range(n)]
    counts, first = combine_stats([s[0] for s in stats], [s[1] for s in stats])
    codes = [encoders[r].stripe_code(counts, first) for r in range(n)]
    summaries = [c[0] for c in codes]
    total = None
    for r in range(n):
        _, _, total = encoders[r].stripe_pack(summaries, r, out_ptr, cap)
    return total


def encode_stripe_dist(enc, rgb_ptr: int, stride: int, width: int, height: int, quality: int, out, maxval: int = 255,
                       group=None, restart: int = 0) -> int:
    """This rank's stripe of a torch.distributed job (rank r of world n takes stripe r).
    rgb_ptr: device RGB of the stripe's rows (stripe_rows() says which); out: a uint8
    torch tensor on this rank's device with whole-file capacity.  After the call rank
    0's `out` holds the whole file; returns its length (every rank).  restart: the
    encoder's restart interval (enc.set_restart), whose boundaries include every
    stripe start — then there is no DC seed exchange and the summaries only place
    byte runs (the RCCL traffic is the histogram all-reduce and the segment gather).

    The exchanges' device work runs on a stream of this module's, never the null stream
    (an operation there makes every later launch on the encoders' lane streams slower,
    DESIGN §2); the call returns once that stream is idle."""
    import torch

    if out.device.type != "cuda":
        return _encode_stripe_dist(enc, rgb_ptr, stride, width, height, quality, out, maxval, group, restart)
    side = _SIDE.get(out.device.index)
    if side is None:
        side = _SIDE[out.device.index] = torch.cuda.Stream(device=out.device)
    with torch.cuda.stream(side):
        total = _encode_stripe_dist(enc, rgb_ptr, stride, width, height, quality, out, maxval, group, restart)
    side.synchronize()
    return total


_SIDE = {}  # device index -> the exchanges' stream


def _encode_stripe_dist(enc, rgb_ptr, stride, width, height, quality, out, maxval, group, restart):
    import torch
    import torch.distributed as dist

    rank, n = dist.get_rank(group), dist.get_world_size(group)
    rows = stripe_rows((height + 15) // 16, n, restart_align(width, restart))
    # exchanges in device memory over RCCL; through host memory for gloo (CPU tests,
    # several ranks sharing one GPU)
    dev = out.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    last = enc.stripe_transform(rgb_ptr, stride, width, height, rows[rank][0], rows[rank][1], quality, maxval)
    if restart:  # every stripe starts a restart interval: its DC chain starts at 0
        seed = np.zeros(3, np.int32)
    else:
        # 1) DC seeds: all-gather of 3 x int32 per rank
        g = [torch.zeros(3, dtype=torch.int32, device=dev) for _ in range(n)]
        dist.all_gather(g, torch.from_numpy(last).to(dev), group=group)
        seed = seeds_from([t.cpu().numpy() for t in g], rank)
    counts, first = enc.stripe_stats(seed)
    # 2) histograms: sum of counts, minimum of first-occurrence keys (int64 view: keys < 2^63)
    tc = torch.from_numpy(counts.astype(np.int64)).to(dev)
    tf = torch.from_numpy(np.minimum(first, np.uint64(2**63 - 1)).astype(np.int64)).to(dev)
    dist.all_reduce(tc, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(tf, op=dist.ReduceOp.MIN, group=group)
    counts = tc.cpu().numpy().astype(np.uint32)
    fk = tf.cpu().numpy().astype(np.uint64)
    first = np.where(counts > 0, fk, np.uint64(2**64 - 1))
    summary, hdr_len = enc.stripe_code(counts, first)
    # 3) summaries: all-gather of 12 x int64 per rank (bits, ff[8], head, tail, restart);
    #    with restart intervals only the byte lengths matter (stitching the segments)
    mine = torch.tensor([summary[0], *summary[1], summary[2], summary[3], summary[4]], dtype=torch.int64,
                        device=dev)
    gs = [torch.zeros(12, dtype=torch.int64, device=dev) for _ in range(n)]
    dist.all_gather(gs, mine, group=group)
    summaries = []
    for t in gs:
        v = [int(x) for x in t.cpu().tolist()]
        summaries.append((v[0], tuple(v[1:9]), v[9], v[10], v[11]))
    off, ln, total = enc.stripe_pack(summaries, rank, out.data_ptr(), out.numel())
    # 4) segments to rank 0: one grouped round of point-to-point transfers (every
    #    stripe's xGMI link busy at once), peers named by their global ranks
    spans = [J.stripe_place(summaries, r, hdr_len) for r in range(n)]
    ends = [spans[r + 1][0] if r + 1 < n else total for r in range(n)]
    ops, staged = [], []
    if rank == 0:
        for r in range(1, n):
            o = spans[r][0]
            buf = out[o:ends[r]] if dev == out.device else torch.empty(ends[r] - o, dtype=torch.uint8, device=dev)
            staged.append((o, buf))
            ops.append(dist.P2POp(dist.irecv, buf, dist.get_global_rank(group, r) if group is not None else r,
                                  group=group))
    else:
        seg = out[off:off + ln] if dev == out.device else out[off:off + ln].to(dev)
        ops.append(dist.P2POp(dist.isend, seg, dist.get_global_rank(group, 0) if group is not None else 0,
                              group=group))
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    for o, buf in staged:
        if buf.device != out.device:
            out[o:o + buf.numel()].copy_(buf)
    return total
