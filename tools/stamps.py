"""Summarise diagnostic phase stamps (diag build, JPGE_STAMPS_FILE) of one frame:
per kernel, the mean/median duration of each phase per workgroup, the spread of
workgroup start/end times, and the accumulated per-tile sub-phase durations
(slots 8-15).  s_memrealtime ticks -> us at --ghz."""
import argparse

import numpy as np

SLOTS = 16
KERNELS = ["fdct", "stats", "entropy_code", "entropy_pack"]
PHASES = {
    "fdct": ["start", "", "", "", "", "", "", "end"],
    "stats": ["start", "data", "tiles", "flush", "", "", "", ""],  # (wave kernel: wave 0's first data)
    "entropy_code": ["start", "emit", "count8", "", "", "", "", ""],
    "entropy_pack": ["start", "scan", "output", "", "", "", "", ""],
}
ACC = {
    "stats": ["stage+fetch", "fields", "blocks", "DC recs"],  # (wave kernel: wave 0)
    "entropy_code": ["sync", "rounds(tail)", "store", "load+bits", "scan", "zero", "pack"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("--ghz", type=float, default=0.1)  # s_memrealtime: 100 MHz
    a = ap.parse_args()
    raw = np.fromfile(a.file, np.uint64)
    nk = len(KERNELS)
    n = raw[:nk].astype(np.int64)
    data = raw[nk:].reshape(nk, 65536, SLOTS).astype(np.int64)
    us = lambda x: x / (a.ghz * 1e3)
    for k, name in enumerate(KERNELS):
        full = data[k, : n[k]]
        labels = PHASES[name]
        used = [i for i, l in enumerate(labels) if l]
        d = full[:, used]
        keep = (d > 0).all(axis=1)  # launched workgroups only
        d, full = d[keep], full[keep]
        if not len(d):
            continue
        t0 = d[:, 0].min()
        starts = np.sort(d[:, 0] - t0)
        ends = d[:, -1] - t0
        tm = np.median(np.concatenate([starts, ends]))
        alive = int(((d[:, 0] - t0 <= tm) & (ends >= tm)).sum())
        print(f"{name}: alive at median time {alive}; start quantiles (us) "
              + " ".join(f"{q}:{us(starts[int(q / 100 * (len(starts) - 1))]):.1f}" for q in (0, 25, 50, 75, 100)))
        print(f"{name}: {n[k]} workgroups, span {us(d[:, -1].max() - t0):.1f} us, "
              f"start spread {us(d[:, 0].max() - t0):.1f} us")
        for j in range(1, len(used)):
            dur = us(d[:, j] - d[:, j - 1])
            print(f"   {labels[used[j - 1]]:>14s} -> {labels[used[j]]:<14s} mean {dur.mean():7.2f}  "
                  f"median {np.median(dur):7.2f}  p95 {np.percentile(dur, 95):7.2f} us")
        life = us(d[:, -1] - d[:, 0])
        print(f"   workgroup lifetime mean {life.mean():.2f} us, max {life.max():.2f} us")
        for j, lab in enumerate(ACC.get(name, [])):
            acc = us(full[:, 8 + j])
            print(f"   [per-workgroup total] {lab:<8s} mean {acc.mean():7.2f}  p95 {np.percentile(acc, 95):7.2f} us")


if __name__ == "__main__":
    main()
