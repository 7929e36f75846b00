"""Concurrency view of a multi-lane run from a rocprofv3 --kernel-trace CSV: per
hardware queue the kernel count and idle time, the time spent with 0/1/2/3+
kernels running, and which kernel pairs overlap for how long.

    python tools/lanes_timeline.py <dir-with-*_kernel_trace.csv> [--skip N] [--bench bench.json]

--bench: only kernels inside the bench line's timed window (windows_monotonic_ns).
"""
import json
import argparse
import collections
import csv
import glob
import itertools
import re


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name.split("(")[0][-24:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=400)
    ap.add_argument("--bench")
    a = ap.parse_args()
    win = None
    if a.bench:
        b = json.loads([l for l in open(a.bench) if l.startswith("{")][-1])
        win = b["windows_monotonic_ns"]["timed"]
    ops = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]))
    ops.sort()
    if win:
        ops = [o for o in ops if o[0] >= win[0] and o[1] <= win[1]]
    else:
        ops = ops[a.skip:]
    if not ops:
        print("no operations")
        return
    t0, t1 = ops[0][0], max(e for _, e, _, _ in ops)
    # per queue
    byq = collections.defaultdict(list)
    for o in ops:
        byq[o[3]].append(o)
    for q, qo in sorted(byq.items()):
        busy = sum(e - s for s, e, _, _ in qo)
        print(f"queue {q}: {len(qo)} kernels, busy {100 * busy / (t1 - t0):.1f}% of the window")
    # concurrency levels (sweep)
    ev = sorted([(s, 1, n) for s, e, n, _ in ops] + [(e, -1, n) for s, e, n, _ in ops])
    level, last, hist = 0, t0, collections.Counter()
    running = collections.Counter()
    pair = collections.Counter()
    for t, d, n in ev:
        dt = t - last
        hist[min(level, 3)] += dt
        names = sorted(k for k, v in running.items() for _ in range(v))
        for x, y in itertools.combinations(names, 2):
            pair[(x, y)] += dt
        level += d
        running[n] += d
        last = t
    span = t1 - t0
    print(f"window {span / 1e3:.1f} us: " + ", ".join(f"{k}{'+' if k == 3 else ''} running {100 * v / span:.1f}%"
                                                     for k, v in sorted(hist.items())))
    durs = collections.defaultdict(list)
    for s, e, n, _ in ops:
        durs[n].append(e - s)
    for n, d in sorted(durs.items(), key=lambda x: -sum(x[1])):
        print(f"  {n:24s} n={len(d):5d} mean {sum(d) / len(d) / 1e3:7.2f} us total {sum(d) / 1e6:7.3f} ms")
    print("overlapping pairs (time both run):")
    for (x, y), v in pair.most_common(10):
        print(f"  {x:22s} + {y:22s} {v / 1e6:7.3f} ms")


if __name__ == "__main__":
    main()
