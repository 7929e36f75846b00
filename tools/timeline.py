"""GPU timeline from a rocprofv3 --kernel-trace CSV (+ memory-copy trace if given):
per-operation duration statistics, the idle gaps between consecutive operations,
and the busy fraction of the window.

    python tools/timeline.py <dir-with-*_kernel_trace.csv> [--skip N]
"""
import argparse
import collections
import csv
import glob
import re


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    if m:
        return m.group(1)
    return name.split("(")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=200, help="drop the first N operations (warm-up)")
    a = ap.parse_args()
    ops = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True) + \
            glob.glob(f"{a.dir}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or ("copy " + r.get("Direction", "?"))
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(name)))
    ops.sort()
    ops = ops[a.skip:]
    if not ops:
        print("no operations")
        return
    dur = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    busy_end = ops[0][0]
    busy = 0
    prev = None
    for s, e, n in ops:
        dur[n].append(e - s)
        if prev is not None:
            gaps[f"{prev} -> {n}"].append(max(0, s - busy_end))
        busy += max(0, e - max(s, busy_end))
        busy_end = max(busy_end, e)
        prev = n
    span = busy_end - ops[0][0]
    print(f"{len(ops)} ops over {span / 1e3:.1f} us, GPU busy {100 * busy / span:.1f}%")
    for n, d in sorted(dur.items(), key=lambda x: -sum(x[1])):
        d.sort()
        print(f"  {n:28s} n={len(d):5d} mean {sum(d) / len(d) / 1e3:8.2f} us  median {d[len(d) // 2] / 1e3:8.2f} us  "
              f"total {sum(d) / 1e6:8.3f} ms")
    print("idle gaps before an operation (by transition):")
    for k, g in sorted(gaps.items(), key=lambda x: -sum(x[1]))[:12]:
        g.sort()
        print(f"  {k:50s} n={len(g):5d} mean {sum(g) / len(g) / 1e3:7.2f} us  median {g[len(g) // 2] / 1e3:7.2f} us  "
              f"total {sum(g) / 1e6:7.3f} ms")


if __name__ == "__main__":
    main()
