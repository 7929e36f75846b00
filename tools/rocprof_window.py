"""Per-kernel mean durations from a rocprofv3 --kernel-trace CSV inside the bench's
timed and solo windows (bench.py's "windows_monotonic_ns"), next to the bench's
HIP-event averages — the agreement check for the roofline's kernel time.

    python tools/rocprof_window.py <trace dir> <bench json line file>
"""
import collections
import csv
import glob
import json
import gzip
import re
import statistics
import sys


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) if m else name.split("(")[0][-30:]


def main():
    tdir, bfile = sys.argv[1], sys.argv[2]
    line = [l for l in open(bfile) if l.startswith("{")][-1]
    b = json.loads(line)
    wins = b["windows_monotonic_ns"]
    ops = []
    for f in glob.glob(f"{tdir}/**/*kernel_trace.csv*", recursive=True):
        for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    for label in ("timed", "solo", "solo_single"):
        w = wins.get(label)
        if not w:
            continue
        d = collections.defaultdict(list)
        for s, e, n in ops:
            if w[0] <= s and e <= w[1]:
                d[n].append(e - s)
        print(f"{label} window ({(w[1] - w[0]) / 1e6:.2f} ms):")
        for n, v in sorted(d.items(), key=lambda x: -sum(x[1])):
            extra = ""
            if label == "solo_single" and len(v) >= 64:  # the single-frame pass's batches of 32 frames
                extra = " (batches: " + " ".join(f"{sum(v[i:i + 32]) / len(v[i:i + 32]) / 1e3:.2f}"
                                                 for i in range(0, len(v), 32)) + ")"
            print(f"   {n:28s} n={len(v):5d} mean {sum(v) / len(v) / 1e3:8.2f} us  median "
                  f"{statistics.median(v) / 1e3:8.2f} us{extra}")
        ev = {"timed": b.get("stages"), "solo": b.get("stages_solo"),
              "solo_single": b.get("stages_solo_single_frame")}[label] or {}
        for k, v in ev.items():
            if v.get("avg_kernel_ms") is None:
                print(f"   bench HIP events {k:18s}     none (no timed launch)")
                continue
            print(f"   bench HIP events {k:18s} {v['avg_kernel_ms'] * 1e3:8.2f} us "
                  f"(entropy = code + pack launches)")


if __name__ == "__main__":
    main()
