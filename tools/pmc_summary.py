"""Summarise rocprofv3 PMC CSVs per kernel (mean over dispatches)."""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) + ("<exact>" if "<true>" in name else "<generic>" if "<false>" in name else "") if m else name[:40]


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/pass*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


if __name__ == "__main__":
    res = load(sys.argv[1])
    for k, d in res.items():
        if "rocclr" in k:
            continue
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {v:16.0f}")
