"""Summarise rocprofv3 PMC CSVs per kernel (mean over dispatches).

    python tools/pmc_summary.py <pmc_dir> [--json OUT --width W --height H]

--json writes the per-launch HBM traffic of every kernel, corrected as
MI355X_MICROARCH.md (HBM section) prescribes: FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is
doubled; WRITE_SIZE is taken as is.
"""
import argparse
import collections
import csv
import glob
import gzip
import json
import re


def short(name):
    m = re.search(r"(\w+_kernel)", name)
    return m.group(1) + ("<exact>" if "<true>" in name else "<generic>" if "<false>" in name else "") if m else name[:40]


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    files += glob.glob(f"{d}/**/*counter_collection.csv.gz", recursive=True)
    for f in sorted(files):
        fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
        for r in csv.DictReader(fh):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    a = ap.parse_args()
    res = load(a.dir)
    out = {"width": a.width, "height": a.height,
           "note": "per-launch HBM bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving corrected)",
           "kernels": {}}
    for k, d in res.items():
        if "rocclr" in k:
            continue
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {v:16.0f}")
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            rd = 2.0 * d["FETCH_SIZE"] * 1024
            wr = d["WRITE_SIZE"] * 1024
            out["kernels"][k] = {"read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes_per_launch": int(rd + wr)}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", a.json)


if __name__ == "__main__":
    main()
