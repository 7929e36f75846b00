#!/bin/bash
# Solo per-kernel durations (diagnostic): rocprofv3 --kernel-trace --stats of the
# single-frame loop over 16 distinct 4K frames; prints each kernel's mean.
#   tools/prof_kernels.sh <tag> [prof_frame args]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
tag=$1; shift
d=$R/gpurun_out/pk_$tag
rm -rf "$d"; mkdir -p "$d"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
  python3 "$R/tools/prof_frame.py" --frames 16 --iters 64 "$@" > "$d/log" 2>&1 || { echo "failed"; tail -5 "$d/log"; exit 1; }
grep -h "bytes" "$d/log"
python3 - "$d/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    import re
    m = re.search(r'(\w+)(<[^>]*>)?\(', r['Name'].replace('(anonymous namespace)', 'anon'))
    print(f"   {(m.group(1) if m else r['Name'])[:28]:28s} calls {int(r['Calls']):5d}  mean {float(r['AverageNs'])/1e3:8.2f} us  min {float(r['MinNs'])/1e3:8.2f} us")
PY
