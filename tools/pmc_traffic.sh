#!/bin/bash
# HBM traffic per kernel launch for the bench workload: two rocprofv3 PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), each with
# --kernel-trace only, never combined with sys/runtime traces.
#   tools/pmc_traffic.sh <tag> [bench args]   ->  gpurun_out/pmc_<tag>/, gpurun_out/pmc_<tag>.json
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
tag=$1; shift
out=$R/gpurun_out/pmc_$tag
mkdir -p "$out"
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$out" -o pass$i -- \
    python3 "$R/bench.py" --no-cpu-baseline "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$out" --json "$R/gpurun_out/pmc_$tag.json" --width "${PMC_W:-3840}" --height "${PMC_H:-2160}"
