#!/bin/bash
# Round profiles in one GPU call (run through gpurun):
#   1. the bench line with the CPU baseline                      -> gpurun_out/rp/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench command -> gpurun_out/rp/trace/
#      + per-kernel means in the bench's timed / solo windows     -> gpurun_out/rp/window.txt
#   3. HBM traffic, two --pmc passes (FETCH_SIZE, WRITE_SIZE)     -> gpurun_out/pmc_rp.json
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 400 python3 bench.py > gpurun_out/rp/bench.json 2> gpurun_out/rp/bench.err || { tail -5 gpurun_out/rp/bench.err; exit 1; }
tail -c 400 gpurun_out/rp/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp/trace -o run -- \
  python3 bench.py --no-cpu-baseline > gpurun_out/rp/prof_bench.json 2> gpurun_out/rp/prof.err || { tail -5 gpurun_out/rp/prof.err; exit 1; }
python3 tools/rocprof_window.py gpurun_out/rp/trace gpurun_out/rp/prof_bench.json | tee gpurun_out/rp/window.txt
bash tools/pmc_traffic.sh rp || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_rp | tail -40
# keep the summaries (gpurun copies back <= 64 MiB): drop the per-dispatch CSVs
find gpurun_out/rp/trace gpurun_out/pmc_rp -name '*kernel_trace.csv' -delete 2>/dev/null
find gpurun_out/pmc_rp -name '*counter_collection.csv' -exec gzip -9 {} + 2>/dev/null
true
