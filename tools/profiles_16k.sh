#!/bin/bash
# 16384^2 4:2:0 Q90 profiles in one GPU call (the HBM-roofline frame):
#   bench line (16 frames per step over 2 distinct inputs)  -> gpurun_out/p16/bench.json
#   rocprofv3 --kernel-trace --stats of the same command    -> gpurun_out/p16/trace/ + window.txt
#   HBM traffic, two --pmc passes (FETCH_SIZE, WRITE_SIZE)  -> gpurun_out/pmc_16k.json
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/p16
A="--width 16384 --height 16384 --frames 16 --distinct 2 --steps 5 --warmup 1 --d2h-steps 0 --solo-batches 1"
timeout -k 10 400 python3 bench.py $A --no-cpu-baseline > gpurun_out/p16/bench.json 2> gpurun_out/p16/bench.err || { tail -5 gpurun_out/p16/bench.err; exit 1; }
tail -c 300 gpurun_out/p16/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p16/trace -o run -- \
  python3 bench.py $A --no-cpu-baseline > gpurun_out/p16/prof_bench.json 2> gpurun_out/p16/prof.err || { tail -5 gpurun_out/p16/prof.err; exit 1; }
python3 tools/rocprof_window.py gpurun_out/p16/trace gpurun_out/p16/prof_bench.json | tee gpurun_out/p16/window.txt
PMC_W=16384 PMC_H=16384 bash tools/pmc_traffic.sh 16k $A || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_16k | tail -20
find gpurun_out/p16/trace gpurun_out/pmc_16k -name '*kernel_trace.csv' -delete 2>/dev/null
find gpurun_out/pmc_16k -name '*counter_collection.csv' -exec gzip -9 {} + 2>/dev/null
true
