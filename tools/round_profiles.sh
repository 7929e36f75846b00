#!/bin/bash
# Round profiles in one GPU call (run through gpurun), on the final tree:
#   1. the bench line with the CPU baseline (default arguments)     -> gpurun_out/rp/bench.json
#   2. rocprofv3 --kernel-trace --stats of a shorter bench run       -> gpurun_out/rp/trace/
#      + per-kernel means in its timed / solo windows next to the bench's
#        kernel-bound event averages                                  -> gpurun_out/rp/window.txt
#   3. HBM traffic, two --pmc passes (FETCH_SIZE, WRITE_SIZE) of a small bench run,
#      one frame per launch (JPGE_SET=1: per-frame bytes)          -> gpurun_out/pmc_rp.json
#   4. SQ counters (2 passes) of the single-frame loop                -> gpurun_out/sq_rp/
#   5. config 4 (batch1080) and 16384^2 bench lines                   -> gpurun_out/rp/{b1080,16k}.json
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 400 python3 bench.py > gpurun_out/rp/bench.json 2> gpurun_out/rp/bench.err || { tail -5 gpurun_out/rp/bench.err; exit 1; }
tail -c 300 gpurun_out/rp/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp/trace -o run -- \
  python3 bench.py --no-cpu-baseline --frames 768 --steps 10 > gpurun_out/rp/prof_bench.json 2> gpurun_out/rp/prof.err || { tail -5 gpurun_out/rp/prof.err; exit 1; }
python3 tools/rocprof_window.py gpurun_out/rp/trace gpurun_out/rp/prof_bench.json | tee gpurun_out/rp/window.txt
JPGE_SET=1 bash tools/pmc_traffic.sh rp --frames 64 --steps 2 --warmup 1 --solo-batches 0 --d2h-steps 0 --no-verify || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_rp | tail -40
bash tools/pmc_sq.sh rp --iters 8 > gpurun_out/rp/sq.txt 2>&1 || { tail -5 gpurun_out/rp/sq.txt; exit 1; }
timeout -k 10 300 python3 bench.py --workload batch1080 > gpurun_out/rp/b1080.json 2> gpurun_out/rp/b1080.err || { tail -5 gpurun_out/rp/b1080.err; exit 1; }
tail -c 300 gpurun_out/rp/b1080.json; echo
timeout -k 10 300 python3 bench.py --width 16384 --height 16384 --frames 16 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/rp/16k.json 2> gpurun_out/rp/16k.err || { tail -5 gpurun_out/rp/16k.err; exit 1; }
tail -c 300 gpurun_out/rp/16k.json; echo
# keep the summaries (gpurun copies back <= 64 MiB): drop the per-dispatch CSVs
find gpurun_out/rp/trace gpurun_out/pmc_rp gpurun_out/sq_rp -name '*kernel_trace.csv' -exec gzip -9 {} + 2>/dev/null
find gpurun_out/pmc_rp gpurun_out/sq_rp -name '*counter_collection.csv' -exec gzip -9 {} + 2>/dev/null
true
