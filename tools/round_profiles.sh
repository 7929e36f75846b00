#!/bin/bash
# Round profiles on the final tree, in two GPU calls (run through gpurun):
#   part A: the GPU test suite and smoke()                            -> gpurun_out/rp/{gpu_tests,smoke}.log
#           the bench line with the CPU baseline (default arguments)  -> gpurun_out/rp/bench.json
#           rocprofv3 --kernel-trace --stats of a shorter bench run   -> gpurun_out/rp/trace/
#             + per-kernel means in its timed / solo windows next to the bench's
#               kernel-bound event averages                           -> gpurun_out/rp/window.txt
#           HBM traffic, two --pmc passes (FETCH_SIZE, WRITE_SIZE) of a small bench run,
#             one frame per launch (JPGE_SET=1: per-frame bytes)      -> gpurun_out/pmc_rp.json
#           SQ counters (2 passes) of the single-frame loop           -> gpurun_out/sq_rp/
#   part B: config 3's quality sweep (Q50, Q100 bench lines)          -> gpurun_out/rp/q{50,100}.json
#           config 4 (batch1080) on one rank and on 2 ranks sharing the GPU
#                                                                     -> gpurun_out/rp/b1080{,x2}.json
#           16384^2 frames through the pipeline                       -> gpurun_out/rp/16k.json
#           config 5 (16k-striped, restart per MCU row) on one GPU    -> gpurun_out/rp/16ks.json
#           rocprofv3 --kernel-trace --stats of the batch1080 and 16k-striped lines, with
#             their solo windows next to the lines' roofline events   -> gpurun_out/rp/{trace_b1080,trace_16ks}/, window_*.txt
#   tools/round_profiles.sh A|B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
O=gpurun_out/rp
mkdir -p $O
line() { tail -c 400 "$1"; echo; }
case "${1:-A}" in
A)
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  line $O/bench.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --no-cpu-baseline --frames 768 --steps 10 --latency-calls 0 > $O/prof_bench.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
  python3 tools/rocprof_window.py $O/trace $O/prof_bench.json | tee $O/window.txt
  JPGE_SET=1 bash tools/pmc_traffic.sh rp --frames 64 --steps 2 --warmup 1 --solo-batches 0 --d2h-steps 0 --latency-calls 0 --no-verify || exit 1
  python3 tools/pmc_summary.py gpurun_out/pmc_rp | tail -40
  bash tools/pmc_sq.sh rp --iters 8 > $O/sq.txt 2>&1 || { tail -5 $O/sq.txt; exit 1; }
  # keep the summaries (gpurun copies back <= 64 MiB): drop the per-dispatch CSVs
  find $O/trace gpurun_out/pmc_rp gpurun_out/sq_rp -name '*kernel_trace.csv' -exec gzip -9 {} + 2>/dev/null
  find gpurun_out/pmc_rp gpurun_out/sq_rp -name '*counter_collection.csv' -exec gzip -9 {} + 2>/dev/null
  ;;
B)
  for q in 50 100; do
    timeout -k 10 400 python3 bench.py --quality $q --no-cpu-baseline > $O/q$q.json 2> $O/q$q.err || { tail -5 $O/q$q.err; exit 1; }
    line $O/q$q.json
  done
  timeout -k 10 300 python3 bench.py --workload batch1080 > $O/b1080.json 2> $O/b1080.err || { tail -5 $O/b1080.err; exit 1; }
  line $O/b1080.json
  timeout -k 10 300 python3 bench.py --workload batch1080 --gpus 2 --allow-shared-gpu > $O/b1080x2.json 2> $O/b1080x2.err || { tail -5 $O/b1080x2.err; exit 1; }
  line $O/b1080x2.json
  timeout -k 10 300 python3 bench.py --width 16384 --height 16384 --frames 16 --steps 5 --warmup 1 --no-cpu-baseline --latency-calls 0 > $O/16k.json 2> $O/16k.err || { tail -5 $O/16k.err; exit 1; }
  line $O/16k.json
  timeout -k 10 300 python3 bench.py --workload 16k-striped > $O/16ks.json 2> $O/16ks.err || { tail -5 $O/16ks.err; exit 1; }
  line $O/16ks.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_b1080 -o run -- \
    python3 bench.py --workload batch1080 --no-cpu-baseline --steps 10 > $O/prof_b1080.json 2> $O/prof_b1080.err || { tail -5 $O/prof_b1080.err; exit 1; }
  python3 tools/rocprof_window.py $O/trace_b1080 $O/prof_b1080.json | tee $O/window_b1080.txt
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_16ks -o run -- \
    python3 bench.py --workload 16k-striped --no-cpu-baseline --steps 10 > $O/prof_16ks.json 2> $O/prof_16ks.err || { tail -5 $O/prof_16ks.err; exit 1; }
  python3 tools/rocprof_window.py $O/trace_16ks $O/prof_16ks.json | tee $O/window_16ks.txt
  find $O/trace_b1080 $O/trace_16ks -name '*kernel_trace.csv' -exec gzip -9 {} + 2>/dev/null
  ;;
esac
true
