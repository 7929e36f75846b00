#!/bin/bash
# Round 3 first GPU call: GPU suite, bench line, rocprof kernel trace of a shorter
# bench (solo window vs the bench's kernel-bound events), VALU issue-rate probe.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03a/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03a/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 60 ./jpgenc_amd/bin/valu_rates > gpurun_out/r03a/valu_rates.txt 2>&1 || exit 1
cat gpurun_out/r03a/valu_rates.txt
timeout -k 10 400 python3 bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { tail -5 gpurun_out/r03a/bench.err; exit 1; }
tail -c 600 gpurun_out/r03a/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03a/trace -o run -- \
  python3 bench.py --no-cpu-baseline --frames 768 --steps 10 > gpurun_out/r03a/prof_bench.json 2> gpurun_out/r03a/prof.err || { tail -5 gpurun_out/r03a/prof.err; exit 1; }
python3 tools/rocprof_window.py gpurun_out/r03a/trace gpurun_out/r03a/prof_bench.json | tee gpurun_out/r03a/window.txt
find gpurun_out/r03a/trace -name '*kernel_trace.csv' -exec gzip -9 {} +
true
