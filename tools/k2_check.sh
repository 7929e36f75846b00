#!/bin/bash
# Round-4 K2 iteration (through gpurun): GPU suite, then an env/lib A/B, then the SQ
# counters of the single-frame loop.  tools/k2_check.sh "<env A>" "<env B>" ...
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/k2_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_env.sh 1 "$@" || exit 1
bash tools/pmc_sq.sh k2 --iters 8 > gpurun_out/sq_k2.txt 2>&1 || { tail -3 gpurun_out/sq_k2.txt; exit 1; }
grep -A16 "^stats" gpurun_out/sq_k2.txt
