#!/bin/bash
# Quick GPU check (through gpurun): the GPU suite (unless NOTESTS=1), then a short
# bench whose solo pass prints each kernel's exclusive time.
#   tools/quick.sh <tag> [bench args]  -> gpurun_out/q_<tag>/
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp
tag=$1; shift
o=gpurun_out/q_$tag
mkdir -p $o
if [ "${NOTESTS:-0}" != 1 ]; then
  timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1
  rc=$?; tail -3 $o/gpu_tests.log; [ $rc -eq 0 ] || exit 1
fi
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --d2h-steps 0 --frames 768 --steps 10 --solo-batches 4 "$@" > $o/bench$i.json 2> $o/bench$i.err || { tail -5 $o/bench$i.err; exit 1; }
  python3 - $o/bench$i.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "host_cpu", d.get("host_cpu"))
print("solo us:", {k: round(v["avg_kernel_ms"] * 1e3, 2) for k, v in (d.get("stages_solo") or {}).items()})
print("in situ us:", {k: round(v["avg_kernel_ms"] * 1e3, 2) for k, v in d["stages"].items()})
PY
done
true
