#!/bin/bash
# bench.py value per libjpge variant, no single-frame loop: tools/ab_bench_only.sh name...
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 0 > gpurun_out/abo_$n.json 2> gpurun_out/abo_$n.err || exit 1
  echo "== bench $n: $(python3 -c "import json;d=json.loads(open('gpurun_out/abo_$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
