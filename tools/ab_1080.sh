#!/bin/bash
# batch1080 (config 4) bench value per libjpge variant: tools/ab_1080.sh name...  (main = the working tree's library)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --workload batch1080 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/a1080_$n.json 2> gpurun_out/a1080_$n.err || { tail -3 gpurun_out/a1080_$n.err; exit 1; }
  echo "== 1080 $n: $(python3 -c "import json;d=json.loads(open('gpurun_out/a1080_$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
