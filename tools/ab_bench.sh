#!/bin/bash
# A/B of libjpge variants: the single-frame loop (tools/ab_frames.sh) and a short
# bench.py run (4k-frames value) per variant.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash tools/ab_frames.sh "$@" || exit 1
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --d2h-steps 0 > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || exit 1
  echo "== bench $n: $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
