#!/bin/bash
# K1's solo time per libjpge variant (bench.py's 1-lane pass, HIP events): tools/solo_k1.sh name...
# (SOLO_ARGS adds bench.py options, e.g. "--width 16384 --height 16384 --frames 4 --distinct 2")
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for n in "$@"; do
  lib=jpgenc_amd/lib/var/$n/libjpge.so
  [ "$n" = main ] && lib=jpgenc_amd/lib/libjpge.so
  JPGE_LIB=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --d2h-steps 0 --no-verify --solo-batches 4 ${SOLO_ARGS:-} > gpurun_out/sk.json 2> gpurun_out/sk.err || exit 1
  echo "== $n: $(python3 -c "import json;d=json.loads(open('gpurun_out/sk.json').read().strip().splitlines()[-1]);s=d['stages_solo'];print({k:round(v['avg_kernel_ms']*1e3,2) for k,v in s.items()}, d['value'])")"
done
