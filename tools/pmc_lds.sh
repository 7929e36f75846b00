#!/bin/bash
# LDS counters of the single-frame loop for libjpge variants (through gpurun):
#   tools/pmc_lds.sh name...  (main = the tree's build, else jpgenc_amd/lib/var/<name>/)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; export TMPDIR=/tmp
for n in "$@"; do
  lib=$R/jpgenc_amd/lib/var/$n/libjpge.so; [ "$n" = main ] && lib=$R/jpgenc_amd/lib/libjpge.so
  out=$R/gpurun_out/lds_$n; mkdir -p $out
  JPGE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d $out -o p -- python3 tools/prof_frame.py --iters 8 > $out/log 2>&1 || { echo "$n failed"; tail -3 $out/log; exit 1; }
  echo "== $n"; python3 tools/pmc_summary.py $out | grep -A9 "^stats"
done
