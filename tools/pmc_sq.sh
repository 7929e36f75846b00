#!/bin/bash
# SQ (shader) counters per kernel on the single-frame profiling loop, in separate
# --pmc passes of <= 8 SQ counters each, --kernel-trace only (no sys/runtime traces).
#   tools/pmc_sq.sh <tag> [prof_frame args]  ->  gpurun_out/sq_<tag>/ + summary on stdout
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
tag=$1; shift
out=$R/gpurun_out/sq_$tag
mkdir -p "$out"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$out" -o pass$i -- \
    python3 "$R/tools/prof_frame.py" "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$out"
