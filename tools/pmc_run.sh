#!/bin/bash
# PMC passes over the single-frame loop (each pass: --pmc with --kernel-trace only;
# never combined with sys/runtime traces).  Usage: tools/pmc_run.sh <tag> [prof_frame args]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
tag=$1; shift
out=$R/gpurun_out/pmc_$tag
mkdir -p $out
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $out -o pass$i -- python3 $R/tools/prof_frame.py "$@" > $out/pass$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "pmc $tag done"
