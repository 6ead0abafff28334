#!/bin/bash
# PMC passes over tools/pmc_trace.py (steady-state config-2 stage runs).
# usage: tools/pmc_trace.sh <label> [ENV=VAL ...]   -> gpurun_out/pmct_<label>/p*/
export TMPDIR=/tmp
label=$1; shift
for kv in "$@"; do export "$kv"; done
O=gpurun_out/pmct_$label
mkdir -p $O
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o p$i --output-format csv -- python3 ${PROG:-tools/pmc_trace.py} > $O/p$i.log 2>&1 || { echo "pass $i failed: $set"; tail -5 $O/p$i.log; exit 1; }
done
echo DONE $label
