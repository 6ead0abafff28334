#!/bin/bash
# Memory-pipeline PMC passes (TA/TD/TCP) over the steady-state pipeline.
export TMPDIR=/tmp
label=$1; shift
for kv in "$@"; do export "$kv"; done
O=gpurun_out/pmct_$label
mkdir -p $O
i=0
for set in "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES" \
           "TD_TD_BUSY TD_TC_STALL" "TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES" \
           "TCP_TCR_TCP_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES" "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ" \
           "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o p$i --output-format csv -- python3 ${PROG:-tools/pmc_pipe.py} > $O/p$i.log 2>&1 || { echo "pass $i failed: $set"; tail -5 $O/p$i.log; exit 1; }
done
echo DONE $label
