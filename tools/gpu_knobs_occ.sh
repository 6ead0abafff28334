#!/bin/bash
# Round-3 session: k_trace resident waves per CU and partitions re-swept with the occluder cache on
set -o pipefail
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_TRACE_WAVES=28" "MCPT_TRACE_WAVES=24" "MCPT_TRACE_PARTS=32" "MCPT_TRACE_PARTS=8" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace"
