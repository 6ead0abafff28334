#!/bin/bash
# Round-3 session g: k_trace launch knobs re-swept on the whole-frame bench at the new slot counts
set -o pipefail
mkdir -p gpurun_out
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_TRACE_PARTS=32" "MCPT_REFILL_MIN=12" "MCPT_REFILL_MIN=28" "MCPT_TRI_MIN=8" "MCPT_TRI_MIN=24" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace"
