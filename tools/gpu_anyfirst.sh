#!/bin/bash
# Round-3 session: any-hit rays first in each partition's sequence (MCPT_ANY_FIRST=1 build) with the
# occluder cache on (the remaining any-hit rays are mostly unoccluded, long traversals)
set -o pipefail
L=$PWD/mc-path-tracer_amd
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfirst.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfirst.so" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfirst.so" 2>&1 | grep -E "==|value|k_trace"
