#!/bin/bash
# Round-3 session: extension rays' closest hits recorded in the occluder cache too (MCPT_OCC_EXT=1 build)
set -o pipefail
L=$PWD/mc-path-tracer_amd
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_occext.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_occext.so" 2>&1 | grep -E "==|value|k_trace|k_material"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_occext.so" 2>&1 | grep -E "==|value|k_trace|k_material"
