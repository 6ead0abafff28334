#!/bin/bash
# Round-3 session k: node width re-checked at the new slot counts (configs 3 and 4)
set -o pipefail
KS_STEPS=1 KS_ARGS="--config 4 --spp 64" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_BVH_WIDTH=4" "MCPT_X=0" "MCPT_BVH_WIDTH=4" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_BVH_WIDTH=2" "MCPT_X=0" "MCPT_BVH_WIDTH=2" 2>&1 | grep -E "==|value|k_trace"
