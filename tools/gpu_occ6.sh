#!/bin/bash
# Round-3 session: occluder-cache table shape with two ways (cells x bins), config 2; configs 3 and 5
set -o pipefail
F="==|value|k_trace|k_material"
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_OCC_B=16" "MCPT_OCC_G=32" "MCPT_OCC_G=32 MCPT_OCC_B=16" "MCPT_OCC_B=4" "MCPT_X=0" 2>&1 | grep -E "$F"
KS_STEPS=1 KS_ARGS="--config 5 --spp 64" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_OCC_G=32 MCPT_OCC_B=16" 2>&1 | grep -E "$F"
