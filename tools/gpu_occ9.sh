#!/bin/bash
# Round-3 session: occluder-cache table shape when the table starts empty with every frame
set -o pipefail
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_OCC_G=16 MCPT_OCC_B=8" "MCPT_OCC_G=16 MCPT_OCC_B=16" "MCPT_OCC_G=24 MCPT_OCC_B=12" "MCPT_OCC_G=8 MCPT_OCC_B=8" "MCPT_OCC_G=16 MCPT_OCC_B=8" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace|k_material"
