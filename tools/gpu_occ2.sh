#!/bin/bash
# Round-3 session: occluder cache table shape (cells G, bins B, ways W) on config 2, and the
# lookup gate on configs 3-5 (cache on vs MCPT_OCC_G=0); GPU parity suite first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_occ.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_occ.log | head -20; tail -5 gpurun_out/pytest_occ.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_occ.log | tail -1
F="==|value|k_trace|k_material|k_shade"
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_OCC_G=0" "MCPT_X=0" "MCPT_OCC_G=16" "MCPT_OCC_WAYS=2" "MCPT_OCC_G=16 MCPT_OCC_WAYS=2" "MCPT_OCC_G=16 MCPT_OCC_B=16" "MCPT_OCC_G=32 MCPT_OCC_B=4" "MCPT_X=0" "MCPT_OCC_G=0" 2>&1 | grep -E "$F"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_OCC_G=0" "MCPT_X=0" 2>&1 | grep -E "$F"
KS_STEPS=1 KS_ARGS="--config 4 --spp 64" bash tools/gpu_kstats.sh "MCPT_OCC_G=0" "MCPT_X=0" 2>&1 | grep -E "$F"
KS_STEPS=1 KS_ARGS="--config 5 --spp 64" bash tools/gpu_kstats.sh "MCPT_OCC_G=0" "MCPT_X=0" 2>&1 | grep -E "$F"
