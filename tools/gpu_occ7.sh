#!/bin/bash
# Round-3 session: hashed occluder-cache table (2^bits cells x 2 ways), cells/bins/bits sweep on config 2
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_occ.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_occ.log | head -20; tail -5 gpurun_out/pytest_occ.log; exit 1; }
grep -E "passed|failed|resolved by the warm" gpurun_out/pytest_occ.log | tail -6
F="==|value|k_trace|k_material"
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_OCC_BITS=23" "MCPT_OCC_BITS=19" "MCPT_OCC_G=16 MCPT_OCC_B=8" "MCPT_OCC_G=48 MCPT_OCC_B=16" "MCPT_OCC_G=0" "MCPT_X=0" 2>&1 | grep -E "$F"
KS_STEPS=1 KS_ARGS="--config 4 --spp 64" bash tools/gpu_kstats.sh "MCPT_OCC_G=0" "MCPT_X=0" 2>&1 | grep -E "$F"
