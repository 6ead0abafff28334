#!/bin/bash
# Round-3 session f: tests, then the k_shade block-done skip A/B on the whole-frame bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1 || { tail -40 gpurun_out/pytest_f.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_f.log | tail -1
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_NO_BLOCK_DONE=1" "MCPT_X=0" "MCPT_NO_BLOCK_DONE=1" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
KS_STEPS=2 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_NO_BLOCK_DONE=1" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
