#!/bin/bash
# Round-3 session c: path-slot sweep of the whole-frame bench on configs 2 and 3
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_kstats.sh "MCPT_BENCH_SLOTS=5" "MCPT_BENCH_SLOTS=8" "MCPT_BENCH_SLOTS=12" "MCPT_BENCH_SLOTS=16" "MCPT_BENCH_SLOTS=8" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_BENCH_SLOTS=3" "MCPT_BENCH_SLOTS=8" "MCPT_BENCH_SLOTS=12" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
