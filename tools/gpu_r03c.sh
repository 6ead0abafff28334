#!/bin/bash
# Round-3 session c: path-slot sweep of the whole-frame bench on configs 2, 3 and 5
set -o pipefail
mkdir -p gpurun_out
KS_STEPS=1 bash tools/gpu_kstats.sh "MCPT_BENCH_SLOTS=16" "MCPT_BENCH_SLOTS=24" "MCPT_BENCH_SLOTS=32" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_BENCH_SLOTS=16" "MCPT_BENCH_SLOTS=24" "MCPT_BENCH_SLOTS=32" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 5 --spp 64" bash tools/gpu_kstats.sh "MCPT_BENCH_SLOTS=4" "MCPT_BENCH_SLOTS=8" "MCPT_BENCH_SLOTS=16" 2>&1 | grep -E "==|value|k_trace"
