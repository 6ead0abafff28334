#!/bin/bash
# Round-3 session: path slots and k_trace hand-out knobs re-swept with the occluder cache on (config 2)
set -o pipefail
F="==|value|k_trace|k_material|k_shade"
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_BENCH_SLOTS=24" "MCPT_BENCH_SLOTS=16" "MCPT_BENCH_SLOTS=32" "MCPT_BENCH_SLOTS=40" "MCPT_BENCH_SLOTS=24" \
  "MCPT_REFILL_MIN=12" "MCPT_REFILL_MIN=28" "MCPT_TRI_MIN=8" "MCPT_TRI_MIN=24" "MCPT_BENCH_SLOTS=24" 2>&1 | grep -E "$F"
