#!/bin/bash
# Round-3 session o: any-hit rays far child first (libmcpt_anyfar.so): parity subset + A/B
# variant library: libmcpt_anyfar.so: git apply tools/experiments/anyhit_far_first.patch, then tools/build_variant.sh anyfar -DMCPT_X_ANYFAR
set -o pipefail
L=$PWD/mc-path-tracer_amd
MCPT_LIB=$L/libmcpt_anyfar.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "trace_parity or gpu_bvh_same_hits or config1_full or quad_nodes" --timeout 120 --timeout-method thread > gpurun_out/pytest_anyfar.log 2>&1 || { tail -30 gpurun_out/pytest_anyfar.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_anyfar.log | tail -1
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfar.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfar.so" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfar.so" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 4 --spp 64" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_anyfar.so" 2>&1 | grep -E "==|value|k_trace"
