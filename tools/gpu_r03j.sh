#!/bin/bash
# Round-3 session j: two parked leaves per lane (libmcpt_leaf2.so): parity subset + whole-frame A/B
# variant library: libmcpt_leaf2.so: git apply tools/experiments/two_leaf_slots.patch, then tools/build_variant.sh leaf2 -DMCPT_X_LEAF2
set -o pipefail
L=$PWD/mc-path-tracer_amd
MCPT_LIB=$L/libmcpt_leaf2.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "trace_parity or gpu_bvh_same_hits or config1_full or quad_nodes" --timeout 120 --timeout-method thread > gpurun_out/pytest_leaf2.log 2>&1 || { tail -30 gpurun_out/pytest_leaf2.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_leaf2.log | tail -1
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_leaf2.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_leaf2.so" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=2 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_leaf2.so" 2>&1 | grep -E "==|value|k_trace"
