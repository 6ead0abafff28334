#!/bin/bash
# Round-3 session d: quantised nodes (libmcpt_q.so) parity and A/B
# variant library: libmcpt_q.so: git apply tools/experiments/quantized_nodes.patch, then tools/build_variant.sh q -DMCPT_QNODES=1
set -o pipefail
mkdir -p gpurun_out
L=$PWD/mc-path-tracer_amd
md5sum $L/libmcpt_q.so $L/libmcpt.so
for b in host ploc; do MCPT_LIB=$L/libmcpt_q.so timeout -k 5 120 python -u tools/q_mismatch.py $b 1 || exit 1; done
MCPT_LIB=$L/libmcpt_q.so timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
grep -E "FAILED|passed|failed" gpurun_out/pytest_q.log | tail -12
VARIANTS="base q" CFGS=2,3,4,5 bash tools/gpu_cfg_lib_ab.sh || exit 1
