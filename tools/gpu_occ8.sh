#!/bin/bash
# Round-3 session: occluder cache emptied with every film clear (working tree) against the table kept
# across frames (libmcpt_head.so); GPU parity first
set -o pipefail
L=$PWD/mc-path-tracer_amd
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_occ.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_occ.log | head -20; tail -5 gpurun_out/pytest_occ.log; exit 1; }
grep -E "passed|failed|resolved by the" gpurun_out/pytest_occ.log | tail -6
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_head.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_head.so" 2>&1 | grep -E "==|value|k_trace|k_material"
