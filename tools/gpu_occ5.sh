#!/bin/bash
# Round-3 session: occluder-cache entries prefetched inside material() + all four candidates in one
# round trip (working tree) against HEAD's sequential lookups (libmcpt_head.so); section profile.
set -o pipefail
L=$PWD/mc-path-tracer_amd
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_occ.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_occ.log | head -20; tail -5 gpurun_out/pytest_occ.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_occ.log | tail -1
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_LIB=$L/libmcpt_head.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_head.so" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
SLOTS=24 MCPT_LIB=$L/libmcpt_sprof.so timeout -k 10 300 python tools/shade_prof.py
