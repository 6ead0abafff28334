#!/bin/bash
# Round-3 session b: GPU tests, the slot sweep of the whole-frame bench, the multi-rank rehearsal
# variant library: libmcpt_head.so: a build of an earlier commit (tools/build_rev_variant.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_b.log 2>&1 || { tail -40 gpurun_out/pytest_b.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_b.log | tail -1
L=$PWD/mc-path-tracer_amd
bash tools/gpu_kstats.sh "MCPT_LIB=$L/libmcpt_head.so MCPT_BENCH_SLOTS=5" "MCPT_BENCH_SLOTS=3" "MCPT_BENCH_SLOTS=4" "MCPT_BENCH_SLOTS=5" "MCPT_BENCH_SLOTS=6" "MCPT_BENCH_SLOTS=8" 2>&1 | grep -E "==|value|k_trace|k_material|k_shade"
# two ranks on the one GPU (gloo): the --gpus launcher, the partitioned frame and the gather to rank 0
MCPT_BENCH_BACKEND=gloo MCPT_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline --gather --verify-gather > gpurun_out/dist2.log 2>&1 || { tail -30 gpurun_out/dist2.log; exit 1; }
grep '^{"metric"' gpurun_out/dist2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dist2', d['n_gpus'], d['value'], d.get('gather_s'), d.get('gather_equals_one_rank_frame'))"
