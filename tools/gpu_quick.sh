#!/bin/bash
# Quick GPU check after a kernel change: every GPU test, then the config-2 bench without the CPU
# baseline (BENCH_ARGS adds flags).  Each step has its own time limit; the chain stops at a failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/quick_test.log 2>&1 || { tail -40 gpurun_out/quick_test.log; exit 1; }
tail -2 gpurun_out/quick_test.log
timeout -k 10 200 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err \
    || { tail -20 gpurun_out/quick_bench.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/quick_bench.json'))
print('value', d['value'], 'stage ms', d['stage_ms_per_step'], 'full frame s', d['full_frame']['seconds'])"
