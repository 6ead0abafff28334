#!/bin/bash
# Path-slot checks on one GPU: the slot parity tests, then config 2 benches at 1..4 slots.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -k "path_slots" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/slots_test.log 2>&1 || { tail -40 gpurun_out/slots_test.log; exit 1; }
tail -4 gpurun_out/slots_test.log
for s in ${SLOTS:-1 2 3 4}; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --slots $s > gpurun_out/bench_s$s.json 2> gpurun_out/bench_s$s.err \
    || { tail -20 gpurun_out/bench_s$s.err; exit 1; }
done
echo DONE
