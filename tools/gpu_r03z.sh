#!/bin/bash
# Round-3 final check on the committed sources: GPU tests, smoke, the default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_final.log | head; tail -5 gpurun_out/pytest_final.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_final.log | tail -1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{"metric"' gpurun_out/bench_final.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['bound'], r['frac'], r.get('traffic'), r.get('pmc_stale'), d['cpu_baseline']['value'])"
