#!/bin/bash
# Round 6: the occluder table pre-filled at upload by probe rays (default) against an empty table
# at every film clear (MCPT_OCC_PREFILL=0): GPU parity tests, rank frames at N = 8 / 1, whole frames.
set -o pipefail
mkdir -p gpurun_out
TEST_K="occluder or bench_layout_band_parity or native_gather or stage_golden or smoke or config2" bash tools/gpu/run.sh test > gpurun_out/t_pf.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/test.log | head; tail -5 gpurun_out/test.log; exit 1; }
grep -E "passed|failed" gpurun_out/test.log | tail -1
for e in "MCPT_X=0" "MCPT_OCC_PREFILL=0"; do
  for w in 8 1; do
    env $e timeout -k 10 200 python -u tools/rank_frames.py --config 2 --world $w --rank 0 --frames 2 > gpurun_out/pf.log 2>&1 || { tail -5 gpurun_out/pf.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/pf.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if not d['warmup']: print('$e'.ljust(20), 'world $w', d['wall_ms'], 'ms trace', d['ms_trace'], 'shade', d['ms_shade'], 'occ', d['occ_resolved_frac'], 'any traversed', d['ray_counts']['any_hit_traversed'])
"
  done
done
for c in 2 3; do
  CONFIG=$c ENVS="MCPT_X=0|MCPT_OCC_PREFILL=0" ROUNDS=2 STEPS=4 bash tools/gpu/run.sh abenv > gpurun_out/ab_pf_c$c.log 2>&1 || { tail -5 gpurun_out/ab_pf_c$c.log; exit 1; }
  grep MCPT gpurun_out/ab_pf_c$c.log | sed "s/^/C$c /"
done
echo ALL DONE
