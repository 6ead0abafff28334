#!/bin/bash
# Occluder-table shape against the rank layout (round 6): one rank of the N = 8 strong split and the
# one-GPU frame, config 2, per MCPT_OCC_G / MCPT_OCC_B setting (tools/rank_frames.py, 2 frames each).
set -o pipefail
mkdir -p gpurun_out
for w in 8 1; do
  for e in "MCPT_X=0" "MCPT_OCC_G=16" "MCPT_OCC_G=12" "MCPT_OCC_G=8" "MCPT_OCC_G=12 MCPT_OCC_B=8"; do
    env $e timeout -k 10 200 python -u tools/rank_frames.py --config 2 --world $w --rank 0 --frames 2 > gpurun_out/occw.log 2>&1 || { tail -5 gpurun_out/occw.log; exit 1; }
    python3 -c "
import json,sys
for l in open('gpurun_out/occw.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if not d['warmup']: print('world $w', '$e'.ljust(28), d['wall_ms'], 'ms trace', d['ms_trace'], 'shade', d['ms_shade'], 'occ', d['occ_resolved_frac'], 'any traversed', d['ray_counts']['any_hit_traversed'])
"
  done
done
echo DONE
