#!/bin/bash
# Round 6: occluder pre-fill probes per key (p1 = product, p2 / p4 = -DMCPT_OCC_PROBES builds)
set -o pipefail
mkdir -p gpurun_out
for lib in p1:mc-path-tracer_amd/libmcpt.so p2:mc-path-tracer_amd/libmcpt_p2.so p4:mc-path-tracer_amd/libmcpt_p4.so; do
  n=${lib%%:*}; l=${lib#*:}
  for w in 8 1; do
    MCPT_LIB=$PWD/$l timeout -k 10 200 python -u tools/rank_frames.py --config 2 --world $w --rank 0 --frames 2 > gpurun_out/pr.log 2>&1 || { tail -5 gpurun_out/pr.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/pr.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if not d['warmup']: print('$n world $w', d['wall_ms'], 'ms trace', d['ms_trace'], 'shade', d['ms_shade'], 'occ', d['occ_resolved_frac'], 'any traversed', d['ray_counts']['any_hit_traversed'])
"
  done
done
LIBS="p1:mc-path-tracer_amd/libmcpt.so p2:mc-path-tracer_amd/libmcpt_p2.so p4:mc-path-tracer_amd/libmcpt_p4.so" CONFIGS="2" ROUNDS=2 STEPS=4 bash tools/gpu/ab_libs.sh || exit 1
echo ALL DONE
