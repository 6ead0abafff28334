#!/bin/bash
# Round 6: the occluder gate's cold first iteration (new: not judged) against HEAD's gate (g0).
set -o pipefail
mkdir -p gpurun_out
TEST_K="occluder or bench_layout_band_parity or native_gather or stage_golden" bash tools/gpu/run.sh test > gpurun_out/t_gate.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/test.log | head; tail -5 gpurun_out/test.log; exit 1; }
grep -E "passed|failed" gpurun_out/test.log | tail -1
for lib in new:mc-path-tracer_amd/libmcpt.so g0:mc-path-tracer_amd/libmcpt_g0.so; do
  n=${lib%%:*}; l=${lib#*:}
  for w in 8 1; do
    MCPT_LIB=$PWD/$l timeout -k 10 200 python -u tools/rank_frames.py --config 2 --world $w --rank 0 --frames 2 > gpurun_out/gate_$n_$w.log 2>&1 || { tail -5 gpurun_out/gate_$n_$w.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/gate_$n_$w.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if not d['warmup']: print('$n world $w', d['wall_ms'], 'ms trace', d['ms_trace'], 'shade', d['ms_shade'], 'occ', d['occ_resolved_frac'], 'any traversed', d['ray_counts']['any_hit_traversed'], 'iters', d['iterations'])
"
  done
done
LIBS="new:mc-path-tracer_amd/libmcpt.so g0:mc-path-tracer_amd/libmcpt_g0.so" CONFIGS="2 3" ROUNDS=2 STEPS=4 bash tools/gpu/ab_libs.sh || exit 1
echo ALL DONE
