#!/bin/bash
# A/B of one env knob on the config-2 bench, interleaved: A B A B (steady state + full frame).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in A B; do
    if [[ $v == A ]]; then E="X=1"; else E="$KNOB"; fi
    env $E timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err \
      || { tail -5 gpurun_out/ab_$v$r.err; exit 1; }
    python -c "
import json; d = json.load(open('gpurun_out/ab_$v$r.json')); print('$v', '$E', d['value'], d['stage_ms_per_step'], d['full_frame']['seconds'])"
  done
done
