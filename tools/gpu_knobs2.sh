#!/bin/bash
# Config-2 steady-state sweep of the refill / triangle-phase thresholds (env knobs), interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-full-frame > gpurun_out/knob_$label.json 2> gpurun_out/knob_$label.err \
    || { tail -5 gpurun_out/knob_$label.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/knob_$label.json')); print('$label', d['value'], d['stage_ms_per_step'])"
}
for r in 1 2; do
  run base$r X=1
  for k in ${REFILLS:-20 24 28 32}; do run r${k}_$r MCPT_REFILL_MIN=$k; done
done
