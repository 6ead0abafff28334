#!/bin/bash
# Config-2 steady-state sweep of launch knobs (env), interleaved rounds.
# KNOBS="label:VAR=value ..." (default: refill thresholds), ROUNDS (default 2); "base" runs with no knob.
set -o pipefail
mkdir -p gpurun_out
run() {
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-full-frame > gpurun_out/knob_$label.json 2> gpurun_out/knob_$label.err \
    || { tail -5 gpurun_out/knob_$label.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/knob_$label.json')); print('$label', d['value'], d['stage_ms_per_step'])"
}
KNOBS=${KNOBS:-"r16:MCPT_REFILL_MIN=16 r24:MCPT_REFILL_MIN=24"}
for r in $(seq ${ROUNDS:-2}); do
  run base_$r X=1
  for kv in $KNOBS; do run ${kv%%:*}_$r ${kv#*:}; done
done
