#!/bin/bash
set -o pipefail
# Configs 3-5 (CFGS) steady state under launch knobs, two rounds: KNOBS="label:VAR=value ..."
# ("base" = no knob).  Default: the k_trace refill thresholds REFILLS.
mkdir -p gpurun_out
if [[ -z $KNOBS ]]; then for r in ${REFILLS:-16 12 20 24}; do KNOBS="$KNOBS r$r:MCPT_REFILL_MIN=$r"; done; fi
for rnd in 1 2; do
for kv in base:X=1 $KNOBS; do
  l=${kv%%:*}
  env ${kv#*:} timeout -k 10 300 python -u tools/configs.py --configs ${CFGS:-3,4,5} --full 0 --out gpurun_out/cfg_$l.json > gpurun_out/cfg_$l.log 2>&1 || { tail -20 gpurun_out/cfg_$l.log; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/cfg_$l.json')); print('$l', [(c['config'], c['mray_s'], c['ms_trace']) for c in d])"
done
done
