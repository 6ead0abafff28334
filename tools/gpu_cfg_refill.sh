#!/bin/bash
set -o pipefail
# Configs 3-5 steady state at several k_trace refill thresholds (MCPT_REFILL_MIN), two rounds.
mkdir -p gpurun_out
for rnd in 1 2; do
for r in ${REFILLS:-16 12 20 24}; do
  MCPT_REFILL_MIN=$r timeout -k 10 300 python -u tools/configs.py --configs 3,4,5 --full 0 --out gpurun_out/cfg_r$r.json > gpurun_out/cfg_r$r.log 2>&1 || { tail -20 gpurun_out/cfg_r$r.log; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/cfg_r$r.json')); print('refill $r', [(c['config'], c['mray_s'], c['ms_trace']) for c in d])"
done
done
