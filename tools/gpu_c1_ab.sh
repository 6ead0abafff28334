#!/bin/bash
# Config-1 whole-frame time under (library, environment) variants, interleaved:
#   VARIANTS="base nosteal base:MCPT_TRACE_PARTS=8" bash tools/gpu_c1_ab.sh
set -o pipefail
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-3}); do
  for v in ${VARIANTS}; do
    n=${v%%:*}; e=""; [[ $v == *:* ]] && e=${v#*:}
    if [[ $n == base ]]; then L=$PWD/mc-path-tracer_amd/libmcpt.so; else L=$PWD/mc-path-tracer_amd/libmcpt_$n.so; fi
    env ${e//,/ } MCPT_LIB=$L timeout -k 10 120 python tools/configs.py --configs 1 --out gpurun_out/c1.json > gpurun_out/c1.log 2>&1 || { tail -5 gpurun_out/c1.log; exit 1; }
    python -c "
import json; d = json.load(open('gpurun_out/c1.json'))[0]; print('%-32s' % '$v', d['full_frame'])"
  done
done
