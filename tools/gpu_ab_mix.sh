#!/bin/bash
# Interleaved config-2 bench (whole-frame steps) over (library, environment) variants, ROUNDS rounds:
#   VARIANTS="base nosteal base:MCPT_TRACE_PARTS=16" bash tools/gpu_ab_mix.sh
# name = libmcpt_<name>.so ("base" = libmcpt.so); ":K=V,K2=V2" adds environment settings.
set -o pipefail
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    n=${v%%:*}; e=""; [[ $v == *:* ]] && e=${v#*:}
    if [[ $n == base ]]; then L=$PWD/mc-path-tracer_amd/libmcpt.so; else L=$PWD/mc-path-tracer_amd/libmcpt_$n.so; fi
    env ${e//,/ } MCPT_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline ${AB_ARGS} > gpurun_out/abm.json 2> gpurun_out/abm.err \
      || { tail -5 gpurun_out/abm.err; exit 1; }
    python -c "
import json; d = json.load(open('gpurun_out/abm.json')); print('%-36s' % '$v', d['value'], d['ms_per_step'], d['config']['iterations_per_step_rank0'], d['stage_ms_per_step'])"
  done
done
