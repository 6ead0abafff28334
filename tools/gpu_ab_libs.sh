#!/bin/bash
# Interleaved config-2 bench over variant libraries: LIBS="name1 name2 ..." (libmcpt_<name>.so;
# "base" = libmcpt.so), ROUNDS rounds.
set -o pipefail
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
  for n in ${LIBS}; do
    if [[ $n == base ]]; then L=$PWD/mc-path-tracer_amd/libmcpt.so; else L=$PWD/mc-path-tracer_amd/libmcpt_$n.so; fi
    MCPT_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline --no-full-frame > gpurun_out/abl_$n$r.json 2> gpurun_out/abl_$n$r.err \
      || { tail -5 gpurun_out/abl_$n$r.err; exit 1; }
    python -c "
import json; d = json.load(open('gpurun_out/abl_$n$r.json')); print('$n', d['value'], d['stage_ms_per_step'])"
  done
done
