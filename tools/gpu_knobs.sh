#!/bin/bash
# Config-2 steady-state sweep of the traversal launch knobs (env) and a variant library.
# variant library: libmcpt_mat5.so: tools/build_variant.sh mat5 -DMCPT_MAT_WPE=5
set -o pipefail
mkdir -p gpurun_out
run() {  # label, env assignments...
  local label=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-full-frame > gpurun_out/knob_$label.json 2> gpurun_out/knob_$label.err \
    || { tail -5 gpurun_out/knob_$label.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/knob_$label.json')); print('$label', d['value'], d['stage_ms_per_step'])"
}
run base X=1
run w24 MCPT_TRACE_WAVES=24
run w32 MCPT_TRACE_WAVES=32
run r8 MCPT_REFILL_MIN=8
run r24 MCPT_REFILL_MIN=24
run t8 MCPT_TRI_MIN=8
run t24 MCPT_TRI_MIN=24
run mat5 MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_mat5.so
run base2 X=1
