#!/bin/bash
# Round-3 session: occluder-cache record of the occluder's record pair (2k, 2k+1: the two triangles of
# a quad, or neighbours in leaf order) in one 8-B store (MCPT_OCC_PAIR=1 build)
set -o pipefail
L=$PWD/mc-path-tracer_amd
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_occpair.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_occpair.so" 2>&1 | grep -E "==|value|k_trace|k_material"
KS_STEPS=1 KS_ARGS="--config 5 --spp 64" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_occpair.so" 2>&1 | grep -E "==|value|k_trace|k_material"
