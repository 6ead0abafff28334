#!/bin/bash
# Round-3 session n: node steps per trip (3/4/5/6) at the new slot counts, configs 2 and 3
# variant library: libmcpt_ns<N>.so: tools/build_variant.sh ns<N> -DMCPT_NODE_STEPS=<N>
set -o pipefail
L=$PWD/mc-path-tracer_amd
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_ns3.so" "MCPT_LIB=$L/libmcpt_ns5.so" "MCPT_LIB=$L/libmcpt_ns6.so" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace"
KS_STEPS=1 KS_ARGS="--config 3" bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_ns5.so" "MCPT_LIB=$L/libmcpt_ns6.so" "MCPT_X=0" 2>&1 | grep -E "==|value|k_trace"
