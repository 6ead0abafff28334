#!/bin/bash
# Round-3 session m: k_material at 5 waves/SIMD (96 VGPRs, 16 spilled) vs 4, whole frames
# variant library: libmcpt_mat5.so: tools/build_variant.sh mat5 -DMCPT_MAT_WPE=5
set -o pipefail
L=$PWD/mc-path-tracer_amd
KS_STEPS=2 bash tools/gpu_kstats.sh "MCPT_X=0" "MCPT_LIB=$L/libmcpt_mat5.so" "MCPT_X=0" "MCPT_LIB=$L/libmcpt_mat5.so" 2>&1 | grep -E "==|value|k_material"
