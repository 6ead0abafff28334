#!/bin/bash
# Round-3 session: k_shade / k_material section profile at the bench's 24 slots (occluder cache on),
# and the whole-frame per-iteration profile
set -o pipefail
mkdir -p gpurun_out
L=$PWD/mc-path-tracer_amd
SLOTS=24 MCPT_LIB=$L/libmcpt_sprof.so timeout -k 10 300 python tools/shade_prof.py
timeout -k 10 300 python tools/frame_profile.py 24
