#!/bin/bash
# Round-3 session h: the 24-slot frame profile and config 4's literal frame (3840x2160, 1024 spp)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/frame_profile.py 24 > gpurun_out/frame_profile24.log 2>&1 || { tail -20 gpurun_out/frame_profile24.log; exit 1; }
cat gpurun_out/frame_profile24.log
timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c4_bench.log 2>&1 || { tail -20 gpurun_out/c4_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/c4_bench.log | cut -c1-300
