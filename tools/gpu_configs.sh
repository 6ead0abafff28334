#!/bin/bash
# All BASELINE configs on one GPU (tools/configs.py) -> gpurun_out/configs.json
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/configs.py --out gpurun_out/configs.json $CFG_ARGS > gpurun_out/configs.log 2>&1 \
  || { tail -20 gpurun_out/configs.log; exit 1; }
cat gpurun_out/configs.log
