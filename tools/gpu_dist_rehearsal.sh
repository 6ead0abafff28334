#!/bin/bash
# N=2 bench rehearsal on a 1-GPU box: both ranks share the device, gloo collectives, film gather.
set -o pipefail
mkdir -p gpurun_out
MCPT_BENCH_BACKEND=gloo MCPT_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus ${NPROC:-2} --steps 20 --warmup 10 --gather \
  > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -30 gpurun_out/dist2.err; exit 1; }
cat gpurun_out/dist2.json
