#!/bin/bash
# quantised-node sanity per config (bounded): base vs libmcpt_q.so
# variant library: libmcpt_q.so: git apply tools/experiments/quantized_nodes.patch, then tools/build_variant.sh q -DMCPT_QNODES=1
mkdir -p gpurun_out
L=$PWD/mc-path-tracer_amd
for c in 2 4 3 5; do
  for lib in libmcpt.so libmcpt_q.so; do
    echo "== $lib"
    MCPT_LIB=$L/$lib timeout -k 5 60 python -u tools/q_diag.py $c || { echo "FAILED rc=$? ($lib config $c)"; exit 1; }
  done
done
