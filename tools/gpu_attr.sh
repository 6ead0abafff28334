#!/bin/bash
# HBM-byte attribution of the shading kernels over diagnostic builds (one frame each)
# variant library: git apply tools/experiments/diag_env_attribution.patch, then tools/build_variant.sh diag_<X> -DMCPT_DIAG_<X>
set -o pipefail
export TMPDIR=/tmp
L=$PWD/mc-path-tracer_amd
A="--no-cpu-baseline --steps 1 --warmup 0"
for v in base diag_NO_RAY diag_NO_HIT diag_NO_ENVL diag_NO_ENVB; do
  if [[ $v == base ]]; then lib=$L/libmcpt.so; else lib=$L/libmcpt_$v.so; fi
  O=gpurun_out/attr_$v; rm -rf $O; mkdir -p $O
  MCPT_LIB=$lib timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch -o f --output-format csv -- python3 bench.py $A > $O/f.log 2>&1 || { tail -5 $O/f.log; exit 1; }
  MCPT_LIB=$lib timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write -o w --output-format csv -- python3 bench.py $A > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
done
python3 tools/diag_attr.py base diag_NO_RAY diag_NO_HIT diag_NO_ENVL diag_NO_ENVB
