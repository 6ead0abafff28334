set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_tprof.so timeout -k 10 120 python -u tools/trace_prof.py > gpurun_out/tprof.log 2>&1 || { cat gpurun_out/tprof.log; exit 1; }
cat gpurun_out/tprof.log
