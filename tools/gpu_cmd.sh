set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_sprof.so timeout -k 10 120 python -u tools/shade_prof.py > gpurun_out/sprof.log 2>&1 || { cat gpurun_out/sprof.log; exit 1; }
cat gpurun_out/sprof.log
run() { timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-full-frame --steps 60 --warmup 30 > gpurun_out/b.json 2>gpurun_out/bench.err || { cat gpurun_out/bench.err; exit 1; }
 echo "$1: $(python -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['value'],d['stage_ms_per_step'])")"; }
run base
MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_sw8.so run shade_wpe8
run base2
