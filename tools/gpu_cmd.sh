set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -2
grep facade gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { tail -20 gpurun_out/quick_bench.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/quick_bench.json'))
print('value', d['value'], 'stage ms', d['stage_ms_per_step'], 'per_ray', d['roofline']['per_ray'])"
