# A/B of the steady-state bench under environment settings: bash tools/gpu_ab.sh "A=1" "A=0 B=2" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ -n "$AB_TEST" ]]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-full-frame --steps 60 --warmup 30 ${AB_ARGS} > gpurun_out/ab.json 2>gpurun_out/ab.err || { cat gpurun_out/ab.err; exit 1; }
  echo "$cfg: $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'],d['stage_ms_per_step'],d['roofline']['per_ray'])")"
done
