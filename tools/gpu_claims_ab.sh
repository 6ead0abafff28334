set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_claims.log 2>&1 || { tail -40 gpurun_out/pytest_claims.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_claims.log | tail -2
VARIANTS="head base base:MCPT_BENCH_SLOTS=4 base:MCPT_BENCH_SLOTS=5 base:MCPT_BENCH_SLOTS=2" ROUNDS=2 bash tools/gpu_ab_mix.sh || exit 1
timeout -k 10 120 python tools/frame_profile.py 3 > gpurun_out/fp3.log 2>&1 && cat gpurun_out/fp3.log
timeout -k 10 120 python tools/frame_profile.py 4 > gpurun_out/fp4.log 2>&1 && cat gpurun_out/fp4.log
