set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/rk8
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 2 --steps 1 --warmup 0 > gpurun_out/c2_phases.json 2> gpurun_out/c2_phases.err || { tail -20 gpurun_out/c2_phases.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/rk8 -o rk --output-format csv -- python3 tools/rank_frames.py --config 2 --world 8 --rank 0 --frames 2 > gpurun_out/rk8.log 2>&1 || { tail -20 gpurun_out/rk8.log; exit 1; }
grep frame gpurun_out/rk8.log
python3 tools/iter_gaps.py 'gpurun_out/rk8/**/*kernel_trace.csv' > gpurun_out/rk8_gaps.json && cat gpurun_out/rk8_gaps.json
