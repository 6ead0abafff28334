set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 2 --steps 2 --warmup 1 > gpurun_out/c2_share.json 2> gpurun_out/c2_share.err || { tail -20 gpurun_out/c2_share.err; exit 1; }
MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_base.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --config 2 --steps 2 --warmup 1 > gpurun_out/c2_base.json 2> gpurun_out/c2_base.err || { tail -20 gpurun_out/c2_base.err; exit 1; }
MCPT_LIB=$PWD/mc-path-tracer_amd/libmcpt_diagshade.so timeout -k 10 300 python -u tools/shade_sections.py --config 2 --out gpurun_out/shade_sections_c2.json > gpurun_out/shade_sections.log 2>&1 || { tail -20 gpurun_out/shade_sections.log; exit 1; }
CONFIG=2 TAG=r06x ENVS="MCPT_TRI_MIN=32|MCPT_TRI_MIN=48|MCPT_TRI_MIN=8" ROUNDS=1 bash tools/gpu/run.sh abenv
