set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="v0 hr" ROUNDS=3 bash tools/gpu_ab_mix.sh || exit 1
