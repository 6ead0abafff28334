#!/bin/bash
# Round-end measurement set on one box (every step time-limited, the chain stops at the first failure):
# GPU tests, smoke, the bench, its kernel-trace stats and PMC passes (config 2), the bench again with
# the fresh summaries in place, the occluder-table-off traffic pass (k_material byte attribution) and
# one N = 8 rank frame's kernel trace.  TAG names the outputs.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r06}
O=gpurun_out
mkdir -p $O
bash tools/gpu/run.sh test smoke || exit 1
TAG=$TAG STEPS=3 bash tools/gpu/run.sh bench kstats pmc || exit 1
# occluder table off: FETCH/WRITE passes only (attribution of k_material's bytes)
if [[ -z "$SKIP_OCC" ]]; then
  MCPT_OCC_G=0 TAG=${TAG}occoff STEPS=3 FETCH_ONLY=1 bash tools/gpu/run.sh kstats pmc || exit 1
fi
# one rank of the N = 8 strong split, kernel trace
rm -rf $O/rk8_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rk8_$TAG -o rk --output-format csv -- python3 tools/rank_frames.py --config 2 --world 8 --rank 0 --frames 2 > $O/rk8_$TAG.log 2>&1 || { tail -20 $O/rk8_$TAG.log; exit 1; }
python3 tools/iter_gaps.py "$O/rk8_$TAG/**/*kernel_trace.csv" > $O/rk8_gaps_$TAG.json
echo FINAL DONE
