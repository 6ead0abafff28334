#!/bin/bash
# Round-3 GPU session: tests, smoke, the FETCH/WRITE calibration, the config-2 bench with its
# rocprofv3 kernel trace + PMC traffic + SQ counter passes, and the same evidence for configs 3
# and 5.  Every GPU step has its own time limit; the chain stops at the first failure.
#   usage: tools/gpu_r03.sh [all|test|calib|bench|prof|detail|cfg]   (TAG=r03)
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-r03}
STEP=${1:-all}
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "FAILED: $name (rc $?)"; tail -30 $O/$name.log; exit 1; }
}
if [[ $STEP == all || $STEP == test ]]; then
  run pytest_gpu 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread
  tail -30 $O/pytest_gpu.log | grep -E "passed|failed|s call" | head -20
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  tail -3 $O/smoke.log
fi
if [[ $STEP == all || $STEP == calib ]]; then
  run calib_run 120 tools/hbm/fetch_calib
  cp $O/calib_run.log $O/calib.jsonl
  run calib_fetch_p 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/calib_fetch -o f --output-format csv -- tools/hbm/fetch_calib
  run calib_write_p 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/calib_write -o w --output-format csv -- tools/hbm/fetch_calib
  python tools/fetch_calib.py $TAG $O
fi
if [[ $STEP == all || $STEP == bench ]]; then
  run bench 600 python bench.py
  cat $O/bench.log | tail -1
fi
B2="--no-cpu-baseline"
if [[ $STEP == all || $STEP == prof ]]; then
  run prof_kt_p 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o kt --output-format csv -- python3 bench.py $B2
  run prof_fetch_p 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/prof_fetch -o fetch --output-format csv -- python3 bench.py $B2 --steps 1 --warmup 0
  run prof_write_p 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/prof_write -o write --output-format csv -- python3 bench.py $B2 --steps 1 --warmup 0
  PMC_ARGS="$B2" python tools/pmc.py $TAG $O > /dev/null
fi
if [[ $STEP == all || $STEP == detail ]]; then
  export PROG="bench.py $B2 --steps 1 --warmup 0"
  run pmct 900 tools/pmc_trace.sh bench
  python tools/pmc_detail.py $TAG bench $O
fi
if [[ $STEP == all || $STEP == bench || $STEP == prof || $STEP == detail ]]; then
  # the bench again, now reading this session's (box-local) traffic and counter summaries
  run bench2 600 python bench.py --no-cpu-baseline
  tail -1 $O/bench2.log
fi
if [[ $STEP == all || $STEP == cfg ]]; then
  for c in 3 5; do
    A="--config $c --no-cpu-baseline --steps 1 --warmup 0"
    [[ $c == 5 ]] && A="$A --spp 64"
    run c${c}_kt_p 600 rocprofv3 --kernel-trace --stats -d $O/c${c}_kt -o kt --output-format csv -- python3 bench.py $A
    run c${c}_fetch_p 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/c${c}_fetch -o fetch --output-format csv -- python3 bench.py $A
    run c${c}_write_p 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/c${c}_write -o write --output-format csv -- python3 bench.py $A
    mkdir -p $O/c${c} && rm -rf $O/c${c}/prof_kt $O/c${c}/prof_fetch $O/c${c}/prof_write
    mv $O/c${c}_kt $O/c${c}/prof_kt && mv $O/c${c}_fetch $O/c${c}/prof_fetch && mv $O/c${c}_write $O/c${c}/prof_write
    PMC_CONFIG=$c PMC_ARGS="$A" PMC_NAME=pmc_c${c}_$TAG STATS_NAME=kernel_stats_c${c}_$TAG python tools/pmc.py $TAG $O/c${c} > /dev/null
    run c${c}_bench 900 python bench.py $A
    tail -1 $O/c${c}_bench.log
  done
fi
echo DONE
