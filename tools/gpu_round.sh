#!/bin/bash
# One GPU session: tests, bench, rocprofv3 kernel trace + PMC passes.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
STEP=${1:-all}
if [[ $STEP == all || $STEP == test ]]; then
  timeout -k 10 900 python -u -m pytest tests/ -v -m gpu -x --timeout 300 --timeout-method thread> $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [[ $STEP == all || $STEP == prof ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-full-frame --steps 60 --warmup 30 > $OUT/prof_kt.log 2>&1 || { echo "rocprof kt failed"; tail -30 $OUT/prof_kt.log; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/prof_fetch -o fetch --output-format csv -- python3 bench.py --no-cpu-baseline --no-full-frame --steps 20 --warmup 10 > $OUT/prof_fetch.log 2>&1 || { echo "rocprof fetch failed"; tail -30 $OUT/prof_fetch.log; exit 1; }
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/prof_write -o write --output-format csv -- python3 bench.py --no-cpu-baseline --no-full-frame --steps 20 --warmup 10 > $OUT/prof_write.log 2>&1 || { echo "rocprof write failed"; tail -30 $OUT/prof_write.log; exit 1; }
  python tools/pmc.py ${TAG:-r02} $OUT > /dev/null  # box-local profiles/ so the bench below reads this run's traffic
fi
if [[ $STEP == all || $STEP == prof || $STEP == bench2 ]]; then
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
echo DONE
