#!/bin/bash
# The one GPU-session driver (gpurun): every step has its own time limit, the chain stops at the
# first failure, outputs land in gpurun_out/.  Steps run in the order given:
#
#   bash tools/gpu/run.sh test smoke bench kstats pmc partition
#
#   test       python -m pytest tests -m gpu (TEST_ARGS adds pytest arguments, TEST_K a -k expression)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py $BENCH_ARGS                      -> gpurun_out/bench_$TAG.json
#   kstats     rocprofv3 --kernel-trace --stats of bench  -> gpurun_out/kt_$TAG/ (profiled runs pass
#              --no-work-counters: no extra counting frame, every launch is a timed or warmup frame's)
#   pmc        FETCH_SIZE and WRITE_SIZE passes (separate runs, gpurun_out/pmcraw_<sfx>/) + four SQ /
#              TCC counter passes of the same bench command (gpurun_out/pmct_<sfx>/), summarised by
#              tools/pmc.py / tools/pmc_detail.py into profiles/ (kernel_stats_*, pmc_*, pmcdetail_*
#              named by TAG and CONFIG; profiles/ on the box is not copied back: re-run both tools
#              here on the merged gpurun_out/).  FETCH_ONLY=1: the two traffic passes only
#   ab         whole-frame A/B of library builds, interleaved (LIBS="a:path.so b:path.so", CONFIGS,
#              ROUNDS; tools/gpu/ab_libs.sh)
#   abenv      the same for environment settings (ENVS="A=1|A=0 B=2", '|'-separated)
#   abargs     the same for bench arguments (ARGSETS="--slots 16|--slots 24")
#   partition  tools/partition_rehearsal.py (PART_ARGS)       -> gpurun_out/partition_$TAG.json
#
# Parameters (environment): CONFIG (2), TAG (r04), STEPS (bench frames, 3), BENCH_ARGS.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CONFIG=${CONFIG:-2}
TAG=${TAG:-r05}
STEPS=${STEPS:-3}
O=gpurun_out
BARGS="--no-cpu-baseline --config $CONFIG --steps $STEPS --warmup 1 ${BENCH_ARGS}"
sfx=$([[ $CONFIG == 2 ]] && echo "$TAG" || echo "c${CONFIG}_$TAG")

fail() { echo "step $1 failed"; tail -${2:-30} "$3"; exit 1; }

for step in "$@"; do
  case $step in
  test)
    timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread ${TEST_ARGS} ${TEST_K:+-k "$TEST_K"} \
      > $O/test.log 2>&1 || { grep -E "FAILED|Error|differ" $O/test.log | head -20; fail test 5 $O/test.log; }
    grep -E "passed|failed" $O/test.log | tail -1 ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke 20 $O/smoke.log
    tail -2 $O/smoke.log ;;
  bench)
    timeout -k 10 600 python -u bench.py $BARGS > $O/bench_$sfx.json 2> $O/bench_$sfx.err || fail bench 20 $O/bench_$sfx.err
    cut -c1-600 $O/bench_$sfx.json ;;
  kstats)
    rm -rf $O/kt_$sfx
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt_$sfx -o kt --output-format csv -- python3 bench.py $BARGS --no-work-counters \
      > $O/kt_$sfx.log 2>&1 || fail kstats 20 $O/kt_$sfx.log
    f=$(find $O/kt_$sfx -name "*kernel_stats.csv" | head -1)
    cp "$f" $O/kernel_stats_$sfx.csv
    grep '^{"metric"' $O/kt_$sfx.log | tail -1 > $O/bench_kt_$sfx.json
    python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "mcpt_dev" in r["Name"]:
        print(f'  {r["Name"][:64]:64s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.2f} total_ms {float(r["TotalDurationNs"])/1e6:9.2f}')
PY
    ;;
  pmc)
    R=$O/pmcraw_$sfx  # per config: one call's configs must not overwrite each other's raw passes
    rm -rf $R && mkdir -p $R
    for c in FETCH_SIZE WRITE_SIZE; do
      d=$R/prof_$([[ $c == FETCH_SIZE ]] && echo fetch || echo write)
      timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace -d $d -o p --output-format csv -- python3 bench.py $BARGS --no-work-counters \
        > $d.log 2>&1 || fail "pmc $c" 20 $d.log
    done
    if [[ "$FETCH_ONLY" == 1 ]]; then echo "fetch/write passes only"; continue; fi
    mkdir -p $R/prof_kt && cp $O/kernel_stats_$sfx.csv $R/prof_kt/kt_kernel_stats.csv 2>/dev/null
    i=0
    rm -rf $O/pmct_$sfx && mkdir -p $O/pmct_$sfx
    for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
               "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
               "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" \
               "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
      i=$((i+1))
      timeout -k 10 600 rocprofv3 --pmc $set --kernel-trace -d $O/pmct_$sfx/p$i -o p$i --output-format csv -- python3 bench.py $BARGS --no-work-counters \
        > $O/pmct_$sfx/p$i.log 2>&1 || fail "pmc pass $i" 10 $O/pmct_$sfx/p$i.log
    done
    PMC_CONFIG=$CONFIG PMC_ARGS="$BARGS" STATS_NAME=kernel_stats_$sfx python3 tools/pmc.py $sfx $R > /dev/null &&
      PMC_CONFIG=$CONFIG PMC_ARGS="$BARGS" python3 tools/pmc_detail.py $sfx $sfx $O || fail "pmc summary" 5 /dev/null
    ls profiles/*_$sfx* ;;
  ab)
    bash tools/gpu/ab_libs.sh || exit 1 ;;
  abenv)
    IFS='|' read -ra envs <<< "$ENVS"
    for r in $(seq ${ROUNDS:-2}); do
      for e in "${envs[@]}"; do
        env $e timeout -k 10 300 python -u bench.py $BARGS > $O/abenv.json 2> $O/abenv.err || fail abenv 20 $O/abenv.err
        python3 -c "
import json; d = json.load(open('$O/abenv.json')); r = d['roofline']; p = r['per_ray']
print('$e'.ljust(30), round(d['value'], 1), 'Mray/s', d['ms_per_step'], 'ms/frame trace', r['avg_launch_ms'], 'shade',
      d['stage_ms_per_step']['k_shade+k_material'], 'ext nodes/tests', p['ext_pair_nodes'], p['ext_tri_tests'],
      'any', p['any_pair_nodes'], p['any_tri_tests'], 'occ', p['any_resolved_by_occluder_cache'])"
      done
    done ;;
  abargs)
    # the same for bench arguments (ARGSETS="--slots 16|--slots 24", '|'-separated), added to BARGS
    IFS='|' read -ra sets <<< "$ARGSETS"
    for r in $(seq ${ROUNDS:-2}); do
      for e in "${sets[@]}"; do
        timeout -k 10 600 python -u bench.py $BARGS $e > $O/abargs.json 2> $O/abargs.err || fail abargs 20 $O/abargs.err
        python3 -c "
import json; d = json.load(open('$O/abargs.json')); r = d['roofline']
print('$e'.ljust(30), round(d['value'], 1), 'Mray/s', d['ms_per_step'], 'ms/frame trace', r['avg_launch_ms'], 'shade',
      d['stage_ms_per_step']['k_shade+k_material'], 'slots', d['config']['path_slots'], 'iterations', d['config']['iterations_per_step_rank0'])"
      done
    done ;;
  partition)
    timeout -k 10 900 python -u tools/partition_rehearsal.py --out $O/partition_$TAG.json ${PART_ARGS} > $O/partition.log 2>&1 || fail partition 20 $O/partition.log
    cat $O/partition.log ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
echo DONE
