#!/bin/bash
# A/B of whole-frame bench runs between library builds on one box (interleaved):
#   LIBS="new:mc-path-tracer_amd/libmcpt.so r3:mc-path-tracer_amd/libmcpt_r3.so" CONFIGS="2 3" ROUNDS=2 \
#   TEST=1 bash tools/gpu/ab_libs.sh
# An entry may set environment variables for its runs: "l3:mc-path-tracer_amd/libmcpt.so:MCPT_SIBLING_LAYOUT=3".
# TEST=1 first runs the GPU test suite on the default library.  Every GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ -n "$TEST" ]]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/ab_test.log 2>&1 || { grep -E "FAILED|Error|differ" gpurun_out/ab_test.log | head -20; tail -5 gpurun_out/ab_test.log; exit 1; }
  grep -E "passed|failed" gpurun_out/ab_test.log | tail -1
fi
for r in $(seq ${ROUNDS:-2}); do
  for cfg in ${CONFIGS:-2}; do
    for lv in ${LIBS}; do
      # name:lib[:VAR=VAL,VAR=VAL] -- optional environment for that entry
      name=${lv%%:*}; spec=${lv#*:}; lib=${spec%%:*}; envs=${spec#"$lib"}; envs=${envs#:}
      ( [[ -n "$envs" ]] && export ${envs//,/ }
      MCPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $cfg --steps ${STEPS:-4} --warmup 1 ${BENCH_ARGS} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -20 gpurun_out/ab_$name.err; exit 1; } ) || exit 1
      python - "$name" "$cfg" "gpurun_out/ab_$name.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[3])); r = d["roofline"]; p = r["per_ray"]
print(f"r{sys.argv[2]} {sys.argv[1]:>6} cfg{d['config']['workload'][16:17]} {d['value']:9.1f} Mray/s {d['ms_per_step']:8.2f} ms/frame "
      f"trace {r['avg_launch_ms']:.4f} ms/launch  ext nodes {p['ext_pair_nodes']} tests {p['ext_tri_tests']} any nodes {p['any_pair_nodes']} tests {p['any_tri_tests']} occ {p['any_resolved_by_occluder_cache']} shade {d['stage_ms_per_step']['k_shade+k_material']}")
PY
    done
  done
done
echo DONE
