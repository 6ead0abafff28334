# Per-kernel durations of the whole-frame bench under environment settings:
#   bash tools/gpu_kstats.sh "A=1" "A=0" ...   (MCPT_LIB=<variant .so> selects a library build;
#   KS_ARGS="--config 3" passes bench arguments)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  rm -rf gpurun_out/ks$i
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks$i -o ks --output-format csv -- python3 bench.py --no-cpu-baseline ${KS_ARGS:-} --steps ${KS_STEPS:-2} --warmup 1 > gpurun_out/ks$i.log 2>&1 || { tail -20 gpurun_out/ks$i.log; exit 1; }
  f=$(find gpurun_out/ks$i -name "*kernel_stats.csv" | head -1)
  echo "== $cfg"; grep '^{"metric"' gpurun_out/ks$i.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  value', d['value'], 'ms/frame', d['ms_per_step'], 'iters', d['config']['iterations_per_step_rank0'], 'per_ray', d['roofline']['per_ray'])"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith(("mcpt_dev", "void mcpt_dev")):
        print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:8.2f} total_ms {float(r["TotalDurationNs"])/1e6:9.2f}')
PY
done
