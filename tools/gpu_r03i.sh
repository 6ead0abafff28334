#!/bin/bash
# Round-3 session i: SQ/TCC counter passes on configs 3, 4, 5 (their whole-frame bench commands)
# and config 4's kernel trace + FETCH/WRITE traffic
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
A4="--config 4 --no-cpu-baseline --steps 1 --warmup 0 --spp 64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4/prof_kt -o kt --output-format csv -- python3 bench.py $A4 > $O/c4_kt.log 2>&1 || { tail -20 $O/c4_kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/c4/prof_fetch -o fetch --output-format csv -- python3 bench.py $A4 > $O/c4_fetch.log 2>&1 || { tail -20 $O/c4_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/c4/prof_write -o write --output-format csv -- python3 bench.py $A4 > $O/c4_write.log 2>&1 || { tail -20 $O/c4_write.log; exit 1; }
timeout -k 10 300 python3 bench.py $A4 > $O/c4_bench64.log 2>&1 || { tail -20 $O/c4_bench64.log; exit 1; }
for c in 3 4 5; do
  P="bench.py --config $c --no-cpu-baseline --steps 1 --warmup 0"
  [[ $c != 3 ]] && P="$P --spp 64"
  PROG="$P" timeout -k 10 900 bash tools/pmc_trace.sh c$c || exit 1
done
echo DONE
