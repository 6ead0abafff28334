set -o pipefail
for w in 28 24 20 16; do
  echo "== waves/CU $w"
  MCPT_TRACE_WAVES=$w timeout -k 10 200 python tools/overlap_exp.py 1 2 || exit 1
done
