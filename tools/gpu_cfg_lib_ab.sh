set -o pipefail
for r in 1 2; do for v in ${VARIANTS:-base}; do
  if [[ $v == base ]]; then L=$PWD/mc-path-tracer_amd/libmcpt.so; else L=$PWD/mc-path-tracer_amd/libmcpt_$v.so; fi
  MCPT_LIB=$L timeout -k 10 400 python tools/configs.py --configs ${CFGS:-3,5} --full 0 --out gpurun_out/c_$v.json > gpurun_out/c_$v.log 2>&1 || { tail -5 gpurun_out/c_$v.log; exit 1; }
  python -c "
import json; [print('$v', d['config'], d['mray_s'], d['ms_trace'], d['ms_shade']) for d in json.load(open('gpurun_out/c_$v.json'))]"
done; done
