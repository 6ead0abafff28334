# variant library: libmcpt_head.so: a build of an earlier commit (tools/build_rev_variant.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libmcpt_head.so libmcpt.so; do
  MCPT_LIB=$PWD/mc-path-tracer_amd/$lib timeout -k 10 400 python -u tools/configs.py --configs 2,3,4,5 --warmup 10 --iters 15 > gpurun_out/cfg_$lib.log 2>&1 || { tail -5 gpurun_out/cfg_$lib.log; exit 1; }
  echo "== $lib"; python -c "
import json
for l in open('gpurun_out/cfg_$lib.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], d['mray_s'], d['ms_trace'], d['ms_shade'])"
done
