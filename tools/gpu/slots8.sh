set -o pipefail
for b in 24 12 8 6; do
  timeout -k 10 200 python -u tools/rank_frames.py --config 2 --world 8 --rank 0 --frames 2 --slots $b > gpurun_out/s8.log 2>&1 || { tail -5 gpurun_out/s8.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/s8.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if not d['warmup']: print('base $b slots', d['slots'], d['wall_ms'], 'ms trace', d['ms_trace'], 'shade', d['ms_shade'], 'occ', d['occ_resolved_frac'], 'iters', d['iterations'])
"
done
