#!/bin/bash
# gpurun with retries while the pool has no free box (exit 3 / transient), never on a failed command:
#   tools/gpu/retry.sh <timeout> '<command>' > log
for i in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > /tmp/gpurun_try.log 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" /tmp/gpurun_try.log && ! grep -q "status=ok" /tmp/gpurun_try.log; then
    echo "[retry $i] $(grep -m1 'gpurun\] .*busy\|no free\|backing' /tmp/gpurun_try.log)"; sleep ${WAIT:-90}; continue
  fi
  cat /tmp/gpurun_try.log; exit $rc
done
cat /tmp/gpurun_try.log; exit 3
