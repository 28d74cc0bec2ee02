#!/bin/bash
# gpurun with retries ONLY for infrastructure failures before the command ran (status=transient /
# no box free); a command that ran (ok, failed, timed out) is never re-run.
# usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for attempt in $(seq 1 ${RETRIES:-8}); do
  out=$(/usr/local/graft/bin/gpurun --timeout $T -- "$@" 2>&1)
  rc=$?
  echo "$out" | tail -25
  if echo "$out" | grep -q "status=transient\|no free box\|has no free box"; then
    echo "[retry] infrastructure transient, attempt $attempt"; sleep 150; continue
  fi
  exit $rc
done
exit $rc
