#!/bin/bash
# merge-phase sweep of a run-time knob: usage tools/gpu_knob_sweep.sh TAG VAR v1 v2 ...
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-timing --keep-corpus > $OUT/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    tail -1 $OUT/$v.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], 'merge_ms', d['phases_ms']['t_merge_ms'], 'dev-res merge_ms', d['device_resident']['phases_ms']['t_merge_ms'])"
  done
done
