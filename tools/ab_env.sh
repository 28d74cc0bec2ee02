#!/bin/bash
# A/B of environment knobs on one box: merge-loop ms from bench --no-file runs, alternating.
# usage: tools/ab_env.sh OUTTAG "ENV=1" "ENV2=x" ...   ("-" = no extra setting)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = "-" ]; then envs=(); else read -r -a envs <<< "$v"; fi
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-encode --no-cpu-baseline --no-file > $OUT/v$i.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/v$i.$rep.log; exit 1; }
    tail -1 $OUT/v$i.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'merge_ms', d['merge_loop']['ms'], 'trips', d['merge_loop']['trips'], 'us/trip', d['merge_loop']['us_per_trip'], 'dev MB/s', d['value'])"
  done
done
