#!/bin/bash
# A/B of environment settings on the end-to-end file path (load phase and step time).
# usage: tools/ab_load.sh OUTTAG "ENV=1" ...   ("-" = no extra setting)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = "-" ]; then envs=(); else read -r -a envs <<< "$v"; fi
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-encode --no-cpu-baseline --no-device-resident --keep-corpus > $OUT/v$i.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/v$i.$rep.log; exit 1; }
    tail -1 $OUT/v$i.$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print('$v', 'MB/s', d['value'], 'ms', d['ms_per_step'], 'load', p['t_load_ms'], 'count', p['t_count_ms'], 'merge', p['t_merge_ms'])"
  done
done
