#!/bin/bash
# A/B/C on one box: variants given as NAME[:ENV=VAL,...] (library under build/variants/NAME),
# bench merge phase + count phase, alternating, REPS rounds.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in ${REPS:-1 2}; do
  for spec in "$@"; do
    v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=$(echo ${spec#*:} | tr ',' ' ')
    log=$OUT/$(echo $spec | tr ':,=' '___').$rep.log
    env $envs BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-timing > $log 2>&1 || { echo "$spec failed"; tail -5 $log; exit 1; }
    python - $log "$spec" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dr=d.get("device_resident") or {}
print(sys.argv[2], d["value"], "merge_ms", d["phases_ms"]["t_merge_ms"], "count_ms", d["phases_ms"]["t_count_ms"], "words_ms", d["phases_ms"]["t_words_ms"], "dev_ms", dr.get("ms_per_step"), dr.get("phases_ms"))
PY
  done
done
