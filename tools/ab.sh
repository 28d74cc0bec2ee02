#!/bin/bash
# A/B timing of library variants on one box: bench merge-phase for each, alternating.
# usage: tools/ab.sh OUTTAG name1 name2 ... (variants under build/variants/)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in ${REPS:-1 2}; do
  for v in "$@"; do
    BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-timing > $OUT/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    python - $OUT/$v.$rep.log $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], "merge_ms", d["phases_ms"]["t_merge_ms"], "count_ms", d["phases_ms"]["t_count_ms"])
PY
  done
done
