#!/bin/bash
# A/B of library variants (build/variants/NAME) on the merge phase: REPS alternating bench runs
# (file + HBM-resident training, no encode).  usage: tools/ab_merge.sh OUTTAG name1 name2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
  for v in "$@"; do
    BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-timing --keep-corpus > $OUT/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    python - $OUT/$v.$rep.log $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], "merge_ms", d["phases_ms"]["t_merge_ms"], "dev-res merge_ms", d.get("device_resident", {}).get("phases_ms", {}).get("t_merge_ms"))
PY
  done
done
