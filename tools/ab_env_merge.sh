#!/bin/bash
# A/B of runtime knobs on the HBM-resident merge phase: REPS alternating bench runs per setting.
# usage: tools/ab_env_merge.sh OUTTAG "KNOB=V ..." "KNOB=V ..." ...   ("-" = no knob)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
for rep in ${REPS:-1 2}; do
  for k in "$@"; do
    name=${k//[ =]/_}
    if [ "$k" = "-" ]; then kv=""; else kv="$k"; fi
    env $kv timeout -k 10 200 python -u bench.py --no-file --steps 2 --warmup 1 --no-encode --no-cpu-baseline --no-timing --keep-corpus > $OUT/$name.$rep.log 2>&1 || { echo "$k failed"; tail -5 $OUT/$name.$rep.log; exit 1; }
    python - $OUT/$name.$rep.log "$k" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dr=d.get("device_resident", d)
print(sys.argv[2], "merge_ms", dr.get("phases_ms", {}).get("t_merge_ms"), d.get("phases_ms", {}).get("t_merge_ms"))
PY
  done
done
rm -f /tmp/bpe355_bench_*
