#!/bin/bash
# A/B of library variants (build/variants/NAME): merge phase over REPS alternating bench runs, then
# one merge-loop probe per variant.  usage: tools/ab_probe.sh OUTTAG name1 name2 ...
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
for v in "$@"; do
  BPE355_PROBE=1 BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing --no-device-resident --keep-corpus > $OUT/$v.probe.log 2> $OUT/$v.probe_err.log || { echo "$v probe failed"; tail -5 $OUT/$v.probe_err.log; exit 1; }
  echo "== $v"; grep -E "sampled trips|last-workgroup tail|by decile" $OUT/$v.probe_err.log | head -3
done
