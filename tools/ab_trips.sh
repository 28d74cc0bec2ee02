#!/bin/bash
# A/B of trips per merge block (BPE355_TRIPS): merge-loop ms from bench --no-file runs
set -o pipefail
OUT=gpurun_out/${1:-abt}
mkdir -p $OUT
export TMPDIR=/tmp
for t in ${TRIPS:-4 8 16 32}; do
  BPE355_TRIPS=$t BPE355_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-file --no-encode --steps 3 > $OUT/b$t.log 2>&1 || { echo "bench $t failed"; tail -20 $OUT/b$t.log; exit 1; }
  echo "trips $t: $(grep 'host clock' $OUT/b$t.log | tail -1)"
  tail -1 $OUT/b$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('  ', d['merge_loop']['ms'], 'ms', d['merge_loop']['trips'], 'trips', d['merges_per_s'])"
done
