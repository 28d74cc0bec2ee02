#!/bin/bash
# count-tail knobs on the file path (BPE355_AGG_SEGS: segments between partial record
# aggregations; BPE355_SEG_MB: segment size) and one traced run for the merge loop's host clock
set -o pipefail
OUT=gpurun_out/${1:-tail}; mkdir -p $OUT; export TMPDIR=/tmp
BPE355_TRACE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing --no-device-resident --keep-corpus > $OUT/trace.log 2> $OUT/trace_err.log || { echo "trace failed"; tail -5 $OUT/trace_err.log; exit 1; }
grep -E "host clock|trips:|words per slot" $OUT/trace_err.log | tail -4
for rep in 1 2; do
for cfg in "4 256" "1 256" "2 256" "2 128"; do
  set -- $cfg
  BPE355_AGG_SEGS=$1 BPE355_SEG_MB=$2 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-encode --no-cpu-baseline --no-timing --no-device-resident --keep-corpus > $OUT/agg$1_seg$2.$rep.log 2>&1 || { echo "bench failed"; tail -5 $OUT/agg$1_seg$2.$rep.log; exit 1; }
  tail -1 $OUT/agg$1_seg$2.$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['phases_ms']; print('agg $1 seg $2', d['value'], 'load', p['t_load_ms'], 'count tail', p['t_count_ms'], 'words', p['t_words_ms'], 'merge', p['t_merge_ms'], 'total', p['t_total_ms'], d['load_ms_per_step'])"
done
done
