set -o pipefail
OUT=gpurun_out/r05zl; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do for v in 1 2 4; do
  BPE355_AGG_SEGS=$v timeout -k 10 300 python -u bench.py --keep-corpus --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/agg_${v}_$rep.log 2>&1 || { echo "failed"; tail -5 $OUT/agg_${v}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); p=d['phases_ms']; print('AGG_SEGS=$v rep $rep ms_per_step', d['ms_per_step'], 'load', p['t_load_ms'], 'count_tail', p['t_count_ms'], 'merge', p['t_merge_ms'], 'parity', d['parity']['parity'])" $OUT/agg_${v}_$rep.log
done; done
rm -f /tmp/bpe355_bench_*
