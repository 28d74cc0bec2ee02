set -o pipefail
OUT=gpurun_out/r05zn; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do for v in default w5; do
  if [ $v = default ]; then E=""; else E="BPE355_LIB=build/variants/w5/libbpe355.so BPE355_GRID=1280"; fi
  env $E timeout -k 10 300 python -u bench.py --no-file --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/w_${v}_$rep.log 2>&1 || { echo "failed"; tail -5 $OUT/w_${v}_$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); m=d['merge_loop']; print('$v rep $rep merge_ms', m['ms'], 'us_per_trip', m['us_per_trip'], 'k_us', m['k_merge_batch_us'], 'parity', d['parity']['parity'])" $OUT/w_${v}_$rep.log
done; done
