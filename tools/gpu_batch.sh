#!/bin/bash
# Batched-round check: train parity tests (default batching and BPE355_BATCH=1), bench lines.
set -o pipefail
OUT=gpurun_out/${1:-batch}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for b in 8 1 0; do
  BPE355_BATCH=$b timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline > $OUT/bench$b.log 2>&1 || { echo "bench $b failed"; tail -20 $OUT/bench$b.log; exit 1; }
  tail -1 $OUT/bench$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch', $b, d['value'], d['phases_ms']['t_merge_ms'], d['counters'], d['roofline']['avg_launch_us'])"
done
