#!/bin/bash
# Single-GPU runs on k x the bench corpus: the merge loop then trains on the union of k slabs'
# words, which is what each rank runs after the word exchange at N = k.
mkdir -p gpurun_out/union
for k in 2 4 8; do
  b=$(python -c "print(11.9e9*$k)")
  timeout -k 10 300 python -u bench.py --bytes $b --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > gpurun_out/union/k$k.log 2>&1 || { echo "k=$k failed"; tail -5 gpurun_out/union/k$k.log; exit 1; }
  python - gpurun_out/union/k$k.log $k <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["phases_ms"], d["counters"]["n_words"])
PY
done
