#!/bin/bash
# Count-kernel breakdown: full, scan only (mode 1), LDS cache only (mode 2); BPE355_TRACE prints
# the kernel's own pretoken/miss counters.
mkdir -p gpurun_out/cm
for m in 0 1 2; do
  BPE355_COUNT_MODE=$m BPE355_TRACE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --vocab 300 --no-encode --no-cpu-baseline > gpurun_out/cm/m$m.log 2> gpurun_out/cm/m$m.err || { echo "mode $m failed"; tail -5 gpurun_out/cm/m$m.err; exit 1; }
  grep "count:" gpurun_out/cm/m$m.err | tail -1
  python - gpurun_out/cm/m$m.log $m <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("mode", sys.argv[2], "count_ms", d["phases_ms"]["t_count_ms"], "kernel", d["roofline"])
PY
done
