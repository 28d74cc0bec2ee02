#!/bin/bash
# Quick GPU check after a merge-loop change: train/sharded parity tests, probe run, bench line.
# usage: tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
BPE355_PROBE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/probe.log 2> $OUT/probe_err.log || { echo "probe failed"; tail -20 $OUT/probe_err.log; exit 1; }
grep probe $OUT/probe_err.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['phases_ms'], d['roofline']['avg_launch_us'])"
