#!/bin/bash
# One GPU call: optional quick tests, then a trace run and the bench line (no profile).
# usage: tools/gpu_bench.sh TAG [test files...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_first.log 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest_first.log; exit 1; }
  tail -2 $OUT/pytest_first.log
fi
BPE355_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-device-resident > $OUT/trace.log 2> $OUT/trace_err.log || { echo "trace failed"; tail -20 $OUT/trace_err.log; exit 1; }
grep "count:" $OUT/trace_err.log | head -3
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d['phases_ms'], 'dev', d['device_resident'], 'roof', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
