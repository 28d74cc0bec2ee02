#!/bin/bash
# One GPU call: the given test files first (stop on failure), then the full GPU suite, smoke,
# bench line and rocprofv3 kernel summary.   usage: tools/gpu_stage.sh TAG [test files...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_first.log 2>&1 || { echo "first tests failed"; tail -40 $OUT/pytest_first.log; exit 1; }
  tail -2 $OUT/pytest_first.log
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
BPE355_DRIVE_TRACE=1 BPE355_TRACE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 0 --no-encode --no-cpu-baseline --no-device-resident > $OUT/trace.log 2> $OUT/trace_err.log || { echo "trace failed"; tail -20 $OUT/trace_err.log; exit 1; }
grep -E "count:|drive" $OUT/trace_err.log | head -6
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-file --steps 2 > $OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/bench_prof.log; exit 1; }
echo done
