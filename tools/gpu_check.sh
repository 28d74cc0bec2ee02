#!/bin/bash
# GPU check after a merge-loop change: train + scale parity, the merge-loop probe, a bench line.
# usage: tools/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
BPE355_PROBE=1 BPE355_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing --no-file > $OUT/probe.log 2> $OUT/probe_err.log || { echo "probe failed"; tail -20 $OUT/probe_err.log; exit 1; }
grep -E "probe|trips:" $OUT/probe_err.log
timeout -k 10 500 python -u bench.py "$@" > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases_ms'], d.get('device_resident',{}) and d['device_resident']['ms_per_step'], d['merge_loop'])"
