#!/bin/bash
# Counter iteration: its GPU tests, the mode breakdown, and the bench line.
set -o pipefail
OUT=gpurun_out/${1:-cnt}
mkdir -p $OUT gpurun_out/cm
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_count.py tests/test_gpu_utf8.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/count_modes.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'phases', d['phases_ms'], 'dev', d['device_resident'], 'roof', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
