#!/bin/bash
# r03o: PMC calibration, k_select two-stage ranking A/B (head vs top2) with its parity tests, and
# the encode_file phases of the bench line.
set -o pipefail
OUT=gpurun_out/r03o; mkdir -p $OUT
bash tools/gpu_pmc_calib.sh r03o/calib || exit 1
BPE355_LIB=build/variants/top2/libbpe355.so timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/top2_tests.log 2>&1 || { echo "top2 tests failed"; tail -30 $OUT/top2_tests.log; exit 1; }
tail -1 $OUT/top2_tests.log
REPS="1 2" bash tools/ab3.sh r03o/ab head top2 || exit 1
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_enc.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_enc.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_enc.log').read().strip().splitlines()[-1]); e=d['encode']; print('device', e['value'], 'e2e', json.dumps(e['end_to_end']))"
