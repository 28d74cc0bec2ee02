#!/bin/bash
# r04s: encode parity (small + full size), the encode_file timeline after the sync fixes, then
# the default bench line.  usage: tools/gpu_r04s.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04s}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PYT="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_encode.py tests/test_gpu_bulk_encode.py tests/test_gpu_encode_full.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
BPE355_ENC_TRACE=$OUT/timeline.txt timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
grep call $OUT/tl.log
rm -f /tmp/bpe355_encfile.txt
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2> $OUT/bench_err.log || { tail -5 $OUT/bench_err.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
