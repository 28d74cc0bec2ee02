#!/bin/bash
# r04zb: the queued region copies and the minimum mid-file region: bulk-encode parity (small
# knobs and the full corpus), then the encode_file timeline.  usage: tools/gpu_r04zb.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04zb}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bulk_encode.py tests/test_gpu_encode_full.py::test_c5_full_encode_file > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
BPE355_ENC_TRACE=$OUT/timeline.txt timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
grep call $OUT/tl.log
BPE355_ENC_MIN_REGION=1 timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl_min1.log 2>&1 || { tail -5 $OUT/tl_min1.log; exit 1; }
grep call $OUT/tl_min1.log
rm -f /tmp/bpe355_encfile.txt
