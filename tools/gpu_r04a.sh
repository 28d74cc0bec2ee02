#!/bin/bash
# r04 first GPU call: the full-size C5 parity tests (+ the bulk-encode tests with the read-error
# regression), then a rocprofv3 kernel summary of the device encode on the bench corpus.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04a}
mkdir -p $OUT
cd $ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_encode_full.py tests/test_gpu_bulk_encode.py -x -v --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o enc -- python $ROOT/tools/enc_bench.py > $OUT/enc_prof.log 2>&1
rc=$?
tail -3 $OUT/enc_prof.log
exit $rc
