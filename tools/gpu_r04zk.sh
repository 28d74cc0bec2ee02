#!/bin/bash
# r04zk: candidate-list cap 128 vs 256 (k_select on 384 vs 512 threads): train parity on the
# 128 build, then the merge phase alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04zk}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
BPE355_LIB=build/variants/lc128/libbpe355.so timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_scale.py -k "not encode" > $OUT/pytest_lc128.log 2>&1
rc=$?; echo "lc128: $(tail -1 $OUT/pytest_lc128.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_lc128.log | head -30; exit $rc; }
REPS="1 2 3" timeout -k 10 800 bash tools/ab_merge.sh $TAG lc256 lc128
