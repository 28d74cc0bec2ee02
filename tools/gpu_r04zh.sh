#!/bin/bash
# r04zh: k_select with 8 / 4 / 2 partial waves (1 / 2 / 4 partials per thread): the train
# parity tests on the 4- and 2-wave builds, then the merge phase alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04zh}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for v in sel4 sel2; do
  BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_scale.py -k "not encode" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_$v.log | head -30; exit $rc; }
done
REPS="1 2" timeout -k 10 800 bash tools/ab_merge.sh $TAG sel8 sel4 sel2
