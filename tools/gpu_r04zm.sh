#!/bin/bash
# r04zm: list target 40 / 48 / 56 (merge phase, train parity on 40 and 56) and the scan cache's
# eviction epoch 8 vs 4 (device encode, encode parity on 8).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04zm}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for v in t40 t56; do
  BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train.py > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_$v.log | head -20; exit $rc; }
done
BPE355_LIB=build/variants/ep8/libbpe355.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode.py > $OUT/pytest_ep8.log 2>&1
rc=$?; echo "ep8: $(tail -1 $OUT/pytest_ep8.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_ep8.log | head -20; exit $rc; }
for rep in 1 2; do
  for v in t48 ep8; do
    BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 300 python tools/enc_bench.py > $OUT/enc_$v.$rep.log 2>&1 || { tail -5 $OUT/enc_$v.$rep.log; exit 1; }
    echo "$v: $(tail -1 $OUT/enc_$v.$rep.log)"
  done
done
REPS="1 2" timeout -k 10 800 bash tools/ab_merge.sh $TAG t48 t40 t56
