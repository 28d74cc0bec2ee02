#!/bin/bash
# Parity (train + scale tests) then merge-phase A/B of library variants built by build_variant.sh.
# usage: tools/ab_batch.sh TAG base variant...   (the base is timed, not re-tested)
set -o pipefail
TAG=$1; shift
BASE=$1; shift
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/$TAG/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/$TAG/pytest_$v.log)"
done
bash tools/ab.sh $TAG $BASE "$@"
