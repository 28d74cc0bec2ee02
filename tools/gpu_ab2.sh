#!/bin/bash
# parity of the in-tree library on the train/scale tests, then an A/B of two variants with probes
# usage: tools/gpu_ab2.sh TAG v1 v2
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_scale.py tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_probe.sh $TAG "$@"
# encoder variants, when present (tools/enc_bench.py: device encode of the bench corpus)
for v in ${ENC_VARIANTS:-}; do
  [ -f build/variants/$v/libbpe355.so ] || continue
  BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 200 python -u tools/enc_bench.py > $OUT/$v.enc.log 2>&1 || { echo "$v enc failed"; tail -5 $OUT/$v.enc.log; exit 1; }
  echo "$v $(tail -1 $OUT/$v.enc.log)"
done
