#!/bin/bash
# r04v: the scan at 3 workgroups per CU (no spills) vs 4 (device encode, alternating), the
# select's diagnostic counters compiled out vs in (merge phase), and the kernel-driven D2H copy at
# 64 / 128 workgroups vs HIP's copy (encode_file).  usage: tools/gpu_r04v.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04v}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PYT="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
for v in scan3 scan3c; do
  BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 400 $PYT tests/test_gpu_encode.py > $OUT/pytest_$v.log 2>&1
  rc=$?; tail -1 $OUT/pytest_$v.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_$v.log | head -30; exit $rc; }
done
for rep in 1 2; do
  for v in cur scan3 scan3c; do
    BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 300 python tools/enc_bench.py > $OUT/enc_$v.$rep.log 2>&1 || { tail -5 $OUT/enc_$v.$rep.log; exit 1; }
    echo "$v: $(tail -1 $OUT/enc_$v.$rep.log)"
  done
done
REPS="1 2" timeout -k 10 600 bash tools/ab_merge.sh $TAG g512 cur
for k in BPE355_D2H_WG=0 BPE355_D2H_WG=64 BPE355_D2H_WG=128; do
  env $k timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/k_${k//=/_}.log 2>&1 || { tail -5 $OUT/k_${k//=/_}.log; exit 1; }
  grep call $OUT/k_${k//=/_}.log
done
rm -f /tmp/bpe355_encfile.txt
