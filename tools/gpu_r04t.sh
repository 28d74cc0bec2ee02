#!/bin/bash
# r04t: the kernel-driven device-to-host copy (encode_file parity + timeline, knob A/B), then the
# apply-grid A/B of the merge loop (build/variants g512 g1024 g2048).  usage: tools/gpu_r04t.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04t}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PYT="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_bulk_encode.py tests/test_gpu_encode_full.py::test_c5_full_encode_file > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
BPE355_ENC_TRACE=$OUT/timeline.txt timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
grep call $OUT/tl.log
for k in BPE355_D2H_WG=0 BPE355_D2H_WG=32 BPE355_D2H_WG=8; do
  env $k timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/k_${k//=/_}.log 2>&1 || { tail -5 $OUT/k_${k//=/_}.log; exit 1; }
  grep call $OUT/k_${k//=/_}.log
done
rm -f /tmp/bpe355_encfile.txt
REPS="1 2" timeout -k 10 900 bash tools/ab_merge.sh $TAG g512 g1024 g2048
