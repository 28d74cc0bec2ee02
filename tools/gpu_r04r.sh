#!/bin/bash
# r04r: encoder knob parity, the encode_file timeline, encoder A/B (finalize modes), then the merge-loop code-size A/B
# (build/variants base vs noprobe: BPE355_PROBE_CODE=0).  usage: tools/gpu_r04r.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04r}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_encode.py tests/test_gpu_bulk_encode.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
BPE355_ENC_TRACE=$OUT/timeline.txt timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
grep call $OUT/tl.log
BPE355_ENC_FINALIZE=2 timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl_f2.log 2>&1 || { tail -5 $OUT/tl_f2.log; exit 1; }
grep call $OUT/tl_f2.log
rm -f /tmp/bpe355_encfile.txt
for rep in 1 2; do
  for f in 1 2; do
    BPE355_ENC_FINALIZE=$f timeout -k 10 300 python tools/enc_bench.py > $OUT/enc_f$f.$rep.log 2>&1 || { tail -5 $OUT/enc_f$f.$rep.log; exit 1; }
    echo "finalize=$f: $(tail -1 $OUT/enc_f$f.$rep.log)"
  done
done
REPS="1 2" timeout -k 10 900 bash tools/ab_probe.sh $TAG base noprobe
