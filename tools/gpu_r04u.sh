#!/bin/bash
# r04u: encode parity (inline three/four-id infos, kernel-driven device-to-host copies), device
# encode timing + SQ counters, the encode_file timeline (D2H kernel vs HIP copy), then the
# apply-grid A/B of the merge loop.  usage: tools/gpu_r04u.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04u}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PYT="python -u -m pytest -x -q --timeout 400 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_encode.py tests/test_gpu_bulk_encode.py tests/test_gpu_encode_full.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
BPE355_TRACE=1 timeout -k 10 300 python tools/enc_bench.py > $OUT/enc.log 2>&1 || { tail -5 $OUT/enc.log; exit 1; }
tail -1 $OUT/enc.log
timeout -k 10 200 bash tools/gpu_pmc_enc_sq.sh $TAG || exit 1
cd $ROOT
BPE355_ENC_TRACE=$OUT/timeline.txt timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
grep call $OUT/tl.log
BPE355_D2H_WG=0 timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl_dma.log 2>&1 || { tail -5 $OUT/tl_dma.log; exit 1; }
grep call $OUT/tl_dma.log
rm -f /tmp/bpe355_encfile.txt
REPS="1 2" timeout -k 10 600 bash tools/ab_merge.sh $TAG g512 g1024 g2048
