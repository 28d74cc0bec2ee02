#!/bin/bash
# Encoder check on the GPU: the encode parity tests (small goldens first, then the 256 MB and
# full-size C5 goldens), then the device encode timing of the bench corpus under rocprofv3.
# usage: tools/gpu_enc.sh TAG [quick]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-enc}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
PYT="python -u -m pytest -x -v --timeout 400 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_encode.py tests/test_gpu_chunks.py tests/test_gpu_stream.py tests/test_gpu_bulk_encode.py > $OUT/pytest_small.log 2>&1
rc=$?; tail -4 $OUT/pytest_small.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_small.log | head -30; exit $rc; }
timeout -k 10 500 $PYT tests/test_gpu_scale.py -k encode tests/test_gpu_c4.py::test_c5_encode_eight_devices tests/test_gpu_large.py > $OUT/pytest_mid.log 2>&1
rc=$?; tail -4 $OUT/pytest_mid.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_mid.log | head -30; exit $rc; }
if [ "$2" != "quick" ]; then
timeout -k 10 700 $PYT tests/test_gpu_encode_full.py > $OUT/pytest_full.log 2>&1
rc=$?; tail -6 $OUT/pytest_full.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_full.log | head -30; exit $rc; }
fi
cd /tmp && export TMPDIR=/tmp
BPE355_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o enc -- python $ROOT/tools/enc_bench.py > $OUT/enc_prof.log 2>&1
rc=$?; tail -2 $OUT/enc_prof.log
[ $rc -eq 0 ] || exit $rc
python $ROOT/tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) > $OUT/kernel_stats.txt 2>&1
grep -E "enc|find_spec|collect|emit" $OUT/kernel_stats.txt | head -20
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/pmc_hit -o hit -- python $ROOT/tools/enc_bench.py > $OUT/pmc_hit.log 2>&1
rc=$?; tail -1 $OUT/pmc_hit.log; [ $rc -eq 0 ] || exit $rc
for knob in ${KNOBS:-BPE355_ENC_FINALIZE=0}; do
  env $knob timeout -k 10 300 python $ROOT/tools/enc_bench.py > $OUT/enc_${knob//=/_}.log 2>&1
  echo "$knob: $(tail -1 $OUT/enc_${knob//=/_}.log)"
done
