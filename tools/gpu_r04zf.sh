#!/bin/bash
# r04zf: the two-entries-per-thread resolve: encode parity with it on (the knob cases and the
# full-size device encode), then the device encode alternating with it off / on.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04zf}
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode.py > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
BPE355_ENC_RESOLVE_ILP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode_full.py::test_c5_full_encode_device tests/test_gpu_scale.py -k encode > $OUT/pytest_full_ilp.log 2>&1
rc=$?; tail -1 $OUT/pytest_full_ilp.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_full_ilp.log | head -30; exit $rc; }
for rep in 1 2; do
  for f in 0 1; do
    BPE355_ENC_RESOLVE_ILP=$f timeout -k 10 300 python tools/enc_bench.py > $OUT/enc_ilp$f.$rep.log 2>&1 || { tail -5 $OUT/enc_ilp$f.$rep.log; exit 1; }
    echo "ilp=$f: $(tail -1 $OUT/enc_ilp$f.$rep.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
BPE355_ENC_RESOLVE_ILP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o enc -- python $ROOT/tools/enc_bench.py > $OUT/prof.log 2>&1 || { tail -3 $OUT/prof.log; exit 1; }
cd $ROOT && python tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) | grep -E "resolve|scan4|finalize|emit" 
