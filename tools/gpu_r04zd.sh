#!/bin/bash
# r04zd: copy-out threads 4 (default) vs 8, paired twice, after the bulk-encode parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-r04zd}
mkdir -p $OUT
cd $ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bulk_encode.py tests/test_gpu_encode_full.py::test_c5_full_encode_file > $OUT/pytest.log 2>&1
rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
for rep in 1 2; do
  for k in BPE355_ENC_COPY_THREADS=4 BPE355_ENC_COPY_THREADS=8; do
    env $k timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/k_${k//=/_}.$rep.log 2>&1 || { tail -5 $OUT/k_${k//=/_}.$rep.log; exit 1; }
    grep call $OUT/k_${k//=/_}.$rep.log
  done
done
rm -f /tmp/bpe355_encfile.txt
