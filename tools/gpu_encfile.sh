#!/bin/bash
# encode_file after an encoder change: the encode / bulk-encode tests, then encode_file timing on
# the 11.9 GB bench corpus file with the reader/copier thread counts given (default: 4 8).
# usage: tools/gpu_encfile.sh TAG [threads...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-encfile}; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_bulk_encode.py tests/test_gpu_chunks.py tests/test_gpu_count.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest.log | head -30; exit $rc; }
for t in ${@:-4 8}; do
  BPE355_ENC_IO_THREADS=$t timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/encfile_t$t.log 2>&1 || { tail -5 $OUT/encfile_t$t.log; exit 1; }
  grep call $OUT/encfile_t$t.log
done
rm -f /tmp/bpe355_encfile.txt
