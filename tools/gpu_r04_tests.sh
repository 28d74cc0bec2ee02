#!/bin/bash
# The round's GPU tests and smoke on the final tree.  usage: tools/gpu_r04_tests.sh TAG
set -o pipefail
TAG=${1:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for k in BPE355_D2H_PRIO=1 BPE355_D2H_PRIO=0 BPE355_D2H_PRIO=1 BPE355_D2H_PRIO=0; do
  env $k timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/k_${k//=/_}.log 2>&1 || { tail -5 $OUT/k_${k//=/_}.log; exit 1; }
  grep call $OUT/k_${k//=/_}.log
done
rm -f /tmp/bpe355_encfile.txt
