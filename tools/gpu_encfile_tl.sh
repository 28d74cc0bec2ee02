#!/bin/bash
# encode_file timeline: 3 calls on the 11.9 GB bench corpus file with BPE355_ENC_TRACE (per slab
# read, per region encode, per copy: the call's clock in ms), then the knob runs given.
# usage: tools/gpu_encfile_tl.sh TAG ["KNOB=V ..." ...]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-encfile_tl}; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
BPE355_ENC_TRACE=$OUT/timeline.txt timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
grep call $OUT/tl.log
for k in "$@"; do
  env $k timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/k_${k//[ =]/_}.log 2>&1 || { tail -5 $OUT/k_${k//[ =]/_}.log; exit 1; }
  grep call $OUT/k_${k//[ =]/_}.log
done
rm -f /tmp/bpe355_encfile.txt
