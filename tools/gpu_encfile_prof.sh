#!/bin/bash
# encode_file profile: the per-region trace (BPE355_ENC_TRACE) and a rocprofv3 kernel summary of
# encode_file on the 11.9 GB bench corpus file.  usage: tools/gpu_encfile_prof.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-encfileprof}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BPE355_ENC_TRACE=$OUT/regions.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o ef -- python -u $ROOT/tools/enc_file_bench.py > $OUT/run.log 2>&1
rc=$?; grep call $OUT/run.log; [ $rc -eq 0 ] || { tail -5 $OUT/run.log; exit $rc; }
python $ROOT/tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) > $OUT/kernel_stats.txt 2>&1
head -24 $OUT/kernel_stats.txt
head -20 $OUT/regions.txt
rm -f /tmp/bpe355_encfile.txt
