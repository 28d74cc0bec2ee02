#!/bin/bash
# rocprofv3 kernel summaries of library variants on the HBM-resident bench (one training each),
# plus the merge phase from bench runs, alternating.  usage: tools/gpu_prof_ab.sh TAG v1 v2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/ab_probe.sh $TAG "$@" | grep -v "^==\|probe\]" || exit 1
for v in "$@"; do
  cd /tmp && BPE355_LIB=$GRAFT_REPO_ROOT/build/variants/$v/libbpe355.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_$v -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-file --no-encode --steps 1 --warmup 0 --keep-corpus > $GRAFT_REPO_ROOT/$OUT/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $GRAFT_REPO_ROOT/$OUT/prof_$v.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  echo "== $v"; python3 tools/rocprof_summary.py $(find $OUT/prof_$v -name "*.db" | head -1) | grep -E "k_select|k_merge_batch|k_apply_batch"
done
