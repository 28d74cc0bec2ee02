#!/bin/bash
# A/B of k_count2 variants (library builds under build/variants/NAME, "-" = the in-tree build):
# k_count2 ms, aggregation ms and records on the bench corpus in HBM (tools/count_modes.py).
# usage: tools/ab_count.sh OUTTAG name...
set -o pipefail
OUT=gpurun_out/${1:-abc}; shift
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = "-" ]; then unset BPE355_LIB; else export BPE355_LIB=build/variants/$v/libbpe355.so; fi
    timeout -k 10 200 python -u tools/count_modes.py > $OUT/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    echo "$v: $(tail -1 $OUT/$v.$rep.log)"
  done
done
