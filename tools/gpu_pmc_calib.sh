#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the access widths the BPE kernels use
# (tools/microbench/pmc_calib.hip): two separate --pmc passes, then tools/pmc_calib.py.
# usage: tools/gpu_pmc_calib.sh TAG   -> gpurun_out/TAG/calib.txt
set -o pipefail
OUT=gpurun_out/${1:-calib}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -- tools/microbench/pmc_calib > $OUT/f.log 2>&1 || { echo "fetch pass failed"; tail -5 $OUT/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -- tools/microbench/pmc_calib > $OUT/w.log 2>&1 || { echo "write pass failed"; tail -5 $OUT/w.log; exit 1; }
F=$(find $OUT/f -name "*counter_collection.csv" | head -1); W=$(find $OUT/w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_calib.py "$F" "$W" | tee $OUT/calib.txt
rm -rf $OUT/f $OUT/w
