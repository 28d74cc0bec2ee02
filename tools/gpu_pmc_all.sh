#!/bin/bash
# HBM traffic per launch of every kernel of a train step and an encode (two separate --pmc passes,
# MI355X_MICROARCH.md HBM section) on the bench corpus: tools/pmc_train_encode.py.
# usage: tools/gpu_pmc_all.sh TAG   -> gpurun_out/TAG/traffic.json
set -o pipefail
OUT=gpurun_out/${1:-pmcall}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -- python3 tools/pmc_train_encode.py > $OUT/f.log 2>&1 || { echo "fetch pass failed"; tail -5 $OUT/f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -- python3 tools/pmc_train_encode.py > $OUT/w.log 2>&1 || { echo "write pass failed"; tail -5 $OUT/w.log; exit 1; }
F=$(find $OUT/f -name "*counter_collection.csv" | head -1); W=$(find $OUT/w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$F" "$W" $OUT/traffic.json && echo pmc done
# the counter CSVs are large (one row per dispatch): keep only the summary
rm -rf $OUT/f $OUT/w
