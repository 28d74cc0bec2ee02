#!/bin/bash
# HBM traffic of the counter kernels (two separate --pmc passes, MI355X_MICROARCH.md HBM section)
# on the bench corpus, count only (tools/count_modes.py: vocab 256, three trainings).
set -o pipefail
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -- python3 tools/count_modes.py > $OUT/f.log 2>&1 || { echo "fetch pass failed"; tail -5 $OUT/f.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -- python3 tools/count_modes.py > $OUT/w.log 2>&1 || { echo "write pass failed"; tail -5 $OUT/w.log; exit 1; }
F=$(find $OUT/f -name "*counter_collection.csv" | head -1); W=$(find $OUT/w -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$F" "$W" $OUT/traffic.json && echo pmc done
