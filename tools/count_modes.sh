#!/bin/bash
# Count-kernel breakdown (k_count2): full, masks only (1), + token bounds (2), + packing/hash (3),
# + LDS cache with misses dropped (4).
mkdir -p gpurun_out/cm; export TMPDIR=/tmp
for m in ${MODES:-0 1 2 3 4}; do
  BPE355_COUNT_MODE=$m timeout -k 10 200 python -u tools/count_modes.py > gpurun_out/cm/m$m.log 2>&1 || { echo "mode $m failed"; tail -5 gpurun_out/cm/m$m.log; exit 1; }
  tail -1 gpurun_out/cm/m$m.log
done
