#!/bin/bash
# Instruction mix / stall counters of the counter kernel (one --pmc pass per count mode):
# SQ wave cycles split into active / waiting / issue-stalled, VALU vs LDS activity, LDS bank
# conflicts.  usage: tools/gpu_pmc_sq.sh TAG [modes...]
set -o pipefail
OUT=gpurun_out/${1:-pmcsq}; shift
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for m in ${@:-0 1}; do
  BPE355_COUNT_MODE=$m timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/m$m -- python3 tools/count_modes.py 2000000000 > $OUT/m$m.log 2>&1 || { echo "pass $m failed"; tail -5 $OUT/m$m.log; exit 1; }
  F=$(find $OUT/m$m -name "*counter_collection.csv" | head -1)
  python3 - "$F" $m <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_count2" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print("mode", sys.argv[2], {k: f"{v:.3e}" for k, v in sorted(acc.items())})
w = acc["SQ_WAVE_CYCLES"]
if w:
    print("  of wave cycles: active %.2f wait %.2f issue-stall %.2f | valu %.2f lds %.2f | bank-conflict/lds-active %.2f" % (
        acc["SQ_ACTIVE_INST_ANY"] / w, acc["SQ_WAIT_ANY"] / w, acc["SQ_WAIT_INST_ANY"] / w,
        acc["SQ_ACTIVE_INST_VALU"] / w, acc["SQ_ACTIVE_INST_LDS"] / w,
        acc["SQ_LDS_BANK_CONFLICT"] / max(acc["SQ_LDS_IDX_ACTIVE"], 1)))
PY
done
