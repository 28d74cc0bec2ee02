#!/bin/bash
# SQ counters of the merge loop's three trip kernels (one --pmc pass; tools/pmc_train_encode.py on
# a 2 GB corpus at 32k): wave cycles split into parked on s_waitcnt/barrier, issue-stalled and
# active, per kernel.  usage: tools/gpu_pmc_trip.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmctrip}
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/sq -- python3 tools/pmc_train_encode.py 2e9 > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
F=$(find $OUT/sq -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY' | tee $OUT/sq_summary.txt
import csv, sys, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", re.sub(r"bpe::\(anonymous namespace\)::|bpe::", "", r["Kernel_Name"])).replace("void ", "")
    k = re.sub(r"<.*", "", k)
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k in sorted(acc, key=lambda k: -acc[k]["SQ_WAVE_CYCLES"]):
    a = acc[k]; w = a["SQ_WAVE_CYCLES"] or 1
    print(f"{k:24s} n={len(disp[k]):6d} wave_cycles/launch {w/len(disp[k]):12.0f} | wait {a['SQ_WAIT_ANY']/w:.2f} issue-stall {a['SQ_WAIT_INST_ANY']/w:.2f} active {a['SQ_ACTIVE_INST_ANY']/w:.2f} (valu {a['SQ_ACTIVE_INST_VALU']/w:.2f} lds {a['SQ_ACTIVE_INST_LDS']/w:.2f} salu {a['SQ_ACTIVE_INST_SCA']/w:.2f} misc {a['SQ_ACTIVE_INST_MISC']/w:.2f})")
PY
rm -rf $OUT/sq
