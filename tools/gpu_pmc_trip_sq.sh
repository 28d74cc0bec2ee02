#!/bin/bash
# Instruction mix / stall counters of the merge loop's trip kernels (one --pmc pass over one
# HBM-resident training, no encode).  usage: tools/gpu_pmc_trip_sq.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-pmctripsq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/sq -- python3 $ROOT/bench.py --no-file --no-encode --no-cpu-baseline --steps 1 --warmup 0 > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
F=$(find $OUT/sq -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY' | tee $OUT/sq_summary.txt
import csv, sys, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("bpe::(anonymous namespace)::", "")).replace("void ", "")
    if not any(x in k for x in ("k_select", "k_merge_batch", "k_apply_batch", "k_count2")): continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, a in acc.items():
    w = a["SQ_WAVE_CYCLES"]
    if not w: continue
    print("%-36s active %.2f wait %.2f issue-stall %.2f | valu %.2f lds %.2f | bank-conflict/lds-active %.2f" % (
        k, a["SQ_ACTIVE_INST_ANY"] / w, a["SQ_WAIT_ANY"] / w, a["SQ_WAIT_INST_ANY"] / w,
        a["SQ_ACTIVE_INST_VALU"] / w, a["SQ_ACTIVE_INST_LDS"] / w,
        a["SQ_LDS_BANK_CONFLICT"] / max(a["SQ_LDS_IDX_ACTIVE"], 1)))
PY
