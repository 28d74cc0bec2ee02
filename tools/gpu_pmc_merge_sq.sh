#!/bin/bash
# SQ counters of k_merge_batch per dispatch (one --pmc pass, kernel filter), split into the first
# 300 launches of the training (the full scans of the early trips) and the rest.
# usage: tools/gpu_pmc_merge_sq.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmcmerge}
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-include-regex k_merge_batch --output-format csv -d $OUT/sq -- python3 tools/pmc_train_encode.py > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_merge_batch --output-format csv -d $OUT/f -- python3 tools/pmc_train_encode.py > $OUT/f.log 2>&1 || { echo "fetch pass failed"; tail -5 $OUT/f.log; exit 1; }
F=$(find $OUT/sq -name "*counter_collection.csv" | head -1); G=$(find $OUT/f -name "*counter_collection.csv" | head -1)
python3 - "$F" "$G" <<'PY' | tee $OUT/merge_sq.txt
import csv, sys, collections
def load(path):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if "k_merge_batch" not in r["Kernel_Name"]: continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]
sq, fe = load(sys.argv[1]), load(sys.argv[2])
print("k_merge_batch dispatches:", len(sq), len(fe))
for name, lo, hi in (("first 300 launches", 0, 300), ("launches 300..end", 300, len(sq))):
    a = collections.defaultdict(float)
    for d in sq[lo:hi]:
        for k, v in d.items(): a[k] += v
    fb = sum(2 * d.get("FETCH_SIZE", 0) for d in fe[lo:hi]) * 1024 / max(1, hi - lo)
    w = a["SQ_WAVE_CYCLES"] or 1
    print(f"{name}: wave cycles {a['SQ_WAVE_CYCLES']:.3e} | active {a['SQ_ACTIVE_INST_ANY']/w:.2f} wait {a['SQ_WAIT_ANY']/w:.2f} "
          f"issue-stall {a['SQ_WAIT_INST_ANY']/w:.2f} | valu {a['SQ_ACTIVE_INST_VALU']/w:.2f} lds {a['SQ_ACTIVE_INST_LDS']/w:.2f} | "
          f"bank-conflict/lds-active {a['SQ_LDS_BANK_CONFLICT']/max(1,a['SQ_LDS_IDX_ACTIVE']):.2f} | fetch {fb/1e6:.1f} MB per launch")
PY
rm -rf $OUT/sq $OUT/f
