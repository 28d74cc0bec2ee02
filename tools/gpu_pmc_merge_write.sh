#!/bin/bash
# WRITE_SIZE of k_merge_batch per dispatch (one --pmc pass, kernel filter): the first 300 launches of
# a training (the early trips, which rewrite most words) vs the rest.  usage: tools/gpu_pmc_merge_write.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmcmergew}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_merge_batch --output-format csv -d $OUT/w -- python3 tools/pmc_train_encode.py > $OUT/w.log 2>&1 || { echo "write pass failed"; tail -5 $OUT/w.log; exit 1; }
F=$(find $OUT/w -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY' | tee $OUT/merge_write.txt
import csv, sys, collections
per = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_merge_batch" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
        per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
w = [per[k] for k in sorted(per)]
print("k_merge_batch dispatches:", len(w))
for name, lo, hi in (("first 100", 0, 100), ("100..300", 100, 300), ("300..end", 300, len(w))):
    print(f"{name}: WRITE_SIZE {sum(w[lo:hi]) * 1024 / max(1, hi - lo) / 1e6:.1f} MB per launch")
PY
rm -rf $OUT/w
