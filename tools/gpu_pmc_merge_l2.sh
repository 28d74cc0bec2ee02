#!/bin/bash
# TCC_HIT_sum and TCC_MISS_sum (L2) of k_merge_batch per dispatch (one --pmc pass, kernel filter): the first 300 launches of
# a training (the early trips, which rewrite most words) vs the rest.  usage: tools/gpu_pmc_merge_l2.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmcmergel2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_merge_batch --output-format csv -d $OUT/w -- python3 tools/pmc_train_encode.py > $OUT/w.log 2>&1 || { echo "L2 pass failed"; tail -5 $OUT/w.log; exit 1; }
F=$(find $OUT/w -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY' | tee $OUT/merge_l2.txt
import csv, sys, collections
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "k_merge_batch" in r["Kernel_Name"]:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
d = [per[k] for k in sorted(per)]
print("k_merge_batch dispatches:", len(d))
for name, lo, hi in (("first 100", 0, 100), ("100..300", 100, 300), ("300..end", 300, len(d))):
    h = sum(x["TCC_HIT_sum"] for x in d[lo:hi]); m = sum(x["TCC_MISS_sum"] for x in d[lo:hi])
    print(f"{name}: L2 requests {(h + m) / max(1, hi - lo) / 1e6:.2f} M per launch, hit rate {h / max(1, h + m):.2f}")
PY
rm -rf $OUT/w
