#!/bin/bash
# Address-translation counters of the merge loop's trip kernels (one --pmc pass; 2 GB corpus at 32k):
# per kernel, UTCL1 translation hits / misses per launch.  usage: tools/gpu_pmc_tlb.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-pmctlb}
mkdir -p $OUT
export TMPDIR=/tmp
C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/t -- python3 tools/pmc_train_encode.py 2e9 > $OUT/t.log 2>&1 || { echo "tlb pass failed"; tail -5 $OUT/t.log; exit 1; }
F=$(find $OUT/t -name "*counter_collection.csv" | head -1)
python3 - "$F" <<'PY' | tee $OUT/tlb_summary.txt
import csv, sys, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"\(.*", "", re.sub(r"bpe::\(anonymous namespace\)::|bpe::", "", r["Kernel_Name"])).replace("void ", "")
    k = re.sub(r"<.*", "", k)
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for k in ("k_select", "k_merge_batch", "k_apply_batch", "k_count2", "k_enc_scan2", "k_rec_reduce"):
    if k not in acc: continue
    a = acc[k]; n = len(disp[k])
    miss, hit = a["TCP_UTCL1_TRANSLATION_MISS_sum"], a["TCP_UTCL1_TRANSLATION_HIT_sum"]
    print(f"{k:16s} n={n:6d} per launch: utcl1 miss {miss/n:10.0f} hit {hit/n:10.0f} (miss rate {miss/max(1,miss+hit):.3f}) "
          f"tcc read req {a['TCP_TCC_READ_REQ_sum']/n:10.0f} cache accesses {a['TCP_TOTAL_CACHE_ACCESSES_sum']/n:10.0f}")
PY
rm -rf $OUT/t
