#!/bin/bash
# r04y: the next chunk's loads issued before the mask phase (scan and count) vs after it:
# parity of the encode tests on the variant, then alternating HBM-resident bench runs (count
# kernel and encode).  usage: tools/gpu_r04y.sh TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04y}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
export TMPDIR=/tmp
BPE355_LIB=build/variants/early/libbpe355.so timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_count.py tests/test_gpu_scale.py > $OUT/pytest_early.log 2>&1
rc=$?; tail -1 $OUT/pytest_early.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/pytest_early.log | head -30; exit $rc; }
for rep in 1 2; do
  for v in base early; do
    BPE355_LIB=build/variants/$v/libbpe355.so timeout -k 10 300 python -u bench.py --no-file --no-cpu-baseline --steps 2 --warmup 1 --keep-corpus > $OUT/$v.$rep.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.$rep.log; exit 1; }
    python - $OUT/$v.$rep.log $v <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dr=d.get("device_resident", d)
print(sys.argv[2], "count_ms", dr.get("phases_ms", {}).get("t_count_ms"), "count kernel us", d.get("roofline_count", {}).get("avg_launch_us"), "encode s", d["encode"]["seconds"], "merge", dr.get("phases_ms", {}).get("t_merge_ms"))
PY
  done
done
rm -f /tmp/bpe355_bench_*
