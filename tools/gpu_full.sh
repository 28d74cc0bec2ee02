#!/bin/bash
# One GPU call for a round's evidence: GPU parity tests, smoke, the default bench line (with the
# CPU baselines), the rocprofv3 kernel summary of the roofline's configuration (corpus in HBM),
# and the PMC traffic passes.  usage: tools/gpu_full.sh TAG   (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-file --no-encode --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
tail -1 $OUT/bench_prof.log | cut -c1-300
bash tools/gpu_pmc_all.sh $TAG/pmc || exit 1
echo done
