#!/bin/bash
# One GPU call: gpu parity tests, smoke, bench line, rocprofv3 kernel summary.
# usage: tools/gpu_round.sh TAG   (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
# the profile of the roofline's own configuration: corpus in HBM, one k_count2 launch per step
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --no-file --steps 2 > $OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/bench_prof.log; exit 1; }
tail -1 $OUT/bench_prof.log
bash tools/gpu_pmc.sh $TAG/pmc || exit 1
echo done
