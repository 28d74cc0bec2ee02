#!/bin/bash
# One GPU call for the round's evidence: GPU parity tests, smoke, the PMC traffic passes (their
# traffic.json also feeds this call's bench line), the default bench line with the CPU baselines,
# the rocprofv3 kernel summary of the roofline's configuration (corpus in HBM), a merge-loop probe.
# usage: tools/gpu_final.sh TAG   (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_pmc_all.sh $TAG/pmc || exit 1
cp $OUT/pmc/traffic.json profiles/r03/traffic.json
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --keep-corpus > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-file --no-encode --steps 2 --warmup 1 --keep-corpus > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) > $OUT/kernel_stats.txt 2>&1 || python3 tools/rocprof_summary.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) > $OUT/kernel_stats.txt
head -12 $OUT/kernel_stats.txt
BPE355_PROBE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing --no-device-resident --keep-corpus > $OUT/probe.log 2> $OUT/probe_err.log || { echo "probe failed"; tail -5 $OUT/probe_err.log; exit 1; }
grep probe $OUT/probe_err.log | head -3
rm -f /tmp/bpe355_bench_*
echo done
