#!/bin/bash
# One GPU call for the round's evidence: the PMC traffic passes (their traffic.json also feeds this
# call's bench line), the default bench line with the CPU baselines, the rocprofv3 kernel summary
# of train AND encode on the roofline's configuration (corpus in HBM), the 8-rank C4 exchange
# timings, a merge-loop probe.  With "tests" first: the GPU tests and smoke.
# usage: tools/gpu_r04_final.sh TAG [tests]   (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT profiles/r04
export TMPDIR=/tmp
if [ "$2" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
bash tools/gpu_pmc_all.sh $TAG/pmc || exit 1
cp $OUT/pmc/traffic.json profiles/r04/traffic.json
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --keep-corpus > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-file --steps 2 --warmup 1 --keep-corpus > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) > $OUT/kernel_stats.txt 2>&1
head -16 $OUT/kernel_stats.txt
BPE355_STATS_OUT=$OUT/c4_exchange.json timeout -k 10 400 python -u -m pytest tests/test_gpu_c4.py::test_c4_eight_ranks_words_full_owt -x -q --timeout 380 --timeout-method thread > $OUT/c4.log 2>&1 || { echo "c4 failed"; tail -20 $OUT/c4.log; exit 1; }
cat $OUT/c4_exchange.json
BPE355_PROBE=1 BPE355_LIB=build/variants/probe/libbpe355.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing --no-device-resident --keep-corpus > $OUT/probe.log 2> $OUT/probe_err.log || { echo "probe failed"; tail -5 $OUT/probe_err.log; exit 1; }
grep probe $OUT/probe_err.log | head -3
rm -f /tmp/bpe355_bench_*
echo done
