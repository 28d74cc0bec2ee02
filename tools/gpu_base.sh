set -o pipefail
OUT=gpurun_out/r03e_base; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
BPE355_PROBE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/probe.log 2> $OUT/probe_err.log || { echo "probe failed"; tail -20 $OUT/probe_err.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
