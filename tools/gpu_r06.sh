#!/bin/bash
# Round-6 GPU call.  usage: tools/gpu_r06.sh TAG [tests|quick|bench|prof|c4] ...
#   quick: the tests this round added or changed; tests: the whole -m gpu suite + smoke;
#   bench: the default bench line (CPU baselines included); prof: rocprofv3 kernel summary of the
#   HBM-resident bench; c4: the 8-rank words exchange stats + rounds-mode stats; pmc: the HBM traffic
#   passes; exactc3: the exact C oracle on the full C3 corpus; ab*/abenc*/trainpar:*: A/Bs and the
#   train parity tests of build/variants/NAME.
set -o pipefail
TAG=${1:-r06}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
  quick)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_release.py tests/test_gpu_limits.py "tests/test_gpu_c4.py::test_c4_ranks_rounds_1g" tests/test_gpu_train.py tests/test_gpu_encode.py > $OUT/pytest_quick.log 2>&1 || { echo "quick tests failed"; tail -40 $OUT/pytest_quick.log; exit 1; }
    tail -1 $OUT/pytest_quick.log ;;
  pmc)   # HBM traffic per launch (two --pmc passes) -> profiles/r06/traffic.json (bench.py reads it)
    bash tools/gpu_pmc_all.sh $TAG/pmc || exit 1
    mkdir -p profiles/r06 && cp $OUT/pmc/traffic.json profiles/r06/traffic.json ;;
  probe1)   # the merge-loop probe of the default configuration
    BPE355_PROBE=1 BPE355_LIB=build/variants/probe/libbpe355.so timeout -k 10 200 python -u bench.py --no-file --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/probe.log 2> $OUT/probe_err.log || { echo "probe failed"; tail -5 $OUT/probe_err.log; exit 1; }
    grep probe $OUT/probe_err.log > $OUT/merge_probe.txt; head -12 $OUT/merge_probe.txt ;;
  count)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_count.py > $OUT/pytest_count.log 2>&1 || { echo "count tests failed"; tail -40 $OUT/pytest_count.log; exit 1; }
    tail -1 $OUT/pytest_count.log ;;
  trainpar)   # the training parity tests (goldens, tie-heavy, scale)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_scale.py > $OUT/pytest_trainpar.log 2>&1 || { echo "train parity tests failed"; tail -40 $OUT/pytest_trainpar.log; exit 1; }
    tail -1 $OUT/pytest_trainpar.log ;;
  trainpar:*)   # the training parity tests on build/variants/NAME
    V=${step#trainpar:}
    BPE355_LIB=build/variants/$V/libbpe355.so timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_scale.py > $OUT/pytest_trainpar_$V.log 2>&1 || { echo "train parity tests ($V) failed"; tail -40 $OUT/pytest_trainpar_$V.log; exit 1; }
    echo "$V: $(tail -1 $OUT/pytest_trainpar_$V.log)" ;;
  scale)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_scale.py > $OUT/pytest_scale.log 2>&1 || { echo "scale tests failed"; tail -40 $OUT/pytest_scale.log; exit 1; }
    tail -1 $OUT/pytest_scale.log ;;
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
    tail -1 $OUT/pytest_gpu.log
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 1; }
    tail -1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 600 python -u bench.py --keep-corpus > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
    tail -1 $OUT/bench.log | cut -c1-600 ;;
  benchfast)
    timeout -k 10 400 python -u bench.py --keep-corpus --no-cpu-baseline --steps 3 > $OUT/benchfast.log 2>&1 || { echo "bench failed"; tail -30 $OUT/benchfast.log; exit 1; }
    tail -1 $OUT/benchfast.log | cut -c1-600 ;;
  prof)
    cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-file --steps 2 --warmup 1 --keep-corpus > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/bench_prof.log; exit 1; }
    cd $GRAFT_REPO_ROOT
    python3 tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) > $OUT/kernel_stats.txt 2>&1
    head -24 $OUT/kernel_stats.txt
    rm -rf $OUT/prof ;;
  proffile)   # rocprofv3 kernel summary of the default (file-path) bench command, CPU baselines off
    cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$OUT/bench_proffile.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/bench_proffile.log; exit 1; }
    cd $GRAFT_REPO_ROOT
    python3 tools/rocprof_summary.py $(find $OUT/prof -name "*.db" | head -1) > $OUT/kernel_stats_file.txt 2>&1
    head -24 $OUT/kernel_stats_file.txt
    rm -rf $OUT/prof ;;
  abfold)   # merge phase, fused trip kernel vs k_select + k_merge_batch, corpus in HBM, alternating
    for rep in 1 2; do for f in 1 0; do
      BPE355_FOLD=$f timeout -k 10 300 python -u bench.py --no-file --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/abfold_${f}_$rep.log 2>&1 || { echo "abfold failed"; tail -20 $OUT/abfold_${f}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); m=d['merge_loop']; print('FOLD=$f rep $rep merge_ms', m['ms'], 'us_per_trip', m['us_per_trip'], 'k_us', m['k_merge_batch_us'], 'parity', d['parity']['parity'])" $OUT/abfold_${f}_$rep.log
    done; done ;;
  ab:*)   # merge phase with an env knob at 1 vs 0 (ab:NAME), corpus in HBM, alternating, 2 reps
    V=${step#ab:}
    for rep in 1 2; do for f in 1 0; do
      env $V=$f timeout -k 10 300 python -u bench.py --no-file --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/ab_${V}_${f}_$rep.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_${V}_${f}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); m=d['merge_loop']; print('$V=$f rep $rep merge_ms', m['ms'], 'us_per_trip', m['us_per_trip'], 'k_us', m['k_merge_batch_us'], 'count_ms', d['device_resident']['phases_ms']['t_count_ms'] if d.get('device_resident') else None, 'parity', d['parity']['parity'])" $OUT/ab_${V}_${f}_$rep.log
    done; done ;;
  abvar:*)   # merge phase and count, the default library vs build/variants/NAME (abvar:NAME), alternating, 2 reps
    V=${step#abvar:}
    for rep in 1 2; do for lib in default $V; do
      if [ $lib = default ]; then LIBENV=""; else LIBENV="BPE355_LIB=build/variants/$V/libbpe355.so"; fi
      env $LIBENV timeout -k 10 300 python -u bench.py --no-file --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/abvar_${lib}_$rep.log 2>&1 || { echo "abvar failed"; tail -20 $OUT/abvar_${lib}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); m=d['merge_loop']; print('$lib rep $rep merge_ms', m['ms'], 'us_per_trip', m['us_per_trip'], 'k_us', m['k_merge_batch_us'], 'trips', m['trips'], 'count_ms', d['device_resident']['phases_ms']['t_count_ms'] if d.get('device_resident') else None, 'parity', d['parity']['parity'])" $OUT/abvar_${lib}_$rep.log
    done; done ;;
  abmulti:*)   # merge phase: the default library and build/variants/{A,B,...} (abmulti:A,B), alternating, 2 reps
    VS="default ${step#abmulti:}"; VS=${VS//,/ }
    for rep in 1 2; do for lib in $VS; do
      if [ $lib = default ]; then LIBENV=""; else LIBENV="BPE355_LIB=build/variants/$lib/libbpe355.so"; fi
      env $LIBENV timeout -k 10 300 python -u bench.py --no-file --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/abm_${lib}_$rep.log 2>&1 || { echo "abmulti failed"; tail -20 $OUT/abm_${lib}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); m=d['merge_loop']; dr=d.get('device_resident') or {}; print('$lib rep $rep merge_ms', m['ms'], 'us_per_trip', m['us_per_trip'], 'k_us', m['k_merge_batch_us'], 'trips', m['trips'], 'count_ms', dr.get('phases_ms',{}).get('t_count_ms'), 'agg_ms', (dr.get('count_aggregation') or {}).get('ms'), 'k_count2_us', (d.get('roofline_count') or {}).get('avg_launch_us'), 'parity', d['parity']['parity'])" $OUT/abm_${lib}_$rep.log
    done; done ;;
  trace:*)   # the select's statistics (a BPE355_STATS_CODE build): k histogram, why batches end
    V=${step#trace:}
    BPE355_TRACE=1 BPE355_LIB=build/variants/$V/libbpe355.so timeout -k 10 200 python -u bench.py --no-file --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/trace_$V.log 2> $OUT/trace_err_$V.log || { echo "trace failed"; tail -5 $OUT/trace_err_$V.log; exit 1; }
    grep -E "trips:|batch ended" $OUT/trace_err_$V.log ;;
  probeab:*)   # the merge-loop probe with an env knob at 1 and 0
    V=${step#probeab:}
    for f in 1 0; do
      env $V=$f BPE355_PROBE=1 BPE355_LIB=build/variants/probe/libbpe355.so timeout -k 10 200 python -u bench.py --no-file --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/probe_${V}_$f.log 2> $OUT/probe_err_${V}_$f.log || { echo "probe failed"; tail -5 $OUT/probe_err_${V}_$f.log; exit 1; }
      grep probe $OUT/probe_err_${V}_$f.log | head -12
    done ;;
  probev:*)   # the merge-loop probe of build/variants/NAME (a BPE355_PROBE_CODE build)
    V=${step#probev:}
    BPE355_PROBE=1 BPE355_LIB=build/variants/$V/libbpe355.so timeout -k 10 200 python -u bench.py --no-file --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/probe_$V.log 2> $OUT/probe_err_$V.log || { echo "probe failed"; tail -5 $OUT/probe_err_$V.log; exit 1; }
    grep probe $OUT/probe_err_$V.log > $OUT/merge_probe_$V.txt; head -12 $OUT/merge_probe_$V.txt ;;
  probe)   # the merge-loop probe (build/variants/probe), fused and unfused
    for f in 1 0; do
      BPE355_FOLD=$f BPE355_PROBE=1 BPE355_LIB=build/variants/probe/libbpe355.so timeout -k 10 200 python -u bench.py --no-file --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing > $OUT/probe_$f.log 2> $OUT/probe_err_$f.log || { echo "probe failed"; tail -5 $OUT/probe_err_$f.log; exit 1; }
      grep probe $OUT/probe_err_$f.log | head -12
    done ;;
  timeline|timeline:*)   # per-trip kernel timeline (rocprofv3 kernel trace, no probe build) of the HBM-resident training
    V=${step#timeline}; V=${V#:}
    if [ -n "$V" ]; then LIBENV="BPE355_LIB=$GRAFT_REPO_ROOT/build/variants/$V/libbpe355.so"; NAME=$V; else LIBENV=""; NAME=default; fi
    cd /tmp && env $LIBENV BPE355_TRIP_LOG=$GRAFT_REPO_ROOT/$OUT/trips_$NAME.bin timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/tl_$NAME -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-file --no-encode --no-timing --steps 1 --warmup 0 --keep-corpus > $GRAFT_REPO_ROOT/$OUT/tl_$NAME.log 2>&1 || { echo "timeline failed"; tail -30 $GRAFT_REPO_ROOT/$OUT/tl_$NAME.log; exit 1; }
    cd $GRAFT_REPO_ROOT
    python3 tools/trip_timeline.py $(find $OUT/tl_$NAME -name "*.db" | head -1) -1 $OUT/trips_$NAME.bin > $OUT/trip_timeline_$NAME.txt 2>&1
    cat $OUT/trip_timeline_$NAME.txt
    cp $(find $OUT/tl_$NAME -name "*.db" | head -1) $OUT/tl_$NAME.db; rm -rf $OUT/tl_$NAME ;;
  trace|trace_host)   # the host's halts and clock (BPE355_TRACE) of the HBM-resident training
    BPE355_TRACE=1 timeout -k 10 200 python -u bench.py --no-file --steps 1 --warmup 0 --no-encode --no-cpu-baseline --no-timing --keep-corpus > $OUT/trace_host.log 2> $OUT/trace_host_err.log || { echo "trace failed"; tail -5 $OUT/trace_host_err.log; exit 1; }
    grep -E "host clock|trips:|batch ended" $OUT/trace_host_err.log; grep -c "halt" $OUT/trace_host_err.log ;;
  abenvs:*)   # merge phase under env settings (abenvs:default,A=1,B=2+C=3), corpus in HBM, alternating, 2 reps
    SPECS=${step#abenvs:}; SPECS=${SPECS//,/ }
    for rep in 1 2; do for sp in $SPECS; do
      if [ "$sp" = default ]; then ENVS=""; else ENVS=${sp//+/ }; fi
      tag=${sp//[=+]/_}
      env $ENVS timeout -k 10 300 python -u bench.py --no-file --no-encode --no-cpu-baseline --steps 3 --warmup 1 > $OUT/abe_${tag}_$rep.log 2>&1 || { echo "abenvs failed"; tail -20 $OUT/abe_${tag}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); m=d['merge_loop']; print('$sp rep $rep merge_ms', m['ms'], 'us_per_trip', m['us_per_trip'], 'k_us', m['k_merge_batch_us'], 'trips', m['trips'], 'parity', d['parity']['parity'])" $OUT/abe_${tag}_$rep.log
    done; done ;;
  abenc:*)   # device encode of the bench corpus under env settings (abenc:default,A=1), corpus in HBM, 2 reps
    SPECS=${step#abenc:}; SPECS=${SPECS//,/ }
    for rep in 1 2; do for sp in $SPECS; do
      if [ "$sp" = default ]; then ENVS=""; else ENVS=${sp//+/ }; fi
      tag=${sp//[=+]/_}
      env $ENVS timeout -k 10 300 python -u bench.py --no-file --no-cpu-baseline --steps 1 --warmup 0 > $OUT/abenc_${tag}_$rep.log 2>&1 || { echo "abenc failed"; tail -20 $OUT/abenc_${tag}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); e=d['encode']; print('$sp rep $rep encode MB/s', e['value'], 's', e['seconds'], 'ids', e['ids_rank0'])" $OUT/abenc_${tag}_$rep.log
    done; done ;;
  exactc3)   # the exact C oracle on the full C3 corpus (generated into host memory), host's share of cores
    timeout -k 10 900 python -u -c "
import json, sys; sys.path[:0] = ['transformer-lm_amd', '.']
from oracle.cpu_bench import exact_leg, host_threads
r = exact_leg(host_threads(), None, 'train_C3')
json.dump(r, open('$OUT/exact_cpu_C3.json', 'w'), indent=1); print(r)" > $OUT/exact_c3.log 2>&1 || { echo "exact C3 failed"; tail -5 $OUT/exact_c3.log; exit 1; }
    tail -1 $OUT/exact_c3.log ;;
  c4)
    BPE355_STATS_OUT=$OUT/c4_exchange.json timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py -x -q --timeout 380 --timeout-method thread -k "words_full or rounds" > $OUT/c4.log 2>&1 || { echo "c4 failed"; tail -20 $OUT/c4.log; exit 1; }
    cat $OUT/c4_exchange*.json ;;
  esac
done
rm -f /tmp/bpe355_bench_*
echo done
