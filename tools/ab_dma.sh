#!/bin/bash
# A/B of the file staging: 8 readers on 2 shared DMA streams (default) vs 16 readers on 16 streams
set -o pipefail
OUT=gpurun_out/ab_dma; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_file.py tests/test_gpu_bulk_encode.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-device-resident --keep-corpus > $OUT/new.$i.log 2>&1 || { echo "bench failed"; tail -20 $OUT/new.$i.log; exit 1; }
  BPE355_IO_THREADS=16 BPE355_DMA_STREAMS=16 timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-device-resident --keep-corpus > $OUT/old.$i.log 2>&1 || { echo "bench failed"; tail -20 $OUT/old.$i.log; exit 1; }
done
for f in $OUT/*.[12].log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['encode']['end_to_end']; print('$f', d['value'], d['load_ms_per_step'], 'enc_file', e['value'], e.get('phases_ms'))"; done
