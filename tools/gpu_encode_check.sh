#!/bin/bash
# Encoder evidence in one call: the encode/bulk/large-text/file parity tests, a bench line (device
# encode, encode_file), encode_file timing over three calls, and every special of the bench corpus
# accounted for (tools/check_specials.py).  usage: tools/gpu_encode_check.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-enccheck}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_bulk_encode.py tests/test_gpu_encode.py tests/test_gpu_chunks.py tests/test_gpu_utf8.py tests/test_gpu_file.py tests/test_gpu_stream.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log


timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.log').read().strip().splitlines()[-1]); e=d['encode']; print('value', d['value'], 'merge', d['phases_ms']['t_merge_ms'], 'device enc', e['value'], e['ids_rank0'], 'e2e', json.dumps(e['end_to_end']))"
timeout -k 10 300 python -u tools/enc_file_bench.py > $OUT/encfile.log 2>&1 || { echo "encfile failed"; tail -20 $OUT/encfile.log; exit 1; }
grep call $OUT/encfile.log
timeout -k 10 500 python -u tools/check_specials.py > $OUT/specials.log 2>&1 || { echo "specials failed"; tail -30 $OUT/specials.log; exit 1; }
grep "^encode" $OUT/specials.log
