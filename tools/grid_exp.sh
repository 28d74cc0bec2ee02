mkdir -p gpurun_out/grid
for g in 128 256 512 1024 2048; do
  BPE355_GRID=$g timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-encode --no-cpu-baseline > gpurun_out/grid/g$g.log 2>&1 || exit 1
  python - $g <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/grid/g{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["value"], d["phases_ms"], d["roofline"]["avg_launch_us"])
PY
done
