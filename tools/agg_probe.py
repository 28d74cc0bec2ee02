"""File path probe: load / count-tail / aggregation times of train_bpe(path) for several
BPE355_AGG_SEGS settings (segments between partial record aggregations; 0 = at the end only).
Usage: python tools/agg_probe.py [agg ...]"""
import os
import pathlib
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "transformer-lm_amd")]
import bench  # noqa: E402
from bpe_amd import _lib, train_bpe  # noqa: E402
from bpe_amd.train import last_train_stats  # noqa: E402

L = _lib.lib()
_lib.require_device()
n = int(11.9e9) // bench.BLOCK * bench.BLOCK
path = pathlib.Path(tempfile.gettempdir()) / f"bpe355_bench_s2_f0_{n}.txt"
if not (path.exists() and path.stat().st_size == n):
    bench.write_corpus(L, path, n, 2, 0)
settings = sys.argv[1:] or ["0", "4", "12"]
train_bpe(path, 32000, ["<|endoftext|>"])   # warm up
for timed in (0, 1):
    L.bpe_set_timing(timed)
    for a in settings:
        os.environ["BPE355_AGG_SEGS"] = a
        for _ in range(2):
            train_bpe(path, 32000, ["<|endoftext|>"])
            s = last_train_stats()
            print(f"timed {timed} agg {a:>3}: total {s['t_total_ms']:.1f} load {s['t_load_ms']:.1f} "
                  f"count tail {s['t_count_ms']:.1f} batches {s['n_count_batches']} "
                  f"partial {s['count_partial_ms']:.1f} final {s['count_reduce_ms']:.1f} "
                  f"count kernels {s['count_kernel_ms']:.1f} merge {s['t_merge_ms']:.1f}", flush=True)
L.bpe_set_timing(0)
path.unlink(missing_ok=True)
