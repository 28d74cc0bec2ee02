"""Where an end-to-end train_bpe(path) step spends the time outside the library's own t_total:
wall time of the ctypes call, of the result conversion, and the stats' phases.  Writes the bench
corpus first (like bench.py).  usage: python tools/e2e_gap.py [bytes] [steps]"""
import ctypes
import pathlib
import sys
import tempfile
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "transformer-lm_amd"), str(ROOT)]

import bench  # noqa: E402
from bpe_amd import _lib  # noqa: E402

n = int(float(sys.argv[1]) if len(sys.argv) > 1 else 11.9e9) // bench.BLOCK * bench.BLOCK
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
L = _lib.lib()
_lib.require_device()
path = pathlib.Path(tempfile.gettempdir()) / f"bpe355_gap_{n}.txt"
if not (path.exists() and path.stat().st_size == n):
    bench.write_corpus(L, path, n, 2, 0)
arr, k, _keep = _lib.c_strings([bench.EOT])
p = bytes(path)
for step in range(steps + 1):
    res = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = L.bpe_train_file(p, 32000, arr, k, 1, ctypes.byref(res))
    t1 = time.perf_counter()
    _lib.check(rc, "train")
    vocab, merges, st = _lib.take_result(res)
    t2 = time.perf_counter()
    ph = {key: round(v, 1) for key, v in st.items() if key.startswith("t_")}
    print(f"step {step}: call {1e3 * (t1 - t0):.1f} ms, result {1e3 * (t2 - t1):.1f} ms, "
          f"gap {1e3 * (t1 - t0) - st['t_total_ms']:.1f} ms, {ph}", flush=True)
path.unlink()
