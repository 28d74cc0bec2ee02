"""A/B of the end-to-end train_bpe(path) step (overlapped load + count) under knob settings.
usage: python tools/exp_e2e.py [KNOB=V,KNOB=V ...]   (each argument = one child process)"""
import ctypes, os, subprocess, sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "transformer-lm_amd"), str(ROOT)]
N = int(float(os.environ.get("N", "11.9e9"))) // 4096 * 4096
PATH = pathlib.Path("/dev/shm/exp_corpus.txt")


def child():
    import torch
    from bpe_amd import _lib, train_bpe
    from bpe_amd.train import last_train_stats
    L = _lib.lib()
    L.bpe_set_timing(int(os.environ.get("TIMING", "0")))
    tag = os.environ.get("TAG", "")
    for i in range(4):
        t = time.perf_counter(); train_bpe(PATH, 32000, ["<|endoftext|>"]); w = (time.perf_counter() - t) * 1e3
        s = last_train_stats()
        print(f"{tag:28s} wall {w:6.0f} total {s['t_total_ms']:6.0f} load {s['t_load_ms']:5.0f} "
              f"count {s['t_count_ms']:4.0f} kcount {s['count_kernel_ms']:5.1f} merge {s['t_merge_ms']:4.0f}", flush=True)


if __name__ == "__main__":
    if os.environ.get("CHILD"):
        child()
        sys.exit(0)
    import bench
    from bpe_amd import _lib
    bench.write_corpus(_lib.lib(), PATH, N, 2, 0)
    try:
        for spec in sys.argv[1:] or [""]:
            env = dict(os.environ, CHILD="1", TAG=spec)
            for kv in filter(None, spec.split(",")):
                k, v = kv.split("=")
                env[k] = v
            r = subprocess.run([sys.executable, __file__], env=env, timeout=120)
            if r.returncode:
                print(f"child {spec} failed rc={r.returncode}", flush=True)
                break
    finally:
        PATH.unlink()
