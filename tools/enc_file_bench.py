"""encode_file timing on the bench corpus file (page-cache warm): 3 calls, wall time and phases,
for A/B of the bulk path's knobs (environment).  usage: python tools/enc_file_bench.py [bytes]"""
import ctypes, os, pathlib, sys, time
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer
from bpe_amd.encode import encode_file, last_phases_ms
from bench import write_corpus

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 11_899_998_208
L = _lib.lib()
path = pathlib.Path("/tmp/bpe355_encfile.txt")
if not path.exists() or path.stat().st_size != n:
    write_corpus(L, path, n, 2, 0)
c = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), c.numel(), 2, 0, 0, None), "synth")
torch.cuda.synchronize()
vocab, merges = train_bpe_device(c.data_ptr(), c.numel(), 32000, ["<|endoftext|>"])
tok = Tokenizer(vocab, merges, ["<|endoftext|>"])
knobs = {k: v for k, v in os.environ.items() if k.startswith("BPE355_")}
for i in range(3):
    t0 = time.perf_counter()
    ids = encode_file(tok, path, keep_device_buffers=True)
    dt = time.perf_counter() - t0
    print(f"{knobs} call {i}: {dt * 1e3:.0f} ms = {n / dt / 1e9:.2f} GB/s, ids {ids.size}, phases "
          f"{ {k: round(v) for k, v in last_phases_ms.items()} }", flush=True)
    del ids
