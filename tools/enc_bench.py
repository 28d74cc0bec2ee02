"""Encode timing on the bench corpus in HBM (train 32k once, then Tokenizer.encode device to
device 3 times): for A/B of encoder variants (BPE355_LIB)."""
import ctypes, sys, time
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 11_899_998_208
L = _lib.lib()
c = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
v, m = train_bpe_device(c.data_ptr(), n, 32000, ["<|endoftext|>"])
tok = Tokenizer(v, m, ["<|endoftext|>"])
h = tok._device()
out = torch.empty(n, dtype=torch.int32, device="cuda")
k = ctypes.c_size_t(0)
ts = []
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _lib.check(L.bpe_tok_encode_device(h, ctypes.c_void_p(c.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                       ctypes.byref(k), None), "encode")
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"encode {n / min(ts[1:]) / 1e9:.2f} GB/s best, times {[round(t * 1e3, 1) for t in ts]} ms, ids {k.value}",
      flush=True)
