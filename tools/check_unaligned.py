"""Encode of a text at an aligned and at an unaligned device address (same bytes): ids must
agree.  usage: python tools/check_unaligned.py bytes[,bytes...] [train_bytes]"""
import ctypes, os, sys
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import numpy as np
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer

sizes = [int(float(x)) for x in sys.argv[1].split(",")]
L = _lib.lib()
nmax = max(sizes)
big = torch.empty(nmax + 64, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(big.data_ptr()), nmax, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
tn = min(nmax, 256 << 20)
vocab, merges = train_bpe_device(big.data_ptr(), tn, 32000, ["<|endoftext|>"])
tok = Tokenizer(vocab, merges, ["<|endoftext|>"])
out = torch.empty(nmax, dtype=torch.int32, device="cuda")
k = ctypes.c_size_t(0)
for n in sizes:
    res = {}
    for shift in (0, 3):
        buf = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        buf[shift:shift + n].copy_(big[:n])
        torch.cuda.synchronize()   # the library encodes on its own stream
        _lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(buf.data_ptr() + shift), n,
                                           ctypes.c_void_p(out.data_ptr()), ctypes.byref(k), None), "enc")
        res[shift] = out[:k.value].cpu().numpy().copy()
        del buf
    a, b = res[0], res[3]
    m = min(a.size, b.size)
    bad = np.flatnonzero(a[:m] != b[:m])
    print(f"n={n} env={os.environ.get('BPE355_NOCACHE', '')}{os.environ.get('BPE355_ENC_SCAN_V1', '')} ids {a.size} vs {b.size} "
          f"equal {a.size == b.size and bad.size == 0} first mismatch {int(bad[0]) if bad.size else None}", flush=True)
