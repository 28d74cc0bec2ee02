"""The encoder's LDS word cache on and off (BPE355_NOCACHE) over the same text: where the ids
first differ, the bytes around it and both id runs, plus the tokenizer, for an oracle check.
usage: python tools/check_cache.py bytes outdir"""
import ctypes, json, os, sys
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import numpy as np
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer

n = int(float(sys.argv[1])); outdir = sys.argv[2]
L = _lib.lib()
c = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
vocab, merges = train_bpe_device(c.data_ptr(), min(n, 256 << 20), 32000, ["<|endoftext|>"])
tok = Tokenizer(vocab, merges, ["<|endoftext|>"])
out = torch.empty(n, dtype=torch.int32, device="cuda")
k = ctypes.c_size_t(0)
res = {}
for mode in ("cache", "nocache", "cache2"):
    if mode == "nocache": os.environ["BPE355_NOCACHE"] = "1"
    else: os.environ.pop("BPE355_NOCACHE", None)
    _lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(c.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                       ctypes.byref(k), None), "enc")
    res[mode] = out[:k.value].cpu().numpy().copy()
    print(mode, k.value, flush=True)
a, b = res["cache"], res["nocache"]
print("cache runs equal", res["cache"].size == res["cache2"].size and bool((res["cache"] == res["cache2"]).all()))
m = min(a.size, b.size)
bad = np.flatnonzero(a[:m] != b[:m])
if bad.size:
    i = int(bad[0])
    lens = np.zeros(max(vocab) + 1, dtype=np.int64)
    for t, bs in vocab.items(): lens[t] = len(bs)
    P = int(lens[a[:i]].sum())
    host = c[max(0, P - 3000):P + 3000].cpu().numpy().tobytes()
    print("first mismatch id", i, "byte", P)
    print("cache  :", [vocab[int(t)] for t in a[i - 5:i + 10]])
    print("nocache:", [vocab[int(t)] for t in b[i - 5:i + 10]])
    os.makedirs(outdir, exist_ok=True)
    with open(f"{outdir}/snippet.bin", "wb") as f: f.write(host)
    json.dump({"P": P, "lo": max(0, P - 3000), "cache": a[i - 400:i + 400].tolist(), "nocache": b[i - 400:i + 400].tolist(),
               "vocab": {str(t): bs.hex() for t, bs in vocab.items()}, "merges": [[x.hex(), y.hex()] for x, y in merges]},
              open(f"{outdir}/case.json", "w"))
