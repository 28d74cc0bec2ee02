"""Every '<|endoftext|>' of the bench corpus must come out as the special's id: positions found
on the host (bytes.find) against the positions of the special id in a device encode of the whole
text (and of a prefix).  usage: python tools/check_specials.py [bytes]"""
import ctypes, sys, time
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import numpy as np
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 11_899_998_208
SP = b"<|endoftext|>"
L = _lib.lib()
c = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
host = c.cpu().numpy()
t0 = time.time()
pos = []
step = 1 << 30
for lo in range(0, n, step):
    hi = min(n, lo + step + len(SP) - 1)
    blob = host[lo:hi].tobytes()
    i = blob.find(SP)
    while i >= 0:
        if lo + i < lo + step: pos.append(lo + i)
        i = blob.find(SP, i + len(SP))
pos = np.array(sorted(set(pos)), dtype=np.int64)
print(f"host: {pos.size} specials in {time.time() - t0:.1f}s", flush=True)
vocab, merges = train_bpe_device(c.data_ptr(), 256 << 20, 32000, ["<|endoftext|>"])
tok = Tokenizer(vocab, merges, ["<|endoftext|>"])
sid = [t for t, b in vocab.items() if b == SP][0]
lens = np.zeros(max(vocab) + 1, dtype=np.int64)
for t, b in vocab.items(): lens[t] = len(b)
out = torch.empty(n, dtype=torch.int32, device="cuda")
for m in (n, min(n, 3_400_000_000), min(n, 1_000_000_000)):
    k = ctypes.c_size_t(0)
    _lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(c.data_ptr()), m, ctypes.c_void_p(out.data_ptr()),
                                       ctypes.byref(k), None), "enc")
    ids = out[:k.value].cpu().numpy().astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lens[ids])[:-1]])
    dpos = off[ids == sid]
    hp = pos[pos + len(SP) <= m]
    missing = np.setdiff1d(hp, dpos)
    extra = np.setdiff1d(dpos, hp)
    print(f"encode [0, {m}): ids {k.value}, specials {dpos.size} of {hp.size}; missing {missing.size} "
          f"(first {missing[:5].tolist()}), extra {extra.size}", flush=True)
    if missing.size:
        p = int(missing[0])
        print("  context", host[p - 40:p + 30].tobytes())
