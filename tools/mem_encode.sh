#!/bin/bash
# device memory after each training, then the encode time (diagnoses encode slowdowns after
# repeated trainings)
timeout -k 10 400 python -u - <<'PY'
import sys, ctypes, time
sys.path.insert(0, "transformer-lm_amd"); sys.path.insert(0, ".")
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer
L = _lib.lib(); _lib.require_device()
n = int(11.9e9) // 4096 * 4096
corpus = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
for it in range(3):
    v, m = train_bpe_device(corpus.data_ptr(), n, 32000, ["<|endoftext|>"])
    torch.cuda.synchronize()
    f, t = torch.cuda.mem_get_info()
    print("train", it, "free GB %.1f of %.1f" % (f / 1e9, t / 1e9), flush=True)
    tok = Tokenizer(v, m, ["<|endoftext|>"])
    h = tok._device()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    n_out = ctypes.c_size_t(0)
    for rep in range(2):
        torch.cuda.synchronize(); te = time.perf_counter()
        _lib.check(L.bpe_tok_encode_device(h, ctypes.c_void_p(corpus.data_ptr()), n, ctypes.c_void_p(out.data_ptr()), ctypes.byref(n_out), None), "encode")
        torch.cuda.synchronize()
        print("  encode", rep, "%.3f s" % (time.perf_counter() - te), "free GB %.1f" % (torch.cuda.mem_get_info()[0] / 1e9), flush=True)
    del out, tok
PY
