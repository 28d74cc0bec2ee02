#!/bin/bash
# bench line with trip statistics (batched merge loop)
timeout -k 10 300 python -u - "$@" <<'PY'
import sys, ctypes, json, time, pathlib
sys.path.insert(0, "transformer-lm_amd"); sys.path.insert(0, ".")
import torch
from bpe_amd import _lib, train_bpe_device
from bpe_amd.train import last_train_stats
L = _lib.lib(); _lib.require_device()
n = int(11.9e9) // 4096 * 4096
corpus = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
for it in range(2):
    t0 = time.perf_counter()
    v, m = train_bpe_device(corpus.data_ptr(), n, 32000, ["<|endoftext|>"])
    torch.cuda.synchronize()
    s = last_train_stats()
    print(it, round(time.perf_counter() - t0, 3), {k: s[k] for k in ("t_count_ms", "t_merge_ms", "n_trips", "n_rounds_batched", "n_rebuilds")}, flush=True)
PY
