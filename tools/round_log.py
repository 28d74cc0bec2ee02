"""Per-round records of one training on the bench corpus in HBM (BPE355_ROUND_LOG): a, b, new id,
posting-list length of the member (~0: full scan) and count, 24 bytes per round.  Analysis only.
usage: python tools/round_log.py OUT.bin [bytes] [vocab]"""
import ctypes, os, sys, time
sys.path[:0] = ["transformer-lm_amd", "."]
os.environ["BPE355_ROUND_LOG"] = sys.argv[1]
os.environ.setdefault("BPE355_TRACE", "1")
import torch
from bpe_amd import _lib, train_bpe_device
from bpe_amd.train import last_train_stats
n = int(float(sys.argv[2])) // 4096 * 4096 if len(sys.argv) > 2 else 11_899_998_208
vocab = int(sys.argv[3]) if len(sys.argv) > 3 else 32000
L = _lib.lib()
c = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
t0 = time.perf_counter()
train_bpe_device(c.data_ptr(), n, vocab, ["<|endoftext|>"])
st = last_train_stats()
print(f"{time.perf_counter() - t0:.3f}s", {k: st[k] for k in ("t_count_ms", "t_merge_ms", "n_trips", "n_rounds_batched",
                                                               "n_rebuilds", "n_index_builds", "n_words")}, flush=True)
