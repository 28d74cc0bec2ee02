"""The program the PMC passes profile (tools/gpu_pmc_all.sh): one training on the bench corpus in
HBM (count, word table, merge loop: every kernel of a train step) and one encode of it with the
result (the encoder's kernels), nothing else.  usage: python tools/pmc_train_encode.py [bytes]"""
import ctypes, sys
import os as _os
_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
sys.path[:0] = [_os.path.join(_ROOT, "transformer-lm_amd"), _ROOT]
import torch
from bpe_amd import _lib, train_bpe_device, Tokenizer
n = int(float(sys.argv[1])) // 4096 * 4096 if len(sys.argv) > 1 else 11_899_998_208
L = _lib.lib()
c = torch.empty(n, dtype=torch.uint8, device="cuda")
_lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(c.data_ptr()), n, 2, 0, 0, None), "synth")
torch.cuda.synchronize()
vocab, merges = train_bpe_device(c.data_ptr(), n, 32000, ["<|endoftext|>"])
tok = Tokenizer(vocab, merges, ["<|endoftext|>"])
out = torch.empty(n, dtype=torch.int32, device="cuda")
n_out = ctypes.c_size_t(0)
_lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(c.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                   ctypes.byref(n_out), None), "encode")
torch.cuda.synchronize()
print("merges", len(merges), "ids", n_out.value, flush=True)
