"""Texts past 2^32 bytes (and id runs past 2^32 ids) on the device.  A dispatch's grid is at most
2^32 work-items (the AQL packet's 32-bit grid size); a kernel launched with one thread per byte
of a larger text wraps silently.  That dropped every special token past byte 11.9e9 mod 2^32 of
the bench corpus (found by tools/check_specials.py); the per-byte and per-id kernels now stride.
Byte-level tokenizer (no merges), so the expected ids follow from the text alone: every byte its
own id, every '<|endoftext|>' the special's id, and decode gives the text back."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SP = b"<|endoftext|>"


def _host_specials(host: np.ndarray) -> int:
    n, cnt, step = host.size, 0, 1 << 30
    for lo in range(0, n, step):   # occurrences starting in [lo, lo + step)
        blob = host[lo:min(n, lo + step + len(SP) - 1)].tobytes()
        i = blob.find(SP)
        while 0 <= i < step:
            cnt += 1
            i = blob.find(SP, i + len(SP))
    return cnt


def test_encode_and_decode_past_4gib():
    import torch
    from bpe_amd import _lib, Tokenizer
    L = _lib.lib()
    n = (4 << 30) + (300 << 20)   # 4.3 GiB: the last 300 MiB past the 32-bit grid
    text = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(text.data_ptr()), n, 2, 0, 0, None), "synth")
    torch.cuda.synchronize()
    n_sp = _host_specials(text.cpu().numpy())
    assert n_sp > 0
    vocab = {i: bytes([i]) for i in range(256)}
    vocab[256] = SP
    tok = Tokenizer(vocab, [], [SP.decode()])
    ids = torch.empty(n, dtype=torch.int32, device="cuda")
    k = ctypes.c_size_t(0)
    _lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(text.data_ptr()), n,
                                       ctypes.c_void_p(ids.data_ptr()), ctypes.byref(k), None), "encode")
    torch.cuda.synchronize()
    assert k.value == n - (len(SP) - 1) * n_sp
    ids = ids[:k.value]
    assert int((ids == 256).sum()) == n_sp
    back = torch.empty(n, dtype=torch.uint8, device="cuda")
    m = ctypes.c_size_t(0)
    _lib.check(L.bpe_dec_decode_device(tok._decoder(), ctypes.c_void_p(ids.data_ptr()), k.value,
                                       ctypes.c_void_p(back.data_ptr()), n, ctypes.byref(m), None), "decode")
    torch.cuda.synchronize()
    assert m.value == n and torch.equal(back, text)
