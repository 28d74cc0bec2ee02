"""train_bpe hands its device memory back.

The reference keeps nothing once train_bpe returns (models/tokenizer/train.py:231), and its caller
trains the LM on the same GPU right after (train.py:230-232).  The drop-in keeps the corpus buffer
and the counter's record pool and bins between calls only when asked (keep_device_buffers=True,
as bench.py does for its repeated steps); by default train_bpe releases them before it returns.
"""
import gzip
import hashlib
import json
import pathlib
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")
torch = pytest.importorskip("torch")

SCALE = pathlib.Path(__file__).resolve().parent / "golden" / "scale"


def _check_c3_1g(o, vocab, merges):
    want = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in o["merges"]]
    assert merges == want
    h = hashlib.sha256()
    for i in range(len(vocab)):
        h.update(struct.pack("<I", len(vocab[i])) + vocab[i])
    assert h.hexdigest() == o["vocab_sha256"]


def test_train_releases_device_memory():
    from bpe_amd import _lib
    _lib.require_device()
    with gzip.open(SCALE / "train_C3_1G.json.gz", "rt") as f:
        o = json.load(f)
    buf = np.empty(o["n"], dtype=np.uint8)
    assert _lib.lib().bpe_synth_corpus_host(buf.ctypes.data, o["n"], o["seed"], o["flavour"], 0, 16) == 0
    data = buf.tobytes()
    del buf
    bpe_amd.release_device_memory()       # whatever earlier tests of this process kept
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info()

    # default: nothing kept once train_bpe returns
    vocab, merges = bpe_amd.train_bpe_bytes(data, o["vocab"], o["specials"])
    _check_c3_1g(o, vocab, merges)
    free1, _ = torch.cuda.mem_get_info()
    assert abs(free1 - free0) <= 0.01 * free0, (free0, free1)

    # kept on request: the pool and the corpus buffer stay until released
    vocab, merges = bpe_amd.train_bpe_bytes(data, o["vocab"], o["specials"], keep_device_buffers=True)
    _check_c3_1g(o, vocab, merges)
    free2, _ = torch.cuda.mem_get_info()
    assert free2 < free0 - o["n"], (free0, free2)   # at least the corpus buffer is held
    freed = bpe_amd.release_device_memory(0)
    assert freed >= o["n"]
    free3, _ = torch.cuda.mem_get_info()
    assert abs(free3 - free0) <= 0.01 * free0, (free0, free3)
    assert bpe_amd.release_device_memory() == 0   # nothing left to hand back
