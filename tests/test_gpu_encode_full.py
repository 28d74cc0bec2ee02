"""BASELINE.json configs[4] at the full OWT size: Tokenizer.encode of the whole 11.9 GB C3 corpus
with C3's 32k merges, against the C oracle's golden (tests/golden/make_encode_full_golden.py).

Three paths, each must reproduce the oracle's id stream exactly:
  * bpe_tok_encode_device on the corpus in HBM -- encode(text), reference
    models/tokenizer/tokenizer.py:111-138;
  * bpe_amd.encode.encode_file(path) -- encode.py:31-37: the file read 1024*1024 characters at a
    time, each piece encoded on its own, np.uint16 ids;
  * bpe_tok_encode_gpus with 8 ranks (threads of this process sharing the card,
    BPE355_INPROC_RANKS=1) -- the 8-GPU encode of configs[4].

The golden holds the sha256 of every ~256 MiB slab of each stream (with its id count), so a
mismatch names the slab where it starts.
"""
from __future__ import annotations

import ctypes
import gzip
import hashlib
import json
import pathlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import bpe_amd
from bpe_amd import _lib, Tokenizer

pytestmark = pytest.mark.gpu

SCALE = pathlib.Path(__file__).resolve().parent / "golden" / "scale"


def _load(name):
    with gzip.open(SCALE / name, "rt") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def golden():
    e = _load("encode_C5_full.json.gz")
    o = _load("train_C3.json.gz")
    merges = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in o["merges"]]
    ids_vocab = {}
    for s in e["specials"]:
        ids_vocab.setdefault(s.encode(), len(ids_vocab))
    for b in range(256):
        ids_vocab.setdefault(bytes([b]), len(ids_vocab))
    for a, b in merges:
        ids_vocab.setdefault(a + b, len(ids_vocab))
    vocab = {i: b for b, i in ids_vocab.items()}
    return e, o, vocab, merges


def _check_slabs(ids, slabs, what):
    """ids (host numpy array) against the golden's per-slab (byte lo, byte hi, n_ids, sha256)"""
    assert ids.size == sum(s[2] for s in slabs), f"{what}: {ids.size} ids, oracle {sum(s[2] for s in slabs)}"
    bounds = np.concatenate([[0], np.cumsum([s[2] for s in slabs])])

    def digest(i):
        return hashlib.sha256(ids[bounds[i]:bounds[i + 1]].tobytes()).hexdigest()

    with ThreadPoolExecutor(16) as ex:
        got = list(ex.map(digest, range(len(slabs))))
    bad = [i for i, (g, s) in enumerate(zip(got, slabs)) if g != s[3]]
    assert not bad, (f"{what}: {len(bad)} of {len(slabs)} slabs differ from the oracle, the first at "
                     f"bytes [{slabs[bad[0]][0]}, {slabs[bad[0]][1]})")


def test_c5_full_encode_device(golden):
    """encode(text) of the whole corpus, HBM to HBM"""
    import torch
    e, o, vocab, merges = golden
    n = e["n"]
    corpus = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(_lib.lib().bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), n, e["seed"], e["flavour"],
                                                  0, None), "synth")
    torch.cuda.synchronize()
    piece, digests = o["digest_piece"], o["piece_sha256"]
    for i in sorted({0, len(digests) // 2, len(digests) - 1}):
        lo = i * piece
        assert hashlib.sha256(corpus[lo:lo + piece].cpu().numpy().tobytes()).hexdigest() == digests[i]
    tok = Tokenizer(vocab, merges, e["specials"])
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    n_out = ctypes.c_size_t(0)
    _lib.check(_lib.lib().bpe_tok_encode_device(tok._device(), ctypes.c_void_p(corpus.data_ptr()), n,
                                                ctypes.c_void_p(out.data_ptr()), ctypes.byref(n_out), None),
               "encode")
    torch.cuda.synchronize()
    del corpus
    w = e["whole"]
    assert n_out.value == w["n_ids"]
    ids = out[:n_out.value].cpu().numpy().view(np.uint32)
    del out
    tok.release_device_buffers()
    torch.cuda.empty_cache()
    assert ids[:4096].tolist() == w["ids_head"]
    assert ids[-4096:].tolist() == w["ids_tail"]
    _check_slabs(ids, w["slabs"], "encode_device")


def test_c5_full_encode_file(golden):
    """encode.py's stream: the corpus file in 1024*1024-character pieces, np.uint16"""
    from test_gpu_c4 import _corpus_file
    from bpe_amd.encode import encode_file
    e, o, vocab, merges = golden
    path = _corpus_file(o)
    tok = Tokenizer(vocab, merges, e["specials"])
    ids = encode_file(tok, path)
    p = e["pieces"]
    assert ids.dtype == np.uint16
    _check_slabs(ids, p["groups"], "encode_file")


def test_c5_full_encode_eight_devices(golden, monkeypatch):
    """configs[4] on 8 ranks: the host text cut at safe points no special spans, one piece per
    rank, the ids concatenated"""
    import torch
    e, o, vocab, merges = golden
    n = e["n"]
    monkeypatch.setenv("BPE355_INPROC_RANKS", "1")
    text = np.empty(n, dtype=np.uint8)
    assert _lib.lib().bpe_synth_corpus_host(text.ctypes.data, n, e["seed"], e["flavour"], 0, 16) == 0
    tok = Tokenizer(vocab, merges, e["specials"])
    out = np.empty(n, dtype=np.uint32)   # cap >= n; only the pages written become resident
    n_out = ctypes.c_size_t(0)
    try:
        _lib.check(_lib.lib().bpe_tok_encode_gpus(tok._device(), text.ctypes.data_as(ctypes.c_char_p), n,
                                                  out.ctypes.data, n, ctypes.byref(n_out), 8), "encode x8")
    finally:
        tok.release_device_buffers()
        bpe_amd.set_num_gpus(None)
    del text
    torch.cuda.empty_cache()
    ids = out[:n_out.value]
    w = e["whole"]
    assert ids[:4096].tolist() == w["ids_head"]
    _check_slabs(ids, w["slabs"], "encode_gpus x8")
