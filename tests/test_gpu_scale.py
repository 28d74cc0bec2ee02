"""Bit-exact parity at the north-star sizes (BASELINE.json configs[1], [2], [4]) and on the code
paths only large corpora reach.

The expected results are committed under tests/golden/scale/ by make_scale_golden.py: the C
oracle (pinned to the reference by the small goldens) trained on the same deterministic corpus,
written on the host by bpe_synth_corpus_host.  Here the device writes the corpus into HBM
(bpe_synth_corpus_device), a sample of its 64 MiB pieces is checked against the fixture's
per-piece sha256, and the GPU trainer must reproduce the oracle's ordered merges (reference
models/tokenizer/train.py:183-231) and id-ordered vocab exactly.
"""
from __future__ import annotations

import ctypes
import gzip
import hashlib
import json
import os
import pathlib
import struct

import numpy as np
import pytest

import bpe_amd
from bpe_amd import _lib, train_bpe_device, Tokenizer
from bpe_amd.train import last_train_stats

pytestmark = pytest.mark.gpu

SCALE = pathlib.Path(__file__).resolve().parent / "golden" / "scale"


def _load(kind, name):
    with gzip.open(SCALE / f"{kind}_{name}.json.gz", "rt") as f:
        return json.load(f)


def _device_corpus(seed, flavour, n):
    import torch
    L = _lib.lib()
    corpus = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), n, seed, flavour, 0,
                                         None), "synth")
    torch.cuda.synchronize()
    return corpus


def _check_pieces(corpus, o):
    """the device bytes equal the oracle's input: first, last and two middle 64 MiB pieces"""
    piece, digests = o["digest_piece"], o["piece_sha256"]
    k = len(digests)
    for i in sorted({0, k // 3, (2 * k) // 3, k - 1}):
        lo = i * piece
        got = hashlib.sha256(corpus[lo:lo + piece].cpu().numpy().tobytes()).hexdigest()
        assert got == digests[i], f"device corpus piece {i} differs from the host generator"


def _vocab_digest(vocab):
    h = hashlib.sha256()
    for i in range(len(vocab)):
        b = vocab[i]
        h.update(struct.pack("<I", len(b)) + b)
    return h.hexdigest()


def _first_diff(got, want):
    for i, (g, w) in enumerate(zip(got, want)):
        if g != w:
            return i, g, w
    return min(len(got), len(want)), None, None


@pytest.mark.parametrize("name", ["C3_1G", "U32", "C2", "C3"])
def test_train_scale_bit_exact(name):
    o = _load("train", name)
    corpus = _device_corpus(o["seed"], o["flavour"], o["n"])
    _check_pieces(corpus, o)
    vocab, merges = train_bpe_device(corpus.data_ptr(), o["n"], o["vocab"], o["specials"])
    st = last_train_stats()
    del corpus
    want = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in o["merges"]]
    assert len(merges) == o["n_merges"]
    if merges != want:
        i, g, w = _first_diff(merges, want)
        pytest.fail(f"{name}: merge {i} differs: GPU {g!r} oracle {w!r}")
    assert len(vocab) == o["n_vocab"] and _vocab_digest(vocab) == o["vocab_sha256"]
    # A1 pinned on its own: the device's unique multi-byte words and their pre-token total
    assert st["n_words"] == o["n_words_multibyte"]
    assert st["n_pretokens"] == o["n_pretokens_multibyte"]


def test_encode_scale_bit_exact():
    """C5: Tokenizer.encode of 256 MB of the C3 corpus with the C3 merges (reference
    tokenizer.py:111-138), id stream equal to the oracle's (sha256, head and tail)."""
    e = _load("encode", "C5_256M")
    o = _load("train", e["train"])
    merges = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in o["merges"]]
    ids_vocab = {}
    for s in e["specials"]:
        ids_vocab.setdefault(s.encode(), len(ids_vocab))
    for b in range(256):
        ids_vocab.setdefault(bytes([b]), len(ids_vocab))
    for a, b in merges:
        ids_vocab.setdefault(a + b, len(ids_vocab))
    vocab = {i: b for b, i in ids_vocab.items()}
    import torch
    corpus = _device_corpus(e["seed"], e["flavour"], e["n"])
    assert hashlib.sha256(corpus.cpu().numpy().tobytes()).hexdigest() == e["corpus_sha256"]
    tok = Tokenizer(vocab, merges, e["specials"])
    L = _lib.lib()
    out = torch.empty(e["n"], dtype=torch.int32, device="cuda")
    n_out = ctypes.c_size_t(0)
    _lib.check(L.bpe_tok_encode_device(tok._device(), ctypes.c_void_p(corpus.data_ptr()), e["n"],
                                       ctypes.c_void_p(out.data_ptr()), ctypes.byref(n_out), None),
               "encode")
    torch.cuda.synchronize()
    ids = out[:n_out.value].cpu().numpy().astype(np.uint32)
    assert ids.size == e["n_ids"]
    assert ids[:4096].tolist() == e["ids_head"]
    assert ids[-4096:].tolist() == e["ids_tail"]
    assert hashlib.sha256(ids.tobytes()).hexdigest() == e["ids_sha256"]


# ------------------------------------------------------------------ forced large-corpus paths
@pytest.fixture
def knob():
    saved = {}

    def set_(k, v):
        saved.setdefault(k, os.environ.get(k))
        os.environ[k] = str(v)

    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _synth_host(seed, flavour, n):
    L = _lib.lib()
    buf = np.empty(n, dtype=np.uint8)
    assert L.bpe_synth_corpus_host(buf.ctypes.data, n, seed, flavour, 0, 8) == 0
    return buf.tobytes()


def test_synth_host_twin_matches_device():
    """bpe_synth_corpus_host writes the bytes the device writes (both flavours, odd sizes,
    a non-zero first block)."""
    import torch
    L = _lib.lib()
    for seed, flavour, n, first in [(2, 0, 48 << 20, 0), (1, 1, 3_000_001, 7), (9, 0, 4095, 123)]:
        d = torch.empty(n, dtype=torch.uint8, device="cuda")
        _lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(d.data_ptr()), n, seed, flavour, first,
                                             None), "synth")
        h = np.empty(n, dtype=np.uint8)
        assert L.bpe_synth_corpus_host(h.ctypes.data, n, seed, flavour, first, 4) == 0
        assert np.array_equal(d.cpu().numpy(), h)


def test_pair_table_growth_vs_oracle(knob):
    """grow_pairs / k_rehash (the bench corpus rehashes twice): a 2^18-slot first table on a
    corpus whose pair table passes 2^17 keys."""
    from oracle import oracle
    data = _synth_host(11, 0, 12 << 20)
    knob("BPE355_PAIR_CAP_LOG2", 18)
    vocab, merges = bpe_amd.train_bpe_bytes(data, 8000, ["<|endoftext|>"])
    assert last_train_stats()["n_pairs_final"] > (1 << 17)
    assert (vocab, merges) == oracle.train_raw(data, 8000, ["<|endoftext|>"])


def test_word_table_recount_vs_oracle(knob):
    """the word-count table overflows and the count reruns with 4x the slots (4 times here)"""
    from oracle import oracle
    data = _synth_host(12, 1, 3 << 20)
    knob("BPE355_WORD_CAP_LOG2", 10)
    vocab, merges = bpe_amd.train_bpe_bytes(data, 3000, ["<|endoftext|>"])
    assert (vocab, merges) == oracle.train_raw(data, 3000, ["<|endoftext|>"])


def test_batched_equals_per_round_bench_corpus(knob):
    """the batched trips (k_select/k_merge_batch/k_apply_batch) and the one-round-per-trip path
    give the same merges on 64 MB of the bench recipe at 32k"""
    import torch
    corpus = _device_corpus(2, 0, 64 << 20)
    a = train_bpe_device(corpus.data_ptr(), corpus.numel(), 32000, ["<|endoftext|>"])
    knob("BPE355_BATCH", 0)
    b = train_bpe_device(corpus.data_ptr(), corpus.numel(), 32000, ["<|endoftext|>"])
    assert a == b
    del torch
