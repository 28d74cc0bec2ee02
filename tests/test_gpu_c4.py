"""The multi-rank protocols at the north-star sizes (BASELINE.json configs[3] and [4]: OWT vocab
32k sharded over 8 GPUs, and Tokenizer.encode on 8 GPUs), on the one GPU this box has.

The ranks are threads of this process sharing the card (BPE355_INPROC_RANKS=1: RCCL refuses two
ranks on one device); their collectives go through the library's in-process communicator, which
keeps RCCL's contracts (sum all-reduce, all-gather of equal-size segments).  Everything else --
slab cuts at safe points, each rank's file read and count, the word exchange or the per-round
delta exchange, the merge loop -- is the code the 8-GPU run executes.  The expected results are
the single-GPU goldens of tests/golden/scale/ (the C oracle, pinned to the reference by the small
goldens), so the sharded result must equal the reference's unsharded one
(models/tokenizer/train.py:183-231, tokenizer.py:111-138) bit for bit.
"""
from __future__ import annotations

import ctypes
import gzip
import hashlib
import json
import mmap
import os
import pathlib
import struct
import tempfile

import numpy as np
import pytest

import bpe_amd
from bpe_amd import _lib, Tokenizer
from bpe_amd.train import last_train_stats

pytestmark = pytest.mark.gpu

SCALE = pathlib.Path(__file__).resolve().parent / "golden" / "scale"


def _load(kind, name):
    with gzip.open(SCALE / f"{kind}_{name}.json.gz", "rt") as f:
        return json.load(f)


def _vocab_digest(vocab):
    h = hashlib.sha256()
    for i in range(len(vocab)):
        b = vocab[i]
        h.update(struct.pack("<I", len(b)) + b)
    return h.hexdigest()


def _check(o, vocab, merges, name):
    want = [(bytes.fromhex(a), bytes.fromhex(b)) for a, b in o["merges"]]
    assert len(merges) == o["n_merges"]
    if merges != want:
        i = next(i for i, (g, w) in enumerate(zip(merges, want)) if g != w)
        pytest.fail(f"{name}: merge {i} differs: sharded {merges[i]!r} oracle {want[i]!r}")
    assert len(vocab) == o["n_vocab"] and _vocab_digest(vocab) == o["vocab_sha256"]


@pytest.fixture
def inproc(monkeypatch):
    monkeypatch.setenv("BPE355_INPROC_RANKS", "1")
    yield monkeypatch
    bpe_amd.set_num_gpus(None)


def _corpus_file(o) -> pathlib.Path:
    """the golden's corpus as a page-cache-warm file (the bench's scratch name, so a bench run in
    the same call reuses it); pieces checked against the golden's per-piece sha256"""
    n = o["n"]
    d = pathlib.Path(os.environ.get("BPE355_BENCH_DIR", tempfile.gettempdir()))
    path = d / f"bpe355_bench_s{o['seed']}_f{o['flavour']}_{n}.txt"
    if not (path.exists() and path.stat().st_size == n):
        tmp = path.with_suffix(".part")
        with open(tmp, "wb+") as f:
            f.truncate(n)
            with mmap.mmap(f.fileno(), n) as m:
                buf = (ctypes.c_char * n).from_buffer(m)
                assert _lib.lib().bpe_synth_corpus_host(ctypes.addressof(buf), n, o["seed"], o["flavour"],
                                                        0, 16) == 0
                del buf
        os.replace(tmp, path)
    piece, digests = o["digest_piece"], o["piece_sha256"]
    k = len(digests)
    with open(path, "rb") as f:
        for i in sorted({0, k // 2, k - 1}):
            f.seek(i * piece)
            assert hashlib.sha256(f.read(piece)).hexdigest() == digests[i], f"corpus piece {i}"
    return path


def test_c4_eight_ranks_words_full_owt(inproc):
    """configs[3] at full size: the 11.9 GB C3 corpus file in 8 slabs, each rank reads and counts
    its own, one all-to-all of the words by owner, one all-gather of the owners' tables, the merge
    loop on the union: the train_C3 golden"""
    o = _load("train", "C3")
    path = _corpus_file(o)
    inproc.setenv("BPE355_EXCHANGE", "words")
    bpe_amd.set_num_gpus(8)
    vocab, merges = bpe_amd.train_bpe(path, o["vocab"], o["specials"])
    st = last_train_stats()
    assert st["n_gpus"] == 8
    assert st["n_bytes"] == o["n"]
    # every rank contributed its slab's words; the union holds the single-GPU word table
    assert st["n_exchanged_words"] >= o["n_words_multibyte"]
    assert st["n_words"] == o["n_words_multibyte"]
    _check(o, vocab, merges, "C4 words x8")
    # the exchange's measured parts (DESIGN.md section 5's table): recorded when asked
    out = os.environ.get("BPE355_STATS_OUT")
    if out:
        keep = ("t_total_ms", "t_load_ms", "t_count_ms", "t_exchange_ms", "t_alltoall_ms", "t_owner_ms",
                "t_gather_ms", "t_union_ms", "exchange_a2a_bytes", "exchange_seg_bytes", "n_exchanged_words",
                "n_words", "t_words_ms", "t_merge_ms", "n_gpus")
        with open(out, "w") as f:
            json.dump({"test": "test_c4_eight_ranks_words_full_owt", "ranks": "8 in-process ranks sharing one "
                       "GPU; the all-to-all by owner and the all-gather of the owners' tables through host "
                       "memory (the in-process communicator)",
                       **{k: st[k] for k in keep}}, f, indent=1)


@pytest.mark.parametrize("ranks", [2, 8])
def test_c4_ranks_rounds_1g(inproc, ranks):
    """the SURVEY's per-round protocol (one sum all-reduce of the delta cells per merge
    round, replicated pair tables and argmax on every rank; reference train.py:183-228) on the
    1 GB C3 prefix at vocab 32k, at 2 and 8 ranks; the driver also requires every rank to have
    chosen the same merges"""
    o = _load("train", "C3_1G")
    buf = np.empty(o["n"], dtype=np.uint8)
    assert _lib.lib().bpe_synth_corpus_host(buf.ctypes.data, o["n"], o["seed"], o["flavour"], 0, 16) == 0
    inproc.setenv("BPE355_EXCHANGE", "rounds")
    bpe_amd.set_num_gpus(ranks)
    vocab, merges = bpe_amd.train_bpe_bytes(buf.tobytes(), o["vocab"], o["specials"])
    st = last_train_stats()
    assert st["n_gpus"] == ranks
    _check(o, vocab, merges, f"C3_1G rounds x{ranks}")
    out = os.environ.get("BPE355_STATS_OUT")
    if out:   # the per-round mode's merge loop beside the words mode
        p = pathlib.Path(out)
        p = p.with_name(f"{p.stem}_rounds{ranks}{p.suffix}")
        keep = ("t_total_ms", "t_count_ms", "t_words_ms", "t_merge_ms", "n_rounds_device", "n_gpus")
        with open(p, "w") as f:
            json.dump({"test": f"test_c4_ranks_rounds_1g[{ranks}]",
                       "ranks": f"{ranks} in-process ranks sharing one GPU; per-round all-reduce through "
                                "host memory (the in-process communicator)",
                       "us_per_round": round(st["t_merge_ms"] * 1e3 / max(1, st["n_rounds_device"]), 2),
                       **{k: st[k] for k in keep}}, f, indent=1)


def test_c5_encode_eight_devices(inproc):
    """configs[4] on 8 devices: 256 MB of the C3 corpus cut at safe points no special spans, one
    piece per rank, ids concatenated -- the C5 golden's id stream (sha256, head, tail)"""
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
    n = e["n"]
    text = np.empty(n, dtype=np.uint8)
    assert _lib.lib().bpe_synth_corpus_host(text.ctypes.data, n, e["seed"], e["flavour"], 0, 16) == 0
    assert hashlib.sha256(text.tobytes()).hexdigest() == e["corpus_sha256"]
    tok = Tokenizer(vocab, merges, e["specials"])
    out = np.empty(n, dtype=np.uint32)
    n_out = ctypes.c_size_t(0)
    _lib.check(_lib.lib().bpe_tok_encode_gpus(tok._device(), text.ctypes.data_as(ctypes.c_char_p), n,
                                              out.ctypes.data, n, ctypes.byref(n_out), 8), "encode x8")
    ids = out[:n_out.value]
    assert ids.size == e["n_ids"]
    assert ids[:4096].tolist() == e["ids_head"]
    assert ids[-4096:].tolist() == e["ids_tail"]
    assert hashlib.sha256(ids.tobytes()).hexdigest() == e["ids_sha256"]
