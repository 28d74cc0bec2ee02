"""GPU parity: libbpe355's train_bpe (HIP, gfx950) against the reference goldens and the oracle.

Bit-exact: ordered merges and the exact id -> bytes vocab must equal the reference's.
"""
import json
import os

import pytest

import golden_cases as G
import gpt2_files
from oracle import oracle

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")


@pytest.fixture(scope="module", autouse=True)
def _device():
    from bpe_amd import _lib
    _lib.require_device()


def test_reference_fixture_corpus_en_500():
    """reference tests/test_train_bpe.py:28-65, through the drop-in train_bpe."""
    vocab, merges = bpe_amd.train_bpe(gpt2_files.FIXTURES / "corpus.en", 500, ["<|endoftext|>"])
    ref_vocab, ref_merges = gpt2_files.load_reference_train_golden()
    assert merges == ref_merges
    assert set(vocab.keys()) == set(ref_vocab.keys())
    assert set(vocab.values()) == set(ref_vocab.values())


def test_merges_are_vocab_objects_and_match_the_flat_view():
    """The result's merges come from bpe_result_merge_ids: each part is the vocab's own bytes
    object (as the reference appends (vocab[a], vocab[b]), train.py:191-196), and the pairs equal
    the byte records of bpe_result_flat(0) (the view the shim falls back to)."""
    import ctypes
    from bpe_amd import _lib
    L = _lib.lib()
    arr, n, _keep = _lib.c_strings(["<|endoftext|>"])
    data = (gpt2_files.FIXTURES / "corpus.en").read_bytes()
    res = ctypes.c_void_p()
    _lib.check(L.bpe_train_buffer(data, len(data), 500, arr, n, None, ctypes.byref(res)), "train")
    lens, buf, nb = ctypes.POINTER(ctypes.c_uint32)(), ctypes.c_void_p(), ctypes.c_size_t(0)
    k = L.bpe_result_flat(res, 0, ctypes.byref(lens), ctypes.byref(buf), ctypes.byref(nb))
    raw = ctypes.string_at(buf, nb.value)
    parts, o = [], 0
    for i in range(k):
        parts.append(raw[o:o + lens[i]])
        o += lens[i]
    ids = ctypes.POINTER(ctypes.c_uint32)()
    assert L.bpe_result_merge_ids(res, ctypes.byref(ids)) == k // 2 > 0
    vocab, merges, _ = _lib.take_result(res)   # (frees res)
    assert merges == list(zip(parts[0::2], parts[1::2]))
    objs = {id(b) for b in vocab.values()}
    assert all(id(a) in objs and id(b) in objs for a, b in merges)


@pytest.mark.parametrize("name", G.names("train"))
def test_train_matches_reference_golden(name):
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    got_vocab, got_merges = bpe_amd.train_bpe_bytes(data, o["vocab_size"], o["special_tokens"])
    assert got_merges == merges
    assert got_vocab == vocab


def test_train_file_path_and_errors(tmp_path):
    with pytest.raises(FileNotFoundError):
        bpe_amd.train_bpe(tmp_path / "missing.txt", 300, [])
    err = json.loads((G.GOLDEN / "error_train_bad_utf8.json").read_text())
    p = tmp_path / "bad.txt"
    p.write_bytes(bytes.fromhex(err["input_hex"]))
    with pytest.raises(UnicodeDecodeError):
        bpe_amd.train_bpe(p, 300, [])


@pytest.mark.parametrize("seed,n_chars,flavour,vocab", [
    (11, 3_000_000, "mixed", 4000),
    (12, 2_000_000, "space", 3000),
    (13, 8_000_000, "ascii", 6000),
])
def test_train_matches_oracle_synthetic(seed, n_chars, flavour, vocab):
    import synth_text
    data = synth_text.generate(seed, n_chars, flavour).encode("utf-8")
    want = oracle.train_raw(data, vocab, ["<|endoftext|>"])
    got = bpe_amd.train_bpe_bytes(data, vocab, ["<|endoftext|>"])
    assert got[1] == want[1]
    assert got[0] == want[0]


def test_deterministic_repeat():
    data = (gpt2_files.FIXTURES / "corpus.en").read_bytes()
    r1 = bpe_amd.train_bpe_bytes(data, 1500, ["<|endoftext|>"])
    r2 = bpe_amd.train_bpe_bytes(data, 1500, ["<|endoftext|>"])
    assert r1 == r2


def _tie_heavy_text(rng, n_words):
    """Short words over a tiny alphabet: pair counts tie constantly, and tied pairs often share a
    token with the top ones -- the cases the batched rounds' rules (1)-(4') must get right."""
    alpha = rng.choice(["ab", "abc", "abcd", "aab", "xyz "])
    words = []
    for _ in range(n_words):
        words.append("".join(rng.choice(alpha) for _ in range(rng.randint(1, 7))))
    sep = rng.choice([" ", "  ", "\n", " \n"])
    return sep.join(words)


@pytest.mark.parametrize("seed", range(16))
def test_train_matches_oracle_tie_heavy(seed):
    import random
    rng = random.Random(9000 + seed)
    data = _tie_heavy_text(rng, rng.choice([200, 2000, 20000])).encode("utf-8")
    vocab = rng.choice([300, 400, 1000])
    want = oracle.train_raw(data, vocab, ["<|endoftext|>"])
    got = bpe_amd.train_bpe_bytes(data, vocab, ["<|endoftext|>"])
    assert got[1] == want[1]
    assert got[0] == want[0]


@pytest.mark.parametrize("knob", ["BPE355_FOLD=1", "BPE355_LDS_CELLS=0",
                                  "BPE355_DENSE_TOK=128+BPE355_SPARSE_FROM=128+BPE355_CHECK_MARKS=1", "BPE355_CELL_MARKS=0"])
def test_train_runtime_variants(knob, monkeypatch):
    """The merge loop's run-time variants against the same goldens: the fused trip
    kernel k_trip (BPE355_FOLD=1: every workgroup decides the batch again while others already
    rewrite) and the 64-bit global delta cells (BPE355_LDS_CELLS=0: the path a batch takes when
    its P1 count reaches 2^32), the touched-block cells with a dense prefix of 128 tokens (every
    later token's cells found through the merge's marks, as at the bench config past 2048 tokens)
    and without marks (every cell scanned) -- each on the reference fixture, tie-heavy text and
    synthetic text, bit-exact."""
    import random
    for kv in knob.split("+"):   # (BPE355_CHECK_MARKS: the library fails the call if a delta cell
        name, val = kv.split("=")  # escaped the marks or two apply workgroups listed other blocks)
        monkeypatch.setenv(name, val)
    vocab, merges = bpe_amd.train_bpe(gpt2_files.FIXTURES / "corpus.en", 500, ["<|endoftext|>"])
    ref_vocab, ref_merges = gpt2_files.load_reference_train_golden()
    assert merges == ref_merges
    assert set(vocab.values()) == set(ref_vocab.values())
    for seed in (3, 7):
        rng = random.Random(9000 + seed)
        data = _tie_heavy_text(rng, 20000).encode("utf-8")
        want = oracle.train_raw(data, 1000, ["<|endoftext|>"])
        assert bpe_amd.train_bpe_bytes(data, 1000, ["<|endoftext|>"]) == want
    import synth_text
    data = synth_text.generate(11, 3_000_000, "mixed").encode("utf-8")
    want = oracle.train_raw(data, 4000, ["<|endoftext|>"])
    assert bpe_amd.train_bpe_bytes(data, 4000, ["<|endoftext|>"]) == want
