"""Tokenizer persistence: pickles (tokenizer.py:50-61, 159-167)
and the GPT-2 text formats (reference tests/common.py:10-59).  Host-side: no GPU needed."""
import pickle
import random

import gpt2_files
from bpe_amd import Tokenizer
from bpe_amd import formats


def test_remap_is_a_bijection_matching_the_fixture_loader():
    table = formats.bytes_to_unicode()
    assert sorted(table) == list(range(256))
    assert len(set(table.values())) == 256
    assert table == gpt2_files.byte_to_printable()


def test_load_gpt2_matches_reference_test_helper():
    got = formats.load_gpt2(gpt2_files.FIXTURES / "gpt2_vocab.json", gpt2_files.FIXTURES / "gpt2_merges.txt",
                            ["<|endoftext|>"])
    want = gpt2_files.load_gpt2(["<|endoftext|>"])
    assert got[0] == want[0]
    assert got[1] == want[1]


def test_gpt2_roundtrip_arbitrary_bytes(tmp_path):
    rng = random.Random(5)
    vocab = {i: bytes([i]) for i in range(256)}
    merges = []
    for k in range(300):
        a, b = rng.choice(list(vocab.values())), rng.choice(list(vocab.values()))
        merges.append((a, b))
        vocab[256 + k] = a + b + bytes([rng.randrange(256)])   # any bytes, incl. space/newline/NUL
    tok = Tokenizer(dict(vocab), list(merges), [])
    tok.save_gpt2(tmp_path / "v.json", tmp_path / "m.txt")
    back = Tokenizer.from_gpt2_files(tmp_path / "v.json", tmp_path / "m.txt")
    first = {}
    for i in sorted(vocab):
        first.setdefault(vocab[i], i)
    assert back.vocab == {i: b for b, i in first.items()}
    assert back.merges == merges


def test_pickle_save_and_from_files(tmp_path):
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    tok.save(str(tmp_path), "t")
    with open(tmp_path / "t-vocab.pkl", "rb") as f:   # this test's own files
        assert pickle.load(f) == tok.vocab
    back = Tokenizer.from_files(str(tmp_path / "t-vocab.pkl"), str(tmp_path / "t-merges.pkl"),
                                ["<|endoftext|>"])
    assert back.vocab == tok.vocab
    assert back.merges == tok.merges
    assert back.vocab_inv == tok.vocab_inv


def test_from_files_is_the_constructor_on_the_pickled_objects(tmp_path):
    # a special missing from the vocab is stored under its BYTES key (tokenizer.py:35-38); saving
    # and loading such a tokenizer re-runs that rule on the pickled dict, as the reference does
    vocab, merges = gpt2_files.load_gpt2([])
    tok = Tokenizer(dict(vocab), list(merges), ["<|pad|>"])
    tok.save(str(tmp_path), "t")
    with open(tmp_path / "t-vocab.pkl", "rb") as f:
        pickled = pickle.load(f)
    back = Tokenizer.from_files(str(tmp_path / "t-vocab.pkl"), str(tmp_path / "t-merges.pkl"), ["<|pad|>"])
    direct = Tokenizer(pickled, list(merges), ["<|pad|>"])
    assert back.vocab == direct.vocab and back.vocab_inv == direct.vocab_inv
