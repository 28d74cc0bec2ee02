"""Tokenizer.decode on the device: tokenizer.py:155-157,
b"".join(self.vocab[i] for i in ids).decode("utf-8", errors="replace")."""
import random

import pytest

import gpt2_files

pytestmark = pytest.mark.gpu


def _ref_decode(vocab, ids):
    return b"".join([vocab[i] for i in ids]).decode("utf-8", errors="replace")


def test_decode_random_ids_including_broken_utf8():
    from bpe_amd import Tokenizer
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    rng = random.Random(3)
    ids_all = sorted(vocab)
    for n in (0, 1, 7, 1000, 200_000):
        ids = [rng.choice(ids_all) for _ in range(n)]   # single-byte ids split UTF-8 sequences
        assert tok.decode(ids) == _ref_decode(tok.vocab, ids)


def test_decode_missing_id_raises_keyerror():
    from bpe_amd import Tokenizer
    vocab, merges = gpt2_files.load_gpt2([])
    tok = Tokenizer(dict(vocab), list(merges), [])
    with pytest.raises(KeyError):
        tok.decode([15496, len(vocab) + 5])
    with pytest.raises(KeyError):
        tok.decode([-1])


def test_decode_roundtrip_encode():
    from bpe_amd import Tokenizer
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = (gpt2_files.FIXTURES / "tinystories_sample.txt").read_text(encoding="utf-8")
    assert tok.decode(tok.encode(text)) == text
