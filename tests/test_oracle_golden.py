"""Pin the oracle (oracle/bpe_oracle.c, CPU restatement) against the reference's golden
vectors before it is trusted as the checker for the HIP path.  CPU only.

Golden sources:
  * the reference's own fixtures: tests/fixtures/train-bpe-reference-{merges.txt,vocab.json}
    (reference tests/test_train_bpe.py:28-65 compares merges exactly and vocab as sets);
  * tests/golden/*.json produced by running the reference itself (tests/golden/make_golden.py).
"""
import pytest

import golden_cases as G
import gpt2_files
from oracle import oracle


def test_reference_fixture_corpus_en_500():
    """The reference's own test (test_train_bpe.py:28-65) against the oracle."""
    vocab, merges = oracle.train_file(gpt2_files.FIXTURES / "corpus.en", 500, ["<|endoftext|>"])
    ref_vocab, ref_merges = gpt2_files.load_reference_train_golden()
    assert merges == ref_merges
    assert set(vocab.keys()) == set(ref_vocab.keys())
    assert set(vocab.values()) == set(ref_vocab.values())


@pytest.mark.parametrize("name", G.names("train"))
def test_oracle_train_matches_reference(name):
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    got_vocab, got_merges = oracle.train_raw(data, o["vocab_size"], o["special_tokens"])
    assert got_merges == merges
    assert got_vocab == vocab          # exact id -> bytes, stricter than the reference test


def test_oracle_bad_utf8_raises():
    import json
    err = json.loads((G.GOLDEN / "error_train_bad_utf8.json").read_text())
    with pytest.raises(UnicodeDecodeError):
        oracle.train_raw(bytes.fromhex(err["input_hex"]), err["vocab_size"], [])
    assert err["error"] == "UnicodeDecodeError"


@pytest.mark.parametrize("name", G.names("words"))
def test_oracle_word_counts_match_reference(name):
    o = G.load("words", name)
    text = oracle.decode_text(G.input_bytes(o["input"]))
    got = oracle.word_counts(text, o["special_tokens"])
    want = {bytes.fromhex(h): c for h, c in o["words"]}
    assert got == want


@pytest.mark.parametrize("name", G.names("encode"))
def test_oracle_encode_matches_reference(name):
    o = G.load("encode", name)
    vocab, merges = G.tokenizer_inputs(o)
    ids = oracle.encode(vocab, merges, o["special_tokens"], G.encode_text(o))
    assert ids == o["ids"]
