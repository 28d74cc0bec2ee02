"""Pin oracle/cpu_ref.py -- the pure-Python restatement of the reference trainer that bench.py
times as `cpu_baseline` -- against every train golden produced by the reference itself
(tests/golden/train_*.json, make_golden.py).  CPU only."""
import pytest

import golden_cases as G
from oracle import cpu_ref
from oracle import oracle


@pytest.mark.parametrize("name", G.names("train"))
def test_cpu_ref_train_matches_reference(name):
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    text = oracle.decode_text(data).decode("utf-8")   # the reference's text-mode read
    got_vocab, got_merges, info = cpu_ref.train(text, o["vocab_size"], o["special_tokens"])
    assert info["complete"]
    assert got_merges == merges
    assert got_vocab == vocab


@pytest.mark.parametrize("name", G.names("encode"))
def test_cpu_ref_encode_matches_reference(name):
    """the encode port bench.py times (cpu_baseline.encode) against every encode golden"""
    o = G.load("encode", name)
    vocab, merges = G.tokenizer_inputs(o)
    enc = cpu_ref.Encoder(vocab, merges, o["special_tokens"])
    assert enc.encode(G.encode_text(o)) == o["ids"]
