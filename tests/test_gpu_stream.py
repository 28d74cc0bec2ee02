"""encode_iterable streaming: tokenizer.py:140-150 concatenates
items until a batch holds >= 2 MiB characters, encodes the batch, yields its ids, and goes on --
memory stays bounded by one batch.  (The reference re-iterates a re-iterable argument forever;
here the argument is consumed once: DESIGN.md section 7.)"""
import pytest

import gpt2_files
from oracle import oracle

pytestmark = pytest.mark.gpu

BATCH = 1024 * 1024 * 2


def _lines(n_lines, consumed):
    base = (gpt2_files.FIXTURES / "tinystories_sample.txt").read_text(encoding="utf-8").splitlines(True)
    for k in range(n_lines):
        consumed[0] += 1
        yield base[k % len(base)]


def test_encode_iterable_is_lazy_and_batch_exact():
    from bpe_amd import Tokenizer
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    consumed = [0]
    n_lines = 120_000   # ~10 MB of text: several batches
    it = tok.encode_iterable(_lines(n_lines, consumed))
    first = next(it)
    assert consumed[0] < n_lines // 2     # yielded after the first batch, not the whole stream
    got = [first] + list(it)
    # expected: the reference's batching (items concatenated until >= 2 MiB characters)
    want, text = [], ""
    for line in _lines(n_lines, [0]):
        text += line
        if len(text) >= BATCH:
            want += oracle.encode(vocab, merges, ["<|endoftext|>"], text)
            text = ""
    if text:
        want += oracle.encode(vocab, merges, ["<|endoftext|>"], text)
    assert got == want
