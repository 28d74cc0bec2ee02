"""Load the GPT-2 vocab / merges fixture files (tests/golden/fixtures) as raw bytes.

The files use GPT-2's printable byte->unicode remapping (the public GPT-2 encoder scheme:
the 188 printable Latin-1 bytes map to themselves, the other 68 bytes map to U+0100..U+0143
in byte order).  Mirrors what the reference's test helper does
(reference tests/test_tokenizer.py:44-79, tests/common.py:10-59) so the GPT-2 goldens can be
rebuilt; written independently here.
"""
from __future__ import annotations

import functools
import json
import pathlib

FIXTURES = pathlib.Path(__file__).resolve().parent / "golden" / "fixtures"


@functools.lru_cache()
def byte_to_printable() -> dict[int, str]:
    keep = set(range(0x21, 0x7F)) | set(range(0xA1, 0xAD)) | set(range(0xAE, 0x100))
    table: dict[int, str] = {}
    shifted = 0
    for b in range(256):
        if b in keep:
            table[b] = chr(b)
        else:
            table[b] = chr(256 + shifted)
            shifted += 1
    return table


@functools.lru_cache()
def printable_to_byte() -> dict[str, int]:
    return {c: b for b, c in byte_to_printable().items()}


def unprintable(s: str) -> bytes:
    dec = printable_to_byte()
    return bytes(dec[c] for c in s)


def load_gpt2(special_tokens=None):
    """Return (vocab: dict[int, bytes], merges: list[tuple[bytes, bytes]]) as the reference's
    test helper builds them, including its rule of appending missing specials to the vocab."""
    with open(FIXTURES / "gpt2_vocab.json", encoding="utf-8") as f:
        raw_vocab = json.load(f)
    vocab = {idx: unprintable(tok) for tok, idx in raw_vocab.items()}
    merges = []
    with open(FIXTURES / "gpt2_merges.txt", encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip().split(" ")
            if len(parts) == 2 and parts[0] and parts[1]:
                merges.append((unprintable(parts[0]), unprintable(parts[1])))
    if special_tokens:
        present = set(vocab.values())
        for sp in special_tokens:
            b = sp.encode("utf-8")
            if b not in present:
                vocab[len(vocab)] = b
    return vocab, merges


def load_reference_train_golden():
    """The reference's own expected output for corpus.en @ vocab 500
    (tests/fixtures/train-bpe-reference-{merges.txt,vocab.json}; compared by
    reference tests/test_train_bpe.py:36-65)."""
    with open(FIXTURES / "train-bpe-reference-merges.txt", encoding="utf-8") as f:
        merges = []
        for line in f:
            a, b = line.rstrip().split(" ")
            merges.append((unprintable(a), unprintable(b)))
    with open(FIXTURES / "train-bpe-reference-vocab.json", encoding="utf-8") as f:
        vocab = {idx: unprintable(tok) for tok, idx in json.load(f).items()}
    return vocab, merges
