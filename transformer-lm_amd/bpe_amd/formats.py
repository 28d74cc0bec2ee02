"""Tokenizer file formats.

* Pickles: Tokenizer.save(path, prefix) / Tokenizer.from_files(...) write and read
  `<prefix>-vocab.pkl` (dict[int, bytes]) and `<prefix>-merges.pkl` (list[tuple[bytes, bytes]]),
  exactly as reference models/tokenizer/tokenizer.py:50-61, 159-167 do (see tokenizer.py).
* GPT-2 text files: `vocab.json` (token string -> id) and `merges.txt` ("a b" per line), whose
  token strings use GPT-2's printable remapping of bytes -- the scheme the reference's tests
  load the GPT-2 fixtures with (reference tests/common.py:10-59, test_tokenizer.py:44-79).
  Provided here as a product API so trained tokenizers can be exchanged with GPT-2 tooling.

The remapping: the 188 printable Latin-1 bytes (0x21-0x7E, 0xA1-0xAC, 0xAE-0xFF) stand for
themselves; the other 68 bytes map to U+0100.. in byte order.
"""
from __future__ import annotations

import functools
import json
from typing import Dict, List, Tuple


@functools.lru_cache()
def bytes_to_unicode() -> Dict[int, str]:
    printable = [b for b in range(256) if 0x21 <= b <= 0x7E or 0xA1 <= b <= 0xAC or 0xAE <= b <= 0xFF]
    table = {b: chr(b) for b in printable}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(0x100 + extra)
            extra += 1
    return table


@functools.lru_cache()
def unicode_to_bytes() -> Dict[str, int]:
    return {c: b for b, c in bytes_to_unicode().items()}


def to_printable(token: bytes) -> str:
    enc = bytes_to_unicode()
    return "".join(enc[b] for b in token)


def from_printable(text: str) -> bytes:
    dec = unicode_to_bytes()
    return bytes(dec[c] for c in text)


def load_gpt2(vocab_path, merges_path, special_tokens=None
              ) -> Tuple[Dict[int, bytes], List[Tuple[bytes, bytes]]]:
    """(vocab, merges) from GPT-2 vocab.json / merges.txt.  Special tokens missing from the
    vocab are appended with the next ids (the reference test helper's rule)."""
    with open(vocab_path, encoding="utf-8") as f:
        raw = json.load(f)
    vocab = {int(i): from_printable(tok) for tok, i in raw.items()}
    merges: List[Tuple[bytes, bytes]] = []
    with open(merges_path, encoding="utf-8") as f:
        for k, line in enumerate(f):
            if k == 0 and line.startswith("#version:"):   # HuggingFace-style header line
                continue
            parts = line.rstrip().split(" ")
            if len(parts) == 2 and parts[0] and parts[1]:
                merges.append((from_printable(parts[0]), from_printable(parts[1])))
    if special_tokens:
        present = set(vocab.values())
        for sp in special_tokens:
            b = sp.encode("utf-8")
            if b not in present:
                vocab[len(vocab)] = b
                present.add(b)
    return vocab, merges


def save_gpt2(vocab: Dict[int, bytes], merges: List[Tuple[bytes, bytes]], vocab_path, merges_path) -> None:
    """Write GPT-2 vocab.json / merges.txt.  Byte strings that repeat keep their first id in
    vocab.json (a JSON object holds each token once)."""
    out: Dict[str, int] = {}
    for i in sorted(vocab):
        out.setdefault(to_printable(vocab[i]), int(i))
    with open(vocab_path, "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False)
    with open(merges_path, "w", encoding="utf-8") as f:   # no header: the fixtures' layout
        for a, b in merges:
            f.write(f"{to_printable(a)} {to_printable(b)}\n")
