"""ORACLE -- TEST INFRASTRUCTURE ONLY: a pure-Python restatement of the reference trainer,
kept structurally like the reference so its speed is representative of it.  It is the
`cpu_baseline` (kind "port") that bench.py times on the GPU box's host cores; the product
never imports it.

Follows reference models/tokenizer/train.py:
  16-28   pre-tokenize with the GPT-2 pattern (`regex` module) and count pre-tokens
  31-49   split words into single bytes; pair counts; pair -> words index
  183-228 per round: max over ALL pairs by (count, pair), rewrite the indexed words, update
          neighbour counts on the partially rewritten word, pop the best pair
  vocab.py:2-34 special tokens, 256 bytes, then each merged token (deduplicated).
The round loop can stop at a deadline so the bench can time a bounded sample.
"""
from __future__ import annotations

import time

import regex

GPT2_SPLIT = regex.compile(
    r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+""", regex.UNICODE)


def count_pretokens(text: str, specials) -> dict:
    skip = set(specials)
    counts: dict = {}
    for m in GPT2_SPLIT.finditer(text, concurrent=True):
        piece = m.group()
        if piece not in skip:
            counts[piece] = counts.get(piece, 0) + 1
    return counts


def train(text: str, vocab_size: int, specials=(), deadline: float | None = None):
    """Returns (vocab, merges, info).  info["complete"] is False if the deadline stopped it."""
    t0 = time.perf_counter()
    vocab_list: list = []
    present = set()
    for tok in [s.encode("utf-8") for s in specials] + [bytes([i]) for i in range(256)]:
        if tok not in present:
            present.add(tok)
            vocab_list.append(tok)
    rounds = vocab_size - len(vocab_list)

    counts = count_pretokens(text, specials)
    t_count = time.perf_counter() - t0
    words = []
    freq = []
    for piece, c in counts.items():
        words.append([bytes([b]) for b in piece.encode("utf-8")])
        freq.append(c)
    pairs: dict = {}
    where: dict = {}
    for wi, w in enumerate(words):
        c = freq[wi]
        for x, y in zip(w, w[1:]):
            pairs[(x, y)] = pairs.get((x, y), 0) + c
            where.setdefault((x, y), set()).add(wi)

    def bump(p, d):
        pairs[p] = pairs.get(p, 0) + d

    merges = []
    done = 0
    for _ in range(max(0, rounds)):
        if not pairs:
            break
        if deadline is not None and time.perf_counter() > deadline:
            break
        a, b = max(pairs, key=lambda p: (pairs[p], p))
        new = a + b
        if new not in present:
            present.add(new)
            vocab_list.append(new)
        for wi in list(where.get((a, b), ())):
            w = words[wi]
            c = freq[wi]
            i = 0
            while i < len(w) - 1:
                if w[i] == a and w[i + 1] == b:
                    if i > 0:
                        bump((w[i - 1], w[i]), -c)
                        bump((w[i - 1], new), c)
                    if i < len(w) - 2:
                        bump((w[i + 1], w[i + 2]), -c)
                        bump((new, w[i + 2]), c)
                    w[i] = new
                    del w[i + 1]
                    if i > 0:
                        where.setdefault((w[i - 1], new), set()).add(wi)
                    if i < len(w) - 1:
                        where.setdefault((new, w[i + 1]), set()).add(wi)
                i += 1
        pairs.pop((a, b))
        where.pop((a, b), None)
        merges.append((a, b))
        done += 1
    info = {"complete": done == max(0, rounds) or not pairs, "rounds_done": done,
            "rounds_total": max(0, rounds), "t_count_s": t_count,
            "t_merge_s": time.perf_counter() - t0 - t_count, "n_words": len(words)}
    return {i: t for i, t in enumerate(vocab_list)}, merges, info
