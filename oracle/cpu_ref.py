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


def train(text: str, vocab_size: int, specials=(), deadline: float | None = None,
          round_cap_s: float | None = None, progress: list | None = None, progress_every: int = 1000):
    """Returns (vocab, merges, info).  info["complete"] is False if the deadline (absolute) or the
    cap on the merge rounds' wall time (from the end of the count) stopped it.  `progress`, when
    given, receives (rounds done, seconds since the start, live pairs) every `progress_every`
    rounds (tools/cpu_port_full.py uses it to check the bench's flat-rate extrapolation)."""
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
    if round_cap_s is not None:
        cap_at = time.perf_counter() + round_cap_s
        deadline = cap_at if deadline is None else min(deadline, cap_at)
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

    t_build = time.perf_counter() - t0 - t_count   # words, pair counts and the pair -> words index

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
        if progress is not None and done % progress_every == 0:
            progress.append((done, time.perf_counter() - t0, len(pairs)))
    info = {"complete": done == max(0, rounds) or not pairs, "rounds_done": done,
            "rounds_total": max(0, rounds), "t_count_s": t_count,
            "t_merge_s": time.perf_counter() - t0 - t_count, "t_build_s": t_build, "n_words": len(words)}
    return {i: t for i, t in enumerate(vocab_list)}, merges, info


class Encoder:
    """Tokenizer.encode restated with the reference's structure (models/tokenizer/tokenizer.py):
      12-38    vocab_inv = {bytes: id} (last id wins); specials deduped, longest first, joined
               into one capture-group split pattern; a missing special gets id len(vocab)
      63-90    segment on the specials; each non-special segment pre-tokenized on its own,
               matches equal to a special dropped
      92-109   merge: every non-overlapping occurrence of the pair, left to right
      111-138  per pre-token: the adjacent pair of minimum merge rank (ties: first position)
               until no pair is ranked; ids by vocab_inv (KeyError when missing)
    inv_merges is rebuilt per encode() call, as the reference does (tokenizer.py:115)."""

    def __init__(self, vocab: dict, merges, specials=None):
        self.vocab = dict(vocab)
        self.vocab_inv = {v: k for k, v in self.vocab.items()}
        self.merges = list(merges)
        self.special_tokens = sorted(set(specials or []), key=len, reverse=True)
        sp = "|".join(regex.escape(t) for t in self.special_tokens)
        self.segment_rgx = f"({sp})" if sp else None
        for t in self.special_tokens:
            if t.encode("utf-8") not in self.vocab_inv:
                self.vocab[t.encode("utf-8")] = len(self.vocab)
                self.vocab_inv[t.encode("utf-8")] = len(self.vocab) - 1

    def pretokenize(self, text: str):
        segments = regex.split(self.segment_rgx, text) if self.segment_rgx else [text]
        out = []
        for seg in segments:
            if seg == "":
                continue
            if seg in self.special_tokens:
                out.append(seg)
                continue
            for m in GPT2_SPLIT.finditer(seg, concurrent=True):
                s = m.group(0)
                if s not in self.special_tokens:
                    out.append(s)
        return out

    @staticmethod
    def merge(tokens, pair, replacement):
        new, i = [], 0
        while i < len(tokens):
            if tokens[i] == pair[0] and i < len(tokens) - 1 and tokens[i + 1] == pair[1]:
                new.append(replacement)
                i += 2
            else:
                new.append(tokens[i])
                i += 1
        return new

    def encode(self, text: str):
        pretokens = self.pretokenize(text)
        inv_merges = {pair: i for i, pair in enumerate(self.merges)}
        ids = []
        inf = float("inf")
        for tok in pretokens:
            if tok in self.special_tokens:
                ids.append(self.vocab_inv[tok.encode("utf-8")])
                continue
            raw = [bytes([b]) for b in tok.encode("utf-8")]
            while len(raw) > 1:
                pair = min(zip(raw, raw[1:]), key=lambda p: inv_merges.get(p, inf))
                if pair not in inv_merges:
                    break
                raw = self.merge(raw, pair, pair[0] + pair[1])
            ids.extend(self.vocab_inv[b] for b in raw)
        return ids
