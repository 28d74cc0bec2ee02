"""Deterministic adversarial text generator for the golden fixtures (test data only).

The golden vectors in this directory were produced by running the reference trainer /
tokenizer on text made by this module (see make_golden.py).  The tests regenerate the
same text from (seed, n_chars, flavour) and check its sha256 before comparing, so only
the generator and the digests are committed, not the text.

Pure Python, integer-only splitmix64 so the output is identical on every machine.
The mix deliberately exercises every branch of the GPT-2 pre-tokenizer pattern
(reference models/tokenizer/train.py:143-146): Unicode letters of many scripts, Unicode
digits (Nd/Nl/No), combining marks (category M: neither L nor N nor \\s), every \\s code
point of the `regex` module plus the U+001C..U+001F separators that Python's
str.isspace() accepts but `regex` does not, contractions in both cases, runs of
whitespace ending in a space/newline/EOF, emoji, and <|endoftext|> separators.
"""
from __future__ import annotations

import hashlib

MASK = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & MASK

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n


_ASCII_SYLL = ["th", "e", "an", "in", "er", "on", "re", "at", "en", "nd", "ti", "es", "or",
               "te", "of", "ed", "is", "it", "al", "ar", "st", "to", "nt", "ng", "se", "ha",
               "a", "o", "i", "u", "y", "s", "t", "k", "z", "qu", "x"]
_UNI_LETTERS = ["é", "ß", "ü", "ñ", "ø", "ł", "ç", "Ω", "λ", "ж", "я", "ш", "א", "ב", "ع", "ل",
                "中", "文", "字", "日", "本", "語", "한", "국", "あ", "カ", "ก", "ข", "अ", "क",
                "ǅ", "ʰ", "ᵃ", "ﬁ"]
_MARKS = ["\u0301", "\u0308", "\u093f", "\u0e31", "\u20dd"]           # Mn / Mc / Me: class "other"
_DIGITS = ["0", "1", "2", "3", "7", "9", "٣", "۴", "३", "３", "²", "½", "Ⅻ", "〇", "𝟙"]
_PUNCT = ["!", "?", ".", ",", ";", ":", "-", "—", "…", "(", ")", "\"", "«", "»", "@", "#",
          "$", "%", "&", "*", "+", "=", "/", "\\", "<", ">", "|", "~", "^", "_", "`", "{", "}",
          "🙃", "👍🏽", "€", "©", "\u200b", "\ufeff", "\x00", "\x7f", "\x93"]
_SPACES_ALL = ["\t", "\n", "\x0b", "\x0c", "\r", " ", "\x85", "\xa0", "\u1680", "\u2000",
               "\u2003", "\u2007", "\u200a", "\u2028", "\u2029", "\u202f", "\u205f", "\u3000"]
_NOT_SPACE_SEP = ["\x1c", "\x1d", "\x1e", "\x1f"]
_CONTRACTIONS = ["'s", "'t", "'re", "'ve", "'m", "'ll", "'d", "'S", "'T", "'RE", "'x", "''",
                 "'"]


def _word(r: SplitMix64, uni: bool) -> str:
    n = 1 + r.below(4)
    parts = []
    for _ in range(n):
        if uni and r.below(6) == 0:
            parts.append(_UNI_LETTERS[r.below(len(_UNI_LETTERS))])
        else:
            parts.append(_ASCII_SYLL[r.below(len(_ASCII_SYLL))])
        if uni and r.below(40) == 0:
            parts.append(_MARKS[r.below(len(_MARKS))])
    w = "".join(parts)
    k = r.below(10)
    if k == 0:
        w = w.capitalize()
    elif k == 1 and r.below(4) == 0:
        w = w.upper()
    return w


def generate(seed: int, n_chars: int, flavour: str = "mixed") -> str:
    """Return exactly n_chars characters.  flavour: 'mixed' (everything), 'ascii'
    (English-like, few oddities: the shape of corpus.en / OWT), 'space' (whitespace-heavy)."""
    r = SplitMix64(seed * 0x100000001B3 + {"mixed": 1, "ascii": 2, "space": 3}[flavour])
    uni = flavour != "ascii"
    # a small lexicon with a Zipf-like rank distribution (rank = floor(L * u^3))
    lex = [_word(r, uni) for _ in range(400 if flavour == "ascii" else 250)]
    out: list[str] = []
    total = 0
    while total < n_chars:
        k = r.below(1000)
        if flavour == "space" and k < 300:
            piece = "".join(_SPACES_ALL[r.below(len(_SPACES_ALL))] for _ in range(1 + r.below(4)))
        elif k < 600:
            u = r.next() >> 11
            rank = (len(lex) * ((u * u >> 53) * u >> 53)) >> 53
            piece = (" " if r.below(5) else "") + lex[rank]
        elif k < 680:
            piece = " " + _word(r, uni)
        elif k < 740:
            piece = _CONTRACTIONS[r.below(len(_CONTRACTIONS) if uni else 7)]
        elif k < 800:
            d = "".join((_DIGITS if uni else _DIGITS[:6])[r.below(15 if uni else 6)]
                        for _ in range(1 + r.below(5)))
            piece = (" " if r.below(2) else "") + d
        elif k < 880:
            p = "".join((_PUNCT if uni else _PUNCT[:12])[r.below(len(_PUNCT) if uni else 12)]
                        for _ in range(1 + r.below(3)))
            piece = (" " if r.below(3) == 0 else "") + p
        elif k < 940:
            piece = ["\n", "\n\n", "  ", "   ", " \n", "\n ", "\t", " \t "][r.below(8)]
        elif k < 970:
            if uni:
                piece = _SPACES_ALL[r.below(len(_SPACES_ALL))]
                if r.below(3) == 0:
                    piece += _NOT_SPACE_SEP[r.below(4)]
            else:
                piece = ". "
        elif k < 985:
            piece = "<|endoftext|>" + ("\n" if r.below(2) else "")
        else:
            piece = "\n\n" if not uni else ["\r\n", "\r", "\n\r\n", " \r "][r.below(4)]
        out.append(piece)
        total += len(piece)
    text = "".join(out)[:n_chars]
    return text


def sha256_text(text: str) -> str:
    return hashlib.sha256(text.encode("utf-8")).hexdigest()
