"""Chunk-boundary stress for the device pre-tokenizer (text.hip k_count_words).

The counter streams the corpus in 16 KiB chunks staged in LDS (+1 KiB halo); each of a
workgroup's 256 threads owns a 64-byte span that it extends to safe points.  These corpora put
every awkward case ON a chunk boundary -- an exact safe point, whitespace runs across it,
multi-byte characters straddling it, letter runs longer than the halo (the global-memory slow
path), no safe point for several chunks -- and mix in the word-length edges of the inline word
keys (7/8, 14/15, 16/17 bytes) and NUL bytes.  The device's pre-token count must equal the
oracle's, and training on it must give the oracle's merges.
"""
import random

import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

CH = 16384
WORDS = [b"the", b"of", b"and", b"a", b"government", b"internation", b"alization", b"x" * 7,
         b"y" * 8, b"z" * 14, b"w" * 15, b"v" * 16, b"u" * 17, b"q" * 40, b"\x00\x00ab",
         b"\x00" * 9, "été".encode(), "naïve".encode(), b"12345", b"2026",
         b"!!", b"...", b"'s", b"'ll", b"don't", b"\xe2\x80\x94"]
SEPS = [b" ", b" ", b" ", b" ", b"  ", b"\n", b"\n\n", b", ", b". ", b"\t", b" \n "]


def _base(rng, n):
    out = bytearray()
    while len(out) < n:
        out += rng.choice(WORDS) + rng.choice(SEPS)
    return out


def _boundary_text(seed, n_chunks=48):
    rng = random.Random(seed)
    parts = bytearray()
    for k in range(n_chunks):
        body = _base(rng, CH)
        # make the piece end exactly at the boundary, then place a pattern across it
        parts += body[:CH - len(parts) % CH] if len(parts) % CH else body[:CH]
        case = k % 8
        if case == 0:      # exact safe point at the boundary
            parts[-1:] = b"a"
            parts += b" b"
        elif case == 1:    # whitespace run across the boundary
            parts[-3:] = b"a  "
            parts += b" \n  x"
        elif case == 2:    # 2-byte character straddling it
            parts[-1:] = "é".encode()[:1]
            parts += "é".encode()[1:] + b"tude "
        elif case == 3:    # letter run longer than the halo across it (slow path)
            parts[-700:] = b"L" * 700
            parts += b"L" * 1500 + b" "
        elif case == 4:    # no safe point for more than a chunk (newline-separated letters)
            parts += (b"word\n" * 4000)
        elif case == 5:    # 3-byte punctuation straddling it
            parts[-2:] = b"a" + "—".encode()[:1]
            parts += "—".encode()[1:] + b"b "
        elif case == 6:    # digits and a contraction at the boundary
            parts[-2:] = b"12"
            parts += b"34's "
        else:              # long word (> 16 bytes) ending on the boundary
            parts[-20:] = b" " + b"k" * 19
            parts += b" m "
    return bytes(parts).decode("utf-8", errors="replace").encode("utf-8")


def _oracle_pretokens(data: bytes) -> int:
    # train_bpe reads text mode: universal newlines first (train.py:22), then pre-tokenizes
    text = oracle.decode_text(data)
    return sum(c for w, c in oracle.word_counts(text, []).items() if len(w) >= 2)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_chunk_boundaries_train(seed):
    from bpe_amd import train_bpe_bytes
    from bpe_amd.train import last_train_stats
    data = _boundary_text(seed)
    assert len(data) > 40 * CH
    vocab, merges = train_bpe_bytes(data, 900, [])
    assert last_train_stats()["n_pretokens"] == _oracle_pretokens(data)
    want_vocab, want_merges = oracle.train_raw(data, 900, [])
    assert merges == want_merges
    assert vocab == want_vocab


# Few workgroups (BPE355_STREAM_WG): each streams ~90 chunks through its LDS word cache,
# across many eviction epochs -- the regime of full-size corpora, at test size.
@pytest.mark.parametrize("wg", [1, 3])
def test_streaming_workgroups_train(monkeypatch, wg):
    import synth_text
    from bpe_amd import train_bpe_bytes
    from bpe_amd.train import last_train_stats
    monkeypatch.setenv("BPE355_STREAM_WG", str(wg))
    data = synth_text.generate(41, 3_000_000, "mixed").encode("utf-8")
    vocab, merges = train_bpe_bytes(data, 2000, ["<|endoftext|>"])
    assert last_train_stats()["n_pretokens"] == _oracle_pretokens(data)
    want_vocab, want_merges = oracle.train_raw(data, 2000, ["<|endoftext|>"])
    assert merges == want_merges
    assert vocab == want_vocab


@pytest.mark.parametrize("wg", [1, 3])
def test_streaming_workgroups_encode(monkeypatch, wg):
    import gpt2_files
    import synth_text
    import bpe_amd
    monkeypatch.setenv("BPE355_STREAM_WG", str(wg))
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    text = synth_text.generate(42, 2_500_000, "mixed") + _boundary_text(4).decode("utf-8")
    tok = bpe_amd.Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    assert tok.encode(text) == oracle.encode(vocab, merges, ["<|endoftext|>"], text)
