"""GPU parity: Tokenizer.encode (HIP) against the reference's encode goldens and the oracle."""
import pytest

import golden_cases as G
import gpt2_files
from oracle import oracle

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")


@pytest.fixture(scope="module", autouse=True)
def _device():
    from bpe_amd import _lib
    _lib.require_device()


@pytest.mark.parametrize("name", G.names("encode"))
def test_encode_matches_reference_golden(name):
    o = G.load("encode", name)
    vocab, merges = G.tokenizer_inputs(o)
    tok = bpe_amd.Tokenizer(dict(vocab), list(merges), o["special_tokens"])
    text = G.encode_text(o)
    ids = tok.encode(text)
    assert ids == o["ids"]
    assert tok.decode(ids) == text.encode("utf-8").decode("utf-8", "replace")


def test_encode_roundtrip_and_iterable():
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = bpe_amd.Tokenizer(vocab, merges, ["<|endoftext|>"])
    with open(gpt2_files.FIXTURES / "tinystories_sample.txt", encoding="utf-8") as f:
        ids_iter = list(tok.encode_iterable(f))
    text = (gpt2_files.FIXTURES / "tinystories_sample.txt").read_text(encoding="utf-8")
    assert ids_iter == tok.encode(text)
    assert tok.decode(ids_iter) == text


@pytest.mark.parametrize("seed,n_chars,flavour", [(21, 2_000_000, "mixed"), (22, 1_000_000, "space")])
def test_encode_matches_oracle_synthetic(seed, n_chars, flavour):
    import synth_text
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    text = synth_text.generate(seed, n_chars, flavour)
    tok = bpe_amd.Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    assert tok.encode(text) == oracle.encode(vocab, merges, ["<|endoftext|>"], text)


def test_encode_bench_corpus_sample_vs_oracle():
    """48 MB of bench.py's own synthetic corpus (every workgroup streams several chunks through
    eviction epochs), merges trained on the device, encode checked against the oracle."""
    import ctypes
    import torch
    from bpe_amd import _lib, train_bpe_device
    L = _lib.lib()
    n = 48 * (1 << 20)
    corpus = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(L.bpe_synth_corpus_device(ctypes.c_void_p(corpus.data_ptr()), n, 7, 0, 0, None), "synth")
    torch.cuda.synchronize()
    vocab, merges = train_bpe_device(corpus.data_ptr(), n, 4000, ["<|endoftext|>"])
    text = corpus.cpu().numpy().tobytes().decode("utf-8")
    tok = bpe_amd.Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    got = tok.encode(text)
    want = oracle.encode(vocab, merges, ["<|endoftext|>"], text)
    assert len(got) == len(want)
    assert got == want


def test_missing_special_after_save_and_from_files(tmp_path):
    """A special missing from the vocab is added by the reference's quirk (tokenizer.py:35-38:
    self.vocab[bytes] = len(self.vocab)); after save() / from_files() that entry comes back keyed
    by bytes (so vocab_inv also holds id -> bytes), the quirk runs again and the special keeps its
    id.  Encode must not trip over the inverted entry and must use that id."""
    import bpe_amd
    vocab, merges = bpe_amd.train_bpe(gpt2_files.FIXTURES / "corpus.en", 300, [])
    sp = "<|x|>"
    v = len(vocab)   # the id the missing special gets
    tok = bpe_amd.Tokenizer(vocab, merges, [sp])
    text = "the cat<|x|>sat on the mat<|x|>"
    ids1 = tok.encode(text)
    assert ids1.count(v) == 2
    tok.save(str(tmp_path), "t")
    tok2 = bpe_amd.Tokenizer.from_files(str(tmp_path / "t-vocab.pkl"), str(tmp_path / "t-merges.pkl"), [sp])
    assert tok2.vocab_inv[sp.encode()] == v and tok2.vocab_inv[v] == sp.encode()
    assert tok2.encode(text) == ids1


@pytest.mark.parametrize("ranks", [2, 3, 5])
def test_encode_several_devices_equals_one(ranks, monkeypatch):
    """bpe_tok_encode_gpus: the text cut at safe points no special spans, one device per piece,
    ids concatenated -- equal to the single-device encode and to the oracle.  A special with
    spaces inside ("<|end of doc|>") puts safe points inside its occurrences, which the cuts must
    avoid.  The ranks share this box's one GPU (BPE355_INPROC_RANKS)."""
    import bpe_amd
    import synth_text
    monkeypatch.setenv("BPE355_INPROC_RANKS", "1")
    specials = ["<|endoftext|>", "<|end of doc|>"]
    vocab, merges = bpe_amd.train_bpe(gpt2_files.FIXTURES / "corpus.en", 600, specials)
    parts = []
    for i in range(40):
        parts.append(synth_text.generate(90 + i, 3000, "mixed" if i % 2 else "ascii"))
        parts.append(specials[i % 2])
    text = "".join(parts)
    tok = bpe_amd.Tokenizer(vocab, merges, specials)
    one = tok.encode(text)
    try:
        bpe_amd.set_num_gpus(ranks)
        many = tok.encode(text)
    finally:
        bpe_amd.set_num_gpus(None)
    assert many == one
    assert one == oracle.encode(vocab, merges, specials, text)


@pytest.mark.parametrize("knobs", [
    {"BPE355_ENC_PEND_CAP": "0"},                                # no pending pool: the scan resolves words
    {"BPE355_ENC_PEND_CAP": "40000", "BPE355_STREAM_WG": "2"},   # the pool runs out part way
    {"BPE355_NOCACHE": "1"},                                     # no LDS cache: every word pending
    {"BPE355_ENC_REC_CAP": "1000"},                              # too few records: the retry
    {"BPE355_ENC_RESOLVE_CACHE": "0"},                           # the resolve without its LDS cache
    {"BPE355_ENC_FINALIZE": "0"},                                # the emit reads resolved records
    {"BPE355_ENC_FINALIZE": "2"},                                # the count pass stores the infos
])
def test_encode_resolution_paths(monkeypatch, knobs):
    """the encoder's record paths against the oracle: pending entries resolved by k_enc_resolve,
    words resolved in the scan itself, no LDS cache, the record buffer's retry -- with the
    dictionary (GPT-2 vocab entries), one-byte words and specials all present"""
    import synth_text
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    text = synth_text.generate(23, 1_500_000, "mixed") + "<|endoftext|>" + synth_text.generate(24, 300_000, "space")
    tok = bpe_amd.Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    assert tok.encode(text) == oracle.encode(vocab, merges, ["<|endoftext|>"], text)


def test_encode_special_in_vocab_and_dictionary_edge_words():
    """words the dictionary must leave out or treat specially: a vocab entry equal to a special
    (0 ids when met as a pre-token is impossible -- re.split takes it -- but the dictionary still
    holds it), merges whose product is missing from the vocab (KeyError, as vocab_inv[...] raises),
    one-byte specials, and several-id dictionary words"""
    vocab = {i: bytes([i]) for i in range(256)}
    merges = [(b" ", b"a"), (b" a", b"b"), (b"c", b"d"), (b"x", b"y")]
    for a, b in merges[:3]:
        vocab[len(vocab)] = a + b
    vocab[len(vocab)] = b"<s>"
    tok = bpe_amd.Tokenizer(dict(vocab), list(merges), ["<s>", "q"])
    text = " ab cd <s> abq cdcd  ab x"
    assert tok.encode(text) == oracle.encode(vocab, merges, ["<s>", "q"], text)
    with pytest.raises(KeyError):
        tok.encode(" xy")   # (x, y) merges to b"xy", which has no id
