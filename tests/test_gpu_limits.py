"""Documented limits fail loudly (include/bpe355.h BPE_E_LIMIT), never with wrong output.

A pre-token of 8 MiB or more cannot be keyed by the word tables (its length would reach bit 63,
the inline-word flag: ADVICE r04), so training and encoding refuse it with BPE_E_LIMIT.  The
reference has no such limit (models/tokenizer/train.py:16-28, tokenizer.py:63-90); the deviation
is listed in DESIGN.md section 7.
"""
import pytest

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")

BIG = (8 << 20) + 4096        # one run of digits: one \p{N}+ pre-token of just over 8 MiB


@pytest.fixture(scope="module", autouse=True)
def _device():
    from bpe_amd import _lib
    _lib.require_device()


def test_train_rejects_8mib_pretoken():
    data = b"a few words " + b"7" * BIG + b" and more words\n"
    with pytest.raises(RuntimeError, match="8 MiB"):
        bpe_amd.train_bpe_bytes(data, 300, ["<|endoftext|>"])


def test_encode_rejects_8mib_pretoken():
    vocab = {i: bytes([i]) for i in range(256)}
    tok = bpe_amd.Tokenizer(vocab, [], ["<|endoftext|>"])
    with pytest.raises(RuntimeError, match="8 MiB"):
        tok.encode("a few words " + "7" * BIG + " and more")
