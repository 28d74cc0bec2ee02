"""GPU: strict UTF-8 validation of the training input (k_validate) against CPython's decoder.

The reference reads the corpus in text mode (models/tokenizer/train.py:22), so ill-formed UTF-8
raises UnicodeDecodeError at the first bad byte.  The kernel checks 16-byte units, one per lane,
with the bytes around a unit taken from the neighbouring lanes; these cases put bad sequences at
unit and wave (1 KiB) boundaries, at the start and at the end of the text.
"""
import random

import pytest

import golden_cases as G

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")

VALID = ["a", "é", "ж", "中", "€", "😀", " ", "\n", "Ω", "ß", "ࠀ", "\U00010000", "\U0010FFFF", "퟿", ""]
BAD = [b"\x80", b"\xbf", b"\xc0\xaf", b"\xc1\x81", b"\xe0\x80\x80", b"\xe0\x9f\xbf", b"\xed\xa0\x80",
       b"\xf0\x80\x80\x80", b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xff", b"\xc3", b"\xe2\x82",
       b"\xf0\x9f\x98", b"\xe2\x28\xa1", b"\xc3\x28"]


@pytest.fixture(scope="module", autouse=True)
def _device():
    from bpe_amd import _lib
    _lib.require_device()


def _text(rng, n):
    out = bytearray()
    while len(out) < n:
        out += rng.choice(VALID).encode("utf-8")
    return bytes(out)


def _gpu_error_pos(data):
    try:
        bpe_amd.train_bpe_bytes(data, 257, [])
    except UnicodeDecodeError as e:
        return e.start
    return None


def _cpu_error_pos(data):
    try:
        data.decode("utf-8")
    except UnicodeDecodeError as e:
        return e.start
    return None


def test_valid_mixed_text_passes():
    rng = random.Random(1)
    for n in (15, 16, 17, 1023, 1024, 1025, 4096 + 7):
        data = _text(rng, n)
        assert _gpu_error_pos(data) is None


@pytest.mark.parametrize("seed", range(6))
def test_first_bad_byte_matches_cpython(seed):
    rng = random.Random(100 + seed)
    for _ in range(12):
        n = rng.choice([40, 300, 2048, 5000])
        data = bytearray(_text(rng, n))
        # one or two bad sequences, often right at a 16-byte or 1 KiB boundary
        for _ in range(rng.choice([1, 1, 2])):
            anchor = rng.choice([16, 1024])
            p = min(len(data), max(0, rng.randrange(0, len(data) + 1) // anchor * anchor + rng.choice([-3, -2, -1, 0, 1, 2])))
            data[p:p] = rng.choice(BAD)
        data = bytes(data)
        assert _gpu_error_pos(data) == _cpu_error_pos(data)


def test_bad_sequence_at_start_and_end():
    rng = random.Random(7)
    body = _text(rng, 3000)
    for bad in BAD:
        for data in (bad + body, body + bad, body[:1024] + bad + body[1024:]):
            assert _gpu_error_pos(data) == _cpu_error_pos(data), (bad, len(data))


def test_crlf_text_with_multibyte_characters():
    rng = random.Random(9)
    data = (_text(rng, 2000).decode() + "\r\n" + _text(rng, 2000).decode() + "\r").encode()
    vocab, merges = bpe_amd.train_bpe_bytes(data, 270, [])
    assert b"\r" not in b"".join(a + b for a, b in merges)


# ------------------------------------------------------------------ A1 on its own
def _device_word_counts(data: bytes, specials):
    import ctypes
    import struct
    from bpe_amd import _lib
    L = _lib.lib()
    arr, k, _keep = _lib.c_strings(specials)
    p, n = ctypes.c_void_p(), ctypes.c_size_t(0)
    _lib.check(L.bpe_word_counts(data, len(data), arr, k, ctypes.byref(p), ctypes.byref(n)), "words")
    try:
        blob = ctypes.string_at(p, n.value) if n.value else b""
    finally:
        L.bpe_blob_free(p)
    out, off = {}, 0
    while off < len(blob):
        ln = struct.unpack_from("<I", blob, off)[0]
        w = blob[off + 4:off + 4 + ln]
        out[w] = struct.unpack_from("<Q", blob, off + 4 + ln)[0]
        off += 12 + ln
    return out


@pytest.mark.parametrize("name", G.names("words"))
def test_device_word_counts_match_reference(name):
    """the device pre-tokenizer + counter (k_validate, k_newline_map, k_count_words) against
    the reference's extract_subword_frequencies table (train.py:16-28): every multi-byte word"""
    o = G.load("words", name)
    want = {bytes.fromhex(h): c for h, c in o["words"]}
    want = {w: c for w, c in want.items() if len(w) > 1}
    got = _device_word_counts(G.input_bytes(o["input"]), o["special_tokens"])
    assert got == want
