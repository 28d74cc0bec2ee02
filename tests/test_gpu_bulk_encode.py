"""Bulk encode output: the reference's dataset encoder
models/tokenizer/encode.py:31-38 and the np.memmap consumer of train.py:230-232.

The device path (bpe_amd.encode) must write exactly the ids the reference's loop produces:
text-mode read (universal newlines), 1 M-character pieces (smaller here), each piece encoded on
its own, concatenated, as np.uint16 -- checked against the oracle encoding each piece.
"""
import ctypes
import random

import numpy as np
import pytest

import gpt2_files
from oracle import oracle

pytestmark = pytest.mark.gpu


def _pieces(text: str, k: int):
    return [text[i:i + k] for i in range(0, len(text), k)]


def _mixed_text(seed: int, n_words: int) -> str:
    rng = random.Random(seed)
    words = ["the", " cat", "été", " naïve", "<|endoftext|>", "\n", "\r\n", "  ", "12", "'s", "!!",
             " 東京", "—", " x" * 3, "\t", "ab<|end", "oftext|>cd"]
    return "".join(rng.choice(words) for _ in range(n_words))


def _device(t):
    return ctypes.c_void_p(t.data_ptr())


def test_chunk_starts_are_character_offsets():
    import torch
    from bpe_amd import _lib
    L = _lib.lib()
    text = _mixed_text(1, 3000)
    data = text.encode("utf-8")
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    for k in (1, 7, 100, 4096):
        ns = ctypes.c_size_t(0)
        _lib.check(L.bpe_utf8_chunk_starts_device(_device(d), len(data), k, None, 0, ctypes.byref(ns), None))
        starts = (ctypes.c_uint64 * max(ns.value, 1))()
        _lib.check(L.bpe_utf8_chunk_starts_device(_device(d), len(data), k, starts, ns.value,
                                                  ctypes.byref(ns), None))
        want = [len(text[:i].encode("utf-8")) for i in range(0, len(text), k)]
        assert list(starts[:ns.value]) == want


def test_text_prepare_is_text_mode_read(tmp_path):
    import torch
    from bpe_amd import _lib
    L = _lib.lib()
    raw = "a\r\nb\rc\n\r\r\nd é\r".encode("utf-8")
    p = tmp_path / "t.txt"
    p.write_bytes(raw)
    with open(p, "r", encoding="utf-8") as f:
        want = f.read().encode("utf-8")
    d = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to("cuda")
    m = ctypes.c_size_t(0)
    _lib.check(L.bpe_text_prepare_device(_device(d), len(raw), _device(d), ctypes.byref(m), None))
    assert bytes(d[:m.value].cpu().numpy()) == want
    bad = torch.tensor([0x61, 0xC3, 0x28], dtype=torch.uint8, device="cuda")
    with pytest.raises(UnicodeDecodeError):
        _lib.check(L.bpe_text_prepare_device(_device(bad), 3, _device(bad), ctypes.byref(m), None))


# (the oracle re-serializes the 50k-entry vocab per call: small pieces only on a short text)
@pytest.mark.parametrize("k,n_words", [(1, 60), (7, 400), (50, 4000), (997, 4000), (100_000, 4000)])
def test_encode_chunks_equals_separate_encodes(k, n_words):
    from bpe_amd import Tokenizer, _lib
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = _mixed_text(2, n_words).replace("\r", "")
    pieces = _pieces(text, k)
    want = []
    for piece in pieces:   # specials straddling a piece boundary are NOT matched
        want += oracle.encode(vocab, merges, ["<|endoftext|>"], piece)
    data = text.encode("utf-8")
    starts = []
    off = 0
    for piece in pieces:
        starts.append(off)
        off += len(piece.encode("utf-8"))
    arr = (ctypes.c_uint64 * max(len(starts), 1))(*starts)
    out = (ctypes.c_uint32 * max(len(data), 1))()
    n_out = ctypes.c_size_t(0)
    _lib.check(_lib.lib().bpe_tok_encode_chunks(tok._device(), data, len(data), arr, len(starts), out,
                                                len(data), ctypes.byref(n_out)))
    assert list(out[:n_out.value]) == want


@pytest.mark.parametrize("k", [2, 3, 5, 11])
def test_prefix_special_fits_when_longest_straddles_a_cut(k):
    """Specials '<|a' and '<|a|>': where a piece cut falls inside '<|a|>', the reference's
    re.split on that piece still matches '<|a' (tokenizer.py:63-66)."""
    from bpe_amd import Tokenizer, _lib
    specials = ["<|a", "<|a|>"]
    vocab, merges = gpt2_files.load_gpt2(specials)
    tok = Tokenizer(dict(vocab), list(merges), specials)
    rng = random.Random(k)
    text = "".join(rng.choice(["<|a|>", "<|a", "|>", " b", "x<|a|>y", "<|", "a|>"]) for _ in range(300))
    pieces = _pieces(text, k)
    want = []
    for piece in pieces:
        want += oracle.encode(vocab, merges, specials, piece)
    data = text.encode("utf-8")
    starts = [0]
    for piece in pieces[:-1]:
        starts.append(starts[-1] + len(piece.encode("utf-8")))
    arr = (ctypes.c_uint64 * len(starts))(*starts)
    out = (ctypes.c_uint32 * len(data))()
    n_out = ctypes.c_size_t(0)
    _lib.check(_lib.lib().bpe_tok_encode_chunks(tok._device(), data, len(data), arr, len(starts), out,
                                                len(data), ctypes.byref(n_out)))
    assert list(out[:n_out.value]) == want


@pytest.mark.parametrize("fmt", ["pt", "bin"])
def test_encode_file_matches_reference_loop(tmp_path, fmt):
    import torch
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = _mixed_text(3, 20000)
    src = tmp_path / "split.txt"
    src.write_bytes(text.encode("utf-8"))
    k = 3000
    with open(src, "r", encoding="utf-8") as f:   # encode.py:31-36, pieces of k characters
        want = []
        while True:
            piece = f.read(k)
            if not piece:
                break
            want += oracle.encode(vocab, merges, ["<|endoftext|>"], piece)
    out = tmp_path / f"tokens.{fmt}"
    got = encode_file(tok, src, out, fmt=fmt, chars_per_piece=k)
    assert got.dtype == np.uint16 and got.tolist() == want
    if fmt == "pt":
        loaded = torch.load(out, weights_only=False)   # this test's own file
        assert isinstance(loaded, np.ndarray) and loaded.dtype == np.uint16
    else:
        loaded = np.memmap(out, dtype=np.uint16, mode="r")   # train.py:230-232
    assert loaded.tolist() == want


def test_ids_above_uint16_are_refused():
    import torch
    from bpe_amd import _lib
    ids = torch.tensor([1, 65535, 65536], dtype=torch.int32, device="cuda")
    out = torch.empty(3, dtype=torch.int16, device="cuda")
    with pytest.raises(RuntimeError, match="uint16"):
        _lib.check(_lib.lib().bpe_ids_to_u16_device(_device(ids), 3, _device(out), None))
    _lib.check(_lib.lib().bpe_ids_to_u16_device(_device(ids), 2, _device(out), None))
    assert out[:2].cpu().numpy().view(np.uint16).tolist() == [1, 65535]


def test_read_file_device_bytes(tmp_path):
    """the library's file reader (pinned staging, several pread threads, 16 MB chunks): exact
    bytes at sizes around the chunk size, and the reference's exceptions for bad paths"""
    import os
    from bpe_amd.encode import read_file_device
    rng = np.random.default_rng(5)
    for size in (0, 1, (16 << 20) - 1, (16 << 20) + 1, 3 * (16 << 20) + 12345):
        p = tmp_path / f"f{size}.bin"
        data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        p.write_bytes(data)
        raw = read_file_device(p)
        assert raw is not None and raw.numel() == size
        assert bytes(raw.cpu().numpy()) == data
    with pytest.raises(FileNotFoundError):
        read_file_device(tmp_path / "missing.txt")
    assert read_file_device(tmp_path) is None   # not a regular file: encode_file reads it itself
    from bpe_amd import _lib
    n = ctypes.c_size_t(0)
    rc = _lib.lib().bpe_read_file_device(os.fsencode(str(tmp_path)), None, 0, ctypes.byref(n))
    assert rc != 0


def test_encode_file_from_fifo_and_directory(tmp_path):
    """a FIFO goes through the host read (as the reference's open().read()); a directory raises
    IsADirectoryError like open() does"""
    import os
    import threading
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = _mixed_text(4, 3000)
    src = tmp_path / "reg.txt"
    src.write_bytes(text.encode("utf-8"))
    want = encode_file(tok, src, chars_per_piece=500)
    fifo = tmp_path / "pipe"
    os.mkfifo(fifo)
    w = threading.Thread(target=lambda: fifo.write_bytes(text.encode("utf-8")))
    w.start()
    got = encode_file(tok, fifo, chars_per_piece=500)
    w.join()
    assert got.tolist() == want.tolist()
    with pytest.raises(IsADirectoryError):
        encode_file(tok, tmp_path)


def test_copy_to_host_bytes():
    """device -> pageable host through the pinned copier threads, sizes around the 16 MB chunk"""
    import torch
    from bpe_amd import _lib
    L = _lib.lib()
    for size in (1, 4097, (16 << 20) + 3, 2 * (16 << 20) + 77):
        src = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda")
        dst = np.zeros(size, dtype=np.uint8)
        _lib.check(L.bpe_copy_to_host(_device(src), size, dst.ctypes.data))
        assert np.array_equal(dst, src.cpu().numpy())


def test_encode_file_refuses_ids_above_uint16(tmp_path):
    """the native bulk path writes np.uint16 on the device: an id past 65535 (here a special
    token's) fails loudly instead of wrapping (encode.py:37 would wrap it silently)"""
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file
    vocab = {i: bytes([i]) for i in range(256)}
    vocab[70000] = b"<|big|>"
    tok = Tokenizer(vocab, [], ["<|big|>"])
    src = tmp_path / "s.txt"
    src.write_bytes(b"ab <|big|> cd")
    with pytest.raises(RuntimeError, match="uint16"):
        encode_file(tok, src)
    src.write_bytes(b"ab cd ef")   # the same handle again, with every id in range
    assert encode_file(tok, src).tolist() == [97, 98, 32, 99, 100, 32, 101, 102]


def _piece_starts(text: str, k: int):
    starts, off = [], 0
    for piece in _pieces(text, k):
        starts.append(off)
        off += len(piece.encode("utf-8"))
    return starts


def _encode_chunks(tok, data: bytes, starts):
    from bpe_amd import _lib
    arr = (ctypes.c_uint64 * max(len(starts), 1))(*starts)
    out = (ctypes.c_uint32 * max(len(data), 1))()
    n_out = ctypes.c_size_t(0)
    _lib.check(_lib.lib().bpe_tok_encode_chunks(tok._device(), data, len(data), arr, len(starts), out,
                                                len(data), ctypes.byref(n_out)))
    return list(out[:n_out.value])


@pytest.mark.parametrize("slab,region,k", [(65536, 100_000, 997), (65536, 1, 4096), (131072, 10 ** 9, 7),
                                           (65536, 50_000, 10 ** 7)])
def test_encode_file_overlapped_regions(tmp_path, monkeypatch, slab, region, k):
    """the overlapped bulk path (file streamed in slabs, pieces validated, counted, encoded and
    copied region by region) against one encode of the whole text cut at the same piece starts
    (bpe_tok_encode_chunks, itself checked against the oracle above): small slabs and regions
    put many region ends, slab ends and piece starts next to each other; a piece longer than a
    region (k = 10^7) is encoded whole"""
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file, last_phases_ms
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = _mixed_text(11, 60000).replace("\r", "")
    data = text.encode("utf-8")
    assert len(data) > 2 * slab
    src = tmp_path / "t.txt"
    src.write_bytes(data)
    want = _encode_chunks(tok, data, _piece_starts(text, k))
    monkeypatch.setenv("BPE355_READ_SLAB", str(slab))
    monkeypatch.setenv("BPE355_ENC_REGION", str(region))
    got = encode_file(tok, src, chars_per_piece=k)
    assert got.dtype == np.uint16 and got.tolist() == want
    assert set(last_phases_ms) == {"read", "decode", "encode", "copy"}


@pytest.mark.parametrize("knobs", [{"BPE355_D2H_WG": "7"}, {"BPE355_ENC_LAST_REGION": "30000"},
                                   {"BPE355_D2H_WG": "64", "BPE355_ENC_LAST_REGION": "1"}])
def test_encode_file_copy_kernel_and_last_region(tmp_path, monkeypatch, knobs):
    """the ids copied out by the workgroup copy kernel (BPE355_D2H_WG, instead of HIP's copy) and
    a short last region once the whole file is in (BPE355_ENC_LAST_REGION): the same ids"""
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = _mixed_text(12, 60000).replace("\r", "")
    data = text.encode("utf-8")
    src = tmp_path / "t.txt"
    src.write_bytes(data)
    want = _encode_chunks(tok, data, _piece_starts(text, 997))
    monkeypatch.setenv("BPE355_READ_SLAB", "65536")
    monkeypatch.setenv("BPE355_ENC_REGION", "100000")
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    got = encode_file(tok, src, chars_per_piece=997)
    assert got.dtype == np.uint16 and got.tolist() == want


def test_encode_file_late_carriage_return_and_bad_utf8(tmp_path, monkeypatch):
    """a carriage return first seen after regions were already encoded: the whole text is redone
    with universal newlines; an ill-formed byte late in the file raises UnicodeDecodeError at its
    position, as decoding the whole file does"""
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    monkeypatch.setenv("BPE355_READ_SLAB", "65536")
    monkeypatch.setenv("BPE355_ENC_REGION", "30000")
    head = _mixed_text(12, 40000).replace("\r", "")
    raw = (head + "tail\r\nmore\rend é").encode("utf-8")
    src = tmp_path / "cr.txt"
    src.write_bytes(raw)
    with open(src, "r", encoding="utf-8") as f:
        text = f.read()
    k = 1500
    want = _encode_chunks(tok, text.encode("utf-8"), _piece_starts(text, k))
    assert encode_file(tok, src, chars_per_piece=k).tolist() == want
    bad = bytearray(head.encode("utf-8"))
    pos = len(bad) - 1000
    while bad[pos] >= 0x80:   # an ASCII byte, replaced by a lone continuation byte
        pos += 1
    bad[pos] = 0x80
    src.write_bytes(bytes(bad))
    with pytest.raises(UnicodeDecodeError) as e:
        encode_file(tok, src, chars_per_piece=k)
    assert e.value.start == pos


@pytest.mark.parametrize("with_cr", [False, True])
def test_encode_file_read_error_raises(tmp_path, monkeypatch, with_cr):
    """a read that fails part way (EIO, a file truncated while read; injected by a test knob)
    raises OSError and leaves no thread behind -- also on the carriage-return path, where the
    text is redone in one pass once read (that path used to end in std::terminate)"""
    from bpe_amd import Tokenizer
    from bpe_amd.encode import encode_file
    vocab, merges = gpt2_files.load_gpt2(["<|endoftext|>"])
    tok = Tokenizer(dict(vocab), list(merges), ["<|endoftext|>"])
    text = _mixed_text(13, 60000).replace("\r", "")
    if with_cr:
        text = "first line\r\n" + text
    src = tmp_path / "t.txt"
    src.write_bytes(text.encode("utf-8"))
    monkeypatch.setenv("BPE355_READ_SLAB", "65536")
    monkeypatch.setenv("BPE355_ENC_REGION", "30000")
    monkeypatch.setenv("BPE355_TEST_READ_FAIL_AT", "150000")
    assert src.stat().st_size > 200000
    with pytest.raises(OSError):
        encode_file(tok, src, chars_per_piece=4096)
    monkeypatch.delenv("BPE355_TEST_READ_FAIL_AT")
    # the tokenizer still works, with its buffers kept or released
    with open(src, "r", encoding="utf-8") as f:
        whole = f.read()
    want = _encode_chunks(tok, whole.encode("utf-8"), _piece_starts(whole, 4096))
    assert encode_file(tok, src, chars_per_piece=4096, keep_device_buffers=True).tolist() == want
    tok.release_device_buffers()
    assert encode_file(tok, src, chars_per_piece=4096).tolist() == want
