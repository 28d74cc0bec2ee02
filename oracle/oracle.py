"""ORACLE -- TEST INFRASTRUCTURE ONLY.  ctypes wrapper over oracle/_build/liboracle.so (the
plain-C restatement of the reference BPE path, oracle/bpe_oracle.c).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
The product package (transformer-lm_amd/bpe_amd) never imports this module.

Functions mirror the reference's semantics:
  train_raw(data, vocab_size, specials)      reference models/tokenizer/train.py:142-231
  word_counts(text_bytes, specials)          reference models/tokenizer/train.py:16-28
  encode(vocab, merges, specials, text)      reference models/tokenizer/tokenizer.py:111-138
  PieceEncoder(...).encode(addr, n, starts)  reference models/tokenizer/encode.py:31-36 (each
                                             piece encoded on its own), ids as numpy uint32
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import struct
import subprocess

HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"


class _Blob(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("n", ctypes.c_size_t)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        u8p = ctypes.c_char_p
        L.oracle_train_raw.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, u8p, ctypes.c_size_t,
                                       ctypes.POINTER(_Blob), ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_train_text.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, u8p, ctypes.c_size_t,
                                        ctypes.POINTER(_Blob)]
        L.oracle_word_counts.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t,
                                         ctypes.POINTER(_Blob)]
        L.oracle_pretokenize.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(_Blob)]
        L.oracle_encode.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p,
                                    ctypes.c_size_t, ctypes.c_int, u8p, ctypes.c_size_t,
                                    ctypes.POINTER(_Blob)]
        L.oracle_encode_pieces.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, u8p,
                                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Blob)]
        L.oracle_decode_text.argtypes = [u8p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                         ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_free.argtypes = [ctypes.POINTER(_Blob)]
        L.oracle_counter_new.restype = ctypes.c_void_p
        L.oracle_counter_new.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_counter_feed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_counter_absorb.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_counter_words.argtypes = [ctypes.c_void_p, ctypes.POINTER(_Blob)]
        L.oracle_counter_train.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(_Blob)]
        L.oracle_counter_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def specials_blob(specials) -> bytes:
    parts = [struct.pack("<I", len(specials or []))]
    for s in specials or []:
        b = s.encode("utf-8")
        parts.append(struct.pack("<I", len(b)) + b)
    return b"".join(parts)


def _take(blob: _Blob) -> bytes:
    data = ctypes.string_at(blob.data, blob.n) if blob.n else b""
    lib().oracle_free(ctypes.byref(blob))
    return data


def _check(rc, what, err_pos=None):
    if rc == 0:
        return
    if rc == -2:
        raise UnicodeDecodeError("utf-8", b"", err_pos or 0, (err_pos or 0) + 1,
                                 f"invalid utf-8 ({what})")
    if rc == -3:
        raise KeyError(what)
    raise RuntimeError(f"oracle {what} failed rc={rc}")


def parse_train_blob(data: bytes):
    off = 0

    def u32():
        nonlocal off
        v = struct.unpack_from("<I", data, off)[0]
        off += 4
        return v

    def chunk():
        nonlocal off
        n = u32()
        b = data[off:off + n]
        off += n
        return b

    merges = [(chunk(), chunk()) for _ in range(u32())]
    vocab = {i: chunk() for i in range(u32())}
    return vocab, merges


def train_raw(data: bytes, vocab_size: int, specials=()):
    blob, err = _Blob(), ctypes.c_size_t(0)
    sb = specials_blob(specials)
    rc = lib().oracle_train_raw(data, len(data), vocab_size, sb, len(sb), ctypes.byref(blob),
                                ctypes.byref(err))
    _check(rc, "train", err.value)
    return parse_train_blob(_take(blob))


def train_file(path, vocab_size: int, specials=()):
    with open(path, "rb") as f:
        return train_raw(f.read(), vocab_size, specials)


def decode_text(data: bytes) -> bytes:
    out = ctypes.POINTER(ctypes.c_uint8)()
    n, err = ctypes.c_size_t(0), ctypes.c_size_t(0)
    rc = lib().oracle_decode_text(data, len(data), ctypes.byref(out), ctypes.byref(n),
                                  ctypes.byref(err))
    _check(rc, "decode", err.value)
    res = ctypes.string_at(out, n.value) if n.value else b""
    ctypes.CDLL(None).free(out)
    return res


def _parse_words(data: bytes):
    off = 4
    out = {}
    for _ in range(struct.unpack_from("<I", data, 0)[0]):
        n = struct.unpack_from("<I", data, off)[0]
        off += 4
        w = data[off:off + n]
        off += n
        out[w] = struct.unpack_from("<Q", data, off)[0]
        off += 8
    return out


def word_counts(text: bytes, specials=()):
    blob = _Blob()
    sb = specials_blob(specials)
    _check(lib().oracle_word_counts(text, len(text), sb, len(sb), ctypes.byref(blob)), "words")
    return _parse_words(_take(blob))


class Counter:
    """extract_subword_frequencies (reference train.py:16-28) over a corpus fed in pieces that
    each end at a safe split point; .train() then runs the merge loop (train.py:155-231).
    feed() releases the GIL (ctypes), so one Counter per thread counts in parallel."""

    def __init__(self, specials=()):
        sb = specials_blob(specials)
        self._h = lib().oracle_counter_new(sb, len(sb))
        if not self._h:
            raise ValueError("bad specials")

    def feed(self, addr: int, n: int):
        err = ctypes.c_size_t(0)
        _check(lib().oracle_counter_feed(self._h, ctypes.c_void_p(addr), n, ctypes.byref(err)),
               "feed", err.value)

    def absorb(self, other: "Counter"):
        _check(lib().oracle_counter_absorb(self._h, other._h), "absorb")

    def words(self):
        blob = _Blob()
        _check(lib().oracle_counter_words(self._h, ctypes.byref(blob)), "words")
        return _parse_words(_take(blob))

    def train(self, vocab_size: int):
        blob = _Blob()
        _check(lib().oracle_counter_train(self._h, vocab_size, ctypes.byref(blob)), "train")
        return parse_train_blob(_take(blob))

    def close(self):
        if self._h:
            lib().oracle_counter_free(self._h)
            self._h = None

    __del__ = close


def pretokenize(text: bytes):
    blob = _Blob()
    _check(lib().oracle_pretokenize(text, len(text), ctypes.byref(blob)), "pretokenize")
    data = _take(blob)
    return [struct.unpack_from("<QQ", data, i) for i in range(0, len(data), 16)]


def vocab_blob(vocab: dict) -> bytes:
    parts = [struct.pack("<I", len(vocab))]
    for i, b in vocab.items():
        parts.append(struct.pack("<qI", int(i), len(b)) + bytes(b))
    return b"".join(parts)


def merges_blob(merges) -> bytes:
    parts = [struct.pack("<I", len(merges))]
    for a, b in merges:
        parts.append(struct.pack("<I", len(a)) + bytes(a) + struct.pack("<I", len(b)) + bytes(b))
    return b"".join(parts)


def encode(vocab: dict, merges, specials, text: str):
    vb, mb = vocab_blob(vocab), merges_blob(merges)
    sb = specials_blob(specials)
    tb = text.encode("utf-8")
    blob = _Blob()
    rc = lib().oracle_encode(vb, len(vb), mb, len(mb), sb, len(sb), int(specials is None), tb,
                             len(tb), ctypes.byref(blob))
    _check(rc, "encode")
    data = _take(blob)
    return list(struct.unpack(f"<{len(data) // 4}I", data)) if data else []


class PieceEncoder:
    """Tokenizer(vocab, merges, specials).encode over raw memory, for corpora too large for
    Python strings: encode(addr, n, starts) encodes text[0:n) at address `addr` cut at the byte
    offsets `starts` (each piece on its own, encode.py:31-36; no starts = encode(text)) and
    returns the ids as a numpy uint32 array.  The call releases the GIL (ctypes), so one
    PieceEncoder serves several threads."""

    def __init__(self, vocab: dict, merges, specials):
        self.vb, self.mb, self.sb = vocab_blob(vocab), merges_blob(merges), specials_blob(specials)

    def encode(self, addr: int, n: int, starts=()):
        import numpy as np
        st = np.ascontiguousarray(np.asarray(starts, dtype=np.uint64))
        blob = _Blob()
        rc = lib().oracle_encode_pieces(self.vb, len(self.vb), self.mb, len(self.mb), self.sb,
                                        len(self.sb), ctypes.c_void_p(addr), n,
                                        ctypes.c_void_p(st.ctypes.data if st.size else 0), st.size,
                                        ctypes.byref(blob))
        _check(rc, "encode")
        ids = np.empty(blob.n // 4, dtype=np.uint32)
        if blob.n:
            ctypes.memmove(ids.ctypes.data, blob.data, blob.n)
        lib().oracle_free(ctypes.byref(blob))
        return ids


if os.environ.get("ORACLE_SELFTEST"):
    print(train_raw(b"abc abc", 270))
