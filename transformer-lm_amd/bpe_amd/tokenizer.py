"""Tokenizer -- drop-in for reference models/tokenizer/tokenizer.py:11-167.

Construction rules, special-token handling and the encode result follow the reference
exactly; encode() runs on the GPU through libbpe355 (segmentation on special tokens,
GPT-2 pre-tokenization, per-word rank-ordered merges, id lookup).  decode(), save() and
from_files() are host-side byte/pickle plumbing, as in the reference.
"""
from __future__ import annotations

import ctypes
import os
import pickle
from typing import Iterable, Iterator, List, Tuple

from . import _lib
from .train import train_bpe


class Tokenizer:
    def __init__(self, vocab: dict[int, bytes], merges: List[Tuple[bytes, bytes]],
                 special_tokens: List[str] | None = []):
        # tokenizer.py:18-38, including its bookkeeping quirks: vocab_inv keeps the LAST id of
        # a repeated byte string, and a missing special is appended as
        # self.vocab[bytes] = len(self.vocab) with vocab_inv[bytes] = len(self.vocab) - 1.
        self.vocab = vocab
        self.vocab_inv = {v: k for k, v in vocab.items()}
        self.merges = merges
        seen = set()
        specials = []
        for t in special_tokens or []:
            if t not in seen:
                seen.add(t)
                specials.append(t)
        # longest first; equal lengths keep first-occurrence order (the reference uses set
        # iteration order there, which only matters for the ids of equal-length missing specials)
        specials.sort(key=len, reverse=True)
        self.special_tokens = specials
        for token in self.special_tokens:
            b = token.encode("utf-8")
            if b not in self.vocab_inv:
                self.vocab[b] = len(self.vocab)
                self.vocab_inv[b] = len(self.vocab) - 1
        self._handle = None
        self._dec = None

    # ------------------------------------------------------------------ constructors
    @classmethod
    def train_from_file(cls, filepath: str, vocab_size: int, special_tokens: List[str]):
        vocab, merges = train_bpe(filepath, vocab_size, special_tokens)
        return cls(vocab, merges, special_tokens)

    @classmethod
    def fit(cls, input_path: str, vocab_size: int, special_tokens: List[str]):
        vocab, merges = train_bpe(input_path, vocab_size, special_tokens)
        return cls(vocab, merges, special_tokens)

    @classmethod
    def from_files(cls, vocab_filepath: str, merges_filepath: str,
                   special_tokens: List[str] = []) -> "Tokenizer":
        # files written by Tokenizer.save (the caller's own artifacts), as in tokenizer.py:50-61
        with open(vocab_filepath, "rb") as f:
            vocab = pickle.load(f)
        with open(merges_filepath, "rb") as f:
            merges = pickle.load(f)
        return cls(vocab, merges, special_tokens=special_tokens)

    @classmethod
    def from_gpt2_files(cls, vocab_json: str, merges_txt: str,
                        special_tokens: List[str] | None = None) -> "Tokenizer":
        """GPT-2 vocab.json / merges.txt (formats.py), as the reference's tests load them."""
        from .formats import load_gpt2
        vocab, merges = load_gpt2(vocab_json, merges_txt, special_tokens)
        return cls(vocab, merges, special_tokens)

    def save_gpt2(self, vocab_json: str, merges_txt: str) -> None:
        from .formats import save_gpt2
        save_gpt2({i: b for i, b in self.vocab.items() if isinstance(i, int)}, self.merges,
                  vocab_json, merges_txt)

    # ------------------------------------------------------------------ device handle
    def _device(self):
        if self._handle is None:
            L = _lib.lib()
            # bytes -> int entries only: after save()/from_files() a missing special added by
            # the reference quirk (self.vocab[b] = len(vocab), tokenizer.py:35-38) comes back as
            # an int -> bytes entry of vocab_inv, which the reference's encode never consults
            inv = [(i, b) for b, i in self.vocab_inv.items()
                   if isinstance(b, (bytes, bytearray)) and isinstance(i, int)]
            vb = _lib.vocab_blob(dict(inv) if len({i for i, _ in inv}) == len(inv) else {})
            if len({i for i, _ in inv}) != len(inv):
                # several byte strings share an id: pass the pairs as they are
                import struct
                vb = struct.pack("<I", len(inv)) + b"".join(
                    struct.pack("<qI", int(i), len(b)) + bytes(b) for i, b in inv)
            mb = _lib.merges_blob(self.merges)
            arr, n, _keep = _lib.c_strings(self.special_tokens)
            h = ctypes.c_void_p()
            _lib.check(L.bpe_tok_create(vb, len(vb), mb, len(mb), arr, n, ctypes.byref(h)),
                       "Tokenizer")
            self._handle = h
        return self._handle

    def __del__(self):
        h = getattr(self, "_handle", None)
        d = getattr(self, "_dec", None)
        if _lib._lib is not None:
            try:
                if h is not None:
                    _lib._lib.bpe_tok_free(h)
                if d is not None:
                    _lib._lib.bpe_dec_free(d)
            except Exception:  # noqa: BLE001
                pass

    def release_device_buffers(self) -> None:
        """Free the device memory the encoder keeps between calls (its per-call arrays and the
        bulk encoder's text and uint16 ids, about 3 bytes per input byte); the tables stay."""
        if self._handle is not None:
            _lib.check(_lib.lib().bpe_tok_release_buffers(self._handle), "release")

    # ------------------------------------------------------------------ encode / decode
    def encode(self, text: str) -> List[int]:
        """tokenizer.py:111-138 on the GPU."""
        data = text.encode("utf-8")
        h = self._device()
        cap = max(1, len(data))
        out = (ctypes.c_uint32 * cap)()
        n_out = ctypes.c_size_t(0)
        from .train import num_gpus
        g = num_gpus()
        if g == 1:
            rc = _lib.lib().bpe_tok_encode(h, data, len(data), out, cap, ctypes.byref(n_out))
        else:   # one process, several devices (bpe_amd.set_num_gpus / BPE355_GPUS)
            rc = _lib.lib().bpe_tok_encode_gpus(h, data, len(data), out, cap, ctypes.byref(n_out), g)
        _lib.check(rc, "encode")
        return list(out[: n_out.value])

    def encode_iterable(self, iterable: Iterable[str]) -> Iterator[int]:
        """tokenizer.py:140-150: concatenate items until >= 2 MiB characters, encode each chunk."""
        it = iter(iterable)
        while True:
            text = ""
            for line in it:
                text += line
                if len(text) >= 1024 * 1024 * 2:
                    break
            if not text:
                break
            yield from self.encode(text)

    def _decoder(self):
        if getattr(self, "_dec", None) is None:
            import struct
            ents = [(i, b) for i, b in self.vocab.items() if isinstance(i, int)]
            blob = struct.pack("<I", len(ents)) + b"".join(
                struct.pack("<qI", int(i), len(b)) + bytes(b) for i, b in ents)
            h = ctypes.c_void_p()
            _lib.check(_lib.lib().bpe_dec_create(blob, len(blob), ctypes.byref(h)), "decoder")
            self._dec = h
        return self._dec

    def decode(self, ids: List[int]) -> str:
        """tokenizer.py:155-157: b"".join(self.vocab[i] for i in ids) gathered on the GPU, then
        CPython's UTF-8 decoder with errors="replace" (its replacement rule, exactly)."""
        ids = list(ids)
        for i in ids:   # ids the uint32 device table cannot hold
            if not isinstance(i, int) or i < 0 or i > 0xFFFFFFFF:
                v = self.vocab[i]   # KeyError, as the reference's lookup raises
                if not isinstance(v, (bytes, bytearray)):   # b"".join of a non-bytes value
                    raise TypeError(f"sequence item: expected a bytes-like object, {type(v).__name__} found")
                raise KeyError(i)   # (a non-int key with a bytes value: not decodable here)
        if not ids:
            return ""
        arr = (ctypes.c_uint32 * len(ids))(*ids)
        L = _lib.lib()
        n_out = ctypes.c_size_t(0)
        rc = L.bpe_dec_decode(self._decoder(), arr, len(ids), None, 0, ctypes.byref(n_out))
        if rc != _lib.BPE_E_ARG or n_out.value == 0:   # size query, or KeyError / empty result
            if rc == _lib.BPE_E_KEY:
                raise KeyError(int((L.bpe_last_error() or b"0").decode()))
            _lib.check(rc, "decode")
        buf = (ctypes.c_uint8 * max(n_out.value, 1))()
        _lib.check(L.bpe_dec_decode(self._decoder(), arr, len(ids), buf, n_out.value, ctypes.byref(n_out)),
                   "decode")
        return bytes(buf[:n_out.value]).decode("utf-8", errors="replace")

    def save(self, path: str, prefix: str = ""):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, prefix + "-vocab.pkl"), "wb+") as f:
            pickle.dump(self.vocab, f)
        with open(os.path.join(path, prefix + "-merges.pkl"), "wb+") as f:
            pickle.dump(self.merges, f)
