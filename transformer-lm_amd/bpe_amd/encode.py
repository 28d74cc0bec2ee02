"""Dataset encoder -- drop-in for reference models/tokenizer/encode.py (and the memmap input of
train.py:230-232).

The reference reads the split in text mode 1 M characters at a time, encodes every piece with
Tokenizer.encode_iterable([piece]) and saves np.array(ids, dtype=np.uint16) with
torch.save(..., pickle_protocol=4).  Here the whole file goes to the device once:

    bytes -> bpe_text_prepare_device    (strict UTF-8 + universal newlines: the text-mode read)
          -> bpe_utf8_chunk_starts_device (where each 1 M-character piece starts)
          -> bpe_tok_encode_chunks_device (one launch sequence for all pieces; a piece boundary
                                          ends every pre-token and no special straddles it, so
                                          the ids equal the per-piece encodes, concatenated)
          -> bpe_ids_to_u16_device        (np.uint16, refusing ids > 65535 instead of wrapping)

and the uint16 ids come back to the host once.  Output formats: "pt" (the reference's file,
torch.save of the np.uint16 array) and "bin" (raw uint16, what train.py's np.memmap reads).

(The reference's loop passes a one-element LIST to encode_iterable, which re-iterates it
forever -- tokenizer.py:140-150; DESIGN.md section 7.  The ids written here are the ones the
loop would produce if it terminated.)
"""
from __future__ import annotations

import argparse
import ctypes
import os
import stat

import numpy as np

from . import _lib
from .tokenizer import Tokenizer

fname = {   # encode.py:8-15
    "tiny/train": "TinyStoriesV2-GPT4-train.txt",
    "tiny/valid": "TinyStoriesV2-GPT4-valid.txt",
    "owt/train": "owt_train.txt",
    "owt/valid": "owt_valid.txt",
    "corpus/train": "corpus.en",
    "corpus/valid": "corpus.en",
}

CHARS_PER_PIECE = 1024 * 1024   # encode.py:33 f.read(1024 * 1024)


def encode_device_u16(tokenizer: Tokenizer, raw, chars_per_piece: int = CHARS_PER_PIECE) -> np.ndarray:
    """The reference's encode.py ids for the raw file bytes held in the device tensor `raw`
    (uint8; overwritten by the text-mode read), as np.uint16 in host memory."""
    import torch
    L = _lib.lib()
    n = raw.numel()
    if n == 0:
        return np.zeros(0, dtype=np.uint16)
    m = ctypes.c_size_t(0)
    _lib.check(L.bpe_text_prepare_device(ctypes.c_void_p(raw.data_ptr()), n, ctypes.c_void_p(raw.data_ptr()),
                                         ctypes.byref(m), None), "read")
    m = m.value
    ns = ctypes.c_size_t(0)
    _lib.check(L.bpe_utf8_chunk_starts_device(ctypes.c_void_p(raw.data_ptr()), m, chars_per_piece, None, 0,
                                              ctypes.byref(ns), None), "chunk starts")
    starts = (ctypes.c_uint64 * max(ns.value, 1))()
    _lib.check(L.bpe_utf8_chunk_starts_device(ctypes.c_void_p(raw.data_ptr()), m, chars_per_piece, starts,
                                              ns.value, ctypes.byref(ns), None), "chunk starts")
    ids = torch.empty(max(m, 1), dtype=torch.int32, device="cuda")
    n_ids = ctypes.c_size_t(0)
    _lib.check(L.bpe_tok_encode_chunks_device(tokenizer._device(), ctypes.c_void_p(raw.data_ptr()), m, starts,
                                              ns.value, ctypes.c_void_p(ids.data_ptr()), ctypes.byref(n_ids),
                                              None), "encode")
    k = n_ids.value
    out16 = torch.empty(max(k, 1), dtype=torch.int16, device="cuda")
    _lib.check(L.bpe_ids_to_u16_device(ctypes.c_void_p(ids.data_ptr()), k, ctypes.c_void_p(out16.data_ptr()),
                                       None), "uint16 ids")
    del ids
    host = np.empty(k, dtype=np.uint16)
    if k:
        _lib.check(L.bpe_copy_to_host(ctypes.c_void_p(out16.data_ptr()), 2 * k, host.ctypes.data), "copy")
    return host


def encode_bytes_u16(tokenizer: Tokenizer, data: bytes, chars_per_piece: int = CHARS_PER_PIECE) -> np.ndarray:
    """The reference's encode.py ids for a file whose raw bytes are `data`, as np.uint16."""
    import torch
    if len(data) == 0:
        return np.zeros(0, dtype=np.uint16)
    raw = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda")
    torch.cuda.synchronize()
    return encode_device_u16(tokenizer, raw, chars_per_piece)


def read_file_device(path):
    """A regular file's raw bytes in HBM (uint8 tensor) through the library's reader: pinned
    staging buffers filled by a pool of pread threads, each DMA'd while the next is read.  None
    for a file that is not regular (a pipe, FIFO or device): the caller reads it itself."""
    import torch
    if not stat.S_ISREG(os.stat(path).st_mode):   # missing: FileNotFoundError, as open() raises
        return None
    L = _lib.lib()
    n = ctypes.c_size_t(0)
    p = os.fsencode(os.fspath(path))
    _lib.check(L.bpe_read_file_device(p, None, 0, ctypes.byref(n)), "read")
    raw = torch.empty(max(n.value, 1), dtype=torch.uint8, device="cuda")[:n.value]
    if n.value:
        _lib.check(L.bpe_read_file_device(p, ctypes.c_void_p(raw.data_ptr()), n.value, ctypes.byref(n)), "read")
    return raw


last_phases_ms = {}   # the last encode_file's read / decode / encode / copy times (library clock)


def encode_file_native(tokenizer: Tokenizer, path, chars_per_piece: int = CHARS_PER_PIECE) -> np.ndarray:
    """A regular file through bpe_tok_encode_file_u16: read into HBM by the library's reader,
    decoded, pieces, encoded straight to uint16 in a device buffer the tokenizer keeps, and copied
    into host memory by copier threads -- no intermediate uint32 ids, no per-call device arrays."""
    L = _lib.lib()
    n = os.stat(path).st_size
    host = np.empty(max(n, 1), dtype=np.uint16)   # ids <= bytes; pages are touched only as written
    k = ctypes.c_size_t(0)
    ph = (ctypes.c_double * 4)()
    _lib.check(L.bpe_tok_encode_file_u16(tokenizer._device(), os.fsencode(os.fspath(path)), chars_per_piece,
                                         host.ctypes.data, host.size, ctypes.byref(k), ph), "encode file")
    last_phases_ms.clear()
    last_phases_ms.update(read=ph[0], decode=ph[1], encode=ph[2], copy=ph[3])
    return host[:k.value]


def encode_file(tokenizer: Tokenizer, input_path, output_path=None, fmt: str = "pt",
                chars_per_piece: int = CHARS_PER_PIECE, keep_device_buffers: bool = False) -> np.ndarray:
    """Encode a text file like encode.py:main; write it if output_path is given.  The device
    buffers of the bulk encoder (about 3 bytes of HBM per file byte) are released afterwards
    unless keep_device_buffers (several files in a row: re-allocating tens of GB costs the driver
    up to seconds per call)."""
    if stat.S_ISREG(os.stat(input_path).st_mode):   # missing: FileNotFoundError, as open() raises
        try:
            pt = encode_file_native(tokenizer, input_path, chars_per_piece)
        finally:
            if not keep_device_buffers:
                tokenizer.release_device_buffers()
    else:
        with open(input_path, "rb") as f:
            data = f.read()
        pt = encode_bytes_u16(tokenizer, data, chars_per_piece)
    if output_path is not None:
        if fmt == "pt":
            import torch
            torch.save(pt, output_path, pickle_protocol=4)   # encode.py:38
        elif fmt == "bin":
            pt.tofile(output_path)                           # np.memmap(path, np.uint16, "r")
        else:
            raise ValueError(f"unknown format {fmt!r}")
    return pt


def main(dataset: str, split: str, fmt: str = "pt"):
    """encode.py:18-38 with the same paths."""
    if dataset == "corpus":
        input_file = "tests/fixtures/corpus.en"
    else:
        input_file = f"/data/{fname[dataset + '/' + split]}"
    tokenizer = Tokenizer.from_files(
        vocab_filepath=f"data/tokenizer/{dataset}-vocab.pkl",
        merges_filepath=f"data/tokenizer/{dataset}-merges.pkl",
        special_tokens=["<|endoftext|>"],
    )
    ext = "pt" if fmt == "pt" else "bin"
    encode_file(tokenizer, input_file, f"data/tokenizer/{dataset}-tokens-{split}.{ext}", fmt=fmt)


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("--dataset", type=str)
    parser.add_argument("--split", type=str)
    parser.add_argument("--format", type=str, default="pt", choices=["pt", "bin"])
    args = parser.parse_args()
    main(args.dataset, args.split, args.format)
