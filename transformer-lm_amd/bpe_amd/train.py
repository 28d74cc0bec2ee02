"""train_bpe -- drop-in for reference models/tokenizer/train.py:142 (train_bpe).

Same signature, same return value (vocab: dict[int, bytes], merges: list[tuple[bytes, bytes]]),
same exceptions (FileNotFoundError / OSError, UnicodeDecodeError), bit-identical output.
The work runs in libbpe355 on an MI355X: pre-tokenization, word counting, the pair histogram
and the merge loop are HIP kernels (transformer-lm_amd/csrc).
"""
from __future__ import annotations

import ctypes
import os
from typing import List

from . import _lib

__all__ = ["train_bpe", "train_bpe_bytes", "train_bpe_device", "last_train_stats", "set_num_gpus",
           "num_gpus", "release_device_memory"]

_last_stats: dict = {}
_num_gpus: int | None = None


def set_num_gpus(n: int | None):
    """GPUs of this process that train_bpe / train_bpe_bytes use (<= 0: every visible one;
    None: back to the default, the BPE355_GPUS environment variable or 1).  The reference's
    signature has no such argument (train.py:142), so it is a module setting."""
    global _num_gpus
    _num_gpus = None if n is None else int(n)


def num_gpus() -> int:
    if _num_gpus is not None:
        return _num_gpus
    return int(os.environ.get("BPE355_GPUS", "1"))


def last_train_stats() -> dict:
    """Timings and counters of the most recent train_bpe call on this process."""
    return dict(_last_stats)


def release_device_memory(device: int = -1) -> int:
    """Hand back the device memory the trainer keeps between calls (the corpus buffer, the
    counter's record pool and bins) on `device` (-1: every device; buffers a call of another
    thread is using are left alone, and the copy streams stay for the process); returns the
    bytes freed.  train_bpe calls it after every call unless keep_device_buffers=True."""
    L = _lib.lib()
    freed = ctypes.c_size_t(0)
    _lib.check(L.bpe_release_device_memory(int(device), ctypes.byref(freed)), "release_device_memory")
    return int(freed.value)


def _finish(rc, res, what, keep_device_buffers=True):
    global _last_stats
    try:
        _lib.check(rc, what)
        vocab, merges, stats = _lib.take_result(res)
    finally:
        # the reference holds nothing once train_bpe returns (train.py:231), and its caller trains
        # the LM on the same GPU next (train.py:230-232)
        if not keep_device_buffers:
            try:
                release_device_memory(-1)
            except Exception:
                if rc == 0:   # never hide the call's own error behind the release's
                    raise
    _last_stats = stats
    return vocab, merges


def train_bpe(input_path: str | os.PathLike, vocab_size: int, special_tokens: List[str] = [],
              comm=None, split_file: bool = False, keep_device_buffers: bool = False):
    """Train a byte-level BPE on the file at input_path (reference train.py:142-231).

    Without comm: one process on num_gpus() devices (set_num_gpus / BPE355_GPUS).
    comm: a bpe_amd.dist.Communicator (one process per GPU); the file is this rank's slab, or
    with split_file=True the whole corpus, of which each rank reads its share.
    keep_device_buffers: keep the corpus buffer and the counter's scratch (~5 bytes of HBM per
    corpus byte) for the next call instead of freeing them on return (bench.py's repeated steps).
    """
    L = _lib.lib()
    arr, n, _keep = _lib.c_strings(special_tokens)
    res = ctypes.c_void_p()
    path = os.fsencode(os.fspath(input_path))
    if comm is not None:
        rc = L.bpe_train_file_comm(path, int(vocab_size), arr, n, comm.handle, int(split_file),
                                   ctypes.byref(res))
    else:
        rc = L.bpe_train_file(path, int(vocab_size), arr, n, num_gpus(), ctypes.byref(res))
    return _finish(rc, res, f"train_bpe({os.fspath(input_path)!r})", keep_device_buffers)


def train_bpe_bytes(data: bytes, vocab_size: int, special_tokens: List[str] = [], comm=None,
                    keep_device_buffers: bool = False):
    """train_bpe on the raw bytes of a file (decoded exactly like the file would be)."""
    L = _lib.lib()
    arr, n, _keep = _lib.c_strings(special_tokens)
    res = ctypes.c_void_p()
    if comm is not None or num_gpus() == 1:
        rc = L.bpe_train_buffer(data, len(data), int(vocab_size), arr, n,
                                comm.handle if comm else None, ctypes.byref(res))
    else:
        rc = L.bpe_train_buffer_gpus(data, len(data), int(vocab_size), arr, n, num_gpus(),
                                     ctypes.byref(res))
    return _finish(rc, res, "train_bpe_bytes", keep_device_buffers)


def train_bpe_device(d_ptr: int, n: int, vocab_size: int, special_tokens: List[str] = [],
                     comm=None, stream: int = 0, keep_device_buffers: bool = False):
    """train_bpe on raw bytes already resident in device memory (e.g. a torch uint8 CUDA
    tensor's data_ptr()); used by bench.py so the timed region starts with data in HBM."""
    L = _lib.lib()
    arr, k, _keep = _lib.c_strings(special_tokens)
    res = ctypes.c_void_p()
    rc = L.bpe_train_device(ctypes.c_void_p(d_ptr), n, int(vocab_size), arr, k,
                            comm.handle if comm else None, ctypes.c_void_p(stream or None),
                            ctypes.byref(res))
    return _finish(rc, res, "train_bpe_device", keep_device_buffers)
