"""ctypes binding of libbpe355 (include/bpe355.h).

This is the whole host<->device boundary: plain pointers and sizes, the library owns result
objects until *_free.  There is deliberately no CPU fallback: if the shared library is missing
or no gfx950 device is visible, every compute call raises.
"""
from __future__ import annotations

import ctypes
import itertools
import errno as _errno
import os
import re
import pathlib
import struct

LIB_PATH = pathlib.Path(__file__).resolve().parent.parent / "lib" / "libbpe355.so"
# experiment knob: an alternative build of the same library (A/B timing of kernel variants)
if os.environ.get("BPE355_LIB"):
    LIB_PATH = pathlib.Path(os.environ["BPE355_LIB"]).resolve()

BPE_OK, BPE_E_IO, BPE_E_UTF8, BPE_E_KEY, BPE_E_HIP, BPE_E_ARG, BPE_E_NOMEM, BPE_E_RCCL, \
    BPE_E_LIMIT = 0, -1, -2, -3, -4, -5, -6, -7, -8


class LibraryMissing(RuntimeError):
    pass


class TrainStats(ctypes.Structure):
    _fields_ = [
        ("t_total_ms", ctypes.c_double), ("t_prepare_ms", ctypes.c_double),
        ("t_count_ms", ctypes.c_double), ("t_words_ms", ctypes.c_double),
        ("t_merge_ms", ctypes.c_double), ("merge_kernel_ms", ctypes.c_double),
        ("merge_kernel_launches", ctypes.c_int64), ("merge_kernel_bytes", ctypes.c_double),
        ("count_kernel_ms", ctypes.c_double), ("count_kernel_bytes", ctypes.c_double),
        ("n_bytes", ctypes.c_int64), ("n_pretokens", ctypes.c_int64), ("n_words", ctypes.c_int64),
        ("n_word_tokens", ctypes.c_int64), ("n_pairs_final", ctypes.c_int64),
        ("n_rebuilds", ctypes.c_int64), ("n_rounds_device", ctypes.c_int64),
        ("n_rounds_host", ctypes.c_int64), ("n_index_builds", ctypes.c_int64),
        ("n_trips", ctypes.c_int64), ("n_rounds_batched", ctypes.c_int64),
        ("t_exchange_ms", ctypes.c_double), ("n_exchanged_words", ctypes.c_int64),
        ("t_load_ms", ctypes.c_double), ("n_gpus", ctypes.c_int64),
        ("count_reduce_ms", ctypes.c_double), ("n_count_records", ctypes.c_int64),
        ("count_partial_ms", ctypes.c_double), ("n_count_batches", ctypes.c_int64),
        ("t_gather_ms", ctypes.c_double), ("t_union_ms", ctypes.c_double),
        ("exchange_seg_bytes", ctypes.c_int64),
        ("t_alltoall_ms", ctypes.c_double), ("t_owner_ms", ctypes.c_double),
        ("exchange_a2a_bytes", ctypes.c_int64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


HOST_ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_int64), ctypes.c_size_t)

_lib = None

# (name, restype, argtypes) for every symbol declared in include/bpe355.h
_P = ctypes.c_void_p
_U8P = ctypes.c_char_p
_SZ = ctypes.c_size_t
_SIGS = [
    ("bpe_abi_version", ctypes.c_int, []),
    ("bpe_runtime_info", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                        ctypes.c_char_p, _SZ]),
    ("bpe_last_error", ctypes.c_char_p, []),
    ("bpe_last_errno", ctypes.c_int, []),
    ("bpe_device_count", ctypes.c_int, []),
    ("bpe_comm_unique_id", ctypes.c_int, [ctypes.c_char_p]),
    ("bpe_comm_init", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(_P)]),
    ("bpe_comm_init_host", ctypes.c_int, [HOST_ALLREDUCE_FN, _P, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(_P)]),
    ("bpe_comm_free", None, [_P]),
    ("bpe_train_file", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                      ctypes.c_int, ctypes.c_int, ctypes.POINTER(_P)]),
    ("bpe_train_file_comm", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, _P,
                                           ctypes.c_int, ctypes.POINTER(_P)]),
    ("bpe_train_buffer", ctypes.c_int, [_U8P, _SZ, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.c_int, _P, ctypes.POINTER(_P)]),
    ("bpe_train_buffer_gpus", ctypes.c_int, [_U8P, _SZ, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                             ctypes.c_int, ctypes.POINTER(_P)]),
    ("bpe_train_device", ctypes.c_int, [_P, _SZ, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.c_int, _P, _P, ctypes.POINTER(_P)]),
    ("bpe_word_counts", ctypes.c_int, [_U8P, _SZ, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                       ctypes.POINTER(_P), ctypes.POINTER(_SZ)]),
    ("bpe_blob_free", None, [_P]),
    ("bpe_result_n_merges", ctypes.c_int64, [_P]),
    ("bpe_result_n_vocab", ctypes.c_int64, [_P]),
    ("bpe_result_merges_blob", _SZ, [_P, ctypes.POINTER(_P)]),
    ("bpe_result_vocab_blob", _SZ, [_P, ctypes.POINTER(_P)]),
    ("bpe_result_flat", ctypes.c_size_t, [_P, ctypes.c_int, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)),
                                           ctypes.POINTER(_P), ctypes.POINTER(_SZ)]),
    ("bpe_result_merge_ids", ctypes.c_size_t, [_P, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32))]),
    ("bpe_result_stats", ctypes.c_int, [_P, ctypes.POINTER(TrainStats)]),
    ("bpe_result_free", None, [_P]),
    ("bpe_release_device_memory", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_SZ)]),
    ("bpe_set_timing", None, [ctypes.c_int]),
    ("bpe_tok_create", ctypes.c_int, [_U8P, _SZ, _U8P, _SZ, ctypes.POINTER(ctypes.c_char_p),
                                      ctypes.c_int, ctypes.POINTER(_P)]),
    ("bpe_tok_special_id", ctypes.c_int64, [_P, ctypes.c_int]),
    ("bpe_tok_encode", ctypes.c_int, [_P, _U8P, _SZ, _P, _SZ, ctypes.POINTER(_SZ)]),
    ("bpe_tok_encode_device", ctypes.c_int, [_P, _P, _SZ, _P, ctypes.POINTER(_SZ), _P]),
    ("bpe_tok_encode_gpus", ctypes.c_int, [_P, _U8P, _SZ, _P, _SZ, ctypes.POINTER(_SZ), ctypes.c_int]),
    ("bpe_tok_encode_chunks", ctypes.c_int, [_P, _U8P, _SZ, _P, _SZ, _P, _SZ, ctypes.POINTER(_SZ)]),
    ("bpe_tok_encode_chunks_device", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, _P, ctypes.POINTER(_SZ), _P]),
    ("bpe_tok_encode_file_u16", ctypes.c_int, [_P, ctypes.c_char_p, _SZ, _P, _SZ, ctypes.POINTER(_SZ),
                                               ctypes.POINTER(ctypes.c_double)]),
    ("bpe_tok_release_buffers", ctypes.c_int, [_P]),
    ("bpe_tok_free", None, [_P]),
    ("bpe_dec_create", ctypes.c_int, [_U8P, _SZ, ctypes.POINTER(_P)]),
    ("bpe_dec_decode", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, ctypes.POINTER(_SZ)]),
    ("bpe_dec_decode_device", ctypes.c_int, [_P, _P, _SZ, _P, _SZ, ctypes.POINTER(_SZ), _P]),
    ("bpe_dec_free", None, [_P]),
    ("bpe_read_file_device", ctypes.c_int, [ctypes.c_char_p, _P, _SZ, ctypes.POINTER(_SZ)]),
    ("bpe_copy_to_host", ctypes.c_int, [_P, _SZ, _P]),
    ("bpe_text_prepare_device", ctypes.c_int, [_P, _SZ, _P, ctypes.POINTER(_SZ), _P]),
    ("bpe_utf8_chunk_starts_device", ctypes.c_int, [_P, _SZ, _SZ, _P, _SZ, ctypes.POINTER(_SZ), _P]),
    ("bpe_ids_to_u16_device", ctypes.c_int, [_P, _SZ, _P, _P]),
    ("bpe_safe_split", _SZ, [_U8P, _SZ, _SZ]),
    ("bpe_synth_corpus_device", ctypes.c_int, [_P, _SZ, ctypes.c_uint64, ctypes.c_int,
                                               ctypes.c_uint64, _P]),
    ("bpe_synth_corpus_host", ctypes.c_int, [_P, _SZ, ctypes.c_uint64, ctypes.c_int,
                                             ctypes.c_uint64, ctypes.c_int]),
]
SYMBOLS = [s[0] for s in _SIGS]


def lib():
    """Load libbpe355.so (built in-tree by __graft_entry__.build()).  Raises if missing."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise LibraryMissing(f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; "
                                 "g.build()'` (hipcc --offload-arch=gfx950)")
        # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64, and whichever
        # copy is loaded first serves every later library that needs that soname.  Loading
        # torch's first keeps torch.cuda usable next to this library (loading ours first left
        # torch with "No HIP GPUs are available").  Importing torch does not touch the GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(str(LIB_PATH))
        for name, res, args in _SIGS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _check_runtime(L)
        _lib = L
    return _lib


RUNTIME = {}   # the HIP runtime this process bound the library to (bpe_runtime_info)


def _check_runtime(L):
    """The library is compiled against the image's ROCm headers; the libamdhip64.so.7 serving it
    is the first copy of that soname the process loaded (torch's bundled runtime when torch is
    imported first).  HIP keeps its C ABI within a major version, so a different minor version
    is recorded (bench line) and a different major version is refused."""
    comp, run = ctypes.c_int(0), ctypes.c_int(0)
    path = ctypes.create_string_buffer(4096)
    rc = L.bpe_runtime_info(ctypes.byref(comp), ctypes.byref(run), path, len(path))
    RUNTIME.update(compiled=comp.value, runtime=run.value if rc == BPE_OK else None,
                   path=path.value.decode("utf-8", "replace"))
    if rc == BPE_OK and run.value // 10_000_000 != comp.value // 10_000_000:
        raise LibraryMissing(f"libbpe355 was compiled for HIP {comp.value} but the process bound HIP "
                             f"runtime {run.value} ({RUNTIME['path']}): major versions differ")


def check(rc: int, what: str = ""):
    if rc == BPE_OK:
        return
    msg = (lib().bpe_last_error() or b"").decode("utf-8", "replace")
    if rc == BPE_E_IO:
        en = lib().bpe_last_errno() or _errno.EIO
        raise OSError(en, os.strerror(en), what or msg)
    if rc == BPE_E_UTF8:
        # start/end name the first ill-formed byte, as CPython's decoder reports it
        m = re.search(r"position (\d+)", msg)
        pos = int(m.group(1)) if m else 0
        raise UnicodeDecodeError("utf-8", b"", pos, pos + 1, msg)
    if rc == BPE_E_KEY:
        raise KeyError(msg)
    raise RuntimeError(f"libbpe355 {what} failed ({rc}): {msg}")


def require_device():
    if lib().bpe_device_count() < 1:
        raise RuntimeError("libbpe355 needs an MI355X (gfx950) GPU; none is visible")


def c_strings(items):
    items = list(items or [])
    arr = (ctypes.c_char_p * max(1, len(items)))()
    keep = [s.encode("utf-8") for s in items]
    for i, b in enumerate(keep):
        arr[i] = b
    return arr, len(items), keep


def iter_records(blob: bytes):
    off, n = 0, len(blob)
    while off < n:
        ln = struct.unpack_from("<I", blob, off)[0]
        off += 4
        yield blob[off:off + ln]
        off += ln


def take_result(res: ctypes.c_void_p):
    """-> (vocab dict[int, bytes], merges list[tuple[bytes, bytes]], stats dict); frees res."""
    L = lib()
    def flat(which):
        lens, data, nb = ctypes.POINTER(ctypes.c_uint32)(), ctypes.c_void_p(), ctypes.c_size_t(0)
        n = L.bpe_result_flat(res, which, ctypes.byref(lens), ctypes.byref(data), ctypes.byref(nb))
        if n == 0:
            return []
        # lengths through a memoryview (one C call) and a list comprehension of slices: the
        # fastest of the forms timed for ~64 K merge parts + 32 K vocab entries
        lv = memoryview((ctypes.c_uint32 * n).from_address(ctypes.addressof(lens.contents))).cast("B").cast("I")
        off = list(itertools.accumulate(lv.tolist(), initial=0))
        buf = ctypes.string_at(data, nb.value)
        return [buf[a:b] for a, b in zip(off, off[1:])]
    try:
        v = flat(1)
        # the merges as vocab ids: each part is the vocab's own bytes object (the reference appends
        # (vocab[a], vocab[b]), train.py:191-196), not one new object per part
        ids = ctypes.POINTER(ctypes.c_uint32)()
        nm = L.bpe_result_merge_ids(res, ctypes.byref(ids))
        if nm:
            iv = memoryview((ctypes.c_uint32 * (2 * nm)).from_address(ctypes.addressof(ids.contents)))
            iv = iv.cast("B").cast("I").tolist()
            g = v.__getitem__
            merges = list(zip(map(g, iv[0::2]), map(g, iv[1::2])))
        else:
            m = flat(0)
            merges = list(zip(m[0::2], m[1::2]))
        st = TrainStats()
        check(L.bpe_result_stats(res, ctypes.byref(st)), "stats")
    finally:
        L.bpe_result_free(res)
    vocab = dict(enumerate(v))
    return vocab, merges, st.as_dict()


def vocab_blob(vocab: dict) -> bytes:
    parts = [struct.pack("<I", len(vocab))]
    for i, b in vocab.items():
        b = bytes(b)
        parts.append(struct.pack("<qI", int(i), len(b)) + b)
    return b"".join(parts)


def merges_blob(merges) -> bytes:
    parts = [struct.pack("<I", len(merges))]
    for a, b in merges:
        a, b = bytes(a), bytes(b)
        parts.append(struct.pack("<I", len(a)) + a + struct.pack("<I", len(b)) + b)
    return b"".join(parts)
