"""CPU-side checks of the drop-in boundary: libbpe355.so loads, exports every entry point
include/bpe355.h declares, and refuses to compute without a GPU (no silent CPU fallback)."""
import ctypes
import pathlib
import re

import pytest

from bpe_amd import _lib

ROOT = pathlib.Path(__file__).resolve().parent.parent


def header_functions():
    text = (ROOT / "include" / "bpe355.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(bpe_[a-z0-9_]+)\s*\(", text)
    return sorted(set(n for n in names if not n.endswith("_fn")))


def test_library_loads_and_exports_header():
    L = _lib.lib()
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(header_functions()) == set(_lib.SYMBOLS)
    assert L.bpe_abi_version() == 2


def test_no_cpu_fallback():
    L = _lib.lib()
    if L.bpe_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        _lib.require_device()
    res = ctypes.c_void_p()
    rc = L.bpe_train_buffer(b"abc abc", 7, 300, None, 0, None, ctypes.byref(res))
    assert rc == _lib.BPE_E_HIP
    import bpe_amd
    with pytest.raises(RuntimeError):
        bpe_amd.train_bpe_bytes(b"abc abc", 300, [])
    tok = bpe_amd.Tokenizer({i: bytes([i]) for i in range(256)}, [], [])
    with pytest.raises(RuntimeError):
        tok.encode("abc")


def test_safe_split_helper():
    L = _lib.lib()
    data = b"hello world, this is a test\n\n  ok"
    for pos in range(len(data)):
        p = L.bpe_safe_split(data, len(data), pos)
        assert p <= max(pos, 0)
        if p:
            assert data[p:p + 1] == b" " and data[p - 1:p] not in b" \t\n\r\x0b\x0c"
            assert data[p + 1:p + 2] not in b" \t\n\r\x0b\x0c"
