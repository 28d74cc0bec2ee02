"""The byte-parallel token-start predicate (csrc/tokstart.h, evaluated 64 bytes per block as the
device counter does) against the serial scanner of the oracle (oracle/bpe_oracle.c pretokenize,
pinned to the reference's pre-tokenization by the golden word tables), on CPU.

Inputs: every golden train input, the adversarial generator's three flavours at many sizes (so
contractions, whitespace runs and multi-byte characters land on every block alignment), and
dense random strings over the characters the pattern treats specially.
"""
from __future__ import annotations

import ctypes
import random

import numpy as np
import pytest

import golden_cases as G
import synth_text
from oracle import oracle

bpe_amd = pytest.importorskip("bpe_amd")
from bpe_amd import _lib  # noqa: E402


def starts_predicate(data: bytes) -> np.ndarray:
    L = _lib.lib()
    out = np.zeros(len(data), dtype=np.uint8)
    fn = L.bpe_pretok_starts_host
    fn.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
    assert fn(data, len(data), out.ctypes.data) == 0
    return out


def starts_oracle(data: bytes) -> np.ndarray:
    out = np.zeros(len(data), dtype=np.uint8)
    for s, _n in oracle.pretokenize(data):
        out[s] = 1
    return out


def check(data: bytes):
    got, want = starts_predicate(data), starts_oracle(data)
    if not np.array_equal(got, want):
        i = int(np.nonzero(got != want)[0][0])
        pytest.fail(f"start flag differs at byte {i}: predicate {got[i]} oracle {want[i]}; "
                    f"context {data[max(0, i - 12):i + 12]!r}")


@pytest.mark.parametrize("name", G.names("train"))
def test_golden_inputs(name):
    o = G.load("train", name)
    data = G.input_bytes(o["input"]).replace(b"\r\n", b"\n").replace(b"\r", b"\n")
    check(data)


@pytest.mark.parametrize("flavour", ["mixed", "ascii", "space"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_generator(flavour, seed):
    for n in (1, 2, 3, 63, 64, 65, 127, 200, 4096 + 17, 60_000):
        check(synth_text.generate(seed * 1000 + n, n, flavour).encode("utf-8"))


_ALPHABET = ["'", "s", "d", "m", "t", "l", "v", "r", "e", "S", "L", "x", " ", " ", "\n", "\t",
             "\xa0", "　", "\x85", "0", "٣", "½", ".", "-", "́", "é", "中", "🙃", "\x00",
             "\x1c", "''", "'ll", "'ve", "'re", "  ", " '"]


@pytest.mark.parametrize("seed", range(8))
def test_dense_random(seed):
    r = random.Random(seed)
    for _ in range(40):
        s = "".join(r.choice(_ALPHABET) for _ in range(r.randrange(1, 400)))
        check(s.encode("utf-8"))
