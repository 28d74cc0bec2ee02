"""train_bpe(input_path) end to end: the file is read by the library's pinned-staging reader
(drive.hip), the way the reference reads it (models/tokenizer/train.py:22, text mode), and the
multi-device driver (n_gpus) splits one file over several ranks in one process.

On a one-GPU box the multi-device driver runs with BPE355_INPROC_RANKS=1: its ranks are threads
that share the device and exchange through an in-process communicator instead of RCCL, so the
slab cutting, the word-table exchange and the error agreement are all exercised.
"""
from __future__ import annotations

import os
import threading

import numpy as np
import pytest

import golden_cases as G
import gpt2_files
from oracle import oracle

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")
from bpe_amd import _lib  # noqa: E402
from bpe_amd.train import last_train_stats  # noqa: E402

EOT = ["<|endoftext|>"]


@pytest.fixture
def inproc(monkeypatch):
    monkeypatch.setenv("BPE355_INPROC_RANKS", "1")
    yield
    bpe_amd.set_num_gpus(None)


def _synth(seed, flavour, n):
    buf = np.empty(n, dtype=np.uint8)
    assert _lib.lib().bpe_synth_corpus_host(buf.ctypes.data, n, seed, flavour, 0, 8) == 0
    return buf.tobytes()


def test_train_from_fifo_matches_reference(tmp_path):
    """a pipe has no size: it is read to EOF (the reference's read() does the same)"""
    data = (gpt2_files.FIXTURES / "corpus.en").read_bytes()
    fifo = tmp_path / "corpus.fifo"
    os.mkfifo(fifo)

    def writer():
        with open(fifo, "wb") as f:
            for i in range(0, len(data), 4096):
                f.write(data[i:i + 4096])

    th = threading.Thread(target=writer)
    th.start()
    vocab, merges = bpe_amd.train_bpe(fifo, 500, EOT)
    th.join()
    ref_vocab, ref_merges = gpt2_files.load_reference_train_golden()
    assert merges == ref_merges
    assert set(vocab.values()) == set(ref_vocab.values())


def test_train_directory_and_missing(tmp_path):
    with pytest.raises(IsADirectoryError):
        bpe_amd.train_bpe(tmp_path, 300, [])
    with pytest.raises(FileNotFoundError):
        bpe_amd.train_bpe(tmp_path / "nope", 300, [])


def test_train_large_file_equals_buffer(tmp_path):
    """48 MB: several 16 MiB staging chunks over several reader threads"""
    data = _synth(21, 0, 48 * (1 << 20) + 12345)
    p = tmp_path / "c.txt"
    p.write_bytes(data)
    got = bpe_amd.train_bpe(p, 4000, EOT)
    st = last_train_stats()
    assert st["t_load_ms"] > 0 and st["n_gpus"] == 1
    assert got == bpe_amd.train_bpe_bytes(data, 4000, EOT)
    assert got == oracle.train_raw(data, 4000, EOT)


@pytest.mark.parametrize("ranks", [2, 3, 5])
def test_multi_device_driver_matches_oracle(tmp_path, inproc, ranks):
    """one process, several ranks: slabs at safe points, word tables exchanged, rank 0 trains"""
    data = _synth(22, 1, 6_000_000 + 77) + (gpt2_files.FIXTURES / "corpus.en").read_bytes()
    p = tmp_path / "c.txt"
    p.write_bytes(data)
    bpe_amd.set_num_gpus(ranks)
    got = bpe_amd.train_bpe(p, 3000, EOT)
    st = last_train_stats()
    assert st["n_gpus"] == ranks and st["n_exchanged_words"] > 0
    assert got == oracle.train_raw(data, 3000, EOT)
    assert bpe_amd.train_bpe_bytes(data, 3000, EOT) == got


@pytest.mark.parametrize("name", ["corpus_en_500", "tiny_1200", "edge_crlf", "edge_empty", "edge_abc"])
def test_multi_device_driver_goldens(inproc, name):
    """reference goldens (including tiny inputs where some slabs are empty) on 4 ranks"""
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    bpe_amd.set_num_gpus(4)
    got_vocab, got_merges = bpe_amd.train_bpe_bytes(data, o["vocab_size"], o["special_tokens"])
    assert got_merges == merges
    assert got_vocab == vocab


def test_multi_device_utf8_error_position(tmp_path, inproc):
    """a bad byte in the last slab: every rank raises, at the byte's whole-file position"""
    data = bytearray(_synth(23, 0, 3_000_000))
    bad = len(data) - 1000
    data[bad] = 0xFF
    try:
        bytes(data).decode("utf-8")
    except UnicodeDecodeError as e:
        want = e.start
    assert want == bad
    p = tmp_path / "bad.txt"
    p.write_bytes(bytes(data))
    bpe_amd.set_num_gpus(3)
    with pytest.raises(UnicodeDecodeError) as ei:
        bpe_amd.train_bpe(p, 1000, EOT)
    assert ei.value.start == want
    bpe_amd.set_num_gpus(1)
    with pytest.raises(UnicodeDecodeError) as ei:
        bpe_amd.train_bpe(p, 1000, EOT)
    assert ei.value.start == want
