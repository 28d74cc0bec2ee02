"""The byte-parallel counter (csrc/count.hip: token-start masks, LDS word cache, record spill and
by-bin LDS aggregation) against the oracle's word table (reference train.py:16-28), on the paths
the bench corpus takes and on the ones only knobs reach on small inputs:

  * records on (BPE355_REC_POOL: the pool, in records; the bench turns it on past 256 MB);
  * the pool spent (a tiny pool: most misses fall back to the global table);
  * few workgroups each streaming many chunks (BPE355_STREAM_WG): pages fill and turn over;
  * the file path's segment launches (BPE355_SEG_MB) continuing each workgroup's page;
  * an unaligned device pointer (the byte-wise staging path);
  * adversarial text (every pattern branch, multi-byte characters at every alignment);
  * text dense in words longer than 16 bytes (the long-word segments, full and not).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import synth_text
from oracle import oracle

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")
from bpe_amd import _lib  # noqa: E402
from bpe_amd.train import last_train_stats  # noqa: E402
from test_gpu_utf8 import _device_word_counts  # noqa: E402

EOT = ["<|endoftext|>"]


@pytest.fixture
def knob(monkeypatch):
    def set_(k, v):
        monkeypatch.setenv(k, str(v))
    return set_


def _synth(seed, flavour, n):
    buf = np.empty(n, dtype=np.uint8)
    assert _lib.lib().bpe_synth_corpus_host(buf.ctypes.data, n, seed, flavour, 0, 8) == 0
    return buf.tobytes()


def _want_words(data, specials):
    text = data.replace(b"\r\n", b"\n").replace(b"\r", b"\n")
    return {w: c for w, c in oracle.word_counts(text, specials).items() if len(w) > 1}


@pytest.mark.parametrize("pool", [None, "1e8", "150000"])
@pytest.mark.parametrize("seed,flavour,n", [(31, 0, 12 << 20), (32, 1, 5 << 20)])
def test_word_table_vs_oracle(knob, pool, seed, flavour, n):
    if pool:
        knob("BPE355_REC_POOL", pool)
    data = _synth(seed, flavour, n)
    assert _device_word_counts(data, EOT) == _want_words(data, EOT)


@pytest.mark.parametrize("flavour", ["mixed", "space", "ascii"])
def test_adversarial_text_records(knob, flavour):
    knob("BPE355_REC_POOL", "1e8")
    data = synth_text.generate(77, 3_000_000, flavour).encode("utf-8")
    assert _device_word_counts(data, EOT) == _want_words(data, EOT)


def test_page_turnover_few_workgroups(knob):
    knob("BPE355_REC_POOL", "1e8")
    knob("BPE355_STREAM_WG", 3)
    data = _synth(33, 0, 24 << 20)
    assert _device_word_counts(data, EOT) == _want_words(data, EOT)


def test_train_records_vs_oracle(knob):
    knob("BPE355_REC_POOL", "1e8")
    data = _synth(34, 0, 16 << 20)
    got = bpe_amd.train_bpe_bytes(data, 6000, EOT)
    assert last_train_stats()["n_count_records"] > 0
    assert got == oracle.train_raw(data, 6000, EOT)


@pytest.mark.parametrize("how", [("BPE355_REC_POOL_FAIL", "1"), ("BPE355_REC_POOL_FIT", "1000")])
def test_pool_does_not_fit_falls_back(knob, how):
    """the record pool is capped by free device memory; when it cannot be had (its
    allocation fails, or the memory left holds less than a page per counting workgroup) the
    counter sends every miss to the global table -- same words, no records"""
    knob("BPE355_REC_POOL", "1e8")
    knob(*how)
    data = _synth(37, 0, 8 << 20)
    got = bpe_amd.train_bpe_bytes(data, 3000, EOT)
    assert last_train_stats()["n_count_records"] == 0
    assert got == oracle.train_raw(data, 3000, EOT)
    assert _device_word_counts(data, EOT) == _want_words(data, EOT)


def test_file_segments_records(knob, tmp_path):
    knob("BPE355_REC_POOL", "1e8")
    knob("BPE355_SEG_MB", 4)
    data = _synth(35, 1, 40 << 20)
    p = tmp_path / "c.txt"
    p.write_bytes(data)
    got = bpe_amd.train_bpe(p, 4000, EOT)
    assert last_train_stats()["n_count_records"] > 0
    assert got == oracle.train_raw(data, 4000, EOT)


@pytest.mark.parametrize("every", [1, 3])
def test_file_partial_aggregation(knob, tmp_path, every):
    # few workgroups fill and leave pages while later segments arrive: those pages are
    # aggregated between segment launches (BPE355_AGG_SEGS), the held ones only at the end
    knob("BPE355_REC_POOL", "1e8")
    knob("BPE355_SEG_MB", 2)
    knob("BPE355_STREAM_WG", 4)
    knob("BPE355_AGG_SEGS", every)
    data = _synth(36, 0, 30 << 20)
    p = tmp_path / "c.txt"
    p.write_bytes(data)
    got = bpe_amd.train_bpe(p, 3000, EOT)
    st = last_train_stats()
    assert st["n_count_records"] > 0
    assert st["n_count_batches"] > 2
    assert got == oracle.train_raw(data, 3000, EOT)


def _long_word_text(seed, n_words):
    """text dense in pre-tokens longer than 16 bytes (ASCII, 2- and 3-byte letters, digits,
    whitespace runs), many of them repeated, between ordinary synthetic text"""
    rng = np.random.default_rng(seed)
    alpha = "abcdefghijklmnopqrstuvwxyz" + "éßøñ" + "жщы" + "中文字"
    vocab = []
    for _ in range(400):
        k = int(rng.integers(9, 40))
        w = "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), k))
        vocab.append(w if rng.random() < 0.8 else "".join(str(int(d)) for d in rng.integers(0, 10, 2 * k)))
    filler = synth_text.generate(seed, 400_000, "mixed")
    parts = []
    for _ in range(n_words):
        parts.append(" " + vocab[int(rng.integers(0, len(vocab)))] if rng.random() < 0.7
                     else " " + "".join(alpha[int(i)] for i in rng.integers(0, len(alpha), int(rng.integers(17, 90)))))
        if rng.random() < 0.1:   # indentation: whitespace runs of 17-40 bytes, the hot long words
            parts.append("\n" + " " * int(rng.integers(17, 41)) + "x")
        if rng.random() < 0.05:
            o = int(rng.integers(0, len(filler) - 300))
            parts.append(filler[o:o + 300])
    return "".join(parts).encode("utf-8")


@pytest.mark.parametrize("seg", [None, "1", "7"])
def test_long_words_listed(knob, seg):
    """words longer than kInline go to each counting workgroup's segment and k_count_long adds
    them after the launch; a full segment (BPE355_LONG_SEG: entries per workgroup) sends the rest
    to the table directly -- the same counts either way"""
    knob("BPE355_REC_POOL", "1e8")
    if seg:
        knob("BPE355_LONG_SEG", seg)
    data = _long_word_text(5, 120_000)
    assert _device_word_counts(data, EOT) == _want_words(data, EOT)


def test_long_words_file_segments(knob, tmp_path):
    # segments are emptied behind every k_count2 launch of the file path
    knob("BPE355_REC_POOL", "1e8")
    knob("BPE355_SEG_MB", 1)
    data = _long_word_text(6, 150_000)
    p = tmp_path / "c.txt"
    p.write_bytes(data)
    got = bpe_amd.train_bpe(p, 800, EOT)
    assert got == oracle.train_raw(data, 800, EOT)


@pytest.mark.parametrize("shift", [1, 3, 7])
def test_unaligned_device_text(shift):
    import torch
    data = synth_text.generate(78, 400_000, "mixed").encode("utf-8").replace(b"\r", b" ")
    buf = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    buf[shift:shift + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    torch.cuda.synchronize()
    got = bpe_amd.train_bpe_device(buf.data_ptr() + shift, len(data), 1500, EOT)
    assert got == oracle.train_raw(data, 1500, EOT)
