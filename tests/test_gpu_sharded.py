"""Sharded (multi-rank) training on the GPU.

A one-GPU box cannot hold two RCCL ranks, so the ranks here are threads of this process that
share the device and exchange through the library's in-process communicator
(BPE355_INPROC_RANKS=1, csrc/comm.hip InProcComm); the slab cutting, the collectives' call
pattern and every kernel are the ones the RCCL path runs.  Both exchange modes are covered:
  words  (default)  one all-to-all of the slabs' unique words by owner (the rank the word's hash
                    names sums its counts), one all-gather of the owners' tables, then rank 0
                    trains on the union (exchange.hip); "words-gather" skips the all-to-all
                    (BPE355_EXCHANGE_OWNER=0: every rank's local table is gathered as it is);
  rounds            local word tables, one all-reduce of the delta cells per merge round, a
                    replicated pair table and argmax on every rank (the driver checks that all
                    ranks chose the same merges).
The result must be exactly the unsharded one.  (Round 1 ran these as two processes sharing the
card through a gloo-backed host communicator; the multi-process protocol is covered on CPU by
test_dist_gloo.py, and one real RCCL rank by test_rccl_comm_single_rank_forced below.)
"""
import multiprocessing as mp
import os

import pytest

import golden_cases as G
from oracle import oracle

pytestmark = pytest.mark.gpu

bpe_amd = pytest.importorskip("bpe_amd")


@pytest.fixture
def ranks(monkeypatch):
    def set_(n, mode):
        monkeypatch.setenv("BPE355_INPROC_RANKS", "1")
        if mode == "words-gather":
            monkeypatch.setenv("BPE355_EXCHANGE_OWNER", "0")
            mode = "words"
        monkeypatch.setenv("BPE355_EXCHANGE", mode)
        bpe_amd.set_num_gpus(n)
    yield set_
    bpe_amd.set_num_gpus(None)


@pytest.mark.parametrize("mode", ["words", "words-gather", "rounds"])
@pytest.mark.parametrize("name", ["corpus_en_1000", "tiny_1200", "synth_mixed_200k"])
def test_sharded_gpu_matches_reference(name, mode, ranks):
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    ranks(2, mode)
    got_vocab, got_merges = bpe_amd.train_bpe_bytes(data, o["vocab_size"], o["special_tokens"])
    assert bpe_amd.last_train_stats()["n_gpus"] == 2
    assert got_merges == merges
    assert got_vocab == vocab


@pytest.mark.parametrize("mode,n", [("words", 2), ("words", 5), ("words-gather", 3), ("rounds", 2), ("rounds", 3)])
def test_sharded_gpu_synthetic_vs_oracle(mode, n, ranks):
    import synth_text
    data = synth_text.generate(31, 4_000_000, "ascii").encode("utf-8")
    want = oracle.train_raw(data, 5000, ["<|endoftext|>"])
    ranks(n, mode)
    got = bpe_amd.train_bpe_bytes(data, 5000, ["<|endoftext|>"])
    assert got[1] == want[1]
    assert got[0] == want[0]


def _rccl_worker(port, q, force):
    """One rank, a real RCCL communicator, and a multi-rank exchange forced on: exercises
    ncclCommInitRank and ncclAllReduce (rounds) or ncclAllGather (words) on the library's
    stream exactly as the N>1 bench does."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    for f in force.split("+"):
        os.environ[f] = "1"
    if force == "BPE355_FORCE_COMM":
        os.environ["BPE355_EXCHANGE"] = "rounds"
    try:
        from bpe_amd import train_bpe_bytes
        from bpe_amd.dist import Communicator
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=0, world_size=1)
        o, _vocab, _merges = G.train_expect("corpus_en_1000")
        data = G.input_bytes(o["input"])
        with Communicator.from_torch(0) as comm:
            out = train_bpe_bytes(data, o["vocab_size"], o["special_tokens"], comm=comm)
        q.put(out)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(repr(e))


@pytest.mark.parametrize("force", ["BPE355_FORCE_COMM", "BPE355_FORCE_EXCHANGE",
                                   "BPE355_FORCE_EXCHANGE+BPE355_EXCHANGE_OWNER"])
def test_rccl_comm_single_rank_forced(force):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(port, q, force))
    p.start()
    try:
        out = q.get(timeout=300)
    finally:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert not isinstance(out, str), out
    o, vocab, merges = G.train_expect("corpus_en_1000")
    assert out[1] == merges
    assert out[0] == vocab
