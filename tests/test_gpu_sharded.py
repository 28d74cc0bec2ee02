"""Sharded (multi-rank) training on the GPU, 2 processes sharing one MI355X.

RCCL refuses two ranks on one device, so the collectives go through the library's host-staged
communicator (bpe_comm_init_host) backed by torch.distributed/gloo; everything else is the same
HIP code the RCCL path runs.  Both exchange modes are covered:
  words  (default)  one all-gather of the slabs' unique-word tables, then each rank trains on
                    the union (exchange.hip);
  rounds            local word tables, one all-reduce of the delta cells per merge round, a
                    replicated pair table and argmax.
Every rank must end with exactly the unsharded result.
"""
import multiprocessing as mp
import os

import pytest

import golden_cases as G
from oracle import oracle

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, slab, vocab_size, specials, q, mode):
    import torch.distributed as dist
    from bpe_amd import train_bpe_bytes
    from bpe_amd.dist import HostCommunicator

    os.environ["BPE355_EXCHANGE"] = mode
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=180))
    try:
        with HostCommunicator() as comm:
            vocab, merges = train_bpe_bytes(slab, vocab_size, specials, comm=comm)
        q.put((rank, (vocab, merges)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _safe_cuts(data, world):
    from bpe_amd.dist import slab_bounds
    return slab_bounds(data, world)


def run_sharded(data, world, vocab_size, specials, mode="words"):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cuts = _safe_cuts(data, world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data[cuts[r]:cuts[r + 1]],
                                               vocab_size, specials, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in procs:
            r, v = q.get(timeout=400)
            out[r] = v
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("mode", ["words", "rounds"])
@pytest.mark.parametrize("name", ["corpus_en_1000", "tiny_1200", "synth_mixed_200k"])
def test_sharded_gpu_matches_reference(name, mode):
    o, vocab, merges = G.train_expect(name)
    data = G.input_bytes(o["input"])
    out = run_sharded(data, 2, o["vocab_size"], o["special_tokens"], mode)
    for r in (0, 1):
        assert not isinstance(out[r], str), out[r]
        assert out[r][1] == merges
        assert out[r][0] == vocab


@pytest.mark.parametrize("mode", ["words", "rounds"])
def test_sharded_gpu_synthetic_vs_oracle(mode):
    import synth_text
    data = synth_text.generate(31, 4_000_000, "ascii").encode("utf-8")
    want = oracle.train_raw(data, 5000, ["<|endoftext|>"])
    out = run_sharded(data, 2, 5000, ["<|endoftext|>"], mode)
    for r in (0, 1):
        assert not isinstance(out[r], str), out[r]
        assert out[r][1] == want[1]
        assert out[r][0] == want[0]


def _rccl_worker(port, q, force):
    """One rank, a real RCCL communicator, and a multi-rank exchange forced on: exercises
    ncclCommInitRank and ncclAllReduce (rounds) or ncclAllGather (words) on the library's
    stream exactly as the N>1 bench does."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ[force] = "1"
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


@pytest.mark.parametrize("force", ["BPE355_FORCE_COMM", "BPE355_FORCE_EXCHANGE"])
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
