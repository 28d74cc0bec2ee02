"""The one-process-per-GPU path (torchrun: bpe_train_file_comm, reference entry
models/tokenizer/train.py:142) with two real processes on this box's one card.

RCCL refuses two ranks on one device, so the ranks' collectives go through the library's
host-staged communicator (bpe_comm_init_host) backed by torch.distributed/gloo; the file split,
each process's read of its share, the error agreement, the word exchange and the merge loop are
the code an 8-GPU torchrun job executes.  Each process binds the HIP runtime on its own (the
check _lib._check_runtime makes at load), and both must end with the oracle's result.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

import gpt2_files
from oracle import oracle

pytestmark = pytest.mark.gpu

EOT = ["<|endoftext|>"]


def _worker(rank, world, port, path, vocab_size, q, mode):
    import datetime
    import torch.distributed as dist
    os.environ["BPE355_EXCHANGE"] = mode
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    try:
        from bpe_amd import train_bpe, _lib
        from bpe_amd.dist import HostCommunicator
        from bpe_amd.train import last_train_stats
        with HostCommunicator() as comm:
            vocab, merges = train_bpe(path, vocab_size, EOT, comm=comm, split_file=True)
        q.put((rank, (vocab, merges, last_train_stats()["n_gpus"], dict(_lib.RUNTIME))))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run(path, world, vocab_size, mode):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(path), vocab_size, q, mode))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in procs:
            r, v = q.get(timeout=240)
            out[r] = v
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


def test_two_processes_file_comm_words(tmp_path):
    buf = np.empty(4_000_000, dtype=np.uint8)
    from bpe_amd import _lib
    assert _lib.lib().bpe_synth_corpus_host(buf.ctypes.data, buf.size, 41, 0, 0, 8) == 0
    data = buf.tobytes() + (gpt2_files.FIXTURES / "corpus.en").read_bytes()
    path = tmp_path / "c.txt"
    path.write_bytes(data)
    want = oracle.train_raw(data, 3000, EOT)
    out = _run(path, 2, 3000, "words")
    for r in (0, 1):
        assert not isinstance(out[r], str), out[r]
        vocab, merges, n_gpus, rt = out[r]
        assert n_gpus == 2
        assert rt["runtime"] // 10_000_000 == rt["compiled"] // 10_000_000
        assert merges == want[1]
        assert vocab == want[0]
