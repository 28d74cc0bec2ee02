"""Communicators for sharded training (one process per GPU).

The default exchange is ONE all-gather of the ranks' unique-word tables after the local counts;
every rank then runs the merge loop on the union.  The per-round protocol
(BPE355_EXCHANGE=rounds: one int64 sum all-reduce of the pair-count delta cells per merge round,
SURVEY.md 8e) is kept and tested but slower.  Two ways to provide the collectives:

  Communicator.from_torch()   RCCL over xGMI (bpe_comm_init): the id is created on rank 0 and
                              broadcast through an initialised torch.distributed group.
  HostCommunicator(group)     host-staged: the library hands a host buffer to a callback that
                              all-reduces it with torch.distributed (e.g. gloo); the library's
                              all-gather goes through it as a sum of zero-padded segments.  For tests and
                              for several ranks sharing one GPU, which RCCL refuses.

Either is passed as `comm=` to train_bpe / train_bpe_bytes / train_bpe_device and must be
closed (or used as a context manager) after training.
"""
from __future__ import annotations

import ctypes
import os

from . import _lib


class Communicator:
    def __init__(self, handle: ctypes.c_void_p, nranks: int, rank: int):
        self.handle = handle
        self.nranks = nranks
        self.rank = rank

    @classmethod
    def from_torch(cls, device: int | None = None, group=None) -> "Communicator":
        import torch.distributed as dist
        L = _lib.lib()
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        uid = ctypes.create_string_buffer(128)
        if rank == 0:
            _lib.check(L.bpe_comm_unique_id(uid), "bpe_comm_unique_id")
        obj = [bytes(uid.raw) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        h = ctypes.c_void_p()
        _lib.check(L.bpe_comm_init(obj[0], world, rank, device, ctypes.byref(h)), "bpe_comm_init")
        return cls(h, world, rank)

    def close(self):
        if self.handle is not None and self.handle.value:
            _lib.lib().bpe_comm_free(self.handle)
        self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class HostCommunicator(Communicator):
    def __init__(self, group=None, device: int = 0):
        import numpy as np
        import torch
        import torch.distributed as dist
        L = _lib.lib()

        @_lib.HOST_ALLREDUCE_FN
        def _allreduce(_ctx, buf, count):
            try:
                t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,)))  # shares memory
                dist.all_reduce(t, group=group)
                return 0
            except Exception:  # noqa: BLE001 -- reported as BPE_E_RCCL by the library
                return -1

        self._fn = _allreduce          # keep the callback alive as long as the handle
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        h = ctypes.c_void_p()
        _lib.check(L.bpe_comm_init_host(_allreduce, None, world, rank, device, ctypes.byref(h)),
                   "bpe_comm_init_host")
        super().__init__(h, world, rank)


def slab_bounds(data: bytes, nranks: int) -> list[int]:
    """Cut points [0, c1, ..., len] that split `data` into nranks slabs at safe points."""
    L = _lib.lib()
    n = len(data)
    return [0] + [L.bpe_safe_split(data, n, n * r // nranks) for r in range(1, nranks)] + [n]
