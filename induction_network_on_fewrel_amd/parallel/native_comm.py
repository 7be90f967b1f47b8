"""Native RCCL communicator (csrc/comm_bindings.cpp) -- the C++ data plane of SURVEY 7.1 / 5.8.

``INA_COMM=native`` splits the distributed runtime in two:
  * control plane: a ``gloo`` process group (barriers, host scalars / objects, the TCP store);
  * data plane:    ONE RCCL communicator per process created here from C++ (``ncclCommInitRank``),
                   bootstrapped by rank 0 publishing the 128-byte ``ncclUniqueId`` in the store.
Gradient buckets are all-reduced on the communicator's own HIP stream: the enqueue waits on an event
of the compute stream and ``wait()`` makes the compute stream wait on the comm stream, so a bucket
launched in the middle of backward overlaps the rest of it without host synchronisation.

The default (``INA_COMM`` unset) is ``torch.distributed`` with the ``nccl`` backend (also RCCL).
"""
from __future__ import annotations

from typing import List

import torch

from ..ops._ext import ops

_UID_KEY = "ina/rccl_unique_id"


class NativeComm:
    def __init__(self, rank: int, world: int, device: torch.device, store, tag: str = "0"):
        o = ops()
        key = f"{_UID_KEY}/{tag}"
        if rank == 0:
            uid = o.comm_unique_id()
            store.set(key, bytes(uid.numpy().tobytes()))
        else:
            uid = torch.frombuffer(bytearray(store.get(key)), dtype=torch.uint8).clone()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        self.h = int(o.comm_init(uid, rank, world, idx))
        self.rank, self.world, self.device = rank, world, device

    def info(self) -> dict:
        r, w, d, v = ops().comm_info(self.h)
        return dict(rank=r, world=w, device=d, rccl_version=v)

    # ------------------------------------------------------------------ collectives (async on the comm stream)
    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> None:
        ops().comm_allreduce_(self.h, t, op)

    def allreduce_many_(self, ts: List[torch.Tensor], op: str = "sum") -> None:
        if ts:
            ops().comm_allreduce_many_(self.h, ts, op)

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> None:
        ops().comm_broadcast_(self.h, t, root)

    def wait(self) -> None:
        """The caller's current stream waits for every collective enqueued so far (host does not block)."""
        ops().comm_wait(self.h)

    def sync(self) -> None:
        """Host-blocking drain + asynchronous-error check (RCCL failure detection)."""
        ops().comm_sync(self.h)

    def destroy(self) -> None:
        if self.h >= 0:
            ops().comm_destroy(self.h)
            self.h = -1


class _NativeWork:
    """The ``wait()`` handle the DistContext bucket paths expect from ``dist.all_reduce(async_op=True)``."""

    def __init__(self, comm: NativeComm):
        self.comm = comm

    def wait(self) -> None:
        self.comm.wait()
