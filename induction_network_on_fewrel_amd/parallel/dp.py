"""Episode-level data parallelism over RCCL (xGMI) -- one process per GPU.

The reference has no distribution at all (one tf.Session, model/base.py:121-123). Here every rank
samples its own episodes (rank-folded seed), computes gradients into ONE flat fp32 buffer
(ops/optim.py::FlatParams) and the buffer is all-reduced in a few large buckets; the fused optimizer
then runs identically on every rank so parameters never diverge (checked by ``params_in_sync``).

Sizing for MI355X / xGMI: the default BiLSTM model's gradient is 0.69 MB -> a single bucket (the
collective is pure latency, so fewer/larger steps = more episodes per GPU is what amortises it).
Large models (BERT encoder) are bucketed at ``bucket_mb`` (default 64 MB: 7 xGMI links x ~153 GB/s
per GPU make a ring all-reduce of 64 MB ~0.5 ms, large enough to run at link rate, small enough to
overlap with the rest of backward). ``torch.distributed`` backend "nccl" is RCCL on ROCm; "gloo" is
used on CPU (tests).  ``INA_COMM=native`` keeps gloo for the control plane and moves every GPU tensor
collective onto the C++ RCCL communicator of csrc/comm_bindings.cpp (parallel/native_comm.py).
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist


def _native_op(op) -> str:
    """torch.distributed ReduceOp -> the native communicator's op name (csrc/comm_bindings.cpp); ops it
    has no equivalent for raise instead of silently becoming a sum."""
    if op is None or op == dist.ReduceOp.SUM:
        return "sum"
    for name in ("MAX", "MIN", "PRODUCT"):
        if op == getattr(dist.ReduceOp, name):
            return {"MAX": "max", "MIN": "min", "PRODUCT": "prod"}[name]
    raise ValueError(f"native communicator: unsupported reduce op {op}")


class DistContext:
    def __init__(self, rank: int = 0, world: int = 1, local_rank: int = 0, device: Optional[torch.device] = None,
                 backend: Optional[str] = None):
        self.rank, self.world, self.local_rank = rank, world, local_rank
        self.device = device or torch.device("cpu")
        self.backend = backend
        self.initialized = False
        self.native = None   # NativeComm when INA_COMM=native (GPU tensors), gloo for the rest

    @classmethod
    def from_env(cls, device: str = "auto", timeout_s: int = 1800) -> "DistContext":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        use_cuda = (device == "cuda") or (device == "auto" and torch.cuda.is_available())
        if use_cuda:
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
            dev = torch.device("cuda", torch.cuda.current_device())
        else:
            dev = torch.device("cpu")
        ctx = cls(rank, world, local_rank, dev, None)
        # INA_FORCE_DIST=1: initialise the process group even at world size 1, so the collective path
        # (RCCL all-reduce / broadcast / barrier) runs on a one-GPU box (tests/test_dp_gpu.py)
        if world > 1 or os.environ.get("INA_FORCE_DIST") == "1":
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            # INA_DIST_BACKEND=gloo: several ranks sharing ONE GPU (RCCL refuses duplicate devices) --
            # the one-card rehearsal of the multi-rank GPU step (tests/test_dp_gpu.py)
            native = use_cuda and os.environ.get("INA_COMM") == "native"
            backend = os.environ.get("INA_DIST_BACKEND") or ("nccl" if use_cuda and not native else "gloo")
            kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
            if use_cuda and backend == "nccl":
                kw["device_id"] = dev
            if not dist.is_initialized():
                dist.init_process_group(**kw)
            ctx.backend = backend
            ctx.initialized = True
            if native:
                from .native_comm import NativeComm
                ctx.native = NativeComm(rank, world, dev, dist.distributed_c10d._get_default_store())
        return ctx

    @property
    def comm_name(self) -> str:
        """Data-plane backend of the GPU collectives ("rccl-native", "nccl" = torch RCCL, "gloo", "none")."""
        if not self.initialized:
            return "none"
        return "rccl-native" if self.native is not None else str(self.backend)

    # ------------------------------------------------------------------
    @property
    def is_main(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.initialized:
            if self.backend == "nccl":
                idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
                dist.barrier(device_ids=[idx])
            else:
                dist.barrier()

    def _native_ok(self, t: torch.Tensor) -> bool:
        return self.native is not None and t.is_cuda

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.initialized:
            if self._native_ok(t):
                self.native.broadcast_(t, src)
                self.native.wait()
            else:
                dist.broadcast(t, src)
        return t

    def allreduce_(self, t: torch.Tensor, op=None) -> torch.Tensor:
        if self.initialized:
            if self._native_ok(t):
                self.native.allreduce_(t, _native_op(op))
                self.native.wait()
            else:
                dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
        return t

    def allreduce_async_(self, t: torch.Tensor):
        """Sum-all-reduce started now; returns a handle whose ``wait()`` orders the caller's stream."""
        if self._native_ok(t):
            from .native_comm import _NativeWork
            self.native.allreduce_(t, "sum")
            return _NativeWork(self.native)
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)

    def allreduce_buckets_(self, flat: torch.Tensor, bucket_mb: float = 64.0) -> None:
        """Sum-all-reduce a flat buffer in ``bucket_mb`` chunks, all issued async then waited."""
        if not self.initialized or flat.numel() == 0:
            return
        n = max(1, int(bucket_mb * 1024 * 1024 // flat.element_size()))
        chunks = [flat[off:off + n] for off in range(0, flat.numel(), n)]
        if self._native_ok(flat):   # one grouped RCCL launch for all buckets
            self.native.allreduce_many_(chunks, "sum")
            self.native.wait()
            return
        works: List = [dist.all_reduce(c, op=dist.ReduceOp.SUM, async_op=True) for c in chunks]
        for w in works:
            w.wait()

    def overlap(self, flat: torch.Tensor, spans: List[tuple], scale: float = 1.0) -> "OverlapAllReduce":
        return OverlapAllReduce(self, flat, spans, scale)

    def max_scalar(self, x: float) -> float:
        if not self.initialized:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def mean_scalars(self, xs: List[float]) -> List[float]:
        if not self.initialized:
            return [float(x) for x in xs]
        t = torch.tensor([float(x) for x in xs], dtype=torch.float64,
                         device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return [float(v) / self.world for v in t.tolist()]

    def all_gather_objects(self, obj) -> list:
        """Every rank's ``obj`` (picklable, small), in rank order, on every rank."""
        if not self.initialized:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    def params_in_sync(self, flat: torch.Tensor) -> bool:
        """Max-abs difference of the flat parameters across ranks is zero."""
        if not self.initialized:
            return True
        ref = flat.detach().clone()
        self.broadcast_(ref, 0)
        diff = (flat.detach() - ref).abs().max().item() if flat.numel() else 0.0
        return self.max_scalar(diff) == 0.0

    def destroy(self) -> None:
        if self.native is not None:
            self.native.sync()
            self.native.destroy()
            self.native = None
        if self.initialized and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized = False


class OverlapAllReduce:
    """Backward-overlapped bucket all-reduce (DDP-style) over one flat gradient buffer.

    ``spans`` = [(offset, numel), ...] buckets of the flat buffer, typically one per transformer layer
    (~28 MB fp32 for BERT-base: large enough to run RCCL at xGMI link rate, issued while the layers
    below are still in backward).  The model calls ``ready(i)`` as soon as bucket i's gradients are
    final; the all-reduce is queued on the process group's stream behind an event on the compute
    stream, so it runs concurrently with the remaining backward kernels.  ``finish()`` reduces every
    part of the buffer not covered by a launched bucket and waits for all of them.
    """

    def __init__(self, ctx: DistContext, flat: torch.Tensor, spans: List[tuple], scale: float = 1.0):
        self.ctx, self.flat, self.spans = ctx, flat, list(spans)
        self.works: List = []
        self.launched = [False] * len(self.spans)
        self.scale = scale

    def ready(self, i: int) -> None:
        if not self.ctx.initialized or self.launched[i]:
            return
        off, n = self.spans[i]
        self.launched[i] = True
        self.works.append(self.ctx.allreduce_async_(self.flat[off:off + n]))

    def finish(self) -> None:
        if not self.ctx.initialized:
            return
        covered = sorted(self.spans[i] for i in range(len(self.spans)) if self.launched[i])
        pos = 0
        rest = []
        for off, n in covered:
            if off > pos:
                rest.append((pos, off - pos))
            pos = max(pos, off + n)
        if pos < self.flat.numel():
            rest.append((pos, self.flat.numel() - pos))
        for off, n in rest:
            self.works.append(self.ctx.allreduce_async_(self.flat[off:off + n]))
        for w in self.works:
            w.wait()
        self.works = []
