"""Bucketed collectives over flat buffers.

Reference: one blocking ``all_reduce(AVG)`` per parameter tensor, 57-201 calls per outer step,
interleaved with pageable H2D copies (REF/nanodiloco/diloco/diloco.py:46-50).

Here a flat buffer is cut into a few large buckets (default 128 MiB: xGMI rings are per-link
bound, so a handful of big messages saturate RCCL's channels; tiny per-tensor calls are
latency-bound).  All buckets are issued back-to-back with ``async_op=True``: RCCL runs them on
its own communicator stream (the side HIP stream), ordered after the producer kernels already
queued on the compute stream.  ``wait(i)`` makes the *compute stream* wait for bucket i only --
the host never blocks -- so a consumer kernel on bucket i overlaps the reduction of bucket i+1.

SUM is used for every backend (gloo has no AVG); the 1/W factor is folded into the consumer
kernel (outer Nesterov) or into the loss scale (inner DDP).

Transport (``impl``): ``"rccl"`` -- the own RCCL communicator of the group (parallel/rccl.py,
csrc/comm/nd_comm.cpp: its own high-priority stream, GPU-side event waits, watchdog), the default on
GPU; ``"c10d"`` -- torch's process group (gloo on CPU; ``--comm-impl c10d`` on GPU for A/B).
"""
from __future__ import annotations

import time
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

Range = Tuple[int, int]


def plan_buckets(start: int, end: int, elem_bytes: int, bucket_bytes: int, align: int = 64) -> List[Range]:
    per = max(align, (bucket_bytes // elem_bytes) // align * align)
    out, a = [], start
    while a < end:
        b = min(end, a + per)
        out.append((a, b))
        a = b
    return out


class CommStats:
    def __init__(self):
        self.calls = 0
        self.bytes = 0
        self.host_time_s = 0.0
        self.events: List[Tuple[torch.cuda.Event, torch.cuda.Event]] = []

    def reset(self):
        self.__init__()


class _RcclWork:
    """c10d-Work-like handle of one own-RCCL collective: ``wait()`` = the current stream waits on the GPU."""

    __slots__ = ("comm", "ticket")

    def __init__(self, comm, ticket: int):
        self.comm, self.ticket = comm, ticket

    def wait(self):
        self.comm.wait(self.ticket)
        return True

    def is_completed(self) -> bool:
        return self.comm.query(self.ticket)


class PendingAllReduce:
    def __init__(self, works, ranges, flat):
        self.works = works
        self.ranges = ranges
        self.flat = flat
        self._done = [False] * len(works)

    def wait(self, i: int):
        if not self._done[i]:
            w = self.works[i]
            if w is not None:
                w.wait()
            self._done[i] = True

    def wait_all(self):
        for i in range(len(self.works)):
            self.wait(i)

    def __len__(self):
        return len(self.works)


class FlatCommunicator:
    """Bucketed async all-reduce / broadcast / all-gather on flat buffers for one process group."""

    def __init__(self, group, group_size: int, bucket_mb: float = 128.0, enabled: bool = True, force: bool = False,
                 impl: str = "c10d", device: Optional[torch.device] = None, timeout_s: float = 1800.0):
        """``force``: issue the collectives even for a one-member group (a one-rank process group from
        ``init_distributed(force_pg=True)``), so the communicator path runs on a single GPU.
        ``impl``: "rccl" (own communicator, GPU) or "c10d" (see module doc)."""
        self.group = group
        self.size = group_size
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.enabled = enabled and (group_size > 1 or force)
        self.stats = CommStats()
        self.impl = impl if self.enabled else "none"
        self.rccl = None
        if self.enabled and impl == "rccl":
            from .rccl import communicator_or_fallback
            self.rccl = communicator_or_fallback(group, device, timeout_s)
            if self.rccl is None:  # every member agreed to carry the bulk traffic on c10d instead
                self.impl = "c10d"

    def check(self, what: str = "step boundary"):
        """Raise if the own RCCL communicator failed (see :meth:`parallel.rccl.RcclCommunicator.check`).
        c10d collectives raise from ``Work.wait`` themselves."""
        if self.rccl is not None:
            self.rccl.check(what)

    def all_reduce_async(self, flat: torch.Tensor, ranges: Optional[Sequence[Range]] = None) -> PendingAllReduce:
        if ranges is None:
            ranges = plan_buckets(0, flat.numel(), flat.element_size(), self.bucket_bytes)
        works = []
        t0 = time.perf_counter()
        for a, b in ranges:
            if self.rccl is not None:
                works.append(_RcclWork(self.rccl, self.rccl.all_reduce(flat[a:b])))
                self.stats.calls += 1
                self.stats.bytes += (b - a) * flat.element_size()
            elif self.enabled:
                works.append(dist.all_reduce(flat[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
                self.stats.calls += 1
                self.stats.bytes += (b - a) * flat.element_size()
            else:
                works.append(None)
        self.stats.host_time_s += time.perf_counter() - t0
        return PendingAllReduce(works, list(ranges), flat)

    def all_reduce(self, flat: torch.Tensor, ranges=None, on_bucket: Optional[Callable[[int, int], None]] = None):
        p = self.all_reduce_async(flat, ranges)
        for i, (a, b) in enumerate(p.ranges):
            p.wait(i)
            if on_bucket is not None:
                on_bucket(a, b)
        return p

    def broadcast(self, flat: torch.Tensor, src_group_rank: int = 0):
        if not self.enabled:
            return
        if self.rccl is not None:
            tickets = [self.rccl.broadcast(flat[a:b], src_group_rank)
                       for a, b in plan_buckets(0, flat.numel(), flat.element_size(), self.bucket_bytes)]
            for t in tickets:
                self.rccl.wait(t)
            return
        src = dist.get_global_rank(self.group, src_group_rank) if self.group not in (None, dist.group.WORLD) \
            else src_group_rank
        for a, b in plan_buckets(0, flat.numel(), flat.element_size(), self.bucket_bytes):
            dist.broadcast(flat[a:b], src=src, group=self.group)

    def all_gather_flat(self, flat: torch.Tensor, shard_ranges: Sequence[Range], my_index: int):
        """Every member contributes ``flat[shard_ranges[my_index]]``; all shards end up everywhere.

        Shards must be equal-sized (the ParamStore pads the flat size to make them so)."""
        if not self.enabled:
            return
        a, b = shard_ranges[my_index]
        n = b - a
        if any((y - x) != n for x, y in shard_ranges):
            raise ValueError("all_gather_flat needs equal shards")
        lo = shard_ranges[0][0]
        out = flat[lo:lo + n * len(shard_ranges)]
        if self.rccl is not None:  # in place: this member's shard already sits at its slot of `out`
            self.rccl.wait(self.rccl.all_gather(out))
            return
        mine = flat[a:b].clone()
        dist.all_gather_into_tensor(out, mine, group=self.group)
