"""Process-group bootstrap and the two-level (inner DDP x outer DiLoCo) topology.

Reference: ``dist.init_process_group("nccl")`` + ``set_device(LOCAL_RANK)``
(REF/nanodiloco/training_utils/utils.py:41-43), one worker per GPU, one flat group.

Here:
* backend ``auto`` = ``nccl`` (RCCL over xGMI on MI355X) when GPUs exist, else ``gloo`` (fixes the
  reference's hard-coded NCCL, SURVEY.md Q8 -- BASELINE config 1 runs on CPU/gloo);
* world size 1 without torchrun works with no process group at all (collectives become no-ops);
  ``force_pg=True`` creates a one-rank process group anyway (in-memory store, no rendezvous) and
  keeps every collective call live, so the RCCL path -- communicator init, bucketed async
  all-reduce, broadcast, sub-group all-gather, device barrier -- runs on a one-GPU box too;
* RCCL groups use a high-priority HIP stream (``_pg_options``) so the side-stream collectives overlap
  the compute stream instead of queueing behind it;
* ``inner_dp = K`` splits the world into W/K DiLoCo workers of K GPUs each (BASELINE config 3).
  Inner groups are blocks of K consecutive ranks (xGMI neighbours on one node); outer groups are
  the ranks with the same index inside their inner group, so an outer all-reduce of shard r only
  involves the r-th GPU of every worker.
"""
from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = dataclasses.field(default_factory=lambda: torch.device("cpu"))
    backend: str = "none"
    inner_dp: int = 1
    inner_rank: int = 0
    worker: int = 0           # DiLoCo worker index  (rank // inner_dp)
    num_workers: int = 1      # world_size // inner_dp
    force_collectives: bool = False  # world size 1 with a live process group (force_pg)
    # with force_collectives: also run the inner-DDP gradient all-reduce of a ONE-GPU worker (a no-op in the
    # math, 12+ collectives per inner step: tests only -- the bench / trainer keep it off, so a one-rank
    # headline step costs what a DiLoCo worker of the N=8 run costs)
    force_inner_ddp: bool = False
    comm_impl: str = "none"   # bulk-traffic transport: "rccl" (own communicator, parallel/rccl.py) | "c10d"
    timeout_s: float = 1800.0
    inner_group: Optional[object] = None
    outer_group: Optional[object] = None
    world_group: Optional[object] = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1 or self.force_collectives

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def _env_int(k, d):
    v = os.environ.get(k)
    return int(v) if v not in (None, "") else d


def _pg_options(backend: str, high_priority: bool, timeout: Optional[datetime.timedelta] = None):
    """RCCL process groups run their collectives on a HIGH-PRIORITY HIP stream: the
    bucketed outer all-reduce that ``--overlap-outer`` issues beside the next round's first inner step
    (and the inner-DDP gradient buckets beside the backward) is then scheduled ahead of the compute
    queue's kernels when both are ready.  The options carry the group's timeout too (torch warns when an
    options object's timeout differs from the ``timeout`` argument it then overrides it with)."""
    if backend != "nccl" or not high_priority or os.environ.get("ND_COMM_PRIORITY", "high") == "normal":
        return None
    try:
        from torch.distributed import ProcessGroupNCCL
    except ImportError:  # torch built without RCCL
        return None
    o = ProcessGroupNCCL.Options(is_high_priority_stream=True)
    if timeout is not None:
        o._timeout = timeout
    return o


def worker_group_namespace(store, rank: int, world: int, timeout_s: float = 300.0) -> str:
    """A key namespace unique to THIS worker group, agreed by all its ranks through ``store``.

    torchrun's agent store outlives the worker groups it starts: after a failure restart
    (TORCHELASTIC_RESTART_COUNT + 1) and after a membership change of an elastic ``--nnodes=min:max`` job
    (the count does NOT move), the new group sees every key the old one wrote -- gloo peer addresses, the
    own RCCL communicators' unique ids -- and would read them.  Rank 0 of the group draws a fresh nonce and
    hands it to every other rank through keys that cannot be stale:

    * rank r counts its incarnations (``add("nd_ns/inc/r", 1)`` = i_r: a number no earlier process of rank
      r had), points ``nd_ns/req/r`` at it and blocks on ``nd_ns/ans/r/<i_r>``, a key nothing wrote before;
    * rank 0 answers whatever incarnation ``nd_ns/req/r`` points at, and repeats until rank r acknowledges
      with rank 0's OWN nonce -- a leftover pointer or acknowledgement of a dead group carries another
      nonce, so it is answered (harmlessly) but never taken for this group's.

    World size may differ between groups and workers may have died at any point: nothing counts arrivals."""
    import time
    import uuid
    deadline = time.monotonic() + timeout_s
    inc = store.add(f"nd_ns/inc/{rank}", 1)
    if rank == 0:
        nonce = f"{inc}-{uuid.uuid4().hex[:12]}"
        todo = set(range(1, world))
        while todo:
            for r in sorted(todo):
                if not store.check([f"nd_ns/req/{r}"]):
                    continue
                i_r = store.get(f"nd_ns/req/{r}").decode()
                store.set(f"nd_ns/ans/{r}/{i_r}", nonce)
                if store.check([f"nd_ns/ack/{r}/{i_r}"]) and store.get(f"nd_ns/ack/{r}/{i_r}").decode() == nonce:
                    todo.discard(r)
            if todo:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"worker-group namespace: ranks {sorted(todo)} never checked in")
                time.sleep(0.005)
        return nonce
    store.set(f"nd_ns/req/{rank}", str(inc))
    nonce = store.get(f"nd_ns/ans/{rank}/{inc}").decode()  # blocks (store timeout) until rank 0 answers
    store.set(f"nd_ns/ack/{rank}/{inc}", nonce)
    return nonce


def comm_stream_high_priority(group=None) -> Optional[bool]:
    """Whether the RCCL backend of ``group`` (default: WORLD) was created with a high-priority stream
    (None: no RCCL backend)."""
    if not dist.is_initialized():
        return None
    g = group if group is not None else dist.group.WORLD
    try:
        be = g._get_backend(torch.device("cuda", torch.cuda.current_device()))
        return bool(be.options.is_high_priority_stream)
    except (RuntimeError, AttributeError):
        return None


def _resolve_comm_impl(comm_impl: str, backend: str) -> str:
    """auto: the own RCCL communicator whenever the backend is RCCL and libnd_comm.so is built; c10d
    otherwise (gloo / CPU)."""
    from . import rccl
    if comm_impl == "auto":
        return "rccl" if backend == "nccl" and rccl.available() else "c10d"
    if comm_impl == "rccl" and backend != "nccl":
        raise ValueError("--comm-impl rccl needs the nccl (RCCL) backend")
    if comm_impl == "rccl" and not rccl.available():
        raise RuntimeError(f"--comm-impl rccl but {rccl.LIB_PATH} is missing (python -m nanodiloco_amd.csrc.build)")
    if comm_impl not in ("rccl", "c10d"):
        raise ValueError(comm_impl)
    return comm_impl


def claim_compute_queues(dev: torch.device) -> None:
    """Give the compute stream and the weight-gradient side stream their HIP hardware queues BEFORE any
    communicator exists.  HIP maps streams onto its hardware queues (GPU_MAX_HW_QUEUES, 4 here) in creation
    / first-use order; when RCCL's and c10d's streams are created first, the two compute streams land on
    other queues and the overlapped backward ran 2 % slower (bench.py, one-rank group vs none, with the
    side stream on: 330.6 vs 323.6 ms per step; serialized: equal -- round 5, gpurun_out r5d / r5g)."""
    torch.zeros(1, device=dev).add_(1)  # first use of the compute (null) stream
    from ..ops.linear import _side_stream
    side = _side_stream(dev)
    with torch.cuda.stream(side):
        torch.zeros(1, device=dev).add_(1)
    torch.cuda.synchronize(dev)


def init_distributed(backend: str = "auto", inner_dp: int = 1, device: Optional[str] = None,
                     timeout_s: float = 1800.0, force_pg: bool = False, high_priority: bool = True,
                     comm_impl: str = "auto") -> DistEnv:
    rank = _env_int("RANK", 0)
    world = _env_int("WORLD_SIZE", 1)
    local_rank = _env_int("LOCAL_RANK", 0)
    use_cuda = torch.cuda.is_available() and device != "cpu"
    if backend == "auto":
        backend = "nccl" if use_cuda else "gloo"
    if backend == "nccl" and not use_cuda:
        raise RuntimeError("backend nccl (RCCL) requested but no GPU is visible")
    if use_cuda:
        torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
        dev = torch.device("cuda", torch.cuda.current_device())
        claim_compute_queues(dev)
    else:
        dev = torch.device("cpu")
    if world % inner_dp:
        raise ValueError(f"world size {world} not divisible by inner_dp {inner_dp}")
    env = DistEnv(rank=rank, world_size=world, local_rank=local_rank, device=dev, backend="none",
                  inner_dp=inner_dp, inner_rank=rank % inner_dp, worker=rank // inner_dp,
                  num_workers=world // inner_dp, timeout_s=timeout_s)
    if world == 1 and not force_pg:
        return env
    # failure detection: a hung / failed collective surfaces as an error on every rank (instead of a
    # silent hang) after `timeout_s`; torchrun --max-restarts + --resume then restart from the last
    # outer-step checkpoint.
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    timeout = datetime.timedelta(seconds=timeout_s)
    # one FRESH Options object per group: torch's _new_process_group_helper writes the group's timeout,
    # split parent / colour, global ranks and name into the object it is given and the backend keeps a
    # pointer to it, so a shared object would let every later new_group overwrite WORLD's settings
    if not dist.is_initialized():
        kw = dict(backend=backend, timeout=timeout)
        if backend == "nccl":
            kw["device_id"] = dev  # eager RCCL communicator init
            kw["pg_options"] = _pg_options(backend, high_priority, timeout)
        launched = "TORCHELASTIC_RUN_ID" in os.environ and "MASTER_PORT" in os.environ
        if world == 1 and not launched:
            # one rank outside torchrun: nothing to rendezvous with (a stray MASTER_ADDR without
            # MASTER_PORT / RANK must not send us into an env:// rendezvous)
            kw.update(store=dist.HashStore(), rank=0, world_size=1)
        elif launched and os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
            # torchrun's agent store is shared by every worker group it starts (failure restarts AND
            # elastic membership changes, which do not move TORCHELASTIC_RESTART_COUNT), while torch's
            # env:// handler assumes a fresh store per attempt and adds no prefix
            # (rendezvous._create_c10d_store): a new group would read the old one's keys (gloo peer
            # addresses: "Connection refused"; the own RCCL unique ids).  Every group, the first one
            # included, works in a namespace of its own (worker_group_namespace).
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, False,
                                 timeout=timeout)
            ns = worker_group_namespace(base, rank, world, timeout_s)
            kw.update(store=dist.PrefixStore(f"nd_group_{ns}", base), rank=rank, world_size=world)
        dist.init_process_group(**kw)
    env.backend = backend
    env.comm_impl = _resolve_comm_impl(comm_impl, backend)
    env.force_collectives = world == 1
    env.world_group = dist.group.WORLD
    if inner_dp == 1:
        env.inner_group = None
        env.outer_group = dist.group.WORLD
    else:
        for w in range(env.num_workers):  # every rank must create every group, in the same order
            ranks = list(range(w * inner_dp, (w + 1) * inner_dp))
            g = dist.new_group(ranks, timeout=timeout, pg_options=_pg_options(backend, high_priority, timeout))
            if w == env.worker:
                env.inner_group = g
        if env.num_workers > 1:
            for r in range(inner_dp):
                ranks = list(range(r, world, inner_dp))
                g = dist.new_group(ranks, timeout=timeout, pg_options=_pg_options(backend, high_priority, timeout))
                if r == env.inner_rank:
                    env.outer_group = g
    return env


def destroy_distributed(abort: bool = False):
    """``abort``: called while an exception propagates -- the own RCCL communicators abort instead of
    draining (a collective may be waiting on a peer that will never arrive)."""
    from .rccl import destroy_communicators
    destroy_communicators(abort)
    if dist.is_initialized():
        dist.destroy_process_group()


def barrier(env: DistEnv):
    if env.is_distributed:
        if env.backend == "nccl":
            dist.barrier(device_ids=[env.device.index])
        else:
            dist.barrier()
