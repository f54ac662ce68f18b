"""DiLoCo for ANY ``torch.nn.Module`` with ANY torch inner / outer optimizers.

Capability parity with ``class Diloco`` (REF/nanodiloco/diloco/diloco.py:8-74), which wraps an
arbitrary model through ``model.parameters()`` and the optimizers' ``param_groups``.  The flagship
path (:class:`~nanodiloco_amd.parallel.diloco.Diloco` on our flat-store Llama) is faster; this one
exists so that a user of the reference can bring their own model (an HF ``LlamaForCausalLM``, a
CNN, ...) and their own optimizers unchanged.  ``Diloco(model, ...)`` dispatches here whenever the
model is not our flat-store Llama.

Same math as the reference, laid out for the device instead of per tensor:

  reference (per parameter tensor)              here (per (device, dtype) flat group)
  --------------------------------------------  ----------------------------------------------
  57+ broadcasts at init (:21-22)               one flat broadcast per group, bucketed
  CPU snapshot, pageable, per tensor (:27-32)   one flat device-resident snapshot per group
                                                (``offload_snapshot=True``: one pinned-host buffer)
  H2D + sub + all_reduce(AVG) per tensor        one fused ``sync - theta`` into a flat buffer, a
  (:44-50), blocking                            few large async SUM buckets on RCCL's stream, one
                                                1/W scale; grads are views into that buffer
  theta <- snapshot, outer.step, zero_grad      same (a single flat copy per group)
  clip(1.0) + step + sched + zero_grad (:56-60) same, torch ``clip_grad_norm_`` (foreach)
  avg_sync_time (always 0, dead code)           real wall seconds per outer step
"""
from __future__ import annotations

import time
from collections import OrderedDict
from typing import List, Optional

import torch
import torch.distributed as dist

from ..utils.schedule import cosine_with_warmup
from .comm import FlatCommunicator


def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class _Group:
    """Parameters of one (device, dtype): flat snapshot + flat pseudo-gradient buffer."""

    def __init__(self, params: List[torch.Tensor], offload: bool, comm_dtype: Optional[torch.dtype]):
        self.params = params
        self.numels = [p.numel() for p in params]
        n = sum(self.numels)
        dev, dt = params[0].device, params[0].dtype
        self.comm_dtype = comm_dtype or dt
        self.delta = torch.empty(n, dtype=self.comm_dtype, device=dev)
        pin = offload and torch.cuda.is_available() and dev.type == "cuda"
        self.snapshot = torch.empty(n, dtype=dt, device="cpu" if offload else dev, pin_memory=pin)
        self.flat_tmp = None

    def views(self, flat: torch.Tensor):
        out, a = [], 0
        for p, k in zip(self.params, self.numels):
            out.append(flat[a:a + k].view_as(p))
            a += k
        return out

    @torch.no_grad()
    def gather(self) -> torch.Tensor:
        return torch.cat([p.detach().reshape(-1) for p in self.params])

    @torch.no_grad()
    def scatter(self, flat: torch.Tensor):
        torch._foreach_copy_([p.data for p in self.params], self.views(flat))

    @torch.no_grad()
    def take_snapshot(self):
        # a device -> pinned-host copy is only asynchronous with respect to the host: block on it so a
        # state_dict() / checkpoint taken right after (before any outer step) never reads a partial
        # snapshot; device-resident snapshots stay stream-ordered
        host = self.snapshot.device.type == "cpu"
        self.snapshot.copy_(self.gather(), non_blocking=not host)


class ModuleDiloco:
    """Same constructor and methods as the reference ``Diloco``; extra keyword arguments:

    * ``comm_dtype``: pseudo-gradient transport dtype (default: the parameter dtype, as the reference);
    * ``offload_snapshot``: keep theta_sync in pinned host memory (the reference always does; the
      default here keeps it in HBM -- 288 GB per MI355X);
    * ``bucket_mb``: all-reduce bucket size;
    * ``max_grad_norm``: inner clip (the reference hard-codes 1.0)."""

    def __init__(self, model: torch.nn.Module, inner_optimizer: torch.optim.Optimizer,
                 outer_optimizer: torch.optim.Optimizer, warmup_steps: int, total_steps: int,
                 inner_steps: int = 100, outer_steps: int = 10, comm_dtype: Optional[torch.dtype] = None,
                 offload_snapshot: bool = False, bucket_mb: float = 128.0, max_grad_norm: float = 1.0,
                 broadcast_init: bool = True):
        self.model = model
        self.inner_optimizer = inner_optimizer
        self.outer_optimizer = outer_optimizer
        self.inner_steps = inner_steps
        self.outer_steps = outer_steps
        self.max_grad_norm = max_grad_norm
        self.scheduler = torch.optim.lr_scheduler.LambdaLR(
            inner_optimizer, lambda s: cosine_with_warmup(s, warmup_steps, total_steps))
        self.world = dist.get_world_size() if _dist_on() else 1
        self.comm = FlatCommunicator(None, self.world, bucket_mb)
        outer_params = [p for g in outer_optimizer.param_groups for p in g["params"]]
        inner_params = [p for g in inner_optimizer.param_groups for p in g["params"]]
        if len(outer_params) != len(inner_params) or any(a is not b for a, b in zip(outer_params, inner_params)):
            raise ValueError("inner and outer optimizers must hold the same parameters in the same order")
        groups = OrderedDict()
        for p in outer_params:
            groups.setdefault((p.device, p.dtype), []).append(p)
        self.groups = [_Group(ps, offload_snapshot, comm_dtype) for ps in groups.values()]
        if broadcast_init and self.world > 1:
            for g in self.groups:
                flat = g.gather()
                self.comm.broadcast(flat, 0)
                g.scatter(flat)
        for g in self.groups:
            g.take_snapshot()
        self._sync_time = 0.0
        self._sync_calls = 0
        self.local_step = 0

    # ------------------------------------------------------------------ reference API
    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def train(self):
        self.model.train()

    def eval(self):
        self.model.eval()

    @property
    def avg_sync_time(self) -> float:
        return self._sync_time / self._sync_calls if self._sync_calls > 0 else 0.0

    def current_lr(self) -> float:
        return self.inner_optimizer.param_groups[0]["lr"]

    def inner_step(self):
        params = [p for g in self.groups for p in g.params]
        torch.nn.utils.clip_grad_norm_(params, max_norm=self.max_grad_norm)
        self.inner_optimizer.step()
        self.scheduler.step()
        self.inner_optimizer.zero_grad()
        self.local_step += 1

    @torch.no_grad()
    def outer_step(self):
        t0 = time.perf_counter()
        pend = []
        for g in self.groups:
            sync = g.snapshot.to(g.delta.device, non_blocking=True)
            torch.sub(sync, g.gather(), out=g.delta) if g.delta.dtype == sync.dtype else \
                g.delta.copy_(sync - g.gather())
            pend.append((g, sync, self.comm.all_reduce_async(g.delta)))
        for g, sync, p in pend:
            p.wait_all()
            if self.world > 1:
                g.delta.mul_(1.0 / self.world)  # SUM -> AVG (gloo has no AVG)
            grad = g.delta if g.delta.dtype == sync.dtype else g.delta.to(sync.dtype)
            for prm, v in zip(g.params, g.views(grad)):
                prm.grad = v
            g.scatter(sync)  # theta <- theta_sync
        self.outer_optimizer.step()
        self.outer_optimizer.zero_grad()
        for g in self.groups:
            g.take_snapshot()
        if any(g.delta.is_cuda for g in self.groups):
            torch.cuda.synchronize()  # wall time of the whole outer step (reference semantics)
        self._sync_time += time.perf_counter() - t0
        self._sync_calls += 1

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self):
        return {"snapshots": [g.snapshot for g in self.groups], "outer": self.outer_optimizer.state_dict(),
                "inner": self.inner_optimizer.state_dict(), "scheduler": self.scheduler.state_dict(),
                "local_step": self.local_step}

    def load_state_dict(self, d):
        for g, s in zip(self.groups, d["snapshots"]):
            g.snapshot.copy_(s)
        self.outer_optimizer.load_state_dict(d["outer"])
        if "inner" in d:  # optional, as in Diloco.load_state_dict (AdamW state may be kept per rank)
            self.inner_optimizer.load_state_dict(d["inner"])
        self.scheduler.load_state_dict(d["scheduler"])
        self.local_step = int(d["local_step"])
