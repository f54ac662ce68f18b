"""DiLoCo: H local AdamW steps per worker, then an outer Nesterov step on the averaged
pseudo-gradient.  Capability parity with ``class Diloco`` (REF/nanodiloco/diloco/diloco.py:7-74):

  reference                                      here
  ---------------------------------------------  ------------------------------------------------
  per-tensor broadcast from rank 0 (:21-22)      one bucketed flat broadcast of the fp32 master
  CPU snapshot, pageable, per tensor (:27-32)    device-resident flat fp32 ``sync`` (288 GB HBM);
                                                 ``offload_snapshot=True`` keeps it in pinned host
  per-tensor H2D, sub, all_reduce(AVG), reset    ``nd_pseudograd`` -> bucketed async all-reduce(SUM)
  then SGD-Nesterov step + zero_grad (:46-53)    on RCCL's stream -> per-bucket fused
                                                 ``nd_outer_nesterov`` (1/W, momentum, Nesterov,
                                                 theta, sync, bf16 shadow in one pass), overlapping
                                                 the reduction of the next bucket
  clip + AdamW + scheduler + zero_grad (:56-60)  fused clip+AdamW kernels + host cosine schedule
  avg_sync_time always 0 (:62-64, dead)          real: wall time of every outer step (host) and
                                                 device time of its collectives (HIP events)

Extensions (north star):
* ``comm_dtype=bf16``: pseudo-gradients travel in bf16 (half the bytes / outer step);
* ``overlap=True``: the all-reduce is launched at the boundary and overlaps the next inner step;
  it is applied one step late as theta <- theta_outer + (theta_local_now - theta_local_boundary)
  (streaming / delayed outer update).  ``overlap=False`` is bit-faithful to the reference order;
* ``inner_dp > 1`` (two-level): the W/K workers' outer all-reduce is sharded over the K GPUs of a
  worker (each reduces 1/K of the pseudo-gradient over its outer group, then the worker
  all-gathers the updated weights), so cross-worker bytes per GPU drop by K.
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from .. import ops
from ..models.llama import LlamaForCausalLM
from ..optim import FlatAdamW, FlatOuterNesterov
from ..utils.schedule import CosineWarmupSchedule
from .comm import FlatCommunicator, PendingAllReduce, plan_buckets
from .dist import DistEnv


class Diloco:
    """Flagship DiLoCo on the flat-store Llama.  Any other ``nn.Module`` (with plain torch optimizers)
    is dispatched to :class:`~nanodiloco_amd.parallel.module_diloco.ModuleDiloco`, which has the
    reference's generic ``model.parameters()`` / ``param_groups`` contract."""

    def __new__(cls, model, *args, **kwargs):
        if not isinstance(model, LlamaForCausalLM):
            from .module_diloco import ModuleDiloco
            return ModuleDiloco(model, *args, **kwargs)
        return super().__new__(cls)

    def __init__(self, model: LlamaForCausalLM, inner_optimizer: FlatAdamW, outer_optimizer: FlatOuterNesterov,
                 warmup_steps: int, total_steps: int, inner_steps: int = 100, outer_steps: Optional[int] = None,
                 env: Optional[DistEnv] = None, comm_dtype: torch.dtype = torch.float32, bucket_mb: float = 128.0,
                 overlap: bool = False, offload_snapshot: bool = False, debug_checks: bool = False,
                 broadcast_init: bool = True):
        self.model = model
        self.store = model.store
        self.inner_optimizer = inner_optimizer
        self.outer_optimizer = outer_optimizer
        self.inner_steps = inner_steps
        self.outer_steps = outer_steps if outer_steps is not None else max(1, total_steps // max(1, inner_steps))
        self.env = env or DistEnv(device=self.store.device)
        self.scheduler = CosineWarmupSchedule(inner_optimizer.lr, warmup_steps, total_steps)
        self.comm_dtype = comm_dtype
        self.overlap = overlap
        self.offload_snapshot = offload_snapshot
        self.debug_checks = debug_checks
        e = self.env
        f = e.force_collectives
        kw = dict(impl=e.comm_impl, device=e.device, timeout_s=e.timeout_s)
        self.outer_comm = FlatCommunicator(e.outer_group, e.num_workers, bucket_mb, force=f, **kw)
        self.inner_comm = FlatCommunicator(e.inner_group, e.inner_dp, bucket_mb, force=f and e.force_inner_ddp, **kw)
        self.world_comm = FlatCommunicator(e.world_group, e.world_size, bucket_mb, force=f, **kw)
        n = self.store.numel
        # shard of the flat vector this GPU reduces over the outer group (two-level mode)
        k = e.inner_dp
        if n % (k * 64):
            raise ValueError("flat size must be divisible by 64*inner_dp (ParamStore pads to 64)")
        self.shards = [(i * n // k, (i + 1) * n // k) for i in range(k)]
        self.my_shard = self.shards[e.inner_rank]

        # ---- replicate the init (reference: 57 per-tensor broadcasts)
        if broadcast_init and e.is_distributed:
            self.world_comm.broadcast(self.store.master, 0)
            self.store.sync_shadow()
        # ---- last-synced snapshot
        if offload_snapshot:
            self.sync = self.store.new_flat(device="cpu", pin=True)
            self.sync.copy_(self.store.master)
        else:
            self.sync = self.store.master.clone()
        a, b = self.my_shard
        self.delta = torch.zeros(b - a, dtype=comm_dtype, device=self.store.device)
        self.drift_base = torch.zeros(b - a, dtype=torch.float32, device=self.store.device) if overlap else None
        self._pending = None
        self._sync_time = 0.0
        self._sync_calls = 0
        self._comm_events = []
        self.local_step = 0
        self.outer_step_count = 0

    # ------------------------------------------------------------------ reference API
    def __call__(self, *args, **kwargs):
        return self.model(*args, **kwargs)

    def train(self):
        self.model.train()

    def eval(self):
        self.model.eval()

    @property
    def avg_sync_time(self) -> float:
        """Mean wall seconds per outer step (host view, includes the device wait when not overlapped)."""
        return self._sync_time / self._sync_calls if self._sync_calls > 0 else 0.0

    @property
    def bytes_per_outer_step(self) -> int:
        """Pseudo-gradient payload each GPU contributes to the outer all-reduce."""
        a, b = self.my_shard
        return (b - a) * torch.tensor([], dtype=self.comm_dtype).element_size() if self.outer_comm.enabled else 0

    def comm_ms(self) -> float:
        """Device time of the last outer step (HIP events on the compute stream, from the pseudo-
        gradient kernel to the last outer-Nesterov / all-gather: i.e. everything the outer step
        costs the compute stream, collectives included; syncs on the end event)."""
        if not self._comm_events:
            return 0.0
        s, e = self._comm_events[-1]
        e.synchronize()
        return s.elapsed_time(e)

    @property
    def buckets_per_outer_step(self) -> int:
        """Number of all-reduce calls one outer step issues (the reference issues one per tensor)."""
        if not self.outer_comm.enabled:
            return 0
        a, b = self.my_shard
        return len(plan_buckets(0, b - a, self.delta.element_size(), self.outer_comm.bucket_bytes))

    def current_lr(self) -> float:
        return self.scheduler.lr()

    # ------------------------------------------------------------------ inner step
    def inner_step(self):
        """clip(1.0) + AdamW at the scheduled lr, advance the schedule, zero grads."""
        lr = self.scheduler.lr()
        self.inner_optimizer.step(lr)
        if getattr(self.model, "fp8", None) is not None:
            self.model.fp8.recipe.update()  # fp8 delayed scaling: roll amax history once per inner step
        self.scheduler.step()
        self.store.zero_grad()
        self.local_step += 1
        if self._pending is not None:  # overlapped outer step from the previous boundary
            self._finish_outer()
        if self.debug_checks and self.env.inner_dp > 1:
            self.check_inner_replicas()

    # ------------------------------------------------------------------ outer step
    def outer_step(self, phases: bool = False):
        """One outer step.  ``phases=True`` (diagnostics, e.g. bench.py after its timed window) runs it
        serialized -- every bucket's all-reduce completes before the first Nesterov update -- and
        records HIP events between the phases, so :meth:`outer_phase_ms` can split the step into
        pseudo-gradient / collective / outer-update time; the default pipelines buckets instead."""
        t0 = time.perf_counter()
        cuda = self.store.device.type == "cuda"
        ev0 = torch.cuda.Event(enable_timing=True) if cuda else None
        if ev0 is not None:
            ev0.record()
        master = self.store.master
        sync = self._sync_on_device()
        a, b = self.my_shard
        ops.pseudograd(sync[a:b], master[a:b], self.delta)
        if self.overlap:
            # fp32 drift base: with bf16 transport, re-applying the local progress from the rounded
            # delta would carry its bf16 rounding error into the weights every outer step
            if self.delta.dtype == torch.float32:
                self.drift_base.copy_(self.delta)
            else:
                ops.pseudograd(sync[a:b], master[a:b], self.drift_base)
        marks = None
        if phases and cuda and not self.overlap:
            marks = [ev0, torch.cuda.Event(enable_timing=True)]
            marks[1].record()
        pend = self.outer_comm.all_reduce_async(self.delta)
        if marks is not None:
            pend.wait_all()  # serialized: the compute stream waits for every bucket here
            marks.append(torch.cuda.Event(enable_timing=True))
            marks[2].record()
        self._pending = (pend, sync, ev0, t0)
        self.outer_step_count += 1
        if not self.overlap:
            self._finish_outer()
            if marks is not None:
                marks.append(self._comm_events[-1][1])
                self._phase_marks = marks
        else:
            self._sync_time += time.perf_counter() - t0

    def outer_phase_ms(self) -> dict:
        """Device time of the last ``outer_step(phases=True)``: pseudo-gradient kernel, bucketed
        all-reduce (from the compute stream's view: issue to last bucket done), outer Nesterov update
        (+ the two-level all-gathers).  Empty if no phased step ran."""
        m = getattr(self, "_phase_marks", None)
        if not m:
            return {}
        m[-1].synchronize()
        return {"pseudograd_ms": m[0].elapsed_time(m[1]), "allreduce_ms": m[1].elapsed_time(m[2]),
                "outer_update_ms": m[2].elapsed_time(m[3])}

    def _finish_outer(self):
        pend, sync, ev0, t0 = self._pending
        t1 = time.perf_counter()
        self._pending = None
        a, b = self.my_shard
        opt = self.outer_optimizer
        first = opt.step_count == 0
        master, shadow, mom = self.store.master, self.store.shadow, opt.momentum_buffer
        inv_w = 1.0 / max(1, self.env.num_workers)
        sh_full = shadow if shadow.data_ptr() != master.data_ptr() else None
        for i, (x, y) in enumerate(pend.ranges):
            pend.wait(i)  # compute stream waits for bucket i only
            ga, gb = a + x, a + y
            ops.outer_nesterov(master[ga:gb], sync[ga:gb], self.delta[x:y], mom[ga:gb],
                               sh_full[ga:gb] if sh_full is not None else None, inv_w, opt.lr, opt.momentum,
                               first, drift_base=self.drift_base[x:y] if self.overlap else None)
        opt.step_count += 1
        self.store.version += 1
        # own RCCL: a watchdog abort still completes the collective's event, so the update above may have
        # consumed a partial reduction -- fail before anything builds on it (c10d raises in Work.wait)
        self.outer_comm.check("the outer update")
        if self.env.inner_dp > 1:
            # every GPU of the worker updated its shard; replicate master and snapshot
            self.inner_comm.all_gather_flat(master, self.shards, self.env.inner_rank)
            self.inner_comm.all_gather_flat(sync, self.shards, self.env.inner_rank)
            if sh_full is not None:
                for j, (x, y) in enumerate(self.shards):
                    if j != self.env.inner_rank:
                        sh_full[x:y].copy_(master[x:y])
        if self.offload_snapshot:
            self.sync.copy_(sync, non_blocking=True)
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._comm_events = [(ev0, ev1)]
        self._sync_time += time.perf_counter() - (t1 if self.overlap else t0)
        self._sync_calls += 1
        if self.debug_checks:
            self.check_replicas()

    def _sync_on_device(self) -> torch.Tensor:
        if not self.offload_snapshot:
            return self.sync
        dev = self.store.master.new_empty(self.store.numel)
        dev.copy_(self.sync, non_blocking=True)
        return dev

    def finalize(self):
        """Apply a still-pending overlapped outer step (end of training / before checkpoint)."""
        if self._pending is not None:
            self._finish_outer()

    def pending_outer_state(self) -> Optional[dict]:
        """An overlapped outer step that is still in flight (a checkpoint between the boundary and its
        one-step-late application): the compute stream waits for its all-reduce, and the reduced
        pseudo-gradient plus this rank's drift base are returned WITHOUT applying the step, so a run
        resumed from the checkpoint applies it at the same point as the uninterrupted run.  None when
        nothing is pending (always, without ``overlap``)."""
        if self._pending is None:
            return None
        self._pending[0].wait_all()
        return {"delta": self.delta, "drift_base": self.drift_base}

    def restore_pending_outer(self, delta: torch.Tensor, drift_base: torch.Tensor):
        """Re-arm the pending outer step saved by :meth:`pending_outer_state` (its all-reduce already
        done): the next :meth:`inner_step` applies it."""
        if not self.overlap:
            raise RuntimeError("checkpoint holds a pending overlapped outer step: resume with --overlap-outer")
        self.delta.copy_(delta)
        self.drift_base.copy_(drift_base)
        ranges = plan_buckets(0, self.delta.numel(), self.delta.element_size(), self.outer_comm.bucket_bytes)
        self._pending = (PendingAllReduce([None] * len(ranges), ranges, self.delta), self._sync_on_device(), None,
                         time.perf_counter())

    # ------------------------------------------------------------------ debug
    @staticmethod
    def _checksum_spread(x: torch.Tensor, group) -> torch.Tensor:
        """MAX-MIN over ``group`` of two order-sensitive fp64 checksums of ``x``."""
        import torch.distributed as dist
        xd = x.double()
        w = torch.arange(1, x.numel() + 1, device=x.device, dtype=torch.float64).remainder(7)
        v = torch.stack([xd.sum(), (xd * w).sum()])
        mx, mn = v.clone(), v.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
        return (mx - mn).abs()

    @torch.no_grad()
    def check_replicas(self, tol: float = 0.0):
        """Replica-consistency assertions, run after every outer step with
        ``debug_checks``:

        * theta_sync is identical on every rank of the job;
        * the GPUs of one DiLoCo worker (inner DDP) hold identical master weights;
        * without the overlapped outer step, the master weights equal theta_sync everywhere.
        (In the overlapped mode the local weights legitimately differ across workers by each
        worker's in-flight inner progress.)"""
        if not self.env.is_distributed:
            return
        spread = self._checksum_spread(self.sync.to(self.store.device), None)
        if spread.max().item() > tol:
            raise RuntimeError(f"DiLoCo replicas diverged: theta_sync checksum spread {spread.tolist()}")
        self.check_inner_replicas(tol)
        if not self.overlap and self._pending is None:
            spread = self._checksum_spread(self.store.master, None)
            if spread.max().item() > tol:
                raise RuntimeError(f"DiLoCo replicas diverged: master checksum spread {spread.tolist()}")

    @torch.no_grad()
    def check_inner_replicas(self, tol: float = 0.0):
        """The K GPUs of one DiLoCo worker apply the same all-reduced gradient every inner step, so
        their master weights must stay bit-identical (run after every inner step with
        ``debug_checks`` when ``inner_dp > 1``)."""
        if self.env.inner_dp <= 1:
            return
        spread = self._checksum_spread(self.store.master, self.env.inner_group)
        if spread.max().item() > tol:
            raise RuntimeError(f"inner-DDP replicas diverged inside worker {self.env.worker}: "
                               f"master checksum spread {spread.tolist()}")

    # ------------------------------------------------------------------ checkpoint state
    def state_dict(self):
        self.finalize()
        return {
            "sync": self.sync,
            "outer": self.outer_optimizer.state_dict(),
            "inner": self.inner_optimizer.state_dict(),
            "scheduler": self.scheduler.state_dict(),
            "local_step": self.local_step,
            "outer_step_count": self.outer_step_count,
        }

    def load_state_dict(self, d):
        """Restore the outer state (``inner`` is optional: the checkpoint keeps AdamW state per rank)."""
        self.sync.copy_(d["sync"])
        self.outer_optimizer.load_state_dict(d["outer"])
        if "inner" in d:
            self.inner_optimizer.load_state_dict(d["inner"])
        self.scheduler.load_state_dict(d["scheduler"])
        self.local_step = int(d["local_step"])
        self.outer_step_count = int(d["outer_step_count"])
