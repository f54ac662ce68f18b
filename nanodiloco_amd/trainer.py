"""Training driver (capability parity with ``train_model``, REF/nanodiloco/main.py:41-130).

Differences from the reference (each documented in SURVEY.md §3.5 and switchable where cheap):
* stops after exactly ``total_steps`` inner steps (reference runs one epoch, Q3);
* gradients are the mean over micro-batches (``legacy_grad_sum=True`` reproduces the reference's
  sum of micro-batch means, Q1);
* logs the true mean loss of the inner step on global rank 0 (Q2, Q6), every ``log_every`` steps,
  so the device is synced only at log points (the reference syncs twice per micro-batch, K10);
* bf16 compute with fp32 master weights / grads / optimizer state by default on GPU.
"""
from __future__ import annotations

import dataclasses
import math
import os
import time
from typing import Any, Dict, Optional

import torch

from . import ops
from .config import LlamaConfig, default_run_config, load_config_from_file, resolve_llama_config
from .data import build_data
from .models import LlamaForCausalLM
from .optim import FlatAdamW, FlatOuterNesterov
from .parallel.diloco import Diloco
from .parallel.dist import DistEnv, init_distributed
from .parallel.inner_ddp import InnerGradSync
from .utils.logging import make_sink
from .utils.profiling import PhaseTimer, torch_profile
from .utils.run_name import create_run_name
from .utils.seed import set_seed_all


@dataclasses.dataclass
class TrainArgs:
    # ---- the 13 reference flags (REF/nanodiloco/main.py:42-56), same defaults
    seed: int = 1337
    batch_size: int = 256
    per_device_batch_size: int = 8     # or "auto": the largest that suits the model (auto_micro_batch)
    seq_length: int = 1024
    warmup_steps: int = 100
    total_steps: int = 10_000
    inner_steps: int = 100
    lr: float = 4e-4
    outer_lr: float = 0.7
    project: str = "nano-diloco"
    dataset_path: str = "/mnt/hf-c4-tiny/datasets/PrimeIntellect/c4-tiny/en/save_to_disk"
    llama_config_file: Optional[str] = None
    wandb_config_file: Optional[str] = None
    # ---- extensions
    dtype: str = "auto"            # auto | fp32 | bf16 | fp8 (= bf16 compute + fp8 decoder projections)
    data: str = "auto"             # auto | synthetic | memmap | hf
    ops: str = "auto"              # auto | hip | torch
    backend: str = "auto"          # auto | nccl | gloo
    comm_impl: str = "auto"        # auto | rccl | c10d: bulk collectives on the own RCCL communicator
                                   # (parallel/rccl.py; auto = whenever the backend is nccl) or torch's group
    device: str = "auto"           # auto | cpu | cuda
    inner_dp: int = 1
    outer_momentum: float = 0.9
    max_grad_norm: float = 1.0
    weight_decay: float = 0.01
    comm_dtype: str = "fp32"
    bucket_mb: float = 128.0
    overlap_outer: bool = False
    offload_snapshot: bool = False
    legacy_grad_sum: bool = False
    activation_checkpointing: bool = False
    residual_dtype: str = "auto"   # fp32 (the autocast recipe) | bf16: residual stream in bf16 (Megatron's default;
                                   # the RMSNorm passes move 4 instead of 6 / 8 tensor units, docs/DESIGN.md) |
                                   # auto: bf16 with --fp8 (the Megatron / Transformer-Engine fp8 recipe), else fp32
    fp8: bool = False              # fp8 e4m3/e5m2 decoder projections (GPU, bf16 compute)
    fp8_wgrad: bool = True         # with fp8: the weight-gradient GEMMs in fp8 too (own kernel on the token-major
                                   # fp8 operands, 1.65-1.73x the bf16 one; profiles/r4_fp8_pp.md)
    fp8_keep_fused: str = "none"   # with fp8: none | rope | mlp | both -- projections kept on the bf16
                                   # fused-epilogue GEMMs (ops/fp8.py set_fp8_keep_fused)
    force_collectives: bool = False  # world size 1: still create a (one-rank) process group and issue
                                     # every collective (exercises the RCCL path on one GPU)
    tuned_gemm: bool = True        # load the pre-tuned hipBLASLt algorithm table (ops/tuned_gemm.py)
    hip_graph: str = "auto"        # capture the micro-batch fwd+bwd in a HIP graph (utils/graphs.py):
                                   # on | off | auto (= on for launch-bound models: GPU, < 100M params,
                                   # --inner-dp 1, no fp8, e.g. the reference's 10M default: 2.5x)
    wgrad_overlap: bool = True     # weight-gradient GEMMs on a side HIP stream, joined before every library
                                   # GEMM (ops/linear.py; GPU only): +0.4 % per step at round 4 HEAD
                                   # (profiles/r4_wgrad_overlap_ab.md)
    checkpoint_dir: Optional[str] = None
    checkpoint_every: int = 0      # in outer steps (0 = only at the end when checkpoint_dir is set)
    stop_at_step: int = 0          # stop early (simulated preemption) after this inner step; 0 = run to total
    resume: Optional[str] = None   # a checkpoint dir, or "auto": the newest complete one in checkpoint_dir (restarts)
    elastic_resume: bool = False   # resume on a different number of DiLoCo workers (utils/checkpoint.py)
    log_every: int = 1
    log_file: Optional[str] = None
    wandb: str = "auto"
    tokenizer: str = "huggyllama/llama-7b"
    debug_checks: bool = False
    mask_pad_labels: bool = True
    deterministic: bool = False    # bitwise-reproducible step: no float atomics (ops/determinism.py)
    skip_nonfinite: bool = False   # device-side skip of inner steps whose grad norm is NaN/Inf (no host sync)
    collective_timeout_s: float = 1800.0
    phase_timing: bool = True      # HIP-event timing of fwd+bwd / inner optimizer / outer step (logged)
    profile_dir: Optional[str] = None   # torch.profiler Chrome trace of `profile_steps` steps
    profile_steps: int = 0


def _dtype(name: str, device: torch.device) -> torch.dtype:
    if name == "auto":
        return torch.bfloat16 if device.type == "cuda" else torch.float32
    return {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
            "bfloat16": torch.bfloat16, "fp8": torch.bfloat16}[name]


def _residual_dtype(name: str, fp8: bool = False) -> torch.dtype:
    if name == "auto":
        return torch.bfloat16 if fp8 else torch.float32
    d = {"fp32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}.get(name)
    if d is None:
        raise ValueError(f"--residual-dtype must be auto, fp32 or bf16, not {name!r}")
    return d


# activation budget of one micro-batch as a share of device memory, and the micro-batch token target
# (128 x 1024 at round-3 HEAD: +0.5 % bf16 / +1.8 % --fp8 over 64 x 1024 for Llama-150M in interleaved
# A/Bs, profiles/r3_micro_batch_ab.md).  Round 5: 45 % of the 288 GB (was 30 %) so Llama-1B gets 64 x 1024
# (~100 GB of activations) instead of 32 x 1024: +0.45 % bf16 with the makespan-planned weight-gradient splits
# (session r5an); optimizer state and flat buffers of the 1B model take < 30 GB
_AUTO_MEM_SHARE = 0.45
_AUTO_TOKENS = 131072


def auto_micro_batch(cfg: LlamaConfig, seq_len: int, batch_size: int, device: torch.device) -> int:
    """``--per-device-batch-size auto``: the largest divisor of ``batch_size`` whose micro-batch holds at
    most ``_AUTO_TOKENS`` = 128k tokens (128 x 1024 for Llama-150M) and whose activations (flash attention, no recompute: ~34 * d bytes per token and
    layer in bf16, plus the chunked lm-head's 4 GiB logits budget) fit in 30 % of the device memory.

    The math does not change: gradients are the mean over the micro-batches of an inner step (each
    micro-batch a mean over its tokens), so with equal tokens per micro-batch (synthetic / packed
    data) any micro-batch size gives the same update up to summation order.  With padded HF batches
    the per-micro-batch token counts differ, exactly as they do for the reference's micro-batch 8.
    On CPU the reference's default (8) is kept."""
    if device.type != "cuda":
        cap = 8
    else:
        mem = torch.cuda.get_device_properties(device).total_memory
        per_tok = 34 * cfg.hidden_size * cfg.num_hidden_layers + 8 * cfg.hidden_size
        budget = _AUTO_MEM_SHARE * mem - (4 << 30)
        cap = max(1, min(_AUTO_TOKENS, int(budget // per_tok)) // max(1, seq_len))
    mb = 1
    for cand in range(1, batch_size + 1):
        if batch_size % cand == 0 and cand <= cap:
            mb = cand
    return mb


def _resolve_data_kind(a: TrainArgs) -> str:
    if a.data != "auto":
        return a.data
    p = a.dataset_path
    if p and os.path.isdir(p):
        import glob
        if glob.glob(os.path.join(p, "*.bin")):
            return "memmap"
        return "hf"
    return "synthetic"


class Trainer:
    def __init__(self, args: TrainArgs, env: Optional[DistEnv] = None):
        self.args = a = args
        if a.total_steps % a.inner_steps:
            raise ValueError("total_steps must be a multiple of inner_steps")  # REF main.py:69
        ops.set_backend(a.ops)
        ops.set_wgrad_overlap(a.wgrad_overlap)
        ops.set_deterministic(a.deterministic)
        self.env = env or init_distributed(a.backend, a.inner_dp, device=None if a.device == "auto" else a.device,
                                           timeout_s=a.collective_timeout_s, force_pg=a.force_collectives,
                                           comm_impl=a.comm_impl)
        e = self.env
        if e.device.type == "cuda" and a.tuned_gemm:
            from .ops.tuned_gemm import enable_tuned_gemms
            enable_tuned_gemms(e.device)
        self.llama_config: LlamaConfig = resolve_llama_config(a.llama_config_file)
        if str(a.per_device_batch_size).lower() == "auto":
            a.per_device_batch_size = auto_micro_batch(self.llama_config, a.seq_length, a.batch_size, e.device)
        a.per_device_batch_size = int(a.per_device_batch_size)
        if a.batch_size % a.per_device_batch_size:
            raise ValueError("batch_size must be a multiple of per_device_batch_size")  # REF main.py:65
        self.run_config = load_config_from_file(a.wandb_config_file) if a.wandb_config_file else default_run_config()
        set_seed_all(a.seed)
        self.grad_accum = a.batch_size // a.per_device_batch_size
        self.outer_steps = a.total_steps // a.inner_steps
        self.compute_dtype = _dtype(a.dtype, e.device)
        if a.fp8 or a.dtype == "fp8":
            from .ops.fp8 import set_fp8_keep_fused
            set_fp8_keep_fused(a.fp8_keep_fused)
        self.model = LlamaForCausalLM(self.llama_config, e.device, self.compute_dtype,
                                      activation_checkpointing=a.activation_checkpointing,
                                      fp8=a.fp8 or a.dtype == "fp8", fp8_wgrad=a.fp8_wgrad,
                                      residual_dtype=_residual_dtype(a.residual_dtype, a.fp8 or a.dtype == "fp8")).init_weights(a.seed)
        inner = FlatAdamW(self.model.store, lr=a.lr, weight_decay=a.weight_decay, max_grad_norm=a.max_grad_norm,
                          skip_nonfinite=a.skip_nonfinite)
        outer = FlatOuterNesterov(self.model.store, lr=a.outer_lr, momentum=a.outer_momentum)
        self.diloco = Diloco(self.model, inner, outer, a.warmup_steps, a.total_steps, a.inner_steps, self.outer_steps,
                             env=e, comm_dtype=_dtype(a.comm_dtype, e.device), bucket_mb=a.bucket_mb,
                             overlap=a.overlap_outer, offload_snapshot=a.offload_snapshot,
                             debug_checks=a.debug_checks)
        self.inner_sync = InnerGradSync(self.model, self.diloco.inner_comm)
        self.loss_scale = (1.0 if a.legacy_grad_sum else 1.0 / self.grad_accum) / e.inner_dp
        self.data_kind = _resolve_data_kind(a)
        self.data = build_data(self.data_kind, vocab_size=self.llama_config.vocab_size, seq_len=a.seq_length,
                               batch_size=a.per_device_batch_size, seed=a.seed, rank=e.rank, world_size=e.world_size,
                               device=e.device, dataset_path=a.dataset_path, tokenizer=a.tokenizer,
                               mask_pad_labels=a.mask_pad_labels)
        self.start_step = 0
        resume = a.resume
        if resume == "auto":  # restart form: the newest complete checkpoint of --checkpoint-dir, else fresh
            from .utils.checkpoint import find_checkpoint
            resume = find_checkpoint(a.checkpoint_dir)
            if e.rank == 0:
                print(f"[resume auto] {'from ' + resume if resume else 'no checkpoint: fresh start'}", flush=True)
        if resume:
            from .utils.checkpoint import load_checkpoint
            st = load_checkpoint(resume, self.model, self.diloco, e, elastic=a.elastic_resume)
            self.start_step = int(st["step"])
            ds = st.get("data_state")
            if st.get("resized_from") is not None and e.rank == 0:
                print(f"[elastic resume] {st['resized_from']} -> {e.world_size} workers", flush=True)
            if st.get("resized_from") is not None and self.data_kind in ("memmap", "hf"):
                # --elastic-resume: the stream restarts where the old workers stopped together (memmap), or
                # the resume refuses (hf: contiguous shards) -- see utils/checkpoint.load_checkpoint
                self.data.load_state_dict(st.get("data_state_rank0") or {}, resized=True)
            elif ds:
                # a data stream that cannot be restored must fail the resume loudly: silently
                # restarting it would re-train on the same tokens
                if not hasattr(self.data, "load_state_dict"):
                    raise RuntimeError(f"checkpoint has data state but data source {self.data_kind!r} "
                                       f"cannot restore it")
                self.data.load_state_dict(ds)
            elif hasattr(self.data, "load_state_dict") and st.get("resized_from") is None:
                # (--elastic-resume: a worker the checkpoint did not have starts a fresh stream by design)
                raise RuntimeError(f"checkpoint {resume} has no data state for rank {e.rank}; "
                                   f"resuming would restart the data stream")
        self.graphed = None
        hg = str(a.hip_graph).lower()
        if hg == "auto":
            # HF batches always carry an attention_mask, which the captured graph does not take:
            # never capture (and hold the graph's memory) for a data source that produces masks
            # a forced one-rank process group arms the inner-DDP communicator (async RCCL all-reduces with
            # host-side pending events), which a captured graph would replay with stale events
            use_graph = (e.device.type == "cuda" and e.inner_dp == 1 and self.model.fp8 is None
                         and self.data_kind != "hf" and not a.force_collectives
                         and self.llama_config.num_params() < 100_000_000)
        else:
            use_graph = hg in ("1", "true", "on", "yes")
        if use_graph:
            if e.device.type != "cuda" or e.inner_dp > 1 or self.model.fp8 is not None or a.force_collectives:
                raise ValueError("--hip-graph needs a GPU, --inner-dp 1, no --fp8 and no --force-collectives")
            from .utils.graphs import GraphedMicroStep
            self.graphed = GraphedMicroStep(self.model)
        self.run_name = create_run_name("nanodiloco", self.run_config, is_debug=False)
        self.timer = PhaseTimer(a.phase_timing)
        self.sink = make_sink(e.rank, a.project, self.run_name, {**self.run_config, **dataclasses.asdict(a)},
                              jsonl_path=a.log_file, use_wandb=a.wandb)

    # ------------------------------------------------------------------ one inner step
    def inner_step(self) -> torch.Tensor:
        """grad_accum micro-batches fwd+bwd, inner-DDP sync, clip+AdamW. Returns mean loss (device)."""
        loss_sum = None
        with self.timer.phase("fwd_bwd"):
            for micro in range(self.grad_accum):
                batch = next(self.data)
                if micro == self.grad_accum - 1:
                    self.inner_sync.arm()
                mask = batch.get("attention_mask")  # HF path: padded batches (reference main.py:79-88,109)
                if self.graphed is not None and mask is None:
                    l = self.graphed(batch["input_ids"], batch["labels"], self.loss_scale).clone()
                else:
                    out = self.model(batch["input_ids"], labels=batch["labels"], attention_mask=mask,
                                     loss_scale=self.loss_scale)
                    out.loss.backward()
                    l = out.loss.detach()
                loss_sum = l if loss_sum is None else loss_sum + l
        with self.timer.phase("inner_opt"):
            self.inner_sync.finish()
            self.diloco.inner_step()
        return loss_sum / self.grad_accum

    def train(self) -> Dict[str, Any]:
        a, e = self.args, self.env
        self.model.train()
        tokens_per_step = a.batch_size * a.seq_length
        last_t, last_step = time.perf_counter(), self.start_step
        last_loss = float("nan")
        prof_at = self.start_step + 2 if (a.profile_dir and a.profile_steps) else -1
        prof_ctx = None
        for step in range(self.start_step, a.total_steps):
            if step == prof_at:
                prof_ctx = torch_profile(a.profile_dir, e.rank)
                prof_ctx.__enter__()
            loss = self.inner_step()
            real_step = step + 1
            did_outer = real_step % a.inner_steps == 0
            if did_outer:
                with self.timer.phase("outer"):
                    self.diloco.outer_step()
            if prof_ctx is not None and step + 1 >= prof_at + a.profile_steps:
                prof_ctx.__exit__(None, None, None)
                prof_ctx = None
            if (a.log_every and real_step % a.log_every == 0) or real_step == a.total_steps:
                lv = float(loss.item())
                now = time.perf_counter()
                dt = now - last_t
                tps = tokens_per_step * (real_step - last_step) * e.world_size / max(dt, 1e-9)
                last_t, last_step, last_loss = now, real_step, lv
                metrics = {
                    "loss": lv,
                    "step": real_step,
                    "lr": self.diloco.inner_optimizer.param_groups[0]["lr"],
                    "Perplexity": math.exp(min(lv, 80.0)),
                    "effective_step": real_step * e.num_workers,
                    "total_samples": real_step * a.batch_size * e.world_size,
                    "tokens_per_s": tps,
                    "grad_norm": float(self.diloco.inner_optimizer.last_grad_norm.item()),
                    "outer_step": self.diloco.outer_step_count,
                }
                if a.skip_nonfinite:
                    metrics["skipped_steps"] = int(self.diloco.inner_optimizer.skipped_steps.item())
                if did_outer:
                    metrics["bytes_outer"] = self.diloco.bytes_per_outer_step
                    metrics["sync_s"] = self.diloco.avg_sync_time
                    metrics["comm_ms"] = self.diloco.comm_ms()
                metrics.update(self.timer.report())
                self.sink.log(metrics)
            if did_outer and a.checkpoint_dir and a.checkpoint_every and \
                    (real_step // a.inner_steps) % a.checkpoint_every == 0:
                self.save(real_step)
            if a.stop_at_step and real_step >= a.stop_at_step:
                break
            _maybe_inject_fault(e.rank, real_step)
        self.diloco.finalize()
        if a.checkpoint_dir and not a.stop_at_step:
            self.save(a.total_steps)
        if e.rank == 0:
            print("Training completed!", flush=True)
        self.sink.finish()
        return {"final_loss": last_loss, "steps": a.total_steps, "outer_steps": self.diloco.outer_step_count}

    def save(self, step: int):
        from .utils.checkpoint import save_checkpoint
        ds = self.data.state_dict() if hasattr(self.data, "state_dict") else None
        save_checkpoint(self.args.checkpoint_dir, self.model, self.diloco, self.env, step, data_state=ds,
                        extra={"run_name": self.run_name})


def _fault_spec():
    """``ND_FAULT_INJECT=<rank>:<step>[:hang]`` (tests / drills): that rank crashes (exit code 17) or hangs right
    after inner step <step> -- only in the first attempt of a torchrun job (``TORCHELASTIC_RESTART_COUNT`` 0), so
    a ``--max-restarts`` restart runs clean."""
    v = os.environ.get("ND_FAULT_INJECT")
    if not v or int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0) != 0:
        return None
    parts = v.split(":")
    return int(parts[0]), int(parts[1]), (parts[2] if len(parts) > 2 else "crash")


_FAULT = {"spec": None, "read": False}


def _maybe_inject_fault(rank: int, step: int) -> None:
    if not _FAULT["read"]:
        _FAULT["spec"], _FAULT["read"] = _fault_spec(), True
    f = _FAULT["spec"]
    if f is None or f[0] != rank or f[1] != step:
        return
    print(f"[fault inject] rank {rank} step {step}: {f[2]}", flush=True)
    if f[2] == "hang":
        while True:
            time.sleep(60)
    os._exit(17)


def train_model(**kwargs) -> Dict[str, Any]:
    """Programmatic entry with the reference's keyword names (REF/nanodiloco/main.py:41-56)."""
    return Trainer(TrainArgs(**kwargs)).train()
