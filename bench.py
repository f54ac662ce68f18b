#!/usr/bin/env python3
"""Headline benchmark: whole-node training tokens/s of Llama-150M DiLoCo workers (H=100), bf16.

BASELINE.json metric: "tokens/sec (whole node) Llama-150M, 8 DiLoCo workers H=100; bytes/outer-step".
One process per GPU (torchrun); every GPU is one DiLoCo worker running the reference's per-worker
inner step (256 sequences x 1024 tokens, clip + AdamW) on synthetic tokens with random-init weights.

Timing contract: W untimed warmup inner steps, then barrier + device sync, K timed inner steps,
barrier + device sync; the elapsed time is the MAX over ranks.  Outer steps fire every H=100 inner
steps as in training; if the timed window contains none, one outer step (pseudo-gradient + bucketed
RCCL all-reduce + outer Nesterov) is executed INSIDE the window anyway -- a conservative charge
(H=100 amortises it 100x in real training).

    python bench.py                       # 1 GPU, defaults
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --steps 20 --warmup 3
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.config import resolve_llama_config  # noqa: E402
from nanodiloco_amd.data import SyntheticTokens  # noqa: E402
from nanodiloco_amd.models import LlamaForCausalLM  # noqa: E402
from nanodiloco_amd.optim import FlatAdamW, FlatOuterNesterov  # noqa: E402
from nanodiloco_amd.parallel.diloco import Diloco  # noqa: E402
from nanodiloco_amd.ops.tuned_gemm import enable_tuned_gemms  # noqa: E402
from nanodiloco_amd.parallel.dist import barrier, init_distributed  # noqa: E402
from nanodiloco_amd.parallel.inner_ddp import InnerGradSync  # noqa: E402

BASELINE_TOKENS_PER_S = None  # the reference publishes no number
METRIC = "tokens/sec (whole node) Llama-150M, 8 DiLoCo workers H=100; bytes/outer-step"  # BASELINE.json
MODEL_NAMES = {"llama_150m": "Llama-150M", "llama_1b": "Llama-1B", "llama_default": "Llama-10M (reference default)",
               "llama_tiny": "tiny-Llama-2L", "llama_large": "Llama-29M"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama_150m.json")
    ap.add_argument("--batch-size", type=int, default=256, help="sequences per worker per inner step (reference)")
    ap.add_argument("--micro-batch", type=int, default=64,
                    help="sequences per forward/backward (64: best of 16/32/64/128/256 on MI355X, same global batch)")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--inner-steps", type=int, default=100)
    ap.add_argument("--inner-dp", type=int, default=1)
    ap.add_argument("--ops", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="collective backend (auto = nccl/RCCL on GPU); gloo lets several ranks share one GPU")
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--bucket-mb", type=float, default=128.0)
    ap.add_argument("--overlap-outer", action="store_true")
    ap.add_argument("--no-tuned-gemm", action="store_true", help="library-default GEMM algorithms (A/B)")
    ap.add_argument("--tuned-gemm-file", default=None, help="alternative TunableOp table (A/B of tunings)")
    ap.add_argument("--hip-graph", action="store_true",
                    help="capture the micro-batch forward+backward in a HIP graph (launch-bound small models)")
    ap.add_argument("--wgrad-overlap", type=int, default=0, choices=[0, 1, 2],
                    help="issue weight-gradient GEMMs on a side HIP stream (overlaps the dgrad chain); off by "
                         "default: beside hipBLASLt's stream-K GEMMs it stalls (docs/DESIGN.md)")
    ap.add_argument("--wgrad-variant", default=None,
                    help="ND_WGRAD_VARIANT for the weight-gradient kernel (A/B of kernel schedules)")
    ap.add_argument("--attn-fused-stats", type=int, default=1, choices=[0, 1],
                    help="attention backward: row statistics inside the dQ kernel (0: separate passes)")
    ap.add_argument("--dgrad-t", type=int, default=1, choices=[0, 1],
                    help="input-gradient GEMMs on transposed weight copies (K-contiguous NT layout)")
    ap.add_argument("--fused-swiglu", type=int, default=0, choices=[0, 1],
                    help="gate|up GEMM with SwiGLU in the own GEMM's epilogue (1) or hipBLASLt + swiglu kernel (0)")
    ap.add_argument("--fp8", action="store_true", help="fp8 (e4m3/e5m2) decoder projections (BASELINE config 5)")
    ap.add_argument("--fp8-wgrad", action="store_true", help="with --fp8: weight-gradient GEMM in fp8 too")
    ap.add_argument("--fp8-gemm", default="hipblaslt", choices=["hip", "hipblaslt"],
                    help="with --fp8: forward / input-gradient fp8 GEMMs on our MFMA kernel or hipBLASLt")
    ap.add_argument("--fp8-fused-quant", type=int, default=1, choices=[0, 1],
                    help="with --fp8: operand quantisation fused into the producing kernels (0: separate casts)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    return ap.parse_args()


def main():
    a = parse()
    ops.set_backend(a.ops)
    ops.set_wgrad_overlap(a.wgrad_overlap)
    ops.set_fused_swiglu(bool(a.fused_swiglu))
    ops.set_dgrad_transposed(bool(a.dgrad_t))
    ops.set_attn_fused_stats(bool(a.attn_fused_stats))
    if a.fp8:
        from nanodiloco_amd.ops import fp8 as _fp8
        _fp8.set_fused_quant(bool(a.fp8_fused_quant))
        _fp8.set_fp8_gemm(a.fp8_gemm)
    if a.wgrad_variant:
        os.environ["ND_WGRAD_VARIANT"] = a.wgrad_variant
    env = init_distributed(a.backend, a.inner_dp)
    if env.world_size != a.gpus and env.rank == 0:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={env.world_size}", file=sys.stderr)
    if env.device.type == "cuda" and not a.no_tuned_gemm:
        if a.tuned_gemm_file:
            enable_tuned_gemms(env.device, a.tuned_gemm_file)
        else:
            enable_tuned_gemms(env.device)
    cfg = resolve_llama_config(a.model)
    dtype = torch.bfloat16 if env.device.type == "cuda" else torch.float32
    model = LlamaForCausalLM(cfg, env.device, dtype, fp8=a.fp8, fp8_wgrad=a.fp8_wgrad).init_weights(1337)
    inner = FlatAdamW(model.store, lr=4e-4)
    outer = FlatOuterNesterov(model.store, lr=0.7, momentum=0.9)
    comm_dtype = torch.bfloat16 if a.comm_dtype == "bf16" else torch.float32
    total = 10_000
    dl = Diloco(model, inner, outer, warmup_steps=100, total_steps=total, inner_steps=a.inner_steps, env=env,
                comm_dtype=comm_dtype, bucket_mb=a.bucket_mb, overlap=a.overlap_outer)
    isync = InnerGradSync(model, dl.inner_comm)
    accum = a.batch_size // a.micro_batch
    data = SyntheticTokens(cfg.vocab_size, a.seq_len, a.micro_batch, seed=1337, rank=env.rank, device=env.device)
    loss_scale = 1.0 / accum / env.inner_dp
    model.train()
    state = {"step": 0}

    graphed = None
    if a.hip_graph:
        if env.inner_dp > 1:
            raise SystemExit("--hip-graph needs --inner-dp 1")
        from nanodiloco_amd.utils.graphs import GraphedMicroStep
        graphed = GraphedMicroStep(model)

    def inner_step():
        loss = None
        for m in range(accum):
            b = next(data)
            if m == accum - 1:
                isync.arm()
            if graphed is not None:
                l_m = graphed(b["input_ids"], b["labels"], loss_scale)
            else:
                out = model(b["input_ids"], labels=b["labels"], loss_scale=loss_scale)
                out.loss.backward()
                l_m = out.loss.detach()
            loss = l_m.clone() if loss is None else loss + l_m
        isync.finish()
        dl.inner_step()
        state["step"] += 1
        outer_done = False
        if state["step"] % a.inner_steps == 0:
            dl.outer_step()
            outer_done = True
        return loss, outer_done

    sync = (lambda: torch.cuda.synchronize()) if env.device.type == "cuda" else (lambda: None)
    for _ in range(a.warmup):
        inner_step()
    if a.warmup:
        dl.outer_step()  # warm the RCCL communicators / bucket path (untimed)
    sync()
    barrier(env)
    sync()
    t0 = time.perf_counter()
    n_outer = 0
    loss = None
    for _ in range(a.steps):
        loss, od = inner_step()
        n_outer += int(od)
    if n_outer == 0:
        dl.outer_step()
        n_outer = 1
    dl.finalize()
    sync()
    barrier(env)
    sync()
    elapsed = time.perf_counter() - t0
    if env.is_distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    outer_ms = dl.comm_ms()  # device time of the last outer step (HIP events; after the timed window)
    if env.is_distributed:
        t = torch.tensor([outer_ms], dtype=torch.float64, device=env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        outer_ms = float(t.item())
    tokens = a.batch_size * a.seq_len * a.steps * env.world_size
    tps = tokens / elapsed
    final_loss = float((loss / accum).item()) if loss is not None else float("nan")
    if a.profile_steps and env.rank == 0:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(a.profile_steps):
                inner_step()
            sync()
        print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=30), file=sys.stderr)
    if env.rank == 0:
        model_name = MODEL_NAMES.get(os.path.splitext(os.path.basename(a.model))[0], a.model)
        mfu_flops = cfg.flops_per_token(a.seq_len) * tps / max(1, env.world_size)
        out = {
            "metric": METRIC if model_name == "Llama-150M" else
            f"tokens/sec (whole node) {model_name}, DiLoCo workers H={a.inner_steps}",
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": env.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * elapsed / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (tps / BASELINE_TOKENS_PER_S) if BASELINE_TOKENS_PER_S else None,
            "dtype": ("fp8" if a.fp8 else "bf16") if dtype == torch.bfloat16 else "fp32",
            "data": "synthetic",
            "config": {
                "model": model_name,
                "global_batch": a.batch_size * env.world_size,
                "seq_len": a.seq_len,
                "parallelism": f"diloco{env.num_workers}" + (f"x_ddp{env.inner_dp}" if env.inner_dp > 1 else ""),
                "per_worker_batch": a.batch_size,
                "micro_batch": a.micro_batch,
                "inner_steps_H": a.inner_steps,
                "params": cfg.num_params(),
            },
            "bytes_per_outer_step": dl.bytes_per_outer_step if env.num_workers > 1 else model.store.numel * (
                2 if comm_dtype == torch.bfloat16 else 4),
            "outer_steps_in_window": n_outer,
            # outer-step cost as seen by the compute stream (HIP events: pseudo-gradient + bucketed
            # RCCL all-reduce + fused Nesterov), host wall time per outer step, and calls per outer step
            "outer_step_ms": round(outer_ms, 3),
            "outer_step_wall_ms": round(1000.0 * dl.avg_sync_time, 3),
            "allreduce_calls_per_outer_step": dl.buckets_per_outer_step,
            "comm_backend": env.backend,
            "comm_dtype": a.comm_dtype,
            "model_tflops_per_gpu": round(mfu_flops / 1e12, 2),
            "final_loss": round(final_loss, 4),
            "tuned_gemm": enable_tuned_gemms(env.device) if env.device.type == "cuda" and not a.no_tuned_gemm else False,
            "wgrad_overlap": ops.wgrad_overlap_enabled(),
            "fused_swiglu_gemm": ops.fused_swiglu_enabled(),
            "fp8_gemm": a.fp8_gemm if a.fp8 else None,
            "dgrad_transposed": ops.dgrad_transposed_enabled(),
            "ops": ops.get_backend() if a.ops != "auto" else ("hip" if env.device.type == "cuda" else "torch"),
        }
        print(json.dumps(out), flush=True)
    if env.is_distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
