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
from nanodiloco_amd.ops.tuned_gemm import enable_tuned_gemms  # noqa: E402
from nanodiloco_amd.parallel.dist import barrier  # noqa: E402
from nanodiloco_amd.trainer import TrainArgs, Trainer  # noqa: E402

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
    ap.add_argument("--micro-batch", default="auto",
                    help="sequences per forward/backward; auto = the trainer's --per-device-batch-size auto "
                         "(128 for Llama-150M: best of 16/32/64/128/256 on MI355X, same global batch; "
                         "profiles/r3_micro_batch_ab.md)")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--inner-steps", type=int, default=100)
    ap.add_argument("--inner-dp", type=int, default=1)
    ap.add_argument("--ops", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--backend", default="auto", choices=["auto", "nccl", "gloo", "none"],
                    help="collective backend (auto = nccl/RCCL on GPU, gloo on CPU); gloo lets several ranks share "
                         "one GPU. At world size 1 every backend but 'none' still creates a one-rank process group "
                         "and issues every collective, so the 1-GPU headline runs the same RCCL path (communicator "
                         "init, bucketed all-reduce on the priority stream) as N=8; 'none' = no process group (A/B)")
    ap.add_argument("--comm-impl", default="auto", choices=["auto", "rccl", "c10d"],
                    help="bulk collectives (initial broadcast, outer all-reduce buckets, inner-DDP spans): the own RCCL "
                         "communicator (auto on GPU; parallel/rccl.py) or torch's process group (c10d, A/B)")
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--bucket-mb", type=float, default=128.0)
    ap.add_argument("--overlap-outer", action="store_true")
    ap.add_argument("--no-tuned-gemm", action="store_true", help="library-default GEMM algorithms (A/B)")
    ap.add_argument("--tuned-gemm-file", default=None, help="alternative TunableOp table (A/B of tunings)")
    ap.add_argument("--hip-graph", action="store_true",
                    help="capture the micro-batch forward+backward in a HIP graph (launch-bound small models)")
    ap.add_argument("--wgrad-overlap", type=int, default=1, choices=[0, 1, 2],
                    help="issue weight-gradient GEMMs on a side HIP stream (overlaps the dgrad chain), joined "
                         "before every hipBLASLt GEMM (1, default: +0.4 %% per step, "
                         "profiles/r4_wgrad_overlap_ab.md); 0 off; 2 unfenced (A/B only)")
    ap.add_argument("--deterministic", action="store_true",
                    help="bitwise-reproducible step (sorted embedding backward, per-row loss sum; A/B)")
    ap.add_argument("--residual-dtype", default="auto", choices=["auto", "fp32", "bf16"],
                    help="residual stream dtype (fp32: the autocast recipe; bf16: Megatron's default; "
                         "auto, the default: bf16 with --fp8, else fp32)")
    ap.add_argument("--wgrad-group", type=int, default=1, choices=[0, 1],
                    help="the MLP's down and gate|up weight gradients as one grouped own-kernel launch (1, default)")
    ap.add_argument("--wgrad-variant", default=None,
                    help="ND_WGRAD_VARIANT for the weight-gradient kernel (A/B of kernel schedules)")
    ap.add_argument("--attn-fused-stats", type=int, default=1, choices=[0, 1],
                    help="attention backward: row statistics inside the dQ kernel (0: separate passes)")
    ap.add_argument("--dgrad-t", type=int, default=1, choices=[0, 1],
                    help="input-gradient GEMMs on transposed weight copies (K-contiguous NT layout)")
    ap.add_argument("--proj-gemm", default="blas", choices=["pp", "blas", "short", "w128"],
                    help="plain projection / lm-head GEMMs: hipBLASLt (blas, default) or the own ping-pong "
                         "MFMA kernel (pp); the fused-epilogue GEMMs always run on the own kernel")
    ap.add_argument("--fused-rope", type=int, default=1, choices=[0, 1],
                    help="RoPE in the q|k|v GEMM epilogue (own kernel) vs a separate rotation pass")
    ap.add_argument("--fused-mlp", type=int, default=1, choices=[0, 1],
                    help="SwiGLU in the gate|up GEMM epilogue and its backward in the down dgrad epilogue")
    ap.add_argument("--mlp-coef", type=int, default=-1, choices=[-1, 0, 1],
                    help="saved-tensor form of the fused SwiGLU pair: 1 derivative coefficients (the library default, "
                         "profiles/r6_mlp_coef_ab.md), 0 gate / up; -1 keeps the library's setting (ND_MLP_COEF)")
    ap.add_argument("--fp8", action="store_true", help="fp8 (e4m3/e5m2) decoder projections (BASELINE config 5)")
    ap.add_argument("--fp8-wgrad", type=int, default=1, choices=[0, 1],
                    help="with --fp8: weight-gradient GEMMs in fp8 too (own kernel on the token-major fp8 "
                         "operands; default on)")
    ap.add_argument("--fp8-gemm", default="pp", choices=["pp", "auto", "hipblaslt"],
                    help="with --fp8: forward / input-gradient fp8 GEMMs: pp (default: the own fp8 ping-pong kernel "
                         "with the fused epilogues for every product), auto (hipBLASLt for the long-K N<=1024 plain "
                         "products) or hipblaslt")
    ap.add_argument("--fp8-fused-epi", type=int, default=1, choices=[0, 1],
                    help="with --fp8 and --fp8-gemm pp: RoPE / SwiGLU fused into the fp8 GEMM epilogues")
    ap.add_argument("--fp8-keep-fused", default="none", choices=["none", "rope", "mlp", "both"],
                    help="with --fp8: projections that stay on the bf16 fused-epilogue GEMMs")
    ap.add_argument("--fp8-lm-head", type=int, default=1, choices=[0, 1],
                    help="with --fp8: the lm head's three GEMMs in fp8 on the own kernels (1, default) or bf16 (0)")
    ap.add_argument("--fp8-fused-quant", type=int, default=1, choices=[0, 1],
                    help="with --fp8: operand quantisation fused into the producing kernels (0: separate casts)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    return ap.parse_args()


def _mlp_form():
    """'coef' / 'gate_up': the fused SwiGLU pair's saved-tensor form that ran (None without the HIP library)."""
    if not torch.cuda.is_available():
        return None
    try:
        from nanodiloco_amd.ops.gemm import mlp_coef
        return "coef" if mlp_coef() else "gate_up"
    except Exception:
        return None


def main():
    a = parse()
    # kernel-path switches the trainer does not own (A/B flags); set before the model is built
    ops.set_proj_gemm(a.proj_gemm)
    ops.set_fused_epilogues(rope=bool(a.fused_rope), mlp=bool(a.fused_mlp))
    if a.mlp_coef >= 0 and torch.cuda.is_available():
        from nanodiloco_amd.ops.gemm import set_mlp_coef
        set_mlp_coef(a.mlp_coef)
    ops.set_dgrad_transposed(bool(a.dgrad_t))
    ops.set_attn_fused_stats(bool(a.attn_fused_stats))
    if a.fp8:
        from nanodiloco_amd.ops import fp8 as _fp8
        _fp8.set_fused_quant(bool(a.fp8_fused_quant))
        _fp8.set_fp8_gemm(a.fp8_gemm)
        _fp8.set_fp8_fused_epilogues(bool(a.fp8_fused_epi))
        _fp8.set_fp8_keep_fused(a.fp8_keep_fused)
        _fp8.set_fp8_lm_head(bool(a.fp8_lm_head))
    if a.wgrad_variant:
        os.environ["ND_WGRAD_VARIANT"] = a.wgrad_variant
    world = int(os.environ.get("WORLD_SIZE", "1"))
    H = a.inner_steps
    # the product's training step: Trainer.inner_step (micro-batch fwd+bwd, inner-DDP sync, clip +
    # AdamW) and Diloco.outer_step, exactly what `python -m nanodiloco_amd` runs
    targs = TrainArgs(
        seed=1337, batch_size=a.batch_size, per_device_batch_size=a.micro_batch, seq_length=a.seq_len,
        warmup_steps=100, total_steps=H * max(1, -(-10_000 // H)), inner_steps=H, lr=4e-4, outer_lr=0.7,
        llama_config_file=a.model, data="synthetic", ops=a.ops, backend="auto" if a.backend == "none" else a.backend,
        inner_dp=a.inner_dp, comm_impl=a.comm_impl,
        comm_dtype=a.comm_dtype, bucket_mb=a.bucket_mb, overlap_outer=a.overlap_outer, fp8=a.fp8,
        fp8_wgrad=bool(a.fp8_wgrad), fp8_keep_fused=a.fp8_keep_fused, tuned_gemm=not a.no_tuned_gemm and not a.tuned_gemm_file,
        hip_graph="on" if a.hip_graph else "off", wgrad_overlap=bool(a.wgrad_overlap), log_every=0, wandb="off",
        phase_timing=False, force_collectives=a.backend != "none" and world == 1, deterministic=a.deterministic,
        residual_dtype=a.residual_dtype)
    tr = Trainer(targs)
    env, cfg, dl = tr.env, tr.llama_config, tr.diloco
    ops.set_wgrad_overlap(a.wgrad_overlap)  # mode 2 (unfenced A/B) is not a trainer option
    ops.set_wgrad_group(bool(a.wgrad_group))
    if env.world_size != a.gpus and env.rank == 0:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={env.world_size}", file=sys.stderr)
    if env.device.type == "cuda" and a.tuned_gemm_file:
        enable_tuned_gemms(env.device, a.tuned_gemm_file)
    micro = targs.per_device_batch_size  # resolved by the trainer
    accum = tr.grad_accum
    tr.model.train()
    state = {"step": 0}

    def inner_step():
        loss = tr.inner_step()
        state["step"] += 1
        outer_done = False
        if state["step"] % H == 0:
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
    # one more outer step, untimed and serialized, split into pseudo-gradient / all-reduce / update
    phases = {}
    if not a.overlap_outer and env.device.type == "cuda":
        dl.outer_step(phases=True)
        phases = dl.outer_phase_ms()
    vals = [outer_ms] + [phases.get(k, 0.0) for k in ("pseudograd_ms", "allreduce_ms", "outer_update_ms")]
    if env.is_distributed:
        t = torch.tensor(vals, dtype=torch.float64, device=env.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = t.tolist()
    outer_ms = vals[0]
    tokens = a.batch_size * a.seq_len * a.steps * env.world_size
    tps = tokens / elapsed
    final_loss = float(loss.item()) if loss is not None else float("nan")
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
        comm_dtype = torch.bfloat16 if a.comm_dtype == "bf16" else torch.float32
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
            "dtype": ("fp8" if a.fp8 else "bf16") if tr.compute_dtype == torch.bfloat16 else "fp32",
            "data": "synthetic",
            "config": {
                "model": model_name,
                "global_batch": a.batch_size * env.world_size,
                "seq_len": a.seq_len,
                "parallelism": f"diloco{env.num_workers}" + (f"x_ddp{env.inner_dp}" if env.inner_dp > 1 else ""),
                "per_worker_batch": a.batch_size,
                "micro_batch": micro,
                "grad_accum": accum,
                "inner_steps_H": a.inner_steps,
                "params": cfg.num_params(),
            },
            "step_driver": "Trainer.inner_step",
            "bytes_per_outer_step": dl.bytes_per_outer_step if dl.outer_comm.enabled else tr.model.store.numel * (
                2 if comm_dtype == torch.bfloat16 else 4),
            "outer_steps_in_window": n_outer,
            # outer-step cost as seen by the compute stream (HIP events: pseudo-gradient + bucketed
            # RCCL all-reduce + fused Nesterov), host wall time per outer step, and calls per outer step
            "outer_step_ms": round(outer_ms, 3),
            # the same step serialized, per phase (untimed, after the window): what RCCL costs per N
            "outer_phase_ms": {k: round(v, 3) for k, v in
                               zip(("pseudograd", "allreduce", "outer_update"), vals[1:])} if phases else None,
            "outer_step_wall_ms": round(1000.0 * dl.avg_sync_time, 3),
            "allreduce_calls_per_outer_step": dl.buckets_per_outer_step,
            "comm_backend": env.backend,
            "comm_impl": dl.outer_comm.impl if dl.outer_comm.enabled else env.comm_impl,  # after any agreed fallback
            "rccl_calls": (dl.outer_comm.rccl.stats()["calls"] if dl.outer_comm.rccl is not None else None),
            "comm_dtype": a.comm_dtype,
            "model_tflops_per_gpu": round(mfu_flops / 1e12, 2),
            "final_loss": round(final_loss, 4),
            "tuned_gemm": enable_tuned_gemms(env.device) if env.device.type == "cuda" and not a.no_tuned_gemm else False,
            "wgrad_overlap": ops.wgrad_overlap_enabled(),
            "wgrad_group": ops.wgrad_group_enabled(),
            "residual_dtype": "bf16" if tr.model.residual_dtype == torch.bfloat16 else "fp32",
            "deterministic": bool(a.deterministic),
            "proj_gemm": ops.proj_gemm(),
            "fused_epilogues": ops.fused_epilogues(),
            "mlp_saved_form": _mlp_form(),
            "fp8_gemm": a.fp8_gemm if a.fp8 else None,
            "fp8_fused_epilogues": bool(a.fp8_fused_epi) if a.fp8 else None,
            "fp8_keep_fused": a.fp8_keep_fused if a.fp8 else None,
            "fp8_lm_head": bool(a.fp8_lm_head) if a.fp8 else None,
            "dgrad_transposed": ops.dgrad_transposed_enabled(),
            "ops": ops.get_backend() if a.ops != "auto" else ("hip" if env.device.type == "cuda" else "torch"),
        }
        print(json.dumps(out), flush=True)
    if env.is_distributed:
        from nanodiloco_amd.parallel.dist import destroy_distributed
        destroy_distributed()


if __name__ == "__main__":
    main()
