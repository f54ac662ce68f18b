#!/usr/bin/env python3
"""Reference-equivalent eager baseline: the reference's training algorithm, verbatim in
structure, on stock PyTorch-ROCm + HF transformers, measured on the same MI355X box.

  * HF ``LlamaForCausalLM(LlamaConfig(**json))`` (REF/nanodiloco/main.py:97-99), eager/SDPA attention
  * ``torch.optim.AdamW(lr)`` + ``SGD(outer_lr, momentum=0.9, nesterov=True)`` (:100-101)
  * per micro-batch ``model(**batch).loss.backward()`` + ``loss.item()`` logging sync (:109-123)
  * inner step: ``clip_grad_norm_(1.0)``, ``opt.step()``, HF cosine schedule, ``zero_grad`` (diloco.py:56-60)
  * outer step every H: per-tensor pageable H2D snapshot, ``all_reduce(AVG)``, Nesterov, CPU re-snapshot
    (diloco.py:34-54)
  * synthetic tokens instead of c4-tiny (no network); ``--autocast bf16`` or fp32 (the reference's dtype)

Prints one JSON line like bench.py so the two can be compared directly.
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="configs/llama_150m.json")
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--micro-batch", type=int, default=8)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--inner-steps", type=int, default=100)
    ap.add_argument("--autocast", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--attn", default="sdpa", choices=["sdpa", "eager"])
    a = ap.parse_args()
    from transformers import LlamaConfig, LlamaForCausalLM, get_cosine_schedule_with_warmup

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    cfg = json.load(open(a.model))
    model = LlamaForCausalLM(LlamaConfig(**cfg, attn_implementation=a.attn)).to(dev)
    inner = torch.optim.AdamW(model.parameters(), lr=4e-4)
    outer = torch.optim.SGD(model.parameters(), lr=0.7, momentum=0.9, nesterov=True)
    sched = get_cosine_schedule_with_warmup(inner, num_warmup_steps=100, num_training_steps=10000)
    if world > 1:
        for p in model.parameters():
            dist.broadcast(p.data, src=0)
    snap = [p.data.detach().clone().to("cpu") for p in model.parameters()]
    accum = a.batch_size // a.micro_batch
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.autocast == "bf16")
    step = {"n": 0}

    def outer_step():
        nonlocal snap
        for p, s in zip(model.parameters(), snap):
            sd = s.to(p.device)
            p.grad = sd - p.data
            if world > 1:
                dist.all_reduce(p.grad, op=dist.ReduceOp.AVG)
            p.data = sd
        outer.step()
        outer.zero_grad()
        snap = [p.data.detach().clone().to("cpu") for p in model.parameters()]

    def inner_step():
        for _ in range(accum):
            ids = torch.randint(0, cfg.get("vocab_size", 32000), (a.micro_batch, a.seq_len), device=dev, generator=g)
            with ac:
                out = model(input_ids=ids, labels=ids)
            loss = out.loss / accum
            out.loss.backward()
            _ = loss.item(), torch.exp(loss).item()  # the reference's per-micro-batch logging syncs
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
        inner.step()
        sched.step()
        inner.zero_grad()
        step["n"] += 1
        if step["n"] % a.inner_steps == 0:
            outer_step()

    for _ in range(a.warmup):
        inner_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        inner_step()
    if a.steps < a.inner_steps:
        outer_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    tps = a.batch_size * a.seq_len * a.steps * world / el
    if rank == 0:
        print(json.dumps({"metric": "reference-equivalent eager tokens/s", "value": round(tps, 1), "n_gpus": world,
                          "ms_per_step": round(1000 * el / a.steps, 2), "micro_batch": a.micro_batch,
                          "autocast": a.autocast, "attn": a.attn, "model": os.path.basename(a.model)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
