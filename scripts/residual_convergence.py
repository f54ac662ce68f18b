#!/usr/bin/env python3
"""Loss curves of Llama-150M with the fp32 and the bf16 residual stream on the same learnable synthetic data.

Every sequence follows a fixed random 'next token' map over the 32k vocabulary with 10 % of the positions
replaced by uniform noise, so the loss falls from ln(32000) = 10.37 towards the noise floor and a precision
difference in the residual stream would show up as a gap between the curves.  Same init, same batches, clip +
AdamW with a linear warmup; prints the 20-step mean loss of both runs."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.config import resolve_llama_config  # noqa: E402
from nanodiloco_amd.models import LlamaForCausalLM  # noqa: E402
from nanodiloco_amd.optim import FlatAdamW  # noqa: E402


def batches(V, B, T, steps, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    nxt = torch.randperm(V, generator=g, device="cuda")
    for _ in range(steps):
        x = torch.empty(B, T, dtype=torch.long, device="cuda")
        x[:, 0] = torch.randint(0, V, (B,), generator=g, device="cuda")
        for t in range(1, T):
            x[:, t] = nxt[x[:, t - 1]]
        noise = torch.rand(B, T, generator=g, device="cuda") < 0.1
        x[noise] = torch.randint(0, V, (int(noise.sum()),), generator=g, device="cuda")
        yield x


def run(rdt, a):
    cfg = resolve_llama_config("llama_150m.json")
    m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16, residual_dtype=rdt).init_weights(0)
    opt = FlatAdamW(m.store, lr=a.lr, weight_decay=0.01, max_grad_norm=1.0)
    losses = []
    for i, ids in enumerate(batches(cfg.vocab_size, a.batch, a.seq, a.steps)):
        out = m(ids, labels=ids)
        out.loss.backward()
        opt.step(lr=a.lr * min(1.0, (i + 1) / a.warmup))
        m.store.zero_grad()
        losses.append(out.loss.detach())
        if (i + 1) % 100 == 0:
            print(f"  {rdt} step {i + 1} loss {losses[-1].item():.4f}", flush=True)
    return torch.stack(losses).float().cpu()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=4e-4)
    ap.add_argument("--warmup", type=int, default=50)
    a = ap.parse_args()
    ops.set_backend("hip")
    t0 = time.time()
    curves = {r: run(r, a) for r in (torch.float32, torch.bfloat16)}
    f, b = curves[torch.float32], curves[torch.bfloat16]
    print(f"{a.steps} steps x {a.batch} x {a.seq} tokens, {time.time() - t0:.0f} s")
    print("steps | fp32 residual | bf16 residual | diff")
    w = 20
    worst = 0.0
    for s in range(0, a.steps, w):
        x, y = f[s:s + w].mean().item(), b[s:s + w].mean().item()
        worst = max(worst, abs(x - y)) if s >= a.warmup else worst
        print(f"{s + 1}-{s + w} | {x:.4f} | {y:.4f} | {y - x:+.4f}")
    print(f"max |diff| of 20-step means after warmup: {worst:.4f}; final 50-step means {f[-50:].mean():.4f} / "
          f"{b[-50:].mean():.4f}")


if __name__ == "__main__":
    main()
