#!/usr/bin/env python3
"""In-process A/B of an attention-kernel environment knob (e.g. ND_ATTN_ORDER=0,1 or ND_ATTN_THR=0,8):
forward and forward+backward on the Llama-150M (B=64, T=1024, 16x64) and 1B GQA (32/4) shapes.

    VAR=ND_ATTN_ORDER VALS=0,1 python scripts/attn_env_ab.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops.attention import rope_cache  # noqa: E402


def bench(fn, iters=8):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


var = os.environ.get("VAR", "ND_ATTN_ORDER")
vals = os.environ.get("VALS", "0,1").split(",")
ops.set_backend("hip")
for (B, T, nh, nkv, hd) in [(64, 1024, 16, 16, 64), (16, 1024, 32, 4, 64)]:
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, "cuda")
    x = qkv.clone().requires_grad_(True)
    do = torch.randn(B * T, nh * hd, device="cuda").bfloat16()

    def fwd():
        return ops.attention(x.detach(), cos, sin, B, T, nh, nkv, hd)

    def fwdbwd():
        o = ops.attention(x, cos, sin, B, T, nh, nkv, hd)
        o.backward(do)

    res = {}
    for rnd in range(3):
        for v in vals:
            os.environ[var] = v
            res.setdefault(("fwd", v), []).append(bench(fwd))
            res.setdefault(("f+b", v), []).append(bench(fwdbwd))
    print(f"B{B} T{T} h{nh}/{nkv} d{hd}: " + "  ".join(
        f"{k[0]} {var}={k[1]}: {min(t) * 1e6:.1f} us" for k, t in res.items()), flush=True)
