#!/usr/bin/env python3
"""In-process A/B of the attention forward's deferred-max threshold (ND_ATTN_THR) on the Llama-150M
attention shape: B=64, T=1024, 16 heads x 64 (and the 1B GQA 32/4 shape)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops.attention import rope_cache  # noqa: E402


def bench(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


ops.set_backend("hip")
for (B, T, nh, nkv, hd) in [(64, 1024, 16, 16, 64), (16, 1024, 32, 4, 64)]:
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, "cuda")
    fl = 2 * 2 * B * nh * T * T * hd / 2
    res = {}
    for rnd in range(3):
        for thr in os.environ.get("THRS", "0,8").split(","):
            os.environ["ND_ATTN_THR"] = thr
            res.setdefault(thr, []).append(bench(lambda: ops.attention(qkv, cos, sin, B, T, nh, nkv, hd)))
    print(f"B{B} T{T} h{nh}/{nkv} d{hd}: " + "  ".join(
        f"thr={k}: {min(v) * 1e6:.1f} us {fl / min(v) / 1e12:.0f} TF/s" for k, v in res.items()), flush=True)
