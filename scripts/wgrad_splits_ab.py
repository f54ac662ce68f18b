#!/usr/bin/env python3
"""Per-kernel time of the bf16 weight gradient at forced split counts (nd_wgrad_force_splits), Llama-150M shapes at
131,072 tokens, interleaved, median of 3 rounds (slab reduction included)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import _ext, gemm as G  # noqa: E402


def timed(fn, iters=6):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ops.set_backend("hip")
    K = int(os.environ.get("TOKENS", 131072))
    L = _ext.lib()
    shapes = {"qkv": (3072, 1024), "o": (1024, 1024), "gu": (5376, 1024), "down": (1024, 2688)}
    arms = [0, 2, 3, 4, 5, 6, 8, 16]
    data = {k: (torch.randn(K, m, device="cuda").bfloat16(), torch.randn(K, n, device="cuda").bfloat16(),
                torch.zeros(m, n, device="cuda")) for k, (m, n) in shapes.items()}
    res = {}
    for _ in range(3):
        for k, (dy, x, gw) in data.items():
            for s in arms:
                L.nd_wgrad_force_splits(s)
                res.setdefault((k, s), []).append(timed(lambda: G.wgrad(gw, dy, x)))
    L.nd_wgrad_force_splits(0)
    for k in shapes:
        plan_s = L.nd_wgrad_splits(*shapes[k], K)
        print(f"{k:5s} plan S={plan_s}: " + " | ".join(f"S{s if s else 'plan'} {sorted(res[(k, s)])[1]:7.1f}" for s in arms),
              flush=True)


if __name__ == "__main__":
    main()
