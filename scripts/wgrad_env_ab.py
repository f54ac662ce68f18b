#!/usr/bin/env python3
"""In-process interleaved A/B of weight-gradient kernel variants (ND_WGRAD_VARIANT is read per call)
on the Llama-150M wgrad shapes at 65,536 tokens (lm head: 16,384-token chunks).

    python scripts/wgrad_env_ab.py --variants ,dma0 --rounds 7   (default = ping-pong kernel, dma0 = round-2 kernel)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops.gemm import wgrad  # noqa: E402


def timed(fn, iters=5):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default=",dma0")
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    vs = a.variants.split(",")
    shapes = [("qkv", 3072, 1024, 65536), ("o", 1024, 1024, 65536), ("gu", 5376, 1024, 65536),
              ("down", 1024, 2688, 65536), ("lm", 32000, 1024, 16384)]
    tot = {v: 0.0 for v in vs}
    for name, M, N, K in shapes:
        dy = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
        gw = torch.zeros(M, N, device="cuda")
        ts = {v: [] for v in vs}
        for _ in range(a.rounds):
            for v in vs:
                os.environ["ND_WGRAD_VARIANT"] = v
                ts[v].append(timed(lambda: wgrad(gw, dy, x)))
        fl = 2.0 * M * N * K
        line = f"{name:6s}"
        for v in vs:
            t = sorted(ts[v])[len(ts[v]) // 2]
            tot[v] += t
            line += f" | {v or 'default':7s} {t:8.1f} us {fl / t / 1e6:6.0f} TF/s"
        print(line, flush=True)
    base = tot[vs[0]]
    print("TOTAL " + " | ".join(f"{v or 'default'} {tot[v]:.1f} us ({base / tot[v]:.3f}x)" for v in vs), flush=True)


if __name__ == "__main__":
    main()
