#!/usr/bin/env python3
"""A/B of the wgrad GEMM variants (LDS-DMA vs register-staged vs hipBLASLt) on the Llama-150M shapes,
interleaved in one process (cdna guide §5.4 rule 24)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops.gemm import wgrad  # noqa: E402


def t(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - s) / iters


def main():
    N = int(os.environ.get("TOKENS", 32768))
    shapes = {"qkv": (3072, 1024, N), "o": (1024, 1024, N), "gate_up": (5376, 1024, N), "down": (1024, 2688, N),
              "lm_head": (32000, 1024, 16640)}
    for name, (M, Nn, K) in shapes.items():
        dy = torch.randn(K, M, device="cuda").bfloat16()
        x = torch.randn(K, Nn, device="cuda").bfloat16()
        gw = torch.zeros(M, Nn, device="cuda")
        fl = 2.0 * M * Nn * K
        res = {}
        for rnd in range(3):
            for v in os.environ.get("VARIANTS", "dma,dma0,blas").split(","):
                if v == "blas":
                    f = lambda: torch.ops.aten.addmm.dtype_out(gw, dy.t(), x, torch.float32, beta=1, alpha=1, out=gw)
                else:
                    os.environ["ND_WGRAD_VARIANT"] = v
                    f = lambda: wgrad(gw, dy, x)
                res.setdefault(v, []).append(t(f))
        print(name, " ".join(f"{v}={fl / min(ts) / 1e12:7.1f}TF" for v, ts in res.items()), flush=True)
    os.environ.pop("ND_WGRAD_VARIANT", None)


if __name__ == "__main__":
    main()
