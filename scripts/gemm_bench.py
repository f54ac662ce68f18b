#!/usr/bin/env python3
"""Micro-benchmark of the Llama-150M GEMM shapes (one 32k-token micro-batch) on the library paths,
to choose the wgrad / lm-head strategy.  Prints TFLOP/s per (shape, variant)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    N = int(os.environ.get("TOKENS", 32768))
    d, F, V = 1024, 2688, 32000
    dev = "cuda"
    shapes = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F), "lm_head": (V, d)}
    torch.manual_seed(0)
    for name, (out, inn) in shapes.items():
        n = N if name != "lm_head" else 16384
        x = torch.randn(n, inn, device=dev).bfloat16()
        dy = torch.randn(n, out, device=dev).bfloat16()
        w = torch.randn(out, inn, device=dev).bfloat16()
        gw = torch.zeros(out, inn, device=dev)
        fl = 2.0 * n * out * inn
        res = {}
        res["fwd x@wT"] = bench(lambda: torch.mm(x, w.t()))
        res["dgrad dy@w"] = bench(lambda: torch.mm(dy, w))
        res["wgrad addmm fp32out"] = bench(
            lambda: torch.ops.aten.addmm.dtype_out(gw, dy.t(), x, torch.float32, beta=1, alpha=1, out=gw))
        res["wgrad mm bf16 + add"] = bench(lambda: gw.add_(torch.mm(dy.t(), x)))
        res["wgrad mm(out fp32) + add"] = bench(lambda: gw.add_(torch.mm(dy.t(), x, out_dtype=torch.float32)))
        res["wgrad x^T dy (transposed) bf16"] = bench(lambda: torch.mm(x.t(), dy))
        xt = x.t().contiguous()
        dyt = dy.t().contiguous()
        res["wgrad contiguousT dyT@x"] = bench(lambda: torch.mm(dyt, xt.t()))
        for k, t in res.items():
            print(f"{name:8s} {k:32s} {t*1e6:9.1f} us  {fl / t / 1e12:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
