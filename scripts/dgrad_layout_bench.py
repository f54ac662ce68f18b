#!/usr/bin/env python3
"""Input-gradient (dgrad) GEMM layout A/B on the Llama-150M shapes (one 64k-token micro-batch).

dX[N, in] = dY[N, out] @ W[out, in] is a row-major x row-major ("NN") product for hipBLASLt.  The
same product with a transposed weight copy Wt[in, out] is dY @ Wt^T -- the "NT" layout of the
forward GEMMs, which hipBLASLt runs faster at K = 1024.  Prints us and TF/s per (shape, layout),
interleaving the arms so clock drift hits both equally."""
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
    if os.environ.get("TUNED", "1") == "1":
        from nanodiloco_amd.ops.tuned_gemm import enable_tuned_gemms
        print("tuned table:", enable_tuned_gemms(torch.device("cuda")))
    N = int(os.environ.get("TOKENS", 65536))
    d, F, V = 1024, 2688, 32000
    shapes = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F), "lm_head": (V, d)}
    torch.manual_seed(0)
    for name, (out, inn) in shapes.items():
        n = N if name != "lm_head" else 16384
        dy = torch.randn(n, out, device="cuda").bfloat16()
        w = (torch.randn(out, inn, device="cuda") * 0.02).bfloat16()
        wt = w.t().contiguous()
        fl = 2.0 * n * out * inn
        res = {"NN dy@W": [], "NT dy@(Wt)^T": []}
        for _ in range(3):
            res["NN dy@W"].append(bench(lambda: torch.mm(dy, w)))
            res["NT dy@(Wt)^T"].append(bench(lambda: torch.mm(dy, wt.t())))
        ref = torch.mm(dy, w).float()
        err = ((torch.mm(dy, wt.t()).float() - ref).norm() / ref.norm()).item()
        tt = bench(lambda: w.t().contiguous(), iters=10)
        for k, ts in res.items():
            t = min(ts)
            print(f"{name:8s} {k:14s} {t*1e6:9.1f} us  {fl / t / 1e12:7.1f} TF/s", flush=True)
        print(f"{name:8s} transpose copy {tt*1e6:9.1f} us   rel err NT vs NN {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
