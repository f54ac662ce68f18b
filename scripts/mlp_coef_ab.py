#!/usr/bin/env python3
"""In-process A/B of the fused SwiGLU pair's saved-tensor form (ops.gemm.set_mlp_coef: 0 gate / up, 1 coefficient
form): the gate|up + SwiGLU and down-dgrad + SwiGLU-backward kernels at the Llama-150M bench shape (131,072 tokens),
bf16 and fp8, interleaved, median of 5 rounds.

    python scripts/mlp_coef_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters=10):
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
    M, F, d = 131072, 2688, 1024
    r = lambda *s: ((torch.rand(*s, device="cuda") * 2 - 1) * 0.05).bfloat16()  # noqa: E731
    x, wgu, dy, wdt, gu = r(M, d), r(2 * F, d), r(M, d), r(F, d), r(M, 2 * F)
    e4, e5 = torch.float8_e4m3fn, torch.float8_e5m2
    x8, wgu8, dy8, wdt8 = x.to(e4), wgu.to(e4), dy.to(e5), wdt.to(e4)
    one = torch.ones(1, device="cuda")
    arms = {
        "swiglu": lambda: G.gemm_pp_swiglu(x, wgu),
        "dswiglu": lambda: G.gemm_pp_dswiglu(dy, wdt, gu),
        "swiglu_f8": lambda: G.gemm_pp_swiglu_f8(x8, wgu8, one, one),
        "dswiglu_f8": lambda: G.gemm_pp_dswiglu_f8(dy8, wdt8, one, one, gu),
    }
    res = {}
    old = G.mlp_coef()
    for _ in range(5):
        for form in (0, 1):
            G.set_mlp_coef(form)
            for k, fn in arms.items():
                res.setdefault((k, form), []).append(timed(fn))
    G.set_mlp_coef(old)
    for k in arms:
        a, b = sorted(res[(k, 0)])[2], sorted(res[(k, 1)])[2]
        print(f"{k:11s} gate/up form {a:8.1f} us | coefficient form {b:8.1f} us | {a / b:.3f}x", flush=True)


if __name__ == "__main__":
    main()
