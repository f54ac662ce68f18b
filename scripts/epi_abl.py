#!/usr/bin/env python3
"""Fused-epilogue ablation timing (round 5; q|k|v + RoPE added in round 6): gemm_pp_dswiglu / gemm_pp_swiglu /
gemm_pp_rope at the Llama-150M bench shape
(131,072 tokens) next to the plain ping-pong GEMM of the same product.  The variant (ND_GEMM_PP_VARIANT: 0
default, 8 no epilogue, 4096 no gate/up loads, 8192 no HBM stores, 16384 no RoPE table loads) is read once per process; the ablation
variants exist only in the -DND_ABLATION library (ND_KERNELS_LIB) and give WRONG results (timing only)."""
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
    dy, wdt, gu = r(M, d), r(F, d), r(M, 2 * F)
    dgu = torch.empty_like(gu)
    x, wgu = r(M, d), r(2 * F, d)
    gu_o, act_o = torch.empty(M, 2 * F, dtype=torch.bfloat16, device="cuda"), torch.empty(M, F, dtype=torch.bfloat16, device="cuda")
    plain_d, plain_s = torch.empty(M, F, dtype=torch.bfloat16, device="cuda"), torch.empty(M, 2 * F, dtype=torch.bfloat16, device="cuda")
    from nanodiloco_amd.ops.attention import rope_cache
    wqkv = r(3 * d, d)
    qkv_o = torch.empty(M, 3 * d, dtype=torch.bfloat16, device="cuda")
    cos, sin = rope_cache(1024, 64, 10000.0, None, "cuda")
    res = {}
    for _ in range(3):
        res.setdefault("dswiglu", []).append(timed(lambda: G.gemm_pp_dswiglu(dy, wdt, gu, dgu)))
        res.setdefault("plain down dgrad", []).append(timed(lambda: G.gemm_pp(dy, wdt, plain_d)))
        res.setdefault("swiglu", []).append(timed(lambda: G.gemm_pp_swiglu(x, wgu, gu_o, act_o)))
        res.setdefault("plain gate|up fwd", []).append(timed(lambda: G.gemm_pp(x, wgu, plain_s)))
        res.setdefault("qkv+rope", []).append(timed(lambda: G.gemm_pp_rope(x, wqkv, cos, sin, 1024, 64, 2048, qkv_o)))
        res.setdefault("plain qkv fwd", []).append(timed(lambda: G.gemm_pp(x, wqkv, qkv_o)))
    v = os.environ.get("ND_GEMM_PP_VARIANT", "0")
    print("variant " + v + " | " + " | ".join(f"{k} {sorted(t)[1]:.1f} us" for k, t in res.items()), flush=True)


if __name__ == "__main__":
    main()
