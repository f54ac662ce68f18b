#!/usr/bin/env python3
"""fp8 ping-pong GEMM (csrc/gemm_pp.hip F8 instantiations) against hipBLASLt fp8 (torch._scaled_mm) and
the bf16 kernels, Llama-150M projection shapes at --tokens, interleaved rounds, medians.

    python scripts/gemm_pp_f8_bench.py [--tokens 131072] [--rounds 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402

E4, E5 = torch.float8_e4m3fn, torch.float8_e5m2


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


def q8(x, dt):
    fmax = 448.0 if dt == E4 else 57344.0
    s = fmax / x.abs().amax().clamp_min(1e-12) / 2
    return (x * s).to(dt), (1.0 / s).reshape(1).float()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    ops.set_backend("hip")
    M, d, F, V = a.tokens, 1024, 2688, 32000
    cases = []

    def plain(name, n, k, adt):
        x = torch.randn(M, k, device="cuda")
        w = torch.randn(n, k, device="cuda") * 0.05
        x8, sa = q8(x, adt)
        w8, sb = q8(w, E4)
        xb, wb = x.bfloat16(), w.bfloat16()
        out = torch.empty(M, n, device="cuda", dtype=torch.bfloat16)
        arms = {"blas f8": lambda: torch._scaled_mm(x8, w8.t(), sa, sb, out_dtype=torch.bfloat16),
                "pp f8": lambda: G.gemm_pp_f8(x8, w8, sa, sb, out),
                "blas bf16": lambda: torch.mm(xb, wb.t(), out=out)}
        err = ((G.gemm_pp_f8(x8, w8, sa, sb).float() - (x8.float() @ w8.float().t()) * sa * sb).norm()
               / ((x8.float() @ w8.float().t()) * sa * sb).norm()).item()
        print(f"check {name}: rel {err:.2e}", flush=True)
        cases.append((name, 2.0 * M * n * k, arms))

    plain("qkv fwd", 3 * d, d, E4)
    plain("o fwd", d, d, E4)
    plain("gu fwd", 2 * F, d, E4)
    plain("down fwd", d, F, E4)
    plain("qkv dgrad", d, 3 * d, E5)
    plain("o dgrad", d, d, E5)
    plain("gu dgrad", d, 2 * F, E5)
    plain("down dgrad", F, d, E5)
    # fused epilogues: fp8 pp vs bf16 pp
    T, hd = 1024, 64
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, "cuda")
    x = torch.randn(M, d, device="cuda")
    wq, wgu, wdt = (torch.randn(n, d, device="cuda") * 0.05 for n in (3 * d, 2 * F, F))
    x8, sx = q8(x, E4)
    dy8, sdy = q8(x, E5)
    wq8, sq = q8(wq, E4)
    wgu8, sgu = q8(wgu, E4)
    wdt8, sdt = q8(wdt, E4)
    xb, wqb, wgub, wdtb = x.bfloat16(), wq.bfloat16(), wgu.bfloat16(), wdt.bfloat16()
    gu, act = G.gemm_pp_swiglu(xb, wgub)
    dgu = torch.empty_like(gu)
    cases.append(("qkv+rope", 2.0 * M * 3 * d * d,
                  {"pp f8": lambda: G.gemm_pp_rope_f8(x8, wq8, sx, sq, cos, sin, T, hd, 2 * d),
                   "pp bf16": lambda: G.gemm_pp_rope(xb, wqb, cos, sin, T, hd, 2 * d)}))
    cases.append(("gu+swiglu", 2.0 * M * 2 * F * d,
                  {"pp f8": lambda: G.gemm_pp_swiglu_f8(x8, wgu8, sx, sgu, gu, act),
                   "pp bf16": lambda: G.gemm_pp_swiglu(xb, wgub, gu, act)}))
    cases.append(("down dgrad+dswiglu", 2.0 * M * F * d,
                  {"pp f8": lambda: G.gemm_pp_dswiglu_f8(dy8, wdt8, sdy, sdt, gu, dgu),
                   "pp bf16": lambda: G.gemm_pp_dswiglu(xb, wdtb, gu, dgu)}))
    # weight gradients: bf16 wgrad_pp vs fp8 wgrad8_pp on the same token-major operands
    for name, m_, n_ in (("wgrad qkv", 3 * d, d), ("wgrad o", d, d), ("wgrad gate|up", 2 * F, d), ("wgrad down", d, F)):
        dyf, xf = torch.randn(M, m_, device="cuda"), torch.randn(M, n_, device="cuda")
        dy8_, sdy_ = q8(dyf, E5)
        x8_, sx_ = q8(xf, E4)
        dyb, xb_ = dyf.bfloat16(), xf.bfloat16()
        gw = torch.zeros(m_, n_, device="cuda")
        cases.append((name, 2.0 * M * m_ * n_,
                      {"wgrad f8": (lambda g=gw, a_=dy8_, b_=x8_, s1=sdy_, s2=sx_: G.wgrad_f8(g, a_, b_, s1, s2)),
                       "wgrad bf16": (lambda g=gw, a_=dyb, b_=xb_: G.wgrad(g, a_, b_))}))
    res = {}
    for _ in range(a.rounds):
        for name, fl, arms in cases:
            for arm, fn in arms.items():
                res.setdefault((name, arm), []).append(timed(fn))
    tot = {}
    for name, fl, arms in cases:
        line = f"{name:19s}"
        for arm in arms:
            t = sorted(res[(name, arm)])[a.rounds // 2]
            tot[arm] = tot.get(arm, 0.0) + t
            line += f" | {arm} {t:8.1f} us {fl / t / 1e6:5.0f} TF"
        print(line, flush=True)
    print("total " + " ".join(f"{k} {v:.0f} us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
