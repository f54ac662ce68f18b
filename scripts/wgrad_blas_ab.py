#!/usr/bin/env python3
"""Weight-gradient GEMM: the own ping-pong kernel (csrc/gemm_wgrad.hip wgrad_pp_kernel, dW += dY^T X into the
fp32 gradient) against hipBLASLt doing the same accumulate (torch.addmm(gw, dY^T, X, out_dtype=float32,
out=gw): bf16 operands, fp32 C = D, beta = 1), Llama-150M shapes at --tokens, interleaved rounds, medians.

    python scripts/wgrad_blas_ab.py [--tokens 131072] [--rounds 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402
from gdma_ab import r, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    ops.set_backend("hip")
    M, d, F, V = a.tokens, 1024, 2688, 32000
    cases = {}
    for name, m_, n_ in (("qkv", 3 * d, d), ("o", d, d), ("gate|up", 2 * F, d), ("down", d, F), ("lm head", V, d)):
        dy, x = r(M, m_), r(M, n_)
        g1 = torch.zeros(m_, n_, device="cuda")
        g2 = torch.zeros(m_, n_, device="cuda")
        G.wgrad(g1, dy, x)
        torch.addmm(g2, dy.t(), x, out_dtype=torch.float32, out=g2)
        err = ((g1 - g2).norm() / g1.norm()).item()
        print(f"{name}: own vs hipBLASLt rel diff {err:.2e}", flush=True)
        cases[name] = (2.0 * M * m_ * n_,
                       {"own": (lambda g=g1, a_=dy, b_=x: G.wgrad(g, a_, b_)),
                        "blas": (lambda g=g2, a_=dy, b_=x: torch.addmm(g, a_.t(), b_, out_dtype=torch.float32, out=g))})
    res = {}
    for _ in range(a.rounds):
        for name, (fl, arms) in cases.items():
            for arm, fn in arms.items():
                res.setdefault((name, arm), []).append(timed(fn))
    tot = {}
    for name, (fl, arms) in cases.items():
        line = f"{name:8s}"
        for arm in arms:
            t = sorted(res[(name, arm)])[a.rounds // 2]
            tot[arm] = tot.get(arm, 0.0) + t
            line += f" | {arm} {t:8.1f} us {fl / t / 1e6:5.0f} TF"
        print(line, flush=True)
    print("total " + " ".join(f"{k} {v:.0f} us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
