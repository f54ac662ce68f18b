#!/usr/bin/env python3
"""A/B of the software-pipelined one-wave-per-SIMD dK/dV kernel (ND_ATTN_DKDV=sp, csrc/attention.hip
attn_bwd_dkdv_sp_kernel) against the default two-waves-per-SIMD one, inside the default fused backward:
bitwise comparison of d(q|k|v), then interleaved timing (medians).  Shapes: Llama-150M (16/16 heads) and
Llama-1B (32/4 GQA), head_dim 64, T = 1024.

    python scripts/attn_dkdv_sp_ab.py [--rounds 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops.attention import rope_cache  # noqa: E402


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    ops.set_backend("hip")
    bad = 0
    for (B, nh, nkv) in ((64, 16, 16), (32, 32, 4)):
        T, hd = 1024, 64
        ld = (nh + 2 * nkv) * hd
        cos, sin = rope_cache(T, hd, 10000.0, None, "cuda")
        x = (torch.randn(B * T, ld, device="cuda") * 2).bfloat16().requires_grad_(True)
        o = ops.attention(x, cos, sin, B, T, nh, nkv, hd, rotated=True)
        do = torch.randn_like(o)
        bwd = lambda: torch.autograd.grad(o, x, do, retain_graph=True)[0]  # noqa: E731
        os.environ.pop("ND_ATTN_DKDV", None)
        g0 = bwd().clone()
        os.environ["ND_ATTN_DKDV"] = "sp"
        g1 = bwd().clone()
        same = torch.equal(g0, g1)
        err = ((g1.float() - g0.float()).norm() / g0.float().norm()).item()
        bad += not (err < 1e-3)
        print(f"B={B} nh={nh} nkv={nkv}: sp == default bitwise {same}, rel diff {err:.2e}", flush=True)
        res = {"default": [], "sp": []}
        for _ in range(a.rounds):
            for arm in res:
                if arm == "sp":
                    os.environ["ND_ATTN_DKDV"] = "sp"
                else:
                    os.environ.pop("ND_ATTN_DKDV", None)
                res[arm].append(timed(bwd))
        os.environ.pop("ND_ATTN_DKDV", None)
        t0 = sorted(res["default"])[a.rounds // 2]
        t1 = sorted(res["sp"])[a.rounds // 2]
        print(f"  backward (dQ + dK/dV): default {t0:8.1f} us | sp {t1:8.1f} us | {t0 / t1:.3f}x", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
