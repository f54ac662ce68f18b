#!/usr/bin/env python3
"""A/B of the dK/dV kernel's Q / dO prefetch depth (csrc/attention.hip attn_bwd_dkdv_dma_kernel NB,
env ND_ATTN_DKDV_NB = 2 | 3 | 4: 64-query tiles with NB LDS buffers; unset: 128-query tiles, 2 buffers)
inside the default fused backward at the bench shape, interleaved rounds, medians.  Every arm's dK / dV
is checked bitwise against the default's.

    python scripts/attn_dkdv_nb.py [--arms 2,3,4] [--rounds 5]   (B, T, NH, NKV, HD env as attn_bench.py)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops.attention import rope_cache  # noqa: E402
from attn_dkdv_abl import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    B = int(os.environ.get("B", 64))
    T = int(os.environ.get("T", 1024))
    nh = int(os.environ.get("NH", 16))
    nkv = int(os.environ.get("NKV", nh))
    hd = int(os.environ.get("HD", 64))
    ops.set_backend("hip")
    ld = (nh + 2 * nkv) * hd
    cos, sin = rope_cache(T, hd, 10000.0, None, "cuda")
    x = torch.randn(B * T, ld, device="cuda").bfloat16().requires_grad_(True)
    o = ops.attention(x, cos, sin, B, T, nh, nkv, hd, rotated=True)
    do = torch.randn_like(o)
    bwd = lambda: torch.autograd.grad(o, x, do, retain_graph=True)[0]  # noqa: E731
    arms = ["default"] + a.arms.split(",")
    ref = bwd().clone()
    for arm in arms[1:]:
        os.environ["ND_ATTN_DKDV_NB"] = arm
        g = bwd()
        print(f"NB={arm}: bitwise equal to default: {torch.equal(g, ref)} "
              f"(max |diff| {(g.float() - ref.float()).abs().max().item():.3e})", flush=True)
    res = {}
    for _ in range(a.rounds):
        for arm in arms:
            if arm == "default":
                os.environ.pop("ND_ATTN_DKDV_NB", None)
            else:
                os.environ["ND_ATTN_DKDV_NB"] = arm
            res.setdefault(arm, []).append(timed(bwd))
    os.environ.pop("ND_ATTN_DKDV_NB", None)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(f"B={B} T={T} nh={nh} nkv={nkv} hd={hd}", flush=True)
    for arm in arms:
        print(f"bwd (dQ + dK/dV) {arm:>7s}: {med[arm]:8.1f} us  {med['default'] / med[arm]:.3f}x", flush=True)


if __name__ == "__main__":
    main()
