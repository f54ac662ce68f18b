#!/usr/bin/env python3
"""Timing ablations of the attention dK/dV kernel (csrc/attention.hip attn_bwd_dkdv_dma_kernel,
ND_ATTN_DKDV_ABL bits: 1 no Q/dO DMA + wait, 2 no barrier, 4 no softmax VALU, 8 no S/dP MFMAs, 16 no
dV/dK MFMAs, 32 fragments read once; WRONG results, timing only) inside the default fused backward
(dQ kernel + dK/dV kernel) at the bench shape, interleaved rounds, medians.  The dQ kernel is the same in
every arm, so differences are the dK/dV kernel's.

    python scripts/attn_dkdv_abl.py [--abl 1,2,4,8,16,32] [--rounds 5]   (B, T, NH, NKV, HD env as attn_bench.py)
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
    ap.add_argument("--abl", default="1,2,3,4,8,16,24,28,32,63")
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
    fwd = lambda: ops.attention(x, cos, sin, B, T, nh, nkv, hd, rotated=True)  # noqa: E731
    bwd = lambda: torch.autograd.grad(o, x, do, retain_graph=True)  # noqa: E731
    arms = ["0"] + a.abl.split(",")
    res = {}
    for _ in range(a.rounds):
        res.setdefault("fwd", []).append(timed(fwd))
        for arm in arms:
            os.environ["ND_ATTN_DKDV_ABL"] = arm
            res.setdefault(arm, []).append(timed(bwd))
    os.environ.pop("ND_ATTN_DKDV_ABL", None)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    fl = 4.0 * B * nh * T * T * hd / 2  # one causal score-matrix GEMM pair
    print(f"B={B} T={T} nh={nh} nkv={nkv} hd={hd}: fwd {med['fwd']:.1f} us ({fl / med['fwd'] / 1e6:.0f} TF)", flush=True)
    for arm in arms:
        print(f"bwd (dQ + dK/dV) abl {arm:>3s}: {med[arm]:8.1f} us  delta vs default {med[arm] - med['0']:+8.1f} us",
              flush=True)


if __name__ == "__main__":
    main()
