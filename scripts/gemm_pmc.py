#!/usr/bin/env python3
"""A few launches of one projection shape on the own ping-pong GEMM and on hipBLASLt (for rocprofv3 --pmc).

    python scripts/gemm_pmc.py [--m 65536 --n 3072 --k 1024] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=65536)
ap.add_argument("--n", type=int, default=3072)
ap.add_argument("--k", type=int, default=1024)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--variants", default="", help="ping-pong ablation variants (G.set_pp_variant)")
a = ap.parse_args()
ops.set_backend("hip")
x = (torch.rand(a.m, a.k, device="cuda") * 2 - 1).bfloat16()
w = ((torch.rand(a.n, a.k, device="cuda") * 2 - 1) * 0.05).bfloat16()
out = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
vs = [int(v) for v in a.variants.split(",")] if a.variants else [None]
for _ in range(a.iters):
    for v in vs:
        if v is not None:
            G.set_pp_variant(v)
        G.gemm_pp(x, w, out)
        G.set_pp_variant(0)
    torch.mm(x, w.t(), out=out)
torch.cuda.synchronize()
print("done")
