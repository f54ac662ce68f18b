#!/usr/bin/env python3
"""A few launches of the attention forward / fused backward kernels at the Llama-150M bench shape
(B=64, T=1024, 16x64, pre-rotated q|k) for rocprofv3 --pmc.

    python scripts/attn_pmc.py [--iters 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops import _ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=3)
ap.add_argument("--shape", default="64,1024,16,16,64")
a = ap.parse_args()
B, T, nh, nkv, hd = (int(x) for x in a.shape.split(","))
L = _ext.lib()
ld = (nh + 2 * nkv) * hd
qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
o = torch.empty(B * T, nh * hd, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B, nh, T, device="cuda")
do = torch.randn(B * T, nh * hd, device="cuda").bfloat16()
dqkv = torch.empty_like(qkv)
dk, dv = dqkv[:, nh * hd:], dqkv[:, (nh + nkv) * hd:]
ws = torch.empty(2, B, nh, T, device="cuda")
st = _ext.stream_ptr(qkv.device)
for _ in range(a.iters):
    for fv in ("d",):
        os.environ["ND_ATTN_FWD"] = fv
        _ext.check(L.nd_attn_fwd_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, nh,
                                    nkv, T, hd, ld, nh * hd, 0, 0, hd ** -0.5, 0, st), "fwd")
    for qv in ("o",):
        _ext.check(L.nd_attn_bwd_fused_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(),
                                          lse.data_ptr(), dqkv.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(),
                                          B, nh, nkv, T, hd, ld, nh * hd, 0, 0, hd ** -0.5, 0, 0, st), "bwd")
torch.cuda.synchronize()
print("done")
