#!/usr/bin/env python3
"""Attention forward kernel A/B on the bench shapes (pre-rotated q|k, the fused-RoPE path): variants are
ND_ATTN_FWD[+ND_ATTN_LOOK] pairs, e.g. d (round-2 LDS-DMA kernel), s1 / s2 (pipelined, 1- / 2-tile
look-ahead).  CUDA-event timing, interleaved rounds, median.

    VARIANTS=d,s1,s2 python scripts/attn_fwd_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops import _ext  # noqa: E402


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


variants = os.environ.get("VARIANTS", "d,s1,s2").split(",")
bwd_variants = os.environ.get("BWD_VARIANTS", "o,s1,s2").split(",")  # ND_ATTN_DQ[+ND_ATTN_LOOK]
L = _ext.lib()
for (B, T, nh, nkv, hd) in [(64, 1024, 16, 16, 64), (16, 1024, 32, 4, 64), (16, 2048, 16, 16, 64)]:
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
    k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
    o = torch.empty(B * T, nh * hd, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, nh, T, device="cuda")
    st = _ext.stream_ptr(qkv.device)

    def run():
        _ext.check(L.nd_attn_fwd_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, nh,
                                    nkv, T, hd, ld, nh * hd, 0, 0, hd ** -0.5, 0, st), "fwd")
    flops = 4.0 * B * nh * T * T * hd / 2
    res = {}
    outs = {}
    for rnd in range(5):
        for var in variants:
            vv, _, abl = var.partition(":")  # "d:3" = round-2 kernel with ablation 3 (ND_ATTN_ABL)
            os.environ["ND_ATTN_FWD"] = vv[0]
            os.environ["ND_ATTN_LOOK"] = vv[1:] or "1"
            os.environ["ND_ATTN_ABL"] = abl or "0"
            res.setdefault(var, []).append(timed(run))
            if rnd == 0:
                outs[var] = o.clone()
    base = outs[variants[0]].float()
    line = f"B{B} T{T} h{nh}/{nkv} d{hd}:"
    for var in variants:
        t = sorted(res[var])[2]
        d = ((outs[var].float() - base).norm() / base.norm()).item()
        line += f"  {var} {t:7.1f} us {flops / t / 1e6:5.0f} TF (diff {d:.1e})"
    print(line, flush=True)
    # fused backward (dQ + row statistics, then dK/dV): the dQ-kernel variants
    os.environ["ND_ATTN_FWD"], os.environ["ND_ATTN_LOOK"], os.environ["ND_ATTN_ABL"] = "d", "1", "0"
    if os.environ.get("FWD_ONLY"):
        continue
    run()
    do = torch.randn(B * T, nh * hd, device="cuda").bfloat16()
    dqkv = torch.empty_like(qkv)
    dk, dv = dqkv[:, nh * hd:], dqkv[:, (nh + nkv) * hd:]
    ws = torch.empty(2, B, nh, T, device="cuda")

    def bwd():
        _ext.check(L.nd_attn_bwd_fused_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(),
                                          lse.data_ptr(), dqkv.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(),
                                          B, nh, nkv, T, hd, ld, nh * hd, 0, 0, hd ** -0.5, 0, 0, st), "bwd")
    res, outs = {}, {}
    for rnd in range(5):
        for var in bwd_variants:
            os.environ["ND_ATTN_DQ"] = var[0]
            os.environ["ND_ATTN_LOOK"] = var[1:] or "1"
            res.setdefault(var, []).append(timed(bwd))
            if rnd == 0:
                outs[var] = dqkv.clone()
    base = outs[bwd_variants[0]].float()
    line = f"  bwd (dQ variants):"
    for var in bwd_variants:
        t = sorted(res[var])[2]
        d = ((outs[var].float() - base).norm() / base.norm()).item()
        line += f"  {var} {t:7.1f} us {2.5 * flops / t / 1e6:5.0f} TF (diff {d:.1e})"
    print(line, flush=True)
