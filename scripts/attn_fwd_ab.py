#!/usr/bin/env python3
"""Attention kernel A/B on the bench shapes (pre-rotated q|k, the fused-RoPE path); CUDA-event timing,
5 interleaved rounds, median.  Forward variants: d (LDS-DMA kernel, 128-query blocks), d8 (256-query
blocks), r (register-staged), with an optional ':<bits>' ND_ATTN_ABL suffix (ablations, or 32 = the
cheaper-mask variant).  Fused-backward variants: o (default), o8 (256-query dQ blocks), k8 (256-key dK/dV
blocks).  Results: profiles/r3_attention_experiments.md.

    VARIANTS=d,d:32,d8 BWD_VARIANTS=o,o8,k8 python scripts/attn_fwd_ab.py   (FWD_ONLY=1: skip the backward)
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


def set_fwd(var):
    vv, _, abl = var.partition(":")
    os.environ["ND_ATTN_FWD"] = vv[0]
    os.environ["ND_ATTN_FWD_W"] = vv[1:] or "4"
    os.environ["ND_ATTN_ABL"] = abl or "0"


def set_bwd(var):
    os.environ["ND_ATTN_DQ_W"] = "8" if var == "o8" else "4"
    os.environ["ND_ATTN_DKDV_W"] = "8" if var == "k8" else "4"


variants = os.environ.get("VARIANTS", "d,d:32,d8").split(",")
bwd_variants = os.environ.get("BWD_VARIANTS", "o,o8,k8").split(",")
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
    res, outs = {}, {}
    for rnd in range(5):
        for var in variants:
            set_fwd(var)
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
    if os.environ.get("FWD_ONLY"):
        continue
    set_fwd("d")
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
            set_bwd(var)
            res.setdefault(var, []).append(timed(bwd))
            if rnd == 0:
                outs[var] = dqkv.clone()
    set_bwd("o")
    base = outs[bwd_variants[0]].float()
    line = "  fused bwd:"
    for var in bwd_variants:
        t = sorted(res[var])[2]
        d = ((outs[var].float() - base).norm() / base.norm()).item()
        line += f"  {var} {t:7.1f} us {2.5 * flops / t / 1e6:5.0f} TF (diff {d:.1e})"
    print(line, flush=True)
