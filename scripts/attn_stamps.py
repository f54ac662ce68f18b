#!/usr/bin/env python3
"""Where the attention forward, dK/dV and dQ kernels spend a wave's cycles: segment stamps of the diagnostic
build (``python -m nanodiloco_amd.csrc.build --rev WT --extra-flags=-DND_ATTN_STAMP --tag stamp``; the product
library has no stamps).  Runs the Llama-150M bench shape (B=64, T=1024, 16x64, pre-rotated q|k) once per
kernel and prints each segment's share of the summed wave cycles (guide cdna_hip_programming.md §7: read
SHARES, the stamped build's run time is not the product's).

    python scripts/attn_stamps.py --lib nanodiloco_amd/_lib/alt/libnd_kernels_stamp.so
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops import _ext  # noqa: E402

SEGS = {
    0: {0: "wait K/V LDS-DMA (vmcnt)", 1: "barrier", 2: "issue next K/V DMA", 3: "K reads + S MFMAs (issue)",
        4: "mask / max / exp / row sum (VALU, waits S)", 5: "P pack + V^T reads + P V MFMAs (issue)",
        6: "epilogue (O / LSE store)", 7: "loop overhead / skipped tiles", 8: "-", 9: "-"},
    1: {0: "wait Q/dO/stat LDS-DMA (vmcnt)", 1: "barrier", 2: "LDS fragment + seed reads (to landed)",
        3: "S / dP MFMAs (issue)", 4: "exp / P*dP (VALU, waits S, dP)", 5: "pack + dV / dK MFMAs (issue)",
        6: "epilogue (dK / dV store)", 7: "loop overhead / skipped steps", 8: "issue row-statistic LDS-DMA pieces",
        9: "issue Q / dO LDS-DMA pieces"},
    2: {0: "wait K/V LDS-DMA (vmcnt)", 1: "barrier", 2: "issue next K/V DMA", 3: "K / V / K^T fragment reads (to landed)",
        4: "S / dP MFMAs (issue)", 5: "exp / dS (VALU, waits S, dP)", 6: "pack + dQ MFMAs (issue)",
        7: "loop overhead / skipped halves", 8: "epilogue (dQ store)", 9: "prologue (Q / dO loads, row statistics)"},
}

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="nanodiloco_amd/_lib/alt/libnd_kernels_stamp.so")
ap.add_argument("--shape", default="64,1024,16,16,64")
a = ap.parse_args()
raw = ctypes.CDLL(os.path.abspath(a.lib), mode=ctypes.RTLD_LOCAL)
raw.nd_attn_stamp_buffer.argtypes = [ctypes.c_void_p]
L = _ext.load_library(os.path.abspath(a.lib))
B, T, nh, nkv, hd = (int(x) for x in a.shape.split(","))
ld = (nh + 2 * nkv) * hd
qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
k, v = qkv[:, nh * hd:], qkv[:, (nh + nkv) * hd:]
o = torch.empty(B * T, nh * hd, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B, nh, T, device="cuda")
do = torch.randn(B * T, nh * hd, device="cuda").bfloat16()
dqkv = torch.empty_like(qkv)
ws = torch.empty(2, B, nh, T, device="cuda")
st = _ext.stream_ptr(qkv.device)
buf = torch.zeros(3 * (1 << 22) + 8, dtype=torch.int64, device="cuda")


def run():
    _ext.check(L.nd_attn_fwd_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, nh, nkv,
                                T, hd, ld, nh * hd, 0, 0, hd ** -0.5, 0, st), "fwd")
    _ext.check(L.nd_attn_bwd_fused_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(),
                                      lse.data_ptr(), dqkv.data_ptr(), dqkv[:, nh * hd:].data_ptr(),
                                      dqkv[:, (nh + nkv) * hd:].data_ptr(), ws.data_ptr(), B, nh, nkv, T, hd, ld,
                                      nh * hd, 0, 0, hd ** -0.5, 0, 0, st), "bwd")


_ext.check(raw.nd_attn_stamp_buffer(ctypes.c_void_p(0)), "stamp buffer")
for _ in range(3):
    run()  # warm (clock, caches), unstamped
torch.cuda.synchronize()
_ext.check(raw.nd_attn_stamp_buffer(ctypes.c_void_p(buf.data_ptr())), "stamp buffer")
run()
torch.cuda.synchronize()
_ext.check(raw.nd_attn_stamp_buffer(ctypes.c_void_p(0)), "stamp buffer")
h = buf.cpu()
for kid, name in ((0, "attn_fwd_kernel"), (1, "attn_bwd_dkdv_dma_kernel"), (2, "attn_bwd_dq_kernel")):
    seg = h[1 + kid * (1 << 22): 1 + kid * (1 << 22) + (1 << 22) // 10 * 10].view(-1, 10)
    seg = seg[seg.sum(1) > 0].double()
    tot = seg.sum(0)
    allc = tot.sum().item()
    print(f"{name}: {seg.shape[0]} waves, {allc / seg.shape[0]:.0f} stamped cycles per wave (mean)")
    for s_ in range(10):
        print(f"  {s_}  {SEGS[kid][s_]:48s} {100 * tot[s_].item() / allc:5.1f} %   "
              f"{tot[s_].item() / seg.shape[0]:9.0f} cyc/wave")
