#!/usr/bin/env python3
"""Flash-attention kernel micro-benchmark (HIP path) on the Llama-150M micro-batch shape, with the
PyTorch SDPA (ROCm: AOTriton/CK) time on the same data for comparison.  Causal FLOPs counted as
half the full score matrix: fwd 2 GEMMs, bwd 5 (dkdv 4 + dq 3 recomputed = 7 executed)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops.attention import rope_cache  # noqa: E402


def bench(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    B = int(os.environ.get("B", 32))
    T = int(os.environ.get("T", 1024))
    nh = int(os.environ.get("NH", 16))
    nkv = int(os.environ.get("NKV", nh))
    hd = int(os.environ.get("HD", 64))
    ops.set_backend("hip")
    ld = (nh + 2 * nkv) * hd
    qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
    cos, sin = rope_cache(T, hd, 10000.0, None, "cuda")
    fl_fwd = 2 * 2 * B * nh * T * T * hd / 2
    x = qkv.clone().requires_grad_(True)
    t_fwd = bench(lambda: ops.attention(x, cos, sin, B, T, nh, nkv, hd))
    o = ops.attention(x, cos, sin, B, T, nh, nkv, hd)
    do = torch.randn_like(o)
    t_bwd = bench(lambda: torch.autograd.grad(o, x, do, retain_graph=True))
    print(f"ours  fwd {t_fwd * 1e6:8.1f} us {fl_fwd / t_fwd / 1e12:6.1f} TF/s | "
          f"bwd {t_bwd * 1e6:8.1f} us {2.5 * fl_fwd / t_bwd / 1e12:6.1f} TF/s (5-GEMM count)", flush=True)
    q = torch.randn(B, nh, T, hd, device="cuda").bfloat16().requires_grad_(True)
    k = torch.randn(B, nkv, T, hd, device="cuda").bfloat16().requires_grad_(True)
    v = torch.randn(B, nkv, T, hd, device="cuda").bfloat16().requires_grad_(True)
    f = lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=nkv != nh)
    try:
        t_sf = bench(f)
        out = f()
        g = torch.randn_like(out)
        t_sb = bench(lambda: torch.autograd.grad(out, (q, k, v), g, retain_graph=True))
        print(f"sdpa  fwd {t_sf * 1e6:8.1f} us {fl_fwd / t_sf / 1e12:6.1f} TF/s | "
              f"bwd {t_sb * 1e6:8.1f} us {2.5 * fl_fwd / t_sb / 1e12:6.1f} TF/s", flush=True)
    except Exception as e:  # noqa: BLE001
        print("sdpa unavailable:", type(e).__name__, e)


if __name__ == "__main__":
    main()
