#!/usr/bin/env python3
"""nd_gemm_nt (C = A B^T, forward-projection layout) vs hipBLASLt torch.mm on the Llama shapes:
correctness vs fp32, then interleaved timing (min over rounds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops import _ext  # noqa: E402


def gemm_nt(a, b, c, dbg=None):
    M, K = a.shape
    N = b.shape[0]
    _ext.check(_ext.lib().nd_gemm_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                     c.stride(0), dbg.data_ptr() if dbg is not None else 0, _ext.stream_ptr()),
               "nd_gemm_nt")


def timed(fn, iters=20):
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
    T = int(os.environ.get("TOKENS", 32768))
    shapes = {"qkv": (3072, 1024), "o": (1024, 1024), "gate_up": (5376, 1024), "down": (1024, 2688),
              "lm_head": (32000, 1024), "odd": (1000, 320)}
    for name, (N, K) in shapes.items():
        M = T if name not in ("lm_head", "odd") else (16384 if name == "lm_head" else 777)
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        gemm_nt(a, b, c)
        ref = a.float() @ b.float().t()
        err = ((c.float() - ref).norm() / ref.norm()).item()
        fl = 2.0 * M * N * K
        t_n, t_b = [], []
        for _ in range(3):
            t_n.append(timed(lambda: gemm_nt(a, b, c)))
            t_b.append(timed(lambda: torch.mm(a, b.t())))
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        dbg = torch.zeros(tiles * 8 * 4, dtype=torch.int64, device="cuda")
        gemm_nt(a, b, c, dbg)
        torch.cuda.synchronize()
        d = dbg.view(-1, 4).double()
        stamp = (f"  [stamps: boundary wait {d[:, 0].sum() / d[:, 2].sum():.0%}, lds wait "
                 f"{d[:, 1].sum() / d[:, 2].sum():.0%} of wave time; clock {d[:, 2].sum() / d[:, 3].sum() * 0.1:.2f} GHz]")
        print(f"{name:8s} M={M} N={N} K={K}  err={err:.1e}  ours {min(t_n):7.1f} us {fl / min(t_n) / 1e6:6.0f} TF/s | "
              f"hipBLASLt {min(t_b):7.1f} us {fl / min(t_b) / 1e6:6.0f} TF/s" + stamp, flush=True)


if __name__ == "__main__":
    main()
