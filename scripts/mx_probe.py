#!/usr/bin/env python3
"""Probe: does this torch/hipBLASLt build run MX (OCP microscaling: e4m3 elements, one e8m0 scale per
32 consecutive K elements) GEMMs on gfx950, and how fast vs bf16 and per-tensor fp8?

The CDNA4 MFMA rates (MI355X_MICROARCH.md): non-scaled fp8 MFMA = the bf16 rate; block-scaled
v_mfma_scale_f32_*_f8f6f4 with e4m3 operands = 2x the bf16 rate.  Per-tensor `_scaled_mm` can only
use the former, so only an MX path can double the fp8 GEMM throughput."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def mx_quant(x):
    """[R, K] fp32 -> (e4m3 [R, K], e8m0 scales [R, K/32]) with power-of-two block scales."""
    R, K = x.shape
    xb = x.view(R, K // 32, 32)
    amax = xb.abs().amax(-1).clamp_min(1e-30)
    # OCP MX: shared exponent = floor(log2(amax)) - emax_elem (e4m3 emax = 8)
    e = torch.floor(torch.log2(amax)) - 8
    scale = torch.exp2(e)
    q = (xb / scale[..., None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(R, K)
    s8 = (e + 127).clamp(0, 254).to(torch.uint8).view(torch.float8_e8m0fnu)
    return q, s8, scale


def main():
    M, N, K = int(os.environ.get("M", 65536)), int(os.environ.get("N", 3072)), int(os.environ.get("K", 1024))
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(N, K, device="cuda") * 0.02
    ref = a @ b.t()
    fl = 2.0 * M * N * K
    ab, bb = a.bfloat16(), b.bfloat16()
    t = bench(lambda: torch.mm(ab, bb.t()))
    print(f"bf16         {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF", flush=True)
    a8 = a.to(torch.float8_e4m3fn)
    b8 = (b * 64).to(torch.float8_e4m3fn)
    one, inv = torch.ones((), device="cuda"), torch.full((), 1 / 64, device="cuda")
    try:
        t = bench(lambda: torch._scaled_mm(a8, b8.t(), one, inv, out_dtype=torch.bfloat16))
        print(f"fp8 tensor   {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF", flush=True)
    except Exception as e:  # noqa: BLE001
        print("fp8 tensorwise failed:", repr(e)[:300])
    qa, sa, _ = mx_quant(a)
    qb, sb, _ = mx_quant(b)
    for name, fn in [
        ("mx legacy", lambda: torch._scaled_mm(qa, qb.t(), sa, sb, out_dtype=torch.bfloat16)),
    ]:
        try:
            out = fn()
            torch.cuda.synchronize()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            t = bench(fn)
            print(f"{name:12s} {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF  rel err {err:.3e}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{name} failed: {repr(e)[:600]}", flush=True)
    try:
        import torch.nn.functional as F
        from torch.nn.functional import ScalingType, SwizzleType
        for sw in (SwizzleType.NO_SWIZZLE, SwizzleType.SWIZZLE_32_4_4):
            try:
                fn = lambda: F.scaled_mm(qa, qb.t(), sa, ScalingType.BlockWise1x32, sb, ScalingType.BlockWise1x32,
                                         swizzle_a=sw, swizzle_b=sw, output_dtype=torch.bfloat16)
                out = fn()
                torch.cuda.synchronize()
                err = ((out.float() - ref).norm() / ref.norm()).item()
                t = bench(fn)
                print(f"mx v2 {sw.name:12s} {t*1e6:8.1f} us {fl/t/1e12:7.1f} TF  rel err {err:.3e}", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"mx v2 {sw} failed: {repr(e)[:600]}", flush=True)
    except Exception as e:  # noqa: BLE001
        print("v2 API unavailable:", repr(e)[:300])


if __name__ == "__main__":
    main()
