#!/usr/bin/env python3
"""fp8 (OCP e4m3 / e5m2) GEMM availability + speed on gfx950 via torch._scaled_mm (hipBLASLt), vs bf16."""
import os
import time

import torch


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    N = int(os.environ.get("TOKENS", 32768))
    d, F = 1024, 2688
    shapes = {"qkv": (3 * d, d), "o": (d, d), "gate_up": (2 * F, d), "down": (d, F)}
    one = torch.ones((), device="cuda")
    for name, (out, inn) in shapes.items():
        x = torch.randn(N, inn, device="cuda")
        w = torch.randn(out, inn, device="cuda")
        dy = torch.randn(N, out, device="cuda")
        xb, wb, dyb = x.bfloat16(), w.bfloat16(), dy.bfloat16()
        x8, w8 = x.to(torch.float8_e4m3fn), w.to(torch.float8_e4m3fn)
        dy8 = dy.to(torch.float8_e5m2)
        wT8 = w.t().contiguous().to(torch.float8_e4m3fn)
        fl = 2.0 * N * out * inn
        r = {}
        r["bf16 fwd"] = bench(lambda: torch.mm(xb, wb.t()))
        r["bf16 dgrad"] = bench(lambda: torch.mm(dyb, wb))
        try:
            r["fp8 fwd"] = bench(lambda: torch._scaled_mm(x8, w8.t(), one, one, out_dtype=torch.bfloat16))
            r["fp8 dgrad(e5m2xe4m3)"] = bench(lambda: torch._scaled_mm(dy8, wT8.t(), one, one, out_dtype=torch.bfloat16))
        except Exception as e:  # noqa: BLE001
            print(name, "scaled_mm failed:", type(e).__name__, str(e)[:300])
        print(name, " ".join(f"{k}={fl / v / 1e12:.0f}TF" for k, v in r.items()), flush=True)
    # numerics sanity
    a = torch.randn(256, 512, device="cuda")
    b = torch.randn(384, 512, device="cuda")
    ref = a @ b.t()
    out = torch._scaled_mm(a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn).t(), one, one, out_dtype=torch.float32)
    print("fp8 rel err", ((out - ref).norm() / ref.norm()).item())


if __name__ == "__main__":
    main()
