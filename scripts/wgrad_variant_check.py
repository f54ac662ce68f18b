#!/usr/bin/env python3
"""Numerics of every wgrad kernel variant (ND_WGRAD_VARIANT) against an fp32 reference, on the
Llama-150M shapes plus a K-tail shape; exits non-zero on a mismatch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd.ops.gemm import wgrad  # noqa: E402


def main():
    torch.manual_seed(0)
    bad = 0
    for M, N, K in [(3072, 1024, 8192), (1024, 2688, 8192), (1024, 1024, 65536), (5376, 1024, 4160), (32000, 1024, 2048)]:
        dy = torch.randn(K, M, device="cuda").bfloat16()
        x = torch.randn(K, N, device="cuda").bfloat16()
        ref = dy.float().t() @ x.float()
        for v in os.environ.get("VARIANTS", "dma0,dmas,b").split(","):
            os.environ["ND_WGRAD_VARIANT"] = v
            gw = torch.ones(M, N, device="cuda")
            wgrad(gw, dy, x)
            torch.cuda.synchronize()
            err = ((gw - 1 - ref).norm() / ref.norm()).item()
            ok = err < 1e-5
            bad += not ok
            print(f"{v:7s} M={M} N={N} K={K} rel err {err:.2e} {'ok' if ok else 'FAIL'}", flush=True)
    os.environ.pop("ND_WGRAD_VARIANT", None)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
