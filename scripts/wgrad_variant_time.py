#!/usr/bin/env python3
"""Per-kernel time of the bf16 weight gradient for the ND_WGRAD_VARIANT this process loaded (read once at library
load), Llama-150M shapes at 131,072 tokens incl. the grouped MLP launch, plus a checksum of the results (priority
variants must be bitwise equal to the default)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters=6):
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
    ops.set_backend("hip")
    K = 131072
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = lambda r, c: torch.randn(r, c, device="cuda", generator=g).bfloat16()  # noqa: E731
    x, xa = mk(K, 1024), mk(K, 2688)
    dq, do, dgu, dd = mk(K, 3072), mk(K, 1024), mk(K, 5376), mk(K, 1024)
    gq, go = torch.zeros(3072, 1024, device="cuda"), torch.zeros(1024, 1024, device="cuda")
    ggu, gdn = torch.zeros(5376, 1024, device="cuda"), torch.zeros(1024, 2688, device="cuda")
    res = {"qkv": timed(lambda: G.wgrad(gq, dq, x)), "o": timed(lambda: G.wgrad(go, do, x)),
           "mlp2": timed(lambda: G.wgrad2(gdn, dd, xa, ggu, dgu, x))}
    for t in (gq, go, ggu, gdn):
        t.zero_()
    G.wgrad(gq, dq, x)
    G.wgrad(go, do, x)
    G.wgrad2(gdn, dd, xa, ggu, dgu, x)
    torch.cuda.synchronize()
    ck = sum(float(t.double().sum()) for t in (gq, go, ggu, gdn))
    v = os.environ.get("ND_WGRAD_VARIANT", "") or "default"
    print(f"{v:8s} " + " ".join(f"{k} {t:7.1f}" for k, t in res.items()) + f" checksum {ck:.10e}", flush=True)


if __name__ == "__main__":
    main()
