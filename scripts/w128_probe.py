#!/usr/bin/env python3
"""Probe the one-wave-per-SIMD GEMM (csrc/gemm_w128.hip) against hipBLASLt on the Llama-150M shapes:

    python scripts/w128_probe.py ablate [--abl 1,2,4,8,16,31]   # timing of ablation builds (wrong results)
    python scripts/w128_probe.py pmc                             # 5 calls per arm, for rocprofv3 --pmc runs
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv fwd": (131072, 3072, 1024), "o fwd": (131072, 1024, 1024), "gu dgrad": (131072, 1024, 5376)}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["ablate", "pmc"])
    ap.add_argument("--abl", default="1,2,4,8,16,31")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    ops.set_backend("hip")
    data = {}
    for nm in a.shapes.split(","):
        m, n, k = SHAPES[nm]
        x = (torch.rand(m, k, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(n, k, device="cuda") * 2 - 1) * 0.05).bfloat16()
        data[nm] = (x, w, torch.empty(m, n, device="cuda", dtype=torch.bfloat16), 2.0 * m * n * k)
    if a.mode == "pmc":
        for nm, (x, w, out, _) in data.items():
            for _ in range(5):
                torch.mm(x, w.t(), out=out)
            for _ in range(5):
                G.gemm_w128(x, w, out)
            for _ in range(5):
                G.gemm_pp(x, w, out)
        torch.cuda.synchronize()
        return
    abl = [int(v) for v in a.abl.split(",") if v]
    res = {}
    for _ in range(a.rounds):
        for nm, (x, w, out, fl) in data.items():
            res.setdefault((nm, "blas"), []).append(timed(lambda: torch.mm(x, w.t(), out=out)))
            res.setdefault((nm, "pp"), []).append(timed(lambda: G.gemm_pp(x, w, out)))
            for v in [0] + abl:
                G.set_w128_ablation(v)
                res.setdefault((nm, f"w{v}"), []).append(timed(lambda: G.gemm_w128(x, w, out)))
            G.set_w128_ablation(0)
    for v in [v for v in abl if v & (32 | 64 | 256 | 512 | 1024 | 2048 | 4096) and not v & (31 | 128)]:  # the correct-result variants: numerics against hipBLASLt
        G.set_w128_ablation(v)
        for nm, (x, w, out, fl) in data.items():
            ref = torch.mm(x, w.t()).float()
            got = G.gemm_w128(x, w).float()
            print(f"check w{v} {nm}: rel {((got - ref).norm() / ref.norm()).item():.2e}", flush=True)
        G.set_w128_ablation(0)
    for nm, (x, w, out, fl) in data.items():
        line = f"{nm:9s}"
        for arm in ["blas", "pp"] + [f"w{v}" for v in [0] + abl]:
            t = sorted(res[(nm, arm)])[len(res[(nm, arm)]) // 2]
            line += f" | {arm}: {t:7.1f} us {fl / t / 1e6:5.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
