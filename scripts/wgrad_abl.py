#!/usr/bin/env python3
"""Timing ablations of the weight-gradient kernel (csrc/gemm_wgrad.hip wgrad_pp_kernel, ND_WGRAD_VARIANT=a<bits>:
1 no LDS-DMA, 2 fragments read once, 4 no barriers, 8 no vmcnt waits, 16 no MFMAs; WRONG results, timing
only) on the Llama-150M shapes at --tokens, interleaved rounds, medians.

    python scripts/wgrad_abl.py [--tokens 131072] [--abl 1,2,4,8,16,31] [--rounds 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import gemm as G  # noqa: E402


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
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--abl", default="1,2,4,8,16,31")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    ops.set_backend("hip")
    M = a.tokens
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()
    shapes = {"qkv": (3072, 1024), "o": (1024, 1024), "gate|up": (5376, 1024), "down": (1024, 2688)}
    arms = [""] + ["a" + v for v in a.abl.split(",")]
    cases = {}
    for nm, (m, n) in shapes.items():
        dy, x, gw = r(M, m), r(M, n), torch.zeros(m, n, device="cuda")
        cases[nm] = (2.0 * M * m * n, dy, x, gw)
    # correct variants (64: half the pieces issued inside the MFMA phase) must match the default bitwise
    for nm, (fl, dy, x, gw) in cases.items():
        for arm in arms:
            if arm not in ("a64",):
                continue
            outs = []
            for v in ("", arm):
                if v:
                    os.environ["ND_WGRAD_VARIANT"] = v
                else:
                    os.environ.pop("ND_WGRAD_VARIANT", None)
                gw.zero_()
                G.wgrad(gw, dy, x)
                outs.append(gw.clone())
            os.environ.pop("ND_WGRAD_VARIANT", None)
            print(f"check {nm} {arm}: bitwise equal to the default: {torch.equal(outs[0], outs[1])}", flush=True)
    res = {}
    for _ in range(a.rounds):
        for nm, (fl, dy, x, gw) in cases.items():
            for arm in arms:
                if arm:
                    os.environ["ND_WGRAD_VARIANT"] = arm
                else:
                    os.environ.pop("ND_WGRAD_VARIANT", None)
                res.setdefault((nm, arm), []).append(timed(lambda: G.wgrad(gw, dy, x)))
    os.environ.pop("ND_WGRAD_VARIANT", None)
    for nm, (fl, *_r) in cases.items():
        line = f"{nm:8s}"
        for arm in arms:
            t = sorted(res[(nm, arm)])[a.rounds // 2]
            line += f" | {arm or 'wgrad_pp'}: {t:7.1f} us {fl / t / 1e6:5.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
