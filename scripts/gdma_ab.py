#!/usr/bin/env python3
"""A/B of the LDS-DMA piece form in the step's own GEMMs: buffer_load ... lds (V#, range-checked) vs
global_load_lds (SGPR base + per-lane offset, the default) for full half-tiles.  Fused ping-pong kernels
(gemm_pp.hip variant 1024 = buffer form) and the weight-gradient kernel (gemm_wgrad.hip, ND_WGRAD_VARIANT=b), Llama-150M shapes at
--tokens.  Checks the two forms produce bitwise-equal outputs, then times them interleaved.

    python scripts/gdma_ab.py [--tokens 131072] [--rounds 5]
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
    return s.elapsed_time(e) / iters * 1e3  # us


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pp-variant", type=int, default=1024, help="gemm_pp variant of the B arm (1024: buffer form)")
    ap.add_argument("--wgrad-variant", default="b", help="ND_WGRAD_VARIANT of the B arm (b: buffer form)")
    a = ap.parse_args()
    ops.set_backend("hip")
    M, d, F, V = a.tokens, 1024, 2688, 32000
    T, hd = 1024, 64
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, "cuda")
    x, wqkv, wgu, wdt, wo = r(M, d), r(3 * d, d) * 0.05, r(2 * F, d) * 0.05, r(F, d) * 0.05, r(d, d) * 0.05
    dy = r(M, d)
    gu, act = G.gemm_pp_swiglu(x, wgu)
    gw_gu = torch.zeros(2 * F, d, device="cuda")
    gw_down = torch.zeros(d, F, device="cuda")
    gw_o = torch.zeros(d, d, device="cuda")
    dgu = torch.empty_like(gu)
    cases = {
        "qkv+rope fwd": (2.0 * M * 3 * d * d, lambda: G.gemm_pp_rope(x, wqkv, cos, sin, T, hd, 2 * d)),
        "gu+swiglu fwd": (2.0 * M * 2 * F * d, lambda: G.gemm_pp_swiglu(x, wgu, gu, act)),
        "down dgrad+dswiglu": (2.0 * M * F * d, lambda: G.gemm_pp_dswiglu(dy, wdt, gu, dgu)),
        "o fwd (plain)": (2.0 * M * d * d, lambda: G.gemm_pp(x, wo)),
        "wgrad gu": (2.0 * M * 2 * F * d, lambda: G.wgrad(gw_gu, dgu, x)),
        "wgrad down": (2.0 * M * F * d, lambda: G.wgrad(gw_down, dy, act)),
        "wgrad o": (2.0 * M * d * d, lambda: G.wgrad(gw_o, dy, x)),
    }

    def arm(name, flat):
        """flat: the default build; else the B arm (--pp-variant / --wgrad-variant)"""
        if name.startswith("wgrad"):
            if flat:
                os.environ.pop("ND_WGRAD_VARIANT", None)
            else:
                os.environ["ND_WGRAD_VARIANT"] = a.wgrad_variant
        else:
            G.set_pp_variant(0 if flat else a.pp_variant)

    bad = 0
    for name, (fl, fn) in cases.items():
        outs = []
        for flat in (False, True):
            arm(name, flat)
            if name.startswith("wgrad"):
                for g_ in (gw_gu, gw_down, gw_o):
                    g_.zero_()
            o = fn()
            if name.startswith("wgrad"):
                o = {"wgrad gu": gw_gu, "wgrad down": gw_down, "wgrad o": gw_o}[name]
            elif name.startswith("gu+swiglu"):
                o = torch.cat([gu.float().flatten(), act.float().flatten()])
            elif name.startswith("down"):
                o = dgu
            outs.append(o.float().clone())
        same = torch.equal(outs[0], outs[1])
        bad += not same
        print(f"check {name}: default == variant bitwise: {same}", flush=True)
    res = {}
    for rd in range(a.rounds):
        for name, (fl, fn) in cases.items():
            for flat in (False, True):
                arm(name, flat)
                res.setdefault((name, flat), []).append(timed(fn))
    arm("wgrad", True)
    arm("pp", True)
    tot = [0.0, 0.0]
    for name, (fl, fn) in cases.items():
        t = [sorted(res[(name, f)])[a.rounds // 2] for f in (False, True)]
        tot[0] += t[0]
        tot[1] += t[1]
        print(f"{name:20s} | variant {t[0]:8.1f} us {fl / t[0] / 1e6:5.0f} TF | default {t[1]:8.1f} us "
              f"{fl / t[1] / 1e6:5.0f} TF | default/variant speed {t[0] / t[1]:.3f}x", flush=True)
    print(f"total variant {tot[0]:.0f} us default {tot[1]:.0f} us ({tot[0] / tot[1]:.3f}x)", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
