#!/usr/bin/env python3
"""Own projection GEMMs (csrc/gemm.hip) vs hipBLASLt (torch.mm) on the Llama-150M / 1B shapes, in one
process, interleaved rounds, random operands; the fused epilogues are compared against the
library GEMM + the separate kernel they replace.

    python scripts/gemm_nt_bench.py [--tokens 65536] [--model 150m|1b] [--rounds 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import _ext  # noqa: E402
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--model", default="150m")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="1,2,3", help="own-kernel schedule variants to A/B (csrc/gemm.hip)")
    ap.add_argument("--only", default="", help="comma list of case-name prefixes")
    ap.add_argument("--fp8", action="store_true", help="fp8 GEMMs (gemm_nt_f8 vs torch._scaled_mm) instead")
    a = ap.parse_args()
    ops.set_backend("hip")
    M = a.tokens
    d, F, nh, nkv, hd, V = (1024, 2688, 16, 16, 64, 32000) if a.model == "150m" else (2048, 5632, 32, 4, 64, 32000)
    qkv_n = (nh + 2 * nkv) * hd
    T = 1024
    cos, sin = ops.rope_cache(T, hd, 10000.0, None, "cuda")
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    cases = []

    def plain(name, m, n, k):
        x, w = r(m, k), r(n, k) * 0.05
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        cases.append((name, 2.0 * m * n * k, lambda: G.gemm_nt(x, w, out), lambda: torch.mm(x, w.t(), out=out)))

    def plain8(name, m, n, k, fa=torch.float8_e4m3fn):
        x8, w8 = r(m, k).to(fa), (r(n, k) * 0.05).to(torch.float8_e4m3fn)
        sa, sb = torch.ones(1, device="cuda"), torch.ones(1, device="cuda")
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        cases.append((name, 2.0 * m * n * k, lambda: G.gemm_nt_f8(x8, w8, sa, sb, out),
                      lambda: torch._scaled_mm(x8, w8.t(), sa, sb, out_dtype=torch.bfloat16)))

    if a.fp8:
        e5 = torch.float8_e5m2
        for nm, n, k in (("qkv", qkv_n, d), ("o", d, nh * hd), ("gu", 2 * F, d), ("down", d, F)):
            plain8(nm + " fwd8", M, n, k)
        for nm, n, k in (("qkv", d, qkv_n), ("o", nh * hd, d), ("gu", d, 2 * F), ("down", F, d)):
            plain8(nm + " dgrad8", M, n, k, e5)
        a.only = a.only or "qkv fwd8,o fwd8,gu fwd8,down fwd8,qkv dgrad8,o dgrad8,gu dgrad8,down dgrad8"
    plain("qkv fwd", M, qkv_n, d)
    plain("o fwd", M, d, nh * hd)
    plain("gu fwd", M, 2 * F, d)
    plain("down fwd", M, d, F)
    plain("qkv dgrad", M, d, qkv_n)
    plain("o dgrad", M, nh * hd, d)
    plain("gu dgrad", M, d, 2 * F)
    plain("down dgrad", M, F, d)
    plain("lm logits", 16384, V, d)
    plain("lm dgrad", 16384, d, V)
    # fused epilogues vs library GEMM + the separate kernel
    x, wq = r(M, d), r(qkv_n, d) * 0.05
    qo = torch.empty(M, qkv_n, device="cuda", dtype=torch.bfloat16)

    def rope_lib():
        torch.mm(x, wq.t(), out=qo)
        _ext.check(_ext.lib().nd_rope_inplace(qo.data_ptr(), 1, cos.data_ptr(), sin.data_ptr(), M, T, nh, nkv, hd,
                                              qkv_n, 0, _ext.stream_ptr()), "rope")

    cases.append(("qkv+rope", 2.0 * M * qkv_n * d, lambda: G.gemm_nt_rope(x, wq, cos, sin, T, hd, (nh + nkv) * hd, qo),
                  rope_lib))
    wg = r(2 * F, d) * 0.05
    gu = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    act = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)

    def swiglu_lib():
        torch.mm(x, wg.t(), out=gu)
        _ext.check(_ext.lib().nd_swiglu_fwd(gu.data_ptr(), act.data_ptr(), 1, M, F, _ext.stream_ptr()), "swiglu")

    cases.append(("gu+swiglu", 2.0 * M * 2 * F * d, lambda: G.gemm_nt_swiglu(x, wg, gu, act), swiglu_lib))
    dy, wdt = r(M, d), r(F, d) * 0.05
    gu_in = r(M, 2 * F)
    dgu = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    dact = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)

    def dswiglu_lib():
        torch.mm(dy, wdt.t(), out=dact)
        _ext.check(_ext.lib().nd_swiglu_bwd(dact.data_ptr(), gu_in.data_ptr(), dgu.data_ptr(), 1, M, F,
                                            _ext.stream_ptr()), "swiglu_bwd")

    cases.append(("down dgrad+dswiglu", 2.0 * M * F * d, lambda: G.gemm_nt_dswiglu(dy, wdt, gu_in, dgu), dswiglu_lib))

    # variant spec "V" or "V:GM" (GM = tile grouping of the 4-wave kernels)
    specs = [tuple(int(x) for x in v.split(":")) if ":" in v else (int(v), 0) for v in a.variants.split(",")]
    variants = list(range(len(specs)))
    only = [p for p in a.only.split(",") if p]
    tot = {v: 0.0 for v in variants}
    tot_b = 0.0
    for name, fl, ours, lib in cases:
        if only and not any(name.startswith(p) for p in only):
            continue
        to = {v: [] for v in variants}
        tb = []
        for _ in range(a.rounds):
            for v in variants:
                if a.fp8:  # --variants then selects the fp8 kernel's schedule (g_f8_variant)
                    G.set_gemm_f8_variant(specs[v][0])
                else:
                    G.set_gemm_variant(specs[v][0])
                G.set_gemm_group_m(specs[v][1])
                to[v].append(timed(ours))
            tb.append(timed(lib))
        b = sorted(tb)[len(tb) // 2]
        tot_b += b
        line = f"{name:20s} lib {b:7.1f} us {fl / b / 1e6:5.0f} TF/s"
        for v in variants:
            o = sorted(to[v])[len(to[v]) // 2]
            tot[v] += o
            line += f" | v{specs[v][0]}:{specs[v][1]} {o:7.1f} us {fl / o / 1e6:5.0f} TF/s {b / o:5.3f}x"
        print(line, flush=True)
    print("TOTAL lib %.1f us | " % tot_b + " | ".join(f"v{specs[v][0]}:{specs[v][1]} {tot[v]:.1f} us {tot_b / tot[v]:.3f}x" for v in variants),
          flush=True)


if __name__ == "__main__":
    main()
