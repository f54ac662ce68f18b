#!/usr/bin/env python3
"""Ping-pong GEMM (csrc/gemm_pp.hip): numerics against an fp32 torch reference, then an interleaved
in-process timing A/B against hipBLASLt (torch.mm) on the
Llama-150M / 1B projection shapes, random operands.

    python scripts/gemm_pp_bench.py [--tokens 65536] [--model 150m|1b] [--rounds 5] [--check-only]
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


def rel(x, ref, name=""):
    err = (x.float() - ref).abs()
    e = (err.max() / ref.abs().max().clamp_min(1e-6)).item()
    if e >= 1e-2 and name:  # where are the wrong elements?
        bad = err > 0.05 * ref.abs().max()
        rows = bad.any(1).nonzero()[:, 0]
        cols = bad.any(0).nonzero()[:, 0]
        print(f"  {name}: {int(bad.sum())} bad of {bad.numel()}; rows {rows.min().item()}..{rows.max().item()} "
              f"({rows.numel()}), cols {cols.min().item()}..{cols.max().item()} ({cols.numel()}); "
              f"first cols {cols[:24].tolist()}; first rows {rows[:12].tolist()}; "
              f"bad-value sample {x.float()[bad][:4].tolist()} ref {ref[bad][:4].tolist()}", flush=True)
    return e


def w128o(x, w, out):
    """the w128 kernel with the epilogue inside each tile's last phase"""
    G.set_w128(ovl=1)
    try:
        return G.gemm_w128(x, w, out)
    finally:
        G.set_w128(ovl=0)


def w128vb(x, w, out):
    """the w128 kernel (epilogue in the last phase) with its B operand staged through VGPRs"""
    G.set_w128(ovl=1)
    old = G.set_w128_vb(1)
    try:
        return G.gemm_w128(x, w, out)
    finally:
        G.set_w128_vb(old)
        G.set_w128(ovl=0)


def check():
    torch.manual_seed(0)
    bad = 0
    for (m, n, k) in [(256, 256, 64), (512, 768, 128), (300, 264, 192), (4096, 3072, 1024), (2048, 2688, 1024),
                      (65536 // 8, 1024, 5376), (1000, 520, 640), (8192, 1024, 32000 // 500 * 64),
                      (16384, 3072, 1024), (32768, 2688, 256), (9000, 1000, 320)]:
        a, b = r(m, k), r(n, k) * 0.05
        ref = a.float() @ b.float().t()
        for nm, fn in (("gemm_pp", G.gemm_pp), ("gemm_w128", G.gemm_w128),
                       ("gemm_w128o", lambda a_, b_: w128o(a_, b_, None)),
                       ("gemm_w128vb", lambda a_, b_: w128vb(a_, b_, None))):
            y = fn(a, b)
            e = rel(y, ref, f"{nm} {m}x{n}x{k}")
            ok = e < 1e-2
            bad += not ok
            print(f"check {nm} {m}x{n}x{k}: rel {e:.2e} {'ok' if ok else 'FAIL'}", flush=True)
    # strided operands / output (views into wider buffers)
    a_w, b_w, o_w = r(512, 1024), r(384, 768) * 0.05, torch.zeros(512, 520, device="cuda", dtype=torch.bfloat16)
    a, b, o = a_w[:, :640], b_w[:, :640], o_w[:, :384]
    G.gemm_pp(a, b, o)
    e = rel(o, a.float() @ b.float().t(), "strided")
    bad += e >= 1e-2
    # strided C only / strided A, B only
    o_w.zero_()
    a2, b2 = a.contiguous(), b.contiguous()
    G.gemm_pp(a2, b2, o)
    e_c = rel(o, a2.float() @ b2.float().t(), "strided-C")
    o2 = G.gemm_pp(a, b)
    e_ab = rel(o2, a.float() @ b.float().t(), "strided-AB")
    bad += (e_c >= 1e-2) + (e_ab >= 1e-2)
    print(f"check gemm_pp strided-C rel {e_c:.2e}, strided-AB rel {e_ab:.2e}", flush=True)
    print(f"check gemm_pp strided: rel {e:.2e} untouched-cols {o_w[:, 384:].abs().max().item()}", flush=True)
    # fused SwiGLU forward
    M, F, K = 1024, 2688 // 4, 1024
    x, w = r(M, K), r(2 * F, K) * 0.05
    gu, act = G.gemm_pp_swiglu(x, w)
    gref = x.float() @ w.float().t()
    e1 = rel(gu, gref, "swiglu-gu")
    g_, u_ = gu[:, :F].float(), gu[:, F:].float()
    e2 = rel(act, torch.nn.functional.silu(g_) * u_)
    bad += e1 >= 1e-2 or e2 >= 1e-2
    print(f"check gemm_pp_swiglu: gu rel {e1:.2e} act rel {e2:.2e}", flush=True)
    # fused SwiGLU backward
    dy, wdt = r(M, K), r(F, K) * 0.05
    dgu = G.gemm_pp_dswiglu(dy, wdt, gu)
    dact = (dy.float() @ wdt.float().t())
    sg = torch.sigmoid(g_)
    dref = torch.cat([dact * u_ * sg * (1 + g_ * (1 - sg)), dact * g_ * sg], 1)
    e3 = rel(dgu, dref)
    bad += e3 >= 1e-2
    print(f"check gemm_pp_dswiglu: rel {e3:.2e}", flush=True)
    # fused RoPE
    for hd in (64, 32):
        T, nq = 128, 4 * hd * 3
        x, wq = r(2 * T, K), r(nq, K) * 0.05
        cos, sin = ops.rope_cache(T, hd, 10000.0, None, "cuda")
        rc = 2 * nq // 3
        y = G.gemm_pp_rope(x, wq, cos, sin, T, hd, rc)
        ref = x.float() @ wq.float().t()
        t = torch.arange(2 * T, device="cuda") % T
        q = ref[:, :rc].view(2 * T, -1, hd)
        c, s_ = cos[t].float()[:, None, :], sin[t].float()[:, None, :]
        rot = torch.cat([-q[..., hd // 2:], q[..., :hd // 2]], -1)
        ref[:, :rc] = (q * c + rot * s_).reshape(2 * T, rc)
        e4 = rel(y, ref)
        bad += e4 >= 1e-2
        print(f"check gemm_pp_rope hd={hd}: rel {e4:.2e}", flush=True)
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--model", default="150m")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--gms", default="", help="comma list of tile-group sizes (G.set_pp_group_m) to A/B")
    ap.add_argument("--ablate", default="", help="comma list of ablation variants (G.set_pp_variant) to time "
                                                 "on the qkv-fwd / gu-dgrad / lm-dgrad shapes instead")
    a = ap.parse_args()
    ops.set_backend("hip")
    if a.ablate or a.gms:
        vs = [int(v) for v in a.ablate.split(",")] if a.ablate else []
        gms = [int(v) for v in a.gms.split(",")] if a.gms else []
        res = {}
        shapes = {"qkv fwd": (65536, 3072, 1024), "gu dgrad": (65536, 1024, 5376), "o fwd": (65536, 1024, 1024),
                  "lm logits": (65536, 32000, 1024)}
        ops_ = {}
        for nm, (m, n, k) in shapes.items():
            x, w = r(m, k), r(n, k) * 0.05
            out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
            ops_[nm] = (x, w, out, 2.0 * m * n * k)
        for rd in range(a.rounds):
            for nm, (x, w, out, fl) in ops_.items():
                res.setdefault((nm, "blas"), []).append(timed(lambda: torch.mm(x, w.t(), out=out)))
                for v in vs:
                    G.set_pp_variant(v)
                    res.setdefault((nm, v), []).append(timed(lambda: G.gemm_pp(x, w, out)))
                G.set_pp_variant(0)
                for gm in gms:
                    old = G.set_pp_group_m(gm)
                    res.setdefault((nm, f"gm{gm}"), []).append(timed(lambda: G.gemm_pp(x, w, out)))
                    G.set_pp_group_m(old)
        for nm, (x, w, out, fl) in ops_.items():
            line = f"{nm:9s}"
            for arm in ["blas"] + vs + [f"gm{gm}" for gm in gms]:
                t = sorted(res[(nm, arm)])[len(res[(nm, arm)]) // 2]
                line += f" | {arm}: {t:7.1f} us {fl / t / 1e6:5.0f} TF"
            print(line, flush=True)
        return
    bad = check()
    if bad:
        print(f"{bad} numerics checks FAILED", flush=True)
    if a.check_only:
        sys.exit(1 if bad else 0)
    M = a.tokens
    d, F, nh, nkv, hd, V = (1024, 2688, 16, 16, 64, 32000) if a.model == "150m" else (2048, 5632, 32, 4, 64, 32000)
    qkv_n = (nh + 2 * nkv) * hd
    cases = []

    def plain(name, m, n, k):
        x, w = r(m, k), r(n, k) * 0.05
        out = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
        arms = {"blas": lambda: torch.mm(x, w.t(), out=out), "pp": lambda: G.gemm_pp(x, w, out),
                "w128": lambda: G.gemm_w128(x, w, out), "w128o": lambda: w128o(x, w, out),
                "w128vb": lambda: w128vb(x, w, out)}
        cases.append((name, 2.0 * m * n * k, arms))

    plain("qkv fwd", M, qkv_n, d)
    plain("o fwd", M, d, nh * hd)
    plain("gu fwd", M, 2 * F, d)
    plain("down fwd", M, d, F)
    plain("qkv dgrad", M, d, qkv_n)
    plain("o dgrad", M, nh * hd, d)
    plain("gu dgrad", M, d, 2 * F)
    plain("down dgrad", M, F, d)
    plain("lm logits", M, V, d)
    plain("lm dgrad", M, d, V)
    res = {}
    for rd in range(a.rounds):
        for name, fl, arms in cases:
            for arm, fn in arms.items():
                res.setdefault((name, arm), []).append(timed(fn))
        print(f"round {rd} done", flush=True)
    tot = {}
    for name, fl, arms in cases:
        line = f"{name:11s}"
        blas = sorted(res[(name, 'blas')])[len(res[(name, 'blas')]) // 2]
        for arm in arms:
            t = sorted(res[(name, arm)])[len(res[(name, arm)]) // 2]
            tot[arm] = tot.get(arm, 0.0) + t
            line += f" | {arm} {t:8.1f} us {fl / t / 1e9:6.0f} TF {blas / t:5.3f}x"
        print(line, flush=True)
    print("total " + " ".join(f"{k} {v:.0f} us ({tot['blas'] / v:.3f}x)" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
