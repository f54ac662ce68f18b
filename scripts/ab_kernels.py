#!/usr/bin/env python3
"""In-process, interleaved A/B of two builds of the kernel library (cdna guide §5.4 rule 24:
device-to-device and call-to-call variance on MI355X is several percent, so code versions are only
compared inside one process, alternating).

  python -m nanodiloco_amd.csrc.build --rev HEAD~1      # -> nanodiloco_amd/_lib/alt/libnd_kernels_<sha>.so
  python scripts/ab_kernels.py --alt nanodiloco_amd/_lib/alt/libnd_kernels_<sha>.so --what attn

--what attn : attention fwd+bwd on the Llama-150M micro-batch (per-kernel times via torch.profiler
              are not needed: each op is timed with HIP events, min over rounds)
--what step : one full forward+backward of Llama-150M (micro-batch 32 x 1024)
--what wgrad: the wgrad GEMM shapes
--what epi  : the fused-epilogue ping-pong GEMMs (q|k|v+RoPE, gate|up+SwiGLU, down dgrad+SwiGLU bwd)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanodiloco_amd import ops  # noqa: E402
from nanodiloco_amd.ops import _ext  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


OUTPUTS = {}  # workload -> tensors it writes (bitwise comparison of the two libraries, --what attnk)


def workloads(what):
    from nanodiloco_amd.ops.attention import rope_cache
    out = {}
    if what == "attn":
        B, T, nh, hd = 32, 1024, 16, 64
        qkv = torch.randn(B * T, 3 * nh * hd, device="cuda").bfloat16()
        cos, sin = rope_cache(T, hd, 10000.0, None, "cuda")
        x = qkv.clone().requires_grad_(True)
        o = ops.attention(x, cos, sin, B, T, nh, nh, hd)
        do = torch.randn_like(o)
        out["attn_fwd"] = lambda: ops.attention(x, cos, sin, B, T, nh, nh, hd)
        out["attn_bwd"] = lambda: torch.autograd.grad(o, x, do, retain_graph=True)
    elif what == "step":
        from nanodiloco_amd.config import resolve_llama_config
        from nanodiloco_amd.models import LlamaForCausalLM
        cfg = resolve_llama_config("llama_150m.json")
        m = LlamaForCausalLM(cfg, "cuda", torch.bfloat16).init_weights(0)
        ids = torch.randint(0, cfg.vocab_size, (32, 1024), device="cuda")

        def step():
            m(ids, labels=ids).loss.backward()
        out["fwd_bwd"] = step
    elif what == "ce":
        V, n = 32000, 16384
        logits = torch.randn(n, V, device="cuda").bfloat16()
        tgt = torch.randint(0, V, (n,), device="cuda")
        loss = torch.zeros(1, device="cuda")
        sc = torch.ones(1, device="cuda")

        def ce():
            _ext.check(_ext.lib().nd_ce_fwd_bwd(logits.data_ptr(), 1, tgt.data_ptr(), loss.data_ptr(), sc.data_ptr(),
                                                n, V, -100, 0, 0, 0.0, _ext.stream_ptr()), "ce")
        out["ce_16k"] = ce
    elif what == "attnk":  # the raw attention kernels at the Llama-150M bench shape (pre-rotated q|k)
        B, T, nh, hd = 64, 1024, 16, 64
        ld = 3 * nh * hd
        qkv = torch.randn(B * T, ld, device="cuda").bfloat16()
        k, v = qkv[:, nh * hd:], qkv[:, 2 * nh * hd:]
        o = torch.empty(B * T, nh * hd, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(B, nh, T, device="cuda")
        do = torch.randn(B * T, nh * hd, device="cuda").bfloat16()
        dqkv = torch.empty_like(qkv)
        ws = torch.empty(2, B, nh, T, device="cuda")

        def fwd():
            _ext.check(_ext.lib().nd_attn_fwd_ks(qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                                 B, nh, nh, T, hd, ld, nh * hd, 0, 0, hd ** -0.5, 0, _ext.stream_ptr()), "f")

        def bwd():
            _ext.check(_ext.lib().nd_attn_bwd_fused_ks(
                qkv.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(), dqkv.data_ptr(),
                dqkv[:, nh * hd:].data_ptr(), dqkv[:, 2 * nh * hd:].data_ptr(), ws.data_ptr(), B, nh, nh, T, hd, ld,
                nh * hd, 0, 0, hd ** -0.5, 0, 0, _ext.stream_ptr()), "b")
        fwd()
        out["attn_fwd"] = fwd
        out["attn_bwd"] = bwd
        OUTPUTS["attn_fwd"] = (o, lse)
        OUTPUTS["attn_bwd"] = (dqkv,)
    elif what == "epi":  # the fused-epilogue ping-pong GEMMs at the Llama-150M bench shapes
        from nanodiloco_amd.ops import gemm as G
        M, d, F = 131072, 1024, 2688
        x = (torch.randn(M, d, device="cuda") * 0.5).bfloat16()
        wq = (torch.randn(3 * d, d, device="cuda") * 0.05).bfloat16()
        wgu = (torch.randn(2 * F, d, device="cuda") * 0.05).bfloat16()
        wdt = (torch.randn(F, d, device="cuda") * 0.05).bfloat16()
        cos, sin = rope_cache(1024, 64, 10000.0, None, "cuda")
        gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
        out["rope"] = lambda: G.gemm_pp_rope(x, wq, cos, sin, 1024, 64, 2 * d)
        out["swiglu"] = lambda: G.gemm_pp_swiglu(x, wgu)
        out["dswiglu"] = lambda: G.gemm_pp_dswiglu(x, wdt, gu)
        # the plain products of the same shapes: what each fused epilogue costs on top
        out["qkv_plain"] = lambda: G.gemm_pp(x, wq)
        out["gu_plain"] = lambda: G.gemm_pp(x, wgu)
        out["down_dgrad_plain"] = lambda: G.gemm_pp(x, wdt)
    elif what == "cast":  # fp8 quantisation of the attention backward's d(q|k|v) at the Llama-150M bench shape
        x = torch.randn(131072, 3072, device="cuda").bfloat16()
        sc = torch.full((1,), 64.0, device="cuda")
        q8 = torch.empty(x.shape, device="cuda", dtype=torch.uint8)
        am = torch.zeros(64, device="cuda")

        def cast():
            _ext.check(_ext.lib().nd_fp8_cast(x.data_ptr(), _ext.dtcode(x), x.numel(), sc.data_ptr(), q8.data_ptr(), 1,
                                              am.data_ptr(), am.numel(), _ext.stream_ptr()), "cast")
        out["cast_e5m2"] = cast
        OUTPUTS["cast_e5m2"] = (q8,)
    elif what == "wgrad":
        from nanodiloco_amd.ops.gemm import wgrad
        # lm: 500 output tiles -> one split (C += acc in place, the S == 1 epilogue)
        for name, (M, N) in {"qkv": (3072, 1024), "o": (1024, 1024), "gate_up": (5376, 1024),
                             "down": (1024, 2688), "lm": (32000, 1024)}.items():
            dy = torch.randn(32768, M, device="cuda").bfloat16()
            xx = torch.randn(32768, N, device="cuda").bfloat16()
            gw = torch.zeros(M, N, device="cuda")
            out[name] = (lambda gw=gw, dy=dy, xx=xx: wgrad(gw, dy, xx))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--alt", required=True)
    ap.add_argument("--what", default="attn", choices=["attn", "attnk", "step", "wgrad", "ce", "epi", "cast"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops.set_backend("hip")
    base = _ext.lib()
    alt = _ext.load_library(a.alt)
    wl = workloads(a.what)
    res = {k: {"new": [], "alt": []} for k in wl}
    for _ in range(a.rounds):
        for k, fn in wl.items():
            res[k]["new"].append(timed(fn, a.iters))
            with _ext.using(alt):
                res[k]["alt"].append(timed(fn, a.iters))
    for k, r in res.items():
        n, o = min(r["new"]), min(r["alt"])
        same = ""
        if k in OUTPUTS:
            wl[k]()
            mine = [t.clone() for t in OUTPUTS[k]]
            with _ext.using(alt):
                wl[k]()
            torch.cuda.synchronize()
            same = " | bitwise " + ("equal" if all(torch.equal(a, b) for a, b in zip(mine, OUTPUTS[k])) else
                                    "DIFFERENT (max %.3g)" % max((a.float() - b.float()).abs().max().item()
                                                                 for a, b in zip(mine, OUTPUTS[k])))
        print(f"{k:10s} working-tree {n:9.1f} us | alt {o:9.1f} us | speedup {o / n:5.3f}x{same}", flush=True)
    del base


if __name__ == "__main__":
    main()
