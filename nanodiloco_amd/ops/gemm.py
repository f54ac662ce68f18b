"""Own MFMA GEMMs (csrc/gemm_pp.hip, csrc/gemm_w128.hip, csrc/gemm_wgrad.hip).

* ``gemm_pp``          C[M, N] = A[M, K] . B[N, K]^T on the ping-pong kernel (two waves per SIMD in
                       opposite load / MFMA phases) -- the plain projection / lm-head products when
                       ``ops.linear.set_proj_gemm`` selects the own kernels (per-shape measurements:
                       profiles/r4_gemm_w128.md, profiles/r5_gemm.md).
* ``gemm_pp_rope``     the q|k|v projection with RoPE on q and k in the epilogue      } on the default
* ``gemm_pp_swiglu``   the gate|up projection writing gu AND act = silu(gate) * up    } path (ops/linear.py
* ``gemm_pp_dswiglu``  the down projection's dgrad fused with the SwiGLU backward     } LinearRopeFn, MLPFn)
* ``wgrad``            ``gW[M, N] (fp32) += dY[K, M]^T @ X[K, N]`` -- the weight gradient of every projection
                       (default path): both operands staged through LDS as they lie in memory, fragments
                       by transposing LDS reads, ping-pong pairing, deterministic split-K.
"""
from __future__ import annotations

import torch

from . import _ext

_WS = {}
_GEMM = {"backend": "hip"}


def set_gemm_backend(name: str) -> None:
    """'hip': the own kernels may run (default); 'blas': ``pp_supported`` refuses every shape (A/B)."""
    if name not in ("hip", "blas"):
        raise ValueError(name)
    _GEMM["backend"] = name


def gemm_backend() -> str:
    return _GEMM["backend"]


def _aligned(t: torch.Tensor) -> bool:
    return t.data_ptr() % 16 == 0 and t.stride(-1) == 1 and t.stride(0) % 8 == 0


_F8_FMT = {torch.float8_e4m3fn: 0, torch.float8_e5m2: 1}


# ---- ping-pong kernels (csrc/gemm_pp.hip): two waves per SIMD in opposite LOAD / COMPUTE phases

def pp_supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Can ``gemm_pp(a, b)`` run: bf16 2-D, K % 64, N % 8, 16-B aligned rows."""
    return (_GEMM["backend"] == "hip" and a.is_cuda and _ext.get_backend() != "torch"
            and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2
            and a.shape[1] == b.shape[1] and a.shape[1] % 64 == 0 and b.shape[0] % 8 == 0
            and _aligned(a) and _aligned(b))


def gemm_pp(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """out[M, N] = a[M, K] . b[N, K]^T on the ping-pong kernel."""
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=a.dtype, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp(_ext.ptr(a), _ext.ptr(b), _ext.ptr(out), M, N, K, a.stride(0), b.stride(0),
                                     out.stride(0), _ext.stream_ptr(a.device)), "nd_gemm_pp")
    return out


def gemm_pp_rope(a, b, cos, sin, T: int, hd: int, rope_cols: int, out=None) -> torch.Tensor:
    """q|k|v projection with RoPE on the first ``rope_cols`` columns (rows are tokens, t = row % T)."""
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=a.dtype, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp_rope(_ext.ptr(a), _ext.ptr(b), _ext.ptr(out), M, N, K, a.stride(0), b.stride(0),
                                          out.stride(0), _ext.ptr(cos), _ext.ptr(sin), T, hd, rope_cols,
                                          _ext.stream_ptr(a.device)), "nd_gemm_pp_rope")
    return out


def gemm_pp_swiglu(a, w_gu, gu_out=None, act_out=None):
    """(gu, act): gu = a . w_gu^T ([M, 2F]), act = silu(gu[:, :F]) * gu[:, F:] ([M, F])."""
    M, K = a.shape
    F = w_gu.shape[0] // 2
    gu = gu_out if gu_out is not None else torch.empty(M, 2 * F, dtype=a.dtype, device=a.device)
    act = act_out if act_out is not None else torch.empty(M, F, dtype=a.dtype, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp_swiglu(_ext.ptr(a), _ext.ptr(w_gu), _ext.ptr(gu), _ext.ptr(act), M, F, K,
                                            a.stride(0), w_gu.stride(0), gu.stride(0), act.stride(0),
                                            _ext.stream_ptr(a.device)), "nd_gemm_pp_swiglu")
    return gu, act


def gemm_pp_dswiglu(dy, w_down_t, gu, dgu_out=None):
    """d(gate|up) [M, 2F] of act = silu(gate) * up, where d(act) = dy . w_down_t^T (never stored)."""
    M, K = dy.shape
    F = w_down_t.shape[0]
    dgu = dgu_out if dgu_out is not None else torch.empty_like(gu)
    _ext.check(_ext.lib().nd_gemm_pp_dswiglu(_ext.ptr(dy), _ext.ptr(w_down_t), _ext.ptr(gu), _ext.ptr(dgu), M, F, K,
                                             dy.stride(0), w_down_t.stride(0), gu.stride(0), dgu.stride(0),
                                             _ext.stream_ptr(dy.device)), "nd_gemm_pp_dswiglu")
    return dgu


# ---- the same ping-pong kernels on fp8 operands (one v_mfma_scale_f32_16x16x128_f8f6f4 per 128-deep K-tile):
# a e4m3 (forward) or e5m2 (input gradient), b e4m3; sa / sb one-element fp32 dequantisation scales
# (the torch._scaled_mm contract); bf16 outputs and the fused epilogues on the dequantised accumulator.

def pp_f8_supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.is_cuda and _ext.get_backend() != "torch" and a.dim() == 2 and b.dim() == 2
            and a.dtype in _F8_FMT and b.dtype == torch.float8_e4m3fn and a.shape[1] == b.shape[1]
            and a.shape[1] % 128 == 0 and b.shape[0] % 8 == 0 and a.stride(1) == 1 and b.stride(1) == 1
            and a.stride(0) % 16 == 0 and b.stride(0) % 16 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def gemm_pp_f8(a, b, sa, sb, out=None) -> torch.Tensor:
    """out[M, N] (bf16) = sa * sb * a[M, K] . b[N, K]^T."""
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp_f8(_ext.ptr(a), _ext.ptr(b), _ext.ptr(out), M, N, K, a.stride(0), b.stride(0),
                                        out.stride(0), _ext.ptr(sa), _ext.ptr(sb), _F8_FMT[a.dtype],
                                        _ext.stream_ptr(a.device)), "nd_gemm_pp_f8")
    return out


def gemm_pp_rope_f8(a, b, sa, sb, cos, sin, T: int, hd: int, rope_cols: int, out=None) -> torch.Tensor:
    """fp8 q|k|v projection (a e4m3) with RoPE on the first ``rope_cols`` columns, bf16 out."""
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp_rope_f8(_ext.ptr(a), _ext.ptr(b), _ext.ptr(out), M, N, K, a.stride(0),
                                             b.stride(0), out.stride(0), _ext.ptr(sa), _ext.ptr(sb), _ext.ptr(cos),
                                             _ext.ptr(sin), T, hd, rope_cols, _ext.stream_ptr(a.device)),
               "nd_gemm_pp_rope_f8")
    return out


def gemm_pp_swiglu_f8(a, w_gu, sa, sb, gu_out=None, act_out=None):
    """fp8 gate|up projection (a, w_gu e4m3) + SwiGLU: (gu [M, 2F], act [M, F]) in bf16."""
    M, K = a.shape
    F = w_gu.shape[0] // 2
    gu = gu_out if gu_out is not None else torch.empty(M, 2 * F, dtype=torch.bfloat16, device=a.device)
    act = act_out if act_out is not None else torch.empty(M, F, dtype=torch.bfloat16, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp_swiglu_f8(_ext.ptr(a), _ext.ptr(w_gu), _ext.ptr(gu), _ext.ptr(act), M, F, K,
                                               a.stride(0), w_gu.stride(0), gu.stride(0), act.stride(0),
                                               _ext.ptr(sa), _ext.ptr(sb), _ext.stream_ptr(a.device)),
               "nd_gemm_pp_swiglu_f8")
    return gu, act


def gemm_pp_dswiglu_f8(dy, w_down_t, sa, sb, gu, dgu_out=None):
    """fp8 down-projection input gradient (dy e5m2 / e4m3, w_down_t e4m3) fused with the SwiGLU backward:
    d(gate|up) [M, 2F] bf16."""
    M, K = dy.shape
    F = w_down_t.shape[0]
    dgu = dgu_out if dgu_out is not None else torch.empty_like(gu)
    _ext.check(_ext.lib().nd_gemm_pp_dswiglu_f8(_ext.ptr(dy), _ext.ptr(w_down_t), _ext.ptr(gu), _ext.ptr(dgu), M, F,
                                                K, dy.stride(0), w_down_t.stride(0), gu.stride(0), dgu.stride(0),
                                                _ext.ptr(sa), _ext.ptr(sb), _F8_FMT[dy.dtype],
                                                _ext.stream_ptr(dy.device)), "nd_gemm_pp_dswiglu_f8")
    return dgu


def gemm_pp_swiglu_f8q(a, w_gu, sa, sb, qscale, qamax, gu_out=None, act8_out=None):
    """As ``gemm_pp_swiglu_f8`` but the SwiGLU output is written ONLY as e4m3 act8 = fp8(bf16(act) * qscale)
    (bitwise a separate cast of the bf16 act), amax folded into the ``qamax`` partial slots."""
    M, K = a.shape
    F = w_gu.shape[0] // 2
    gu = gu_out if gu_out is not None else torch.empty(M, 2 * F, dtype=torch.bfloat16, device=a.device)
    act8 = act8_out if act8_out is not None else torch.empty(M, F, dtype=torch.float8_e4m3fn, device=a.device)
    _ext.check(_ext.lib().nd_gemm_pp_swiglu_f8q(_ext.ptr(a), _ext.ptr(w_gu), _ext.ptr(gu), _ext.ptr(act8), M, F, K,
                                                a.stride(0), w_gu.stride(0), gu.stride(0), act8.stride(0),
                                                _ext.ptr(sa), _ext.ptr(sb), _ext.ptr(qscale), _ext.ptr(qamax),
                                                qamax.numel(), _ext.stream_ptr(a.device)), "nd_gemm_pp_swiglu_f8q")
    return gu, act8


def gemm_pp_dswiglu_f8q(dy, w_down_t, sa, sb, gu, qscale, qamax, dgu8_out=None):
    """As ``gemm_pp_dswiglu_f8`` but d(gate|up) is written ONLY as e5m2 dgu8 = fp8(bf16(dgu) * qscale)."""
    M, K = dy.shape
    F = w_down_t.shape[0]
    dgu8 = dgu8_out if dgu8_out is not None else torch.empty(M, 2 * F, dtype=torch.float8_e5m2, device=dy.device)
    _ext.check(_ext.lib().nd_gemm_pp_dswiglu_f8q(_ext.ptr(dy), _ext.ptr(w_down_t), _ext.ptr(gu), _ext.ptr(dgu8), M, F,
                                                 K, dy.stride(0), w_down_t.stride(0), gu.stride(0), dgu8.stride(0),
                                                 _ext.ptr(sa), _ext.ptr(sb), _F8_FMT[dy.dtype], _ext.ptr(qscale),
                                                 _ext.ptr(qamax), qamax.numel(), _ext.stream_ptr(dy.device)),
               "nd_gemm_pp_dswiglu_f8q")
    return dgu8


def gemm_w128(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """out[M, N] = a[M, K] . b[N, K]^T on the one-wave-per-SIMD kernel (csrc/gemm_w128.hip: 4 waves,
    128 x 128 outputs per wave, one continuous MFMA stream per K-tile -- the hipBLASLt K-loop shape)."""
    M, K = a.shape
    N = b.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=a.dtype, device=a.device)
    _ext.check(_ext.lib().nd_gemm_w128(_ext.ptr(a), _ext.ptr(b), _ext.ptr(out), M, N, K, a.stride(0), b.stride(0),
                                       out.stride(0), _ext.stream_ptr(a.device)), "nd_gemm_w128")
    return out


def set_w128(group_m: int = -1, nt: int = -1, ovl: int = -1) -> int:
    """Tile grouping (m-panels per group) / non-temporal C stores / epilogue overlapped with the next
    tile's first phase, of the w128 kernel (-1: unchanged); returns the previous group size."""
    return int(_ext.lib().nd_gemm_w128_set(int(group_m), int(nt), int(ovl)))


def set_pp_variant(v: int) -> int:
    """Ablation builds of the ping-pong kernel (profiling only -- WRONG results): 1 no LDS-DMA in the
    loop, 2 no fragment reads, 3 both, 4 no barriers, 8 no epilogue stores, 15 all; 0 = the kernel."""
    return int(_ext.lib().nd_gemm_pp_set_variant(int(v)))


def set_mlp_coef(v: int) -> int:
    """Saved-tensor form of the fused SwiGLU pair (gemm_pp_swiglu* -> gemm_pp_dswiglu*, every dtype): 0 the
    forward keeps gu = [gate | up] and the backward recomputes sigmoid(gate); 1 the forward keeps the SwiGLU
    derivative coefficients [A | B] (A = d act / d gate, B = d act / d up) in the same buffer, so the backward is
    two multiplies per unit (the default since round 6: profiles/r6_mlp_coef_ab.md).  Set it only between steps (a
    saved tensor must be read back in its own form); v < 0 only reads it.  Returns the previous setting."""
    return int(_ext.lib().nd_mlp_coef_set(int(v)))


def mlp_coef() -> int:
    return set_mlp_coef(-1)


def set_pp_group_m(g: int) -> int:
    """m-panels per tile group of the ping-pong kernel (XCD L2 locality); returns the old value."""
    return int(_ext.lib().nd_gemm_pp_set_group_m(int(g)))


def _workspace(device, numel):
    """Split-K slab workspace, one per (device, stream): wgrads issued on the side stream
    (ops/linear.py overlap) and on the compute stream (lm head) must not share slabs."""
    stream = torch.cuda.current_stream(device)
    key = (str(device), stream.cuda_stream)
    t = _WS.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        _WS[key] = t
    return t


def wgrad_supported(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> bool:
    return (gw.is_cuda and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and gw.dtype == torch.float32
            and dy.dim() == 2 and x.dim() == 2 and dy.stride(1) == 1 and x.stride(1) == 1 and gw.stride(1) == 1
            and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0 and dy.stride(0) % 8 == 0 and x.stride(0) % 8 == 0
            and gw.stride(0) % 4 == 0)


def wgrad(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    K, M = dy.shape
    N = x.shape[1]
    assert x.shape[0] == K and tuple(gw.shape) == (M, N)
    L = _ext.lib()
    S = L.nd_wgrad_splits(M, N, K)
    ws = _workspace(gw.device, S * M * N) if S > 1 else None
    _ext.check(L.nd_wgrad(_ext.ptr(dy), _ext.ptr(x), _ext.ptr(gw), _ext.ptr(ws), M, N, K, dy.stride(0), x.stride(0),
                          gw.stride(0), _ext.stream_ptr(gw.device)), "nd_wgrad")


def wgrad2(gw0: torch.Tensor, dy0: torch.Tensor, x0: torch.Tensor,
           gw1: torch.Tensor, dy1: torch.Tensor, x1: torch.Tensor) -> bool:
    """Both weight gradients ``gw_i += dy_i^T x_i`` (same token count K) in ONE ping-pong launch whose split
    count is chosen for the pair (csrc/gemm_wgrad.hip nd_wgrad2): e.g. the Llama-150M MLP's down (44 tiles)
    and gate|up (84 tiles) products fill exactly 256 CUs together with 2 K-splits, where alone they leave
    36 / 4 CUs idle.  Returns False (nothing issued) when the pair cannot be grouped -- the caller then
    runs ``wgrad`` twice."""
    K, M0 = dy0.shape
    N0, M1, N1 = x0.shape[1], dy1.shape[1], x1.shape[1]
    if dy1.shape[0] != K or x0.shape[0] != K or x1.shape[0] != K:
        return False
    if tuple(gw0.shape) != (M0, N0) or tuple(gw1.shape) != (M1, N1):
        return False
    L = _ext.lib()
    S = L.nd_wgrad2_splits(M0, N0, M1, N1, K)
    if S <= 0:
        return False
    ws0 = ws1 = None
    if S > 1:
        ws = _workspace(gw0.device, S * (M0 * N0 + M1 * N1))
        ws0, ws1 = ws, ws[S * M0 * N0:]
    _ext.check(L.nd_wgrad2(_ext.ptr(dy0), _ext.ptr(x0), _ext.ptr(gw0), _ext.ptr(ws0), M0, N0, dy0.stride(0),
                           x0.stride(0), gw0.stride(0), _ext.ptr(dy1), _ext.ptr(x1), _ext.ptr(gw1), _ext.ptr(ws1), M1,
                           N1, dy1.stride(0), x1.stride(0), gw1.stride(0), K, _ext.stream_ptr(gw0.device)), "nd_wgrad2")
    return True


def wgrad_f8_supported(gw: torch.Tensor, dy8: torch.Tensor, x8: torch.Tensor) -> bool:
    """Can ``wgrad_f8`` run: fp8 token-major operands (dy e4m3 / e5m2, x e4m3), tokens % 128, M, N >= 256."""
    return (gw.is_cuda and _ext.get_backend() != "torch" and gw.dtype == torch.float32 and dy8.dim() == 2
            and x8.dim() == 2 and dy8.dtype in _F8_FMT and x8.dtype == torch.float8_e4m3fn
            and dy8.shape[0] == x8.shape[0] and dy8.shape[0] % 128 == 0 and dy8.shape[1] % 16 == 0
            and x8.shape[1] % 16 == 0 and dy8.shape[1] >= 256 and x8.shape[1] >= 256 and dy8.stride(1) == 1
            and x8.stride(1) == 1 and gw.stride(1) == 1 and dy8.stride(0) % 16 == 0 and x8.stride(0) % 16 == 0
            and gw.stride(0) % 4 == 0 and dy8.data_ptr() % 16 == 0 and x8.data_ptr() % 16 == 0)


def wgrad_f8(gw: torch.Tensor, dy8: torch.Tensor, x8: torch.Tensor, s_dy: torch.Tensor, s_x: torch.Tensor) -> None:
    """gw[M, N] (fp32) += s_dy * s_x * dy8[K, M]^T . x8[K, N]: the fp8 weight gradient straight from the
    token-major fp8 operands the forward / input-gradient GEMMs already use (csrc/gemm_wgrad.hip
    wgrad8_pp_kernel: transposing ds_read_b64_tr_b8 fragments, 16x16x128 f8f6f4 MFMA)."""
    K, M = dy8.shape
    N = x8.shape[1]
    assert x8.shape[0] == K and tuple(gw.shape) == (M, N)
    L = _ext.lib()
    S = L.nd_wgrad_f8_splits(M, N, K)
    ws = _workspace(gw.device, S * M * N) if S > 1 else None
    _ext.check(L.nd_wgrad_f8(_ext.ptr(dy8), _ext.ptr(x8), _ext.ptr(gw), _ext.ptr(ws), M, N, K, dy8.stride(0),
                             x8.stride(0), gw.stride(0), _ext.ptr(s_dy), _ext.ptr(s_x), _F8_FMT[dy8.dtype],
                             _ext.stream_ptr(gw.device)), "nd_wgrad_f8")


def set_w128_vb(v: int) -> int:
    """1: the w128 kernel stages its B operand through VGPRs (buffer_load + ds_write) instead of LDS-DMA, the
    A operand stays DMA-fed (A/B, round 6); 0: both DMA-fed (default).  Returns the previous setting."""
    return int(_ext.lib().nd_gemm_w128_set_vb(int(v)))


def set_w128_ablation(v: int) -> int:
    """Ablation builds of the w128 kernel (profiling only -- WRONG results): 1 no LDS-DMA, 2 no fragment
    reads, 4 no barriers, 8 no epilogue stores, 16 no vmcnt waits in the loop, 31 all; 0 = the kernel."""
    return int(_ext.lib().nd_gemm_w128_set_ablation(int(v)))
