"""Projection GEMMs with gradient routing into the flat fp32 grad buffer.

``y = x @ W^T`` for W of shape [out, in].  Plain forward and dgrad products go to the selected plain GEMM
(``set_proj_gemm``: hipBLASLt through ``torch.mm`` by default, or the own kernels); the fused ones
(``LinearRopeFn``, ``MLPFn``) always run on the own kernel.  The weight gradient is accumulated straight into the fp32
``ParamStore.grad`` view: bf16 operands, fp32 accumulate, beta=1 -- one GEMM, no bf16 grad
tensor, no separate accumulate pass.  On the HIP path that GEMM is our own ``nd_wgrad`` kernel
(ops/gemm.py); otherwise hipBLASLt ``addmm(out_dtype=fp32)`` (this replaces autograd's per-parameter AccumulateGrad,
K11 in SURVEY.md §2.3).  Fused weights (q|k|v, gate|up) are single views, so one GEMM covers
all three / both projections.

Weight-gradient overlap (``set_wgrad_overlap(True)``): the wgrad GEMM is off the backward's
critical path (nothing downstream reads it until the optimizer), so it is issued on a side HIP
stream forked from the compute stream at that point; the dgrad chain (dgrad GEMM -> SwiGLU /
RMSNorm / attention backward, several of them HBM-bound) continues on the compute stream and the
hardware co-schedules the two queues.  The compute stream joins the side stream at the end of the
backward (``join_wgrad``: embedding backward, inner-DDP layer hooks, optimizer step) -- a GPU-side
wait, never a host sync.  dY / X stay referenced until that join (then the compute stream, which
allocated them, is ordered after the side stream, so the caching allocator may reuse them at once;
``record_stream`` instead defers every such free behind an event and made the allocator fall
back to fresh hipMalloc calls -- host stalls of hundreds of ms per step).

GEMM fence: the compute stream also joins before every LIBRARY GEMM (``library_gemm_fence``).
hipBLASLt's stream-K kernels keep one workgroup per CU and make workgroups wait on each other's
partial tiles; when a side-stream wgrad holds CUs, part of that grid cannot become resident and
the resident part spins -- measured 2-8x slower steps.  Fenced, a wgrad co-runs only with our own
kernels (SwiGLU / RMSNorm backward, the attention backward), which never wait on each other.
"""
from __future__ import annotations

import torch

from . import _ext

_DTYPE_OUT_OK = {"checked": False, "ok": False}
_OVERLAP = {"enabled": False, "fence": True, "streams": {}, "pending": set(), "keep": []}
_DGRAD_T = {"enabled": True}


def transpose_into(dst: torch.Tensor, w: torch.Tensor) -> None:
    """dst[in, out] = w[out, in]^T (bf16 HIP kernel on the GPU; strided copy otherwise)."""
    if w.is_cuda and w.dtype == torch.bfloat16 and _ext.get_backend() != "torch":
        _ext.check(_ext.lib().nd_transpose_bf16(_ext.ptr(w), _ext.ptr(dst), w.shape[0], w.shape[1], w.stride(0),
                                                 dst.stride(0), _ext.stream_ptr(w.device)), "nd_transpose_bf16")
    else:
        dst.copy_(w.t())


def set_dgrad_transposed(enabled: bool) -> None:
    """Input-gradient GEMMs read a transposed weight copy (see ``LinearFn``)."""
    _DGRAD_T["enabled"] = bool(enabled)


def dgrad_transposed_enabled() -> bool:
    return _DGRAD_T["enabled"]


def set_wgrad_overlap(mode) -> None:
    """Issue projection weight-gradient GEMMs on a side stream (GPU only).  0/False: off;
    1/True: on, fenced before every library GEMM; 2: on, unfenced (A/B only, see module doc)."""
    _OVERLAP["enabled"] = int(mode) != 0
    _OVERLAP["fence"] = int(mode) != 2


def wgrad_overlap_enabled() -> bool:
    return _OVERLAP["enabled"]


def _side_stream(device: torch.device) -> torch.cuda.Stream:
    key = device.index if device.index is not None else torch.cuda.current_device()
    s = _OVERLAP["streams"].get(key)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _OVERLAP["streams"][key] = s
    return s


def join_wgrad(device=None) -> None:
    """Make the current stream wait for every weight-gradient GEMM issued on the side stream
    (no-op when nothing is outstanding)."""
    if not _OVERLAP["pending"]:
        return
    keys = list(_OVERLAP["pending"]) if device is None else [
        torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()]
    for k in keys:
        if k in _OVERLAP["pending"]:
            torch.cuda.current_stream(k).wait_stream(_OVERLAP["streams"][k])
            _OVERLAP["pending"].discard(k)
    if not _OVERLAP["pending"]:
        _OVERLAP["keep"].clear()  # operands of the joined wgrads: safe to free on the compute stream


def library_gemm_fence(device=None) -> None:
    """Call right before a hipBLASLt GEMM on the compute stream (see module doc: GEMM fence)."""
    if _OVERLAP["pending"] and _OVERLAP["fence"]:
        join_wgrad(device)


def _wgrad_on_side_stream(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor) -> None:
    cur = torch.cuda.current_stream(gw.device)
    side = _side_stream(gw.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        wgrad_accumulate(gw, dy, x)
    _OVERLAP["keep"].append((dy, x))
    _OVERLAP["pending"].add(side.device.index)


def wgrad_accumulate(gw: torch.Tensor, dy: torch.Tensor, x: torch.Tensor):
    """gw[out, in] (fp32) += dy[N, out]^T @ x[N, in]."""
    if dy.dtype == torch.float32:
        gw.addmm_(dy.t(), x)
        return
    if gw.is_cuda and _ext.get_backend() != "torch":
        from .gemm import wgrad, wgrad_supported
        if wgrad_supported(gw, dy, x):
            wgrad(gw, dy, x)
            return
    if gw.is_cuda:
        st = _DTYPE_OUT_OK
        if not st["checked"] or st["ok"]:
            try:
                torch.ops.aten.addmm.dtype_out(gw, dy.t(), x, torch.float32, beta=1, alpha=1, out=gw)
                st["checked"], st["ok"] = True, True
                return
            except (RuntimeError, NotImplementedError):
                st["checked"], st["ok"] = True, False
    gw.add_(torch.mm(dy.t(), x).float())


# ---- which GEMM runs the PLAIN projection products (forward / input gradient, lm head)
#   "blas" hipBLASLt through torch.mm -- the default: over the ten plain Llama-150M products the own kernels
#          reach 0.924x (pp) / 0.920x (w128) of it per shape, and the bf16 step is 1.9 % (pp) / 3.2 % (w128)
#          slower with them (round 5, gpurun_out r5a / r5k; profiles/r5_gemm.md); the task brief allows a
#          library for PLAIN GEMMs -- every fused product and every weight gradient is on the own kernels
#   "pp"   own ping-pong MFMA kernel (csrc/gemm_pp.hip; ops.gemm.gemm_pp) for every projection
#   "short" own kernel for the short-K products (K <= 1024: o forward / dgrad, lm-head logits); hipBLASLt for
#          the long-K dgrads (0.86-0.94x there)
#   "w128" own one-wave-per-SIMD kernel (csrc/gemm_w128.hip: hipBLASLt's K-loop shape, 128 x 128 per wave)
# The FUSED products always run on the own kernel (they exist only there): RoPE in the q|k|v
# projection's epilogue, SwiGLU in the gate|up projection's, the SwiGLU backward in the down
# projection's dgrad.  Under --fp8 every product (lm head included) runs on the own fp8 kernel.
_PROJ = {"gemm": "blas", "rope": True, "mlp": True}


def set_proj_gemm(name: str) -> None:
    if name not in ("pp", "blas", "short", "w128"):
        raise ValueError(name)
    _PROJ["gemm"] = name


def proj_gemm() -> str:
    return _PROJ["gemm"]


def set_fused_epilogues(rope: bool = None, mlp: bool = None) -> None:
    """RoPE-in-q|k|v-GEMM and SwiGLU-in-MLP-GEMMs fusions (own kernel only)."""
    if rope is not None:
        _PROJ["rope"] = bool(rope)
    if mlp is not None:
        _PROJ["mlp"] = bool(mlp)


def fused_epilogues() -> dict:
    return {"rope": _PROJ["rope"], "mlp": _PROJ["mlp"]}


def _pp_ok(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None, fused: bool = False) -> bool:
    """Shape / layout check for the own kernel; plain products also need the 'pp' selection (the
    fused-epilogue ops exist only on the own kernel and are switched by set_fused_epilogues)."""
    if not a.is_cuda or not (fused or _PROJ["gemm"] in ("pp", "w128") or (_PROJ["gemm"] == "short" and a.shape[-1] <= 1024)):
        return False
    from .gemm import pp_supported
    return pp_supported(a, b) and (out is None or (out.stride(-1) == 1 and out.stride(0) % 8 == 0
                                                   and out.data_ptr() % 16 == 0))


def mm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """a[M, K] . b[N, K]^T on the selected projection GEMM (the own kernel when 'pp' is selected and
    it takes the shape; hipBLASLt otherwise)."""
    if _pp_ok(a, b, out):
        from .gemm import gemm_pp, gemm_w128
        return gemm_w128(a, b, out) if _PROJ["gemm"] == "w128" else gemm_pp(a, b, out)
    library_gemm_fence(a.device if a.is_cuda else None)
    return torch.mm(a, b.t(), out=out) if out is not None else torch.mm(a, b.t())


def _wgrad(gw, dy, x):
    if gw is None:
        return
    if _OVERLAP["enabled"] and gw.is_cuda:
        _wgrad_on_side_stream(gw, dy, x)
    else:
        wgrad_accumulate(gw, dy, x)


# Grouped weight gradients (round 5): the MLP's down and gate|up weight gradients as ONE own-kernel launch
# (ops.gemm.wgrad2), issued after the gate|up input-gradient GEMM instead of one before and one after it.
_GROUP = {"enabled": True}


def set_wgrad_group(enabled: bool) -> None:
    _GROUP["enabled"] = bool(enabled)


def wgrad_group_enabled() -> bool:
    return _GROUP["enabled"]


def wgrad2_accumulate(gw0, dy0, x0, gw1, dy1, x1) -> None:
    """gw0 += dy0^T x0 and gw1 += dy1^T x1, grouped into one launch when the own kernel takes both."""
    if (gw0.is_cuda and _ext.get_backend() != "torch" and dy0.dtype == torch.bfloat16 and dy1.dtype == torch.bfloat16):
        from .gemm import wgrad2, wgrad_supported
        if wgrad_supported(gw0, dy0, x0) and wgrad_supported(gw1, dy1, x1) and wgrad2(gw0, dy0, x0, gw1, dy1, x1):
            return
    wgrad_accumulate(gw0, dy0, x0)
    wgrad_accumulate(gw1, dy1, x1)


def _wgrad2(gw0, dy0, x0, gw1, dy1, x1):
    if gw0 is None or gw1 is None:
        _wgrad(gw0, dy0, x0)
        _wgrad(gw1, dy1, x1)
        return
    if _OVERLAP["enabled"] and gw0.is_cuda:
        cur = torch.cuda.current_stream(gw0.device)
        side = _side_stream(gw0.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            wgrad2_accumulate(gw0, dy0, x0, gw1, dy1, x1)
        _OVERLAP["keep"].append((dy0, x0, dy1, x1))
        _OVERLAP["pending"].add(side.device.index)
    else:
        wgrad2_accumulate(gw0, dy0, x0, gw1, dy1, x1)


class LinearFn(torch.autograd.Function):
    """``wt`` (optional) is W^T stored [in, out] contiguous: the input gradient is then dY . (W^T)^T,
    the same K-contiguous "NT" operand layout as the forward GEMM, which hipBLASLt runs 14-16 %
    faster than dY . W (row-major x row-major) on every Llama-150M shape
    (scripts/dgrad_layout_bench.py); the model keeps the copies in step with the optimizer."""

    @staticmethod
    def forward(ctx, x, w, gw, wt=None):
        ctx.save_for_backward(x, w if wt is None else wt)
        ctx.gw = gw
        ctx.transposed = wt is not None
        return mm_nt(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.needs_input_grad[0]:
            if ctx.transposed:
                dx = mm_nt(dy, w)
            else:
                library_gemm_fence(dy.device if dy.is_cuda else None)
                dx = torch.mm(dy, w)
        else:
            dx = None
        _wgrad(ctx.gw, dy, x)
        return dx, None, None, None


def linear(x: torch.Tensor, w: torch.Tensor, gw: torch.Tensor, wt: torch.Tensor = None) -> torch.Tensor:
    return LinearFn.apply(x, w, gw, wt)




# ---------------------------------------------------------------------------------------------
# Fused epilogues on the own GEMM (csrc/gemm_pp.hip)

def linear_rope_supported(x: torch.Tensor, w: torch.Tensor, wt, hd: int, rope_cols: int) -> bool:
    return (_PROJ["rope"] and wt is not None and _pp_ok(x, w, fused=True) and hd in (32, 64) and rope_cols % 64 == 0)


class LinearRopeFn(torch.autograd.Function):
    """q|k|v projection with RoPE applied to the q and k columns in the GEMM epilogue (replaces the
    separate in-place rotation pass over the projection output).  The attention backward returns the
    gradient w.r.t. the UN-rotated projection (its dq/dk store epilogue applies the inverse
    rotation), so this backward is the plain projection backward."""

    @staticmethod
    def forward(ctx, x, w, gw, wt, cos, sin, T, hd, rope_cols):
        from .gemm import gemm_pp_rope
        ctx.save_for_backward(x, wt)
        ctx.gw = gw
        return gemm_pp_rope(x, w, cos, sin, T, hd, rope_cols)

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        dy = dy.contiguous()
        dx = mm_nt(dy, wt) if ctx.needs_input_grad[0] else None
        _wgrad(ctx.gw, dy, x)
        return dx, None, None, None, None, None, None, None, None


def linear_rope(x, w, gw, wt, cos, sin, T: int, hd: int, rope_cols: int) -> torch.Tensor:
    return LinearRopeFn.apply(x, w, gw, wt, cos, sin, int(T), int(hd), int(rope_cols))


def mlp_fused_supported(y: torch.Tensor, w_gu: torch.Tensor, wt_gu, w_down: torch.Tensor, wt_down) -> bool:
    F = w_gu.shape[0] // 2
    return (_PROJ["mlp"] and wt_gu is not None and wt_down is not None and _pp_ok(y, w_gu, fused=True) and F % 8 == 0
            and w_down.shape[1] == F and w_down.shape[0] % 8 == 0)


class MLPFn(torch.autograd.Function):
    """The whole SwiGLU MLP on the own GEMM with both activation passes fused away:

      forward   gu, act = [gate|up GEMM + SwiGLU epilogue](y)      (gu kept for the backward; by default in the
                                                                  coefficient form [d act/d gate | d act/d up],
                                                                  ops.gemm.set_mlp_coef)
                m       = act . W_down^T
      backward  dgu     = [down dgrad GEMM + SwiGLU-backward epilogue](dm, W_down^T copy, gu)
                          -- d(act) is never stored
                gW_down += dm^T act,  dy = dgu . W_gu (W_gu^T copy),  gW_gu += dgu^T y

    Same math as linear(swiglu(linear(y))) (tests/test_gemm_gpu.py checks it against that chain)."""

    @staticmethod
    def forward(ctx, y, w_gu, gw_gu, wt_gu, w_down, gw_down, wt_down):
        from .gemm import gemm_pp_swiglu
        gu, act = gemm_pp_swiglu(y, w_gu)
        m = mm_nt(act, w_down)
        ctx.save_for_backward(y, gu, act, wt_gu, wt_down)
        ctx.gw = (gw_gu, gw_down)
        return m

    @staticmethod
    def backward(ctx, dm):
        from .gemm import gemm_pp_dswiglu
        y, gu, act, wt_gu, wt_down = ctx.saved_tensors
        gw_gu, gw_down = ctx.gw
        dm = dm.contiguous()
        dgu = gemm_pp_dswiglu(dm, wt_down, gu)
        if _GROUP["enabled"]:  # both weight gradients in one launch, after the input gradient
            dy = mm_nt(dgu, wt_gu) if ctx.needs_input_grad[0] else None
            _wgrad2(gw_down, dm, act, gw_gu, dgu, y)
            return dy, None, None, None, None, None, None
        _wgrad(gw_down, dm, act)
        dy = mm_nt(dgu, wt_gu) if ctx.needs_input_grad[0] else None
        _wgrad(gw_gu, dgu, y)
        return dy, None, None, None, None, None, None


def mlp_fused(y, w_gu, gw_gu, wt_gu, w_down, gw_down, wt_down) -> torch.Tensor:
    return MLPFn.apply(y, w_gu, gw_gu, wt_gu, w_down, gw_down, wt_down)
