"""fp8 inner step (BASELINE config 5): OCP fp8 GEMMs for the decoder projections on gfx950.

Recipe (per-tensor scaling, the common "delayed scaling" scheme):
* forward  ``y = x @ W^T`` with x, W in e4m3 on the own ping-pong GEMM in its fp8 form (``gemm.gemm_pp_f8``,
  csrc/gemm_pp.hip F8: one ``v_mfma_scale_f32_16x16x128_f8f6f4`` per 128-deep K-tile of the same LDS image
  as the bf16 kernel; default ``set_fp8_gemm("pp")``), bf16 out.  The q|k|v projection keeps RoPE and the
  MLP keeps SwiGLU / its backward in that GEMM's epilogues (``Fp8RopeFn``, ``Fp8MLPFn``; on the dequantised
  fp32 accumulator).  ``"hipblaslt"`` (``torch._scaled_mm``) is the A/B alternative; it runs the RoPE /
  SwiGLU passes separately;
* dgrad    ``dx = dy @ W`` with dy in e5m2 (range for gradients), W^T in e4m3, same kernels;
* wgrad    ``dW = dy^T x``: bf16 ``nd_wgrad`` by default; with ``wgrad_fp8`` the own fp8 kernel
  (``gemm.wgrad_f8``, csrc/gemm_wgrad.hip wgrad8_pp_kernel) straight from the token-major fp8 operands
  the other two GEMMs already use -- ``ds_read_b64_tr_b8`` transposes them on the way out of LDS, so no
  transposed copies are written, and the forward keeps x8 (half the bytes of x) for the backward;
* activations / gradients are quantised by ``nd_fp8_cast`` (one pass: scale, saturate, convert,
  and record amax) with a scale derived from the amax history of previous steps (``Fp8Recipe``;
  device-side, no host sync); the very first use of a tensor role is scaled from its current amax;
* weights are re-quantised once per optimizer update (current amax), together with their transpose;
* lm_head, attention, norms stay bf16/fp32; fp32 master weights and optimizer state are unchanged.
* fused operand quantisation: once a slot's scale exists (delayed scaling: known before the
  producer runs), the PRODUCER of an operand writes its fp8 copy in the same pass as its bf16
  output (``QuantTarget``): RMSNorm forward -> x of q|k|v and gate|up, SwiGLU forward -> x of down,
  SwiGLU backward -> dy of gate|up, RMSNorm backward -> dy of o and down.  (The attention
  epilogues stay plain: their fused variants cost occupancy -- measured -2.6 % end to end.)  The backward side
  reaches the consuming ``Fp8LinearFn.backward`` through ``Fp8Recipe.stash`` (keyed by slot, checked
  against the gradient tensor's storage).  Bitwise the separate cast over the bf16 tensor.  With the
  fused-epilogue MLP the SwiGLU outputs come from the GEMM epilogue and act / d(gate|up) get one cast each.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _ext
from .gemm import (gemm_pp_dswiglu_f8, gemm_pp_dswiglu_f8q, gemm_pp_f8, gemm_pp_rope_f8,
                   gemm_pp_swiglu_f8, gemm_pp_swiglu_f8q, pp_f8_supported, wgrad, wgrad_f8, wgrad_f8_supported,
                   wgrad_supported)

E4M3, E5M2 = 0, 1
FMAX = {E4M3: 448.0, E5M2: 57344.0}
TORCH_DT = {E4M3: torch.float8_e4m3fn, E5M2: torch.float8_e5m2}


AMAX_PARTS = 64
_FUSED = {"enabled": True}
# "pp" (default): the ping-pong kernel on fp8 operands (csrc/gemm_pp.hip F8, 16x16x128 f8f6f4 MFMA), which
# also carries the fused RoPE / SwiGLU epilogues; "hipblaslt": torch._scaled_mm (A/B).  (The round-2
# one-wave-per-SIMD fp8 kernel, 0.95x hipBLASLt, was removed in round 5.)  Shapes the own kernels do not take fall back to
# torch._scaled_mm.
_GEMM = {"backend": "pp"}
# fp8 projections with their fused epilogues on the own fp8 GEMM: q|k|v + RoPE, gate|up + SwiGLU and the
# down input gradient + SwiGLU backward (backend "pp" only)
_EPI = {"enabled": True}


def set_fp8_gemm(backend: str) -> None:
    """fp8 forward / input-gradient GEMMs: "pp" (default: the own fp8 ping-pong kernel for every product),
    "auto" (hipBLASLt for the three long-K N <= 1024 plain products, where the own kernel runs 0.8x;
    +0.2 % per step, within noise: profiles/r4_fp8_pp.md) or "hipblaslt"."""
    if backend not in ("auto", "pp", "hipblaslt"):
        raise ValueError(backend)
    _GEMM["backend"] = backend


def set_fp8_fused_epilogues(enabled: bool) -> None:
    """RoPE / SwiGLU fused into the fp8 GEMMs (default on; needs the "pp" backend)."""
    _EPI["enabled"] = bool(enabled)


def fp8_fused_epilogues() -> bool:
    return _EPI["enabled"] and _GEMM["backend"] in ("auto", "pp")


def _own_plain(a8: torch.Tensor, b8: torch.Tensor) -> bool:
    """"auto": plain products the own fp8 kernel runs at >= 0.95x hipBLASLt (profiles/r4_fp8_pp.md: K = 1024
    0.95-1.07x; N = 1024 with K = 2688-5376 0.80-0.82x, where hipBLASLt's stream-K kernels win)."""
    return not (b8.shape[0] <= 1024 and a8.shape[1] > 1024)


def fp8_gemm_backend() -> str:
    return _GEMM["backend"]


def mm8(a8: torch.Tensor, b8: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """bf16 sa * sb * a8 . b8^T (a8 [M, K], b8 [N, K] fp8)."""
    be = _GEMM["backend"]
    if (be == "pp" or (be == "auto" and _own_plain(a8, b8))) and pp_f8_supported(a8, b8):
        return gemm_pp_f8(a8, b8, sa, sb)
    from .linear import library_gemm_fence  # hipBLASLt stream-K must not co-run with side-stream wgrads
    library_gemm_fence(a8.device if a8.is_cuda else None)
    return torch._scaled_mm(a8, b8.t(), sa, sb, out_dtype=torch.bfloat16)


# Projections that stay on the bf16 fused-epilogue GEMMs under --fp8 (ops/linear.py): "rope" keeps
# q|k|v + RoPE, "mlp" keeps gate|up + SwiGLU and the down dgrad + SwiGLU backward.  An fp8 GEMM
# followed by the separate RoPE / SwiGLU pass can cost more than the fused bf16 GEMM it replaces.
_KEEP = {"rope": False, "mlp": False}


def set_fp8_keep_fused(mode: str) -> None:
    """'none' (every decoder projection in fp8), 'rope', 'mlp' or 'both'."""
    if mode not in ("none", "rope", "mlp", "both"):
        raise ValueError(mode)
    _KEEP["rope"] = mode in ("rope", "both")
    _KEEP["mlp"] = mode in ("mlp", "both")


def fp8_keep_fused() -> dict:
    return dict(_KEEP)


# the lm head under --fp8: e4m3 logits GEMM, e5m2 dlogits for its input / weight gradients, all on the own
# fp8 kernels (ops/cross_entropy.py) -- no library GEMM left in the fp8 step; False: the bf16 lm head
_LM = {"enabled": True}


def set_fp8_lm_head(enabled: bool) -> None:
    _LM["enabled"] = bool(enabled)


def fp8_lm_head() -> bool:
    return _LM["enabled"]


def fp8_projection(kind: str) -> bool:
    """Whether projection ``kind`` (qkv / o / gu / down; lm = the lm head) runs in fp8 under --fp8."""
    if kind == "lm":
        return _LM["enabled"]
    if kind == "qkv":
        return not _KEEP["rope"]
    if kind in ("gu", "down"):
        return not _KEEP["mlp"]
    return True


def set_fused_quant(enabled: bool) -> None:
    """Fused producer-side quantisation (default on) vs a separate cast per GEMM operand (A/B)."""
    _FUSED["enabled"] = bool(enabled)


def cast(x: torch.Tensor, scale: torch.Tensor, fmt: int, amax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp8(x * scale) with saturation.  ``amax`` (fp32, zero-initialised; any length P) accumulates
    max|x| as P partial maxima (true amax = ``amax.max()``), which keeps the atomics uncontended."""
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=TORCH_DT[fmt], device=x.device)
    _ext.check(_ext.lib().nd_fp8_cast(_ext.ptr(x), _ext.dtcode(x), x.numel(), _ext.ptr(scale), _ext.ptr(out), fmt,
                                      _ext.ptr(amax), amax.numel() if amax is not None else 1,
                                      _ext.stream_ptr(x.device)), "nd_fp8_cast")
    return out


def absmax_into(x: torch.Tensor, amax: torch.Tensor) -> None:
    """amax (zeroed by the caller; P partial slots) <- max|x| in one read of x (no output written)."""
    x = x.contiguous()
    _ext.check(_ext.lib().nd_fp8_cast(_ext.ptr(x), _ext.dtcode(x), x.numel(), 0, 0, E4M3, _ext.ptr(amax), amax.numel(),
                                      _ext.stream_ptr(x.device)), "nd_fp8_cast(amax)")


def cast_t(x: torch.Tensor, scale: torch.Tensor, fmt: int, amax: Optional[torch.Tensor] = None,
           want_plain: bool = True):
    """(fp8(x * scale) or None, its transpose) in one pass; x is [rows, cols] with rows, cols % 64 == 0."""
    rows, cols = x.shape
    if x.stride(1) != 1:
        x = x.contiguous()
    out = torch.empty(rows, cols, dtype=TORCH_DT[fmt], device=x.device) if want_plain else None
    outT = torch.empty(cols, rows, dtype=TORCH_DT[fmt], device=x.device)
    _ext.check(_ext.lib().nd_fp8_cast_t(_ext.ptr(x), _ext.dtcode(x), rows, cols, x.stride(0), _ext.ptr(scale),
                                        _ext.ptr(out), _ext.ptr(outT), fmt, _ext.ptr(amax),
                                        amax.numel() if amax is not None else 1, _ext.stream_ptr(x.device)),
               "nd_fp8_cast_t")
    return out, outT


def _t_ok(x: torch.Tensor) -> bool:
    return x.dim() == 2 and x.shape[0] % 64 == 0 and x.shape[1] % 64 == 0


class QuantTarget:
    """Where a producer kernel writes the fused fp8 copy of its bf16 output: recipe slot k's scale
    and amax partials, fp8 format; ``out`` is set by the producer (forward), or the copy is stashed
    for slot k (backward)."""

    __slots__ = ("recipe", "k", "fmt", "out")

    def __init__(self, recipe: "Fp8Recipe", k: int, fmt: int):
        self.recipe, self.k, self.fmt, self.out = recipe, k, fmt, None

    def alloc(self, shape, device) -> torch.Tensor:
        return torch.empty(shape, dtype=TORCH_DT[self.fmt], device=device)

    def args(self, q: torch.Tensor):
        """(q ptr, scale ptr, amax ptr, parts, fmt) for the ``*_q`` launchers."""
        r = self.recipe
        return (_ext.ptr(q), r.scale[self.k:self.k + 1].data_ptr(), r.amax[self.k].data_ptr(), AMAX_PARTS, self.fmt)

    def stash(self, grad: torch.Tensor, q: torch.Tensor) -> None:
        self.recipe.stash[self.k] = (grad.data_ptr(), q)


class Fp8Recipe:
    """Amax history / scale bookkeeping for every quantised tensor role, in a few flat device tensors."""

    def __init__(self, device, history: int = 16, margin: int = 1, capacity: int = 1024):
        self.device = torch.device(device)
        self.H, self.margin, self.n, self.pos = history, margin, 0, 0
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        self.amax, self.hist = z(capacity, AMAX_PARTS), z(capacity, history)
        self.scale = torch.ones(capacity, dtype=torch.float32, device=self.device)
        self.inv = torch.ones(capacity, dtype=torch.float32, device=self.device)
        self.fmax = z(capacity)
        self.ready = [False] * capacity
        self.stash: Dict[int, tuple] = {}  # slot -> (grad storage ptr, fp8 copy) from a fused producer
        self._scr: Optional[torch.Tensor] = None  # first-use amax partials

    def new_slot(self, fmt: int) -> int:
        k = self.n
        self.n += 1
        self.fmax[k] = FMAX[fmt]
        return k

    def _first_use(self, x: torch.Tensor, k: int):
        if not self.ready[k]:  # first use: current scaling from this tensor's own amax
            # one amax-only read of x by the own cast kernel (no output), not torch's abs + reduce passes
            if self._scr is None:
                self._scr = torch.zeros(AMAX_PARTS, dtype=torch.float32, device=self.device)
            self._scr.zero_()
            absmax_into(x.detach(), self._scr)
            a = self._scr.amax().clamp_min(1e-30)
            s = self.fmax[k] / (a * 2.0 ** self.margin)
            self.scale[k:k + 1].copy_(s.reshape(1))
            self.inv[k:k + 1].copy_((1.0 / s).reshape(1))
            self.ready[k] = True

    def quantize(self, x: torch.Tensor, k: int, fmt: int) -> torch.Tensor:
        self._first_use(x, k)
        return cast(x, self.scale[k:k + 1], fmt, self.amax[k])

    def take_stashed(self, k: int, g: torch.Tensor) -> Optional[torch.Tensor]:
        st = self.stash.pop(k, None)
        if st is not None and st[0] == g.data_ptr() and st[1].shape == g.shape:
            return st[1]
        return None

    def target(self, k: int, fmt: int) -> Optional[QuantTarget]:
        """A fused-producer target for slot k, once its scale exists (the first use of a slot is
        scaled from the tensor's own amax, which only the separate cast can do)."""
        return QuantTarget(self, k, fmt) if (self.ready[k] and _FUSED["enabled"]) else None

    def quantize_t(self, x: torch.Tensor, k: int, fmt: int, want_plain: bool = True):
        """(x8, x8^T) with the slot's scale (falls back to a separate transpose off the fast shapes)."""
        self._first_use(x, k)
        if _t_ok(x):
            return cast_t(x, self.scale[k:k + 1], fmt, self.amax[k], want_plain)
        q = cast(x, self.scale[k:k + 1], fmt, self.amax[k])
        return q, q.t().contiguous()

    @torch.no_grad()
    def update(self):
        """Roll the amax history and refresh every scale (call once per inner step)."""
        n = self.n
        if n == 0:
            return
        self.hist[:n, self.pos] = self.amax[:n].amax(dim=1)
        self.pos = (self.pos + 1) % self.H
        m = self.hist[:n].amax(dim=1)
        s = torch.where(m > 0, self.fmax[:n] / (m * 2.0 ** self.margin), self.scale[:n])
        self.scale[:n] = s
        self.inv[:n] = 1.0 / s
        self.amax[:n] = 0.0


class Fp8Weight:
    """e4m3 copies of one weight (and its transpose) for the current optimizer version, with current
    scaling: one amax-only read of W, then ONE cast+transpose pass writing W8 and W8^T (was: torch
    abs + amax + two casts + a transposing copy, ~8 ms per optimizer step for Llama-150M)."""

    def __init__(self):
        self.version = -1
        self.w8 = self.wT8 = None
        self.inv = None
        self.amax = None

    def get(self, w: torch.Tensor, version: int):
        if version != self.version:
            with torch.no_grad():
                if self.amax is None:
                    self.amax = torch.zeros(AMAX_PARTS, dtype=torch.float32, device=w.device)
                self.amax.zero_()
                absmax_into(w, self.amax)
                s = (FMAX[E4M3] / self.amax.amax().clamp_min(1e-30)).reshape(1)
                if _t_ok(w):
                    self.w8, self.wT8 = cast_t(w, s, E4M3)
                else:
                    self.w8 = cast(w, s, E4M3)
                    self.wT8 = cast(w.t().contiguous(), s, E4M3)
                self.inv = (1.0 / s).contiguous()
            self.version = version
        return self


class Fp8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gw, wq: Fp8Weight, recipe: Fp8Recipe, kx: int, kdy: int, wgrad_fp8: bool, x8=None):
        if x8 is None or x8.shape != x.shape:
            x8 = recipe.quantize(x, kx, E4M3)
        # fp8 weight gradient: keep x8 (half the bytes of x) for dW = dy8^T x8
        ctx.save_for_backward(x8 if wgrad_fp8 else x)
        inv_x = recipe.inv[kx:kx + 1]
        y = mm8(x8, wq.w8, inv_x, wq.inv)
        ctx.gw, ctx.wq, ctx.recipe, ctx.kdy, ctx.inv_x, ctx.wgrad_fp8 = gw, wq, recipe, kdy, inv_x, wgrad_fp8
        return y

    @staticmethod
    def backward(ctx, dy):
        (xs,) = ctx.saved_tensors
        dy = dy.contiguous()
        r, k = ctx.recipe, ctx.kdy
        dy8 = _dy8(r, k, dy)
        inv_dy = r.inv[k:k + 1]
        dx = mm8(dy8, ctx.wq.wT8, inv_dy, ctx.wq.inv)
        if ctx.wgrad_fp8:
            _wgrad_f8(ctx.gw, dy8, xs, inv_dy, ctx.inv_x, dy)
        else:
            _wgrad_bf16(ctx.gw, dy, xs)
        return dx, None, None, None, None, None, None, None, None


def _wgrad_bf16(gw, dy, x):
    if gw is None:
        return
    from .linear import _wgrad  # side stream when the weight-gradient overlap is on
    _wgrad(gw, dy, x)


def _wgrad_f8(gw, dy8, x8, inv_dy, inv_x, dy=None):
    """gw += dy^T x from the fp8 operands (own kernel, csrc/gemm_wgrad.hip wgrad8_pp_kernel); shapes it does
    not take fall back to the bf16 kernel on the dequantised operands (``dy``: the bf16 gradient if kept).
    With the weight-gradient overlap on (ops/linear.py ``set_wgrad_overlap``) it runs on the side stream like
    the bf16 weight gradients: joined before every library GEMM and before the optimizer."""
    if gw is None:
        return
    if wgrad_f8_supported(gw, dy8, x8):
        from .linear import _OVERLAP, _side_stream
        if _OVERLAP["enabled"] and gw.is_cuda:
            cur = torch.cuda.current_stream(gw.device)
            side = _side_stream(gw.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                wgrad_f8(gw, dy8, x8, inv_dy, inv_x)
            _OVERLAP["keep"].append((dy8, x8))
            _OVERLAP["pending"].add(side.device.index)
        else:
            wgrad_f8(gw, dy8, x8, inv_dy, inv_x)
    else:
        if dy is None:
            dy = (dy8.float() * inv_dy).to(torch.bfloat16)
        _wgrad_bf16(gw, dy, (x8.float() * inv_x).to(dy.dtype))


def _dy8(r: Fp8Recipe, k: int, dy: torch.Tensor) -> torch.Tensor:
    dy8 = r.take_stashed(k, dy)  # written by a fused producer (RMSNorm backward)
    return dy8 if dy8 is not None else r.quantize(dy, k, E5M2)


class Fp8RopeFn(torch.autograd.Function):
    """fp8 q|k|v projection with RoPE in the epilogue of the own fp8 GEMM (bf16 output, rotated q|k).
    The attention backward returns the gradient of the UN-rotated projection, so the backward is the
    plain fp8 projection backward (e5m2 dy x e4m3 W^T) plus the bf16 weight gradient."""

    @staticmethod
    def forward(ctx, x, w, gw, wq: "Fp8Weight", recipe: Fp8Recipe, kx: int, kdy: int, x8, cos, sin, T: int, hd: int,
                rope_cols: int, wgrad_fp8: bool):
        if x8 is None or x8.shape != x.shape:
            x8 = recipe.quantize(x, kx, E4M3)
        inv_x = recipe.inv[kx:kx + 1]
        y = gemm_pp_rope_f8(x8, wq.w8, inv_x, wq.inv, cos, sin, T, hd, rope_cols)
        ctx.save_for_backward(x8 if wgrad_fp8 else x)
        ctx.gw, ctx.wq, ctx.recipe, ctx.kdy, ctx.inv_x, ctx.wgrad_fp8 = gw, wq, recipe, kdy, inv_x, wgrad_fp8
        return y

    @staticmethod
    def backward(ctx, dy):
        (xs,) = ctx.saved_tensors
        dy = dy.contiguous()
        r, k = ctx.recipe, ctx.kdy
        dy8 = _dy8(r, k, dy)
        dx = mm8(dy8, ctx.wq.wT8, r.inv[k:k + 1], ctx.wq.inv)
        if ctx.wgrad_fp8:
            _wgrad_f8(ctx.gw, dy8, xs, r.inv[k:k + 1], ctx.inv_x, dy)
        else:
            _wgrad_bf16(ctx.gw, dy, xs)
        return (dx,) + (None,) * 13


class Fp8MLPFn(torch.autograd.Function):
    """The SwiGLU MLP with every projection in fp8 and both activation passes fused into the own fp8 GEMMs:

      forward   gu, act = [e4m3 gate|up GEMM + SwiGLU epilogue](y8)
                m       = act8 . W_down8^T            (act8: one cast of act, slot down.x)
      backward  dgu     = [e5m2 down dgrad GEMM + SwiGLU-backward epilogue](dm8, W_down8^T copy, gu)
                dy      = dgu8 . W_gu8               (dgu8: one cast of dgu, slot gu.dy)
                gW_down += dm^T act, gW_gu += dgu^T y (bf16 weight-gradient kernel)"""

    @staticmethod
    def forward(ctx, y, w_gu, w_dn, gw_gu, gw_dn, wq_gu: "Fp8Weight", wq_dn: "Fp8Weight", recipe: Fp8Recipe,
                ks, y8, wgrad_fp8: bool):
        k_gx, k_gdy, k_dx, k_ddy = ks
        if y8 is None or y8.shape != y.shape:
            y8 = recipe.quantize(y, k_gx, E4M3)
        # with fp8 weight gradients nothing needs the bf16 act: once the slot has a scale, the epilogue writes
        # act8 directly (bitwise the cast of the bf16 act) and no bf16 act exists
        q = wgrad_fp8 and recipe.ready[k_dx] and _FUSED["enabled"] and y.shape[0] % 128 == 0
        if q:
            gu, act8 = gemm_pp_swiglu_f8q(y8, wq_gu.w8, recipe.inv[k_gx:k_gx + 1], wq_gu.inv,
                                          recipe.scale[k_dx:k_dx + 1], recipe.amax[k_dx])
            act = None
        else:
            gu, act = gemm_pp_swiglu_f8(y8, wq_gu.w8, recipe.inv[k_gx:k_gx + 1], wq_gu.inv)
            act8 = recipe.quantize(act, k_dx, E4M3)
        m = mm8(act8, wq_dn.w8, recipe.inv[k_dx:k_dx + 1], wq_dn.inv)
        # fp8 weight gradients keep the fp8 operands (y8, act8) instead of the bf16 ones
        ctx.save_for_backward(y8 if wgrad_fp8 else y, gu, act8 if wgrad_fp8 else act)
        ctx.gw, ctx.wq, ctx.recipe, ctx.ks, ctx.wgrad_fp8 = (gw_gu, gw_dn), (wq_gu, wq_dn), recipe, ks, wgrad_fp8
        return m

    @staticmethod
    def backward(ctx, dm):
        ys, gu, acts = ctx.saved_tensors
        gw_gu, gw_dn = ctx.gw
        wq_gu, wq_dn = ctx.wq
        r = ctx.recipe
        k_gx, k_gdy, k_dx, k_ddy = ctx.ks
        dm = dm.contiguous()
        dm8 = _dy8(r, k_ddy, dm)
        if ctx.wgrad_fp8 and r.ready[k_gdy] and _FUSED["enabled"] and dm.shape[0] % 128 == 0:
            # only the e5m2 d(gate|up) is consumed (dgrad and fp8 wgrad): the epilogue writes it directly
            dgu8 = gemm_pp_dswiglu_f8q(dm8, wq_dn.wT8, r.inv[k_ddy:k_ddy + 1], wq_dn.inv, gu,
                                       r.scale[k_gdy:k_gdy + 1], r.amax[k_gdy])
            dgu = None
        else:
            dgu = gemm_pp_dswiglu_f8(dm8, wq_dn.wT8, r.inv[k_ddy:k_ddy + 1], wq_dn.inv, gu)
            dgu8 = r.quantize(dgu, k_gdy, E5M2)
        if ctx.wgrad_fp8:
            _wgrad_f8(gw_dn, dm8, acts, r.inv[k_ddy:k_ddy + 1], r.inv[k_dx:k_dx + 1], dm)
        else:
            _wgrad_bf16(gw_dn, dm, acts)
        dy = mm8(dgu8, wq_gu.wT8, r.inv[k_gdy:k_gdy + 1], wq_gu.inv)
        if ctx.wgrad_fp8:
            _wgrad_f8(gw_gu, dgu8, ys, r.inv[k_gdy:k_gdy + 1], r.inv[k_gx:k_gx + 1], dgu)
        else:
            _wgrad_bf16(gw_gu, dgu, ys)
        return (dy,) + (None,) * 10


class Fp8Linears:
    """Per-model fp8 state: one recipe, one (x, dy) slot pair and one weight cache per projection."""

    def __init__(self, device, wgrad_fp8: bool = False):
        self.recipe = Fp8Recipe(device)
        self.wgrad_fp8 = wgrad_fp8
        self.slots: Dict[str, tuple] = {}
        self.weights: Dict[str, Fp8Weight] = {}

    def _slots(self, key: str):
        if key not in self.slots:
            self.slots[key] = (self.recipe.new_slot(E4M3), self.recipe.new_slot(E5M2))
            self.weights[key] = Fp8Weight()
        return self.slots[key]

    def x_target(self, key: str) -> Optional[QuantTarget]:
        """Fused-producer target for the projection ``key``'s input (e4m3)."""
        return self.recipe.target(self._slots(key)[0], E4M3)

    def dy_target(self, key: str) -> Optional[QuantTarget]:
        """Fused-producer target for the gradient of projection ``key``'s output (e5m2)."""
        return self.recipe.target(self._slots(key)[1], E5M2)

    def rope_ok(self, x: torch.Tensor, w: torch.Tensor, hd: int, rope_cols: int) -> bool:
        """Can the q|k|v projection run as fp8 GEMM + fused RoPE (own kernel)."""
        return (fp8_fused_epilogues() and x.is_cuda and x.dim() == 2 and x.stride(1) == 1
                and x.shape[1] % 128 == 0 and w.shape[0] % 8 == 0 and hd in (32, 64) and rope_cols % 64 == 0)

    def rope(self, key: str, x, w, gw, version: int, x8, cos, sin, T: int, hd: int, rope_cols: int):
        kx, kdy = self._slots(key)
        wq = self.weights[key].get(w, version)
        return Fp8RopeFn.apply(x, w, gw, wq, self.recipe, kx, kdy, x8, cos, sin, int(T), int(hd), int(rope_cols),
                               self.wgrad_fp8)

    def mlp_ok(self, y: torch.Tensor, w_gu: torch.Tensor, w_dn: torch.Tensor) -> bool:
        """Can the MLP run as fp8 GEMMs with the fused SwiGLU forward / backward epilogues."""
        F = w_gu.shape[0] // 2
        return (fp8_fused_epilogues() and y.is_cuda and y.dim() == 2 and y.stride(1) == 1
                and y.shape[1] % 128 == 0 and F % 128 == 0 and w_dn.shape[1] == F and w_dn.shape[0] % 128 == 0)

    def mlp(self, kgu: str, kdn: str, y, w_gu, w_dn, gw_gu, gw_dn, version: int, y8=None):
        k_gx, k_gdy = self._slots(kgu)
        k_dx, k_ddy = self._slots(kdn)
        wq_gu = self.weights[kgu].get(w_gu, version)
        wq_dn = self.weights[kdn].get(w_dn, version)
        return Fp8MLPFn.apply(y, w_gu, w_dn, gw_gu, gw_dn, wq_gu, wq_dn, self.recipe, (k_gx, k_gdy, k_dx, k_ddy), y8,
                              self.wgrad_fp8)

    def __call__(self, key: str, x: torch.Tensor, w: torch.Tensor, gw: Optional[torch.Tensor], version: int,
                 x8: Optional[torch.Tensor] = None):
        kx, kdy = self._slots(key)
        wq = self.weights[key].get(w, version)
        return Fp8LinearFn.apply(x, w, gw, wq, self.recipe, kx, kdy, self.wgrad_fp8, x8)
