"""fp8 inner step (BASELINE config 5): OCP fp8 GEMMs for the decoder projections on gfx950.

Recipe (per-tensor scaling, the common "delayed scaling" scheme):
* forward  ``y = x @ W^T`` with x, W in e4m3 -> hipBLASLt fp8 GEMM (``torch._scaled_mm``), bf16 out;
* dgrad    ``dx = dy @ W`` with dy in e5m2 (range for gradients), W^T in e4m3;
* wgrad    stays bf16 on our ``nd_wgrad`` kernel (fp32 accumulate into the flat grad buffer), so the
  master-weight update sees full-precision gradients;
* activations / gradients are quantised by ``nd_fp8_cast`` (one pass: scale, saturate, convert,
  and record amax) with a scale derived from the amax history of previous steps (``Fp8Recipe``;
  device-side, no host sync); the very first use of a tensor role is scaled from its current amax;
* weights are re-quantised once per optimizer update (current amax), together with their transpose;
* lm_head, attention, norms stay bf16/fp32; fp32 master weights and optimizer state are unchanged.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import _ext
from .gemm import wgrad, wgrad_supported

E4M3, E5M2 = 0, 1
FMAX = {E4M3: 448.0, E5M2: 57344.0}
TORCH_DT = {E4M3: torch.float8_e4m3fn, E5M2: torch.float8_e5m2}


AMAX_PARTS = 64


def cast(x: torch.Tensor, scale: torch.Tensor, fmt: int, amax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp8(x * scale) with saturation.  ``amax`` (fp32, zero-initialised; any length P) accumulates
    max|x| as P partial maxima (true amax = ``amax.max()``), which keeps the atomics uncontended."""
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=TORCH_DT[fmt], device=x.device)
    _ext.check(_ext.lib().nd_fp8_cast(_ext.ptr(x), _ext.dtcode(x), x.numel(), _ext.ptr(scale), _ext.ptr(out), fmt,
                                      _ext.ptr(amax), amax.numel() if amax is not None else 1,
                                      _ext.stream_ptr(x.device)), "nd_fp8_cast")
    return out


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

    def new_slot(self, fmt: int) -> int:
        k = self.n
        self.n += 1
        self.fmax[k] = FMAX[fmt]
        return k

    def quantize(self, x: torch.Tensor, k: int, fmt: int) -> torch.Tensor:
        if not self.ready[k]:  # first use: current scaling from this tensor's own amax
            a = x.detach().abs().amax().float().clamp_min(1e-30)
            s = self.fmax[k] / (a * 2.0 ** self.margin)
            self.scale[k:k + 1].copy_(s.reshape(1))
            self.inv[k:k + 1].copy_((1.0 / s).reshape(1))
            self.ready[k] = True
        return cast(x, self.scale[k:k + 1], fmt, self.amax[k])

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
    """e4m3 copies of one weight (and its transpose) for the current optimizer version."""

    def __init__(self):
        self.version = -1
        self.w8 = self.wT8 = None
        self.inv = None

    def get(self, w: torch.Tensor, version: int):
        if version != self.version:
            with torch.no_grad():
                a = w.abs().amax().float().clamp_min(1e-30)
                s = (FMAX[E4M3] / a).reshape(1)
                self.w8 = cast(w, s, E4M3)
                self.wT8 = cast(w.t().contiguous(), s, E4M3)
                self.inv = (1.0 / s).contiguous()
            self.version = version
        return self


class Fp8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gw, wq: Fp8Weight, recipe: Fp8Recipe, kx: int, kdy: int):
        x8 = recipe.quantize(x, kx, E4M3)
        y = torch._scaled_mm(x8, wq.w8.t(), recipe.inv[kx:kx + 1], wq.inv, out_dtype=torch.bfloat16)
        ctx.save_for_backward(x)
        ctx.gw, ctx.wq, ctx.recipe, ctx.kdy = gw, wq, recipe, kdy
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        r, k = ctx.recipe, ctx.kdy
        dy8 = r.quantize(dy, k, E5M2)
        dx = torch._scaled_mm(dy8, ctx.wq.wT8.t(), r.inv[k:k + 1], ctx.wq.inv, out_dtype=torch.bfloat16)
        if ctx.gw is not None:
            if wgrad_supported(ctx.gw, dy, x):
                wgrad(ctx.gw, dy, x)
            else:
                ctx.gw.add_(torch.mm(dy.t(), x).float())
        return dx, None, None, None, None, None, None


class Fp8Linears:
    """Per-model fp8 state: one recipe, one (x, dy) slot pair and one weight cache per projection."""

    def __init__(self, device):
        self.recipe = Fp8Recipe(device)
        self.slots: Dict[str, tuple] = {}
        self.weights: Dict[str, Fp8Weight] = {}

    def __call__(self, key: str, x: torch.Tensor, w: torch.Tensor, gw: Optional[torch.Tensor], version: int):
        if key not in self.slots:
            self.slots[key] = (self.recipe.new_slot(E4M3), self.recipe.new_slot(E5M2))
            self.weights[key] = Fp8Weight()
        kx, kdy = self.slots[key]
        wq = self.weights[key].get(w, version)
        return Fp8LinearFn.apply(x, w, gw, wq, self.recipe, kx, kdy)
