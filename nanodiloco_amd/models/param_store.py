"""Flat parameter / gradient storage.

The reference keeps one ``nn.Parameter`` per tensor and loops over 57-201 of them in every
optimizer, clip, pseudo-gradient and collective call (REF/nanodiloco/diloco/diloco.py:21-22,46-50;
SURVEY.md §7.1).  Here every per-worker state vector is ONE contiguous allocation and each
parameter is a view into it:

* ``master``  fp32 master weights (what AdamW / the outer step update)
* ``grad``    fp32 gradient accumulator (written directly by our backward kernels / GEMM epilogues)
* ``shadow``  compute-dtype copy (bf16) the forward reads; refreshed by the fused optimizer kernels.
              For fp32 compute it aliases ``master``.

Each view starts on a 64-element (256 B for fp32) boundary so vectorised kernels can run over the
whole flat buffer (padding stays zero: zero grad -> zero update, and weight-decay of 0 is 0).
Parameters of one decoder layer are contiguous and in HF state_dict order, so ``q|k|v`` and
``gate|up`` form single fused ``[3d, d]`` / ``[2F, d]`` GEMM weights without any copy.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

ALIGN = 64


def _numel(shape: Sequence[int]) -> int:
    n = 1
    for s in shape:
        n *= int(s)
    return n


class ParamStore:
    def __init__(self, specs: Iterable[Tuple[str, Tuple[int, ...]]], device="cpu",
                 compute_dtype: torch.dtype = torch.float32, align: int = ALIGN,
                 fuse_groups: Optional[List[List[str]]] = None):
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.names: List[str] = []
        self.shapes: Dict[str, Tuple[int, ...]] = {}
        self.offsets: Dict[str, int] = {}
        off = 0
        fused_members = set()
        for g in fuse_groups or []:
            fused_members.update(g[1:])  # members after the first are packed without padding
        for name, shape in specs:
            shape = tuple(int(s) for s in shape)
            if name not in fused_members:
                off = (off + align - 1) // align * align
            self.names.append(name)
            self.shapes[name] = shape
            self.offsets[name] = off
            off += _numel(shape)
        # pad so the flat vector splits into 1..8 equal, 64-aligned shards (lcm(1..8) = 840):
        # the two-level outer step shards it over the GPUs of one DiLoCo worker.
        q = align * 840
        self.numel = (off + q - 1) // q * q
        self.num_params = sum(_numel(s) for s in self.shapes.values())
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        if compute_dtype == torch.float32:
            self.shadow = self.master
        else:
            self.shadow = torch.zeros(self.numel, dtype=compute_dtype, device=self.device)
        self._views: Dict[Tuple[str, str], torch.Tensor] = {}
        self.version = 0  # bumped whenever the weights change (optimizer / outer step / load)

    # ------------------------------------------------------------------ views
    def range(self, name: str) -> Tuple[int, int]:
        o = self.offsets[name]
        return o, o + _numel(self.shapes[name])

    def _view(self, buf: torch.Tensor, name: str, shape=None) -> torch.Tensor:
        a, b = self.range(name)
        return buf[a:b].view(shape or self.shapes[name])

    def view(self, which: str, name: str) -> torch.Tensor:
        key = (which, name)
        v = self._views.get(key)
        if v is None:
            v = self._view(getattr(self, which), name)
            self._views[key] = v
        return v

    def master_view(self, name):
        return self.view("master", name)

    def grad_view(self, name):
        return self.view("grad", name)

    def shadow_view(self, name):
        return self.view("shadow", name)

    def fused_view(self, which: str, names: Sequence[str]) -> torch.Tensor:
        """Single [sum(rows), cols] view over consecutive, unpadded 2-D params (e.g. q|k|v)."""
        key = (which, "|".join(names))
        v = self._views.get(key)
        if v is not None:
            return v
        cols = self.shapes[names[0]][1]
        start = self.offsets[names[0]]
        rows = 0
        for n in names:
            if self.shapes[n][1] != cols or self.offsets[n] != start + rows * cols:
                raise ValueError(f"params {names} are not contiguous; cannot fuse")
            rows += self.shapes[n][0]
        buf = getattr(self, which)
        v = buf[start:start + rows * cols].view(rows, cols)
        self._views[key] = v
        return v

    def span(self, prefix: str) -> Tuple[int, int]:
        """Smallest [start, end) covering every param whose name starts with ``prefix``."""
        rs = [self.range(n) for n in self.names if n.startswith(prefix)]
        return min(r[0] for r in rs), max(r[1] for r in rs)

    # ------------------------------------------------------------------ state
    def sync_shadow(self):
        if self.shadow is not self.master:
            self.shadow.copy_(self.master)

    def zero_grad(self):
        self.grad.zero_()

    def state_dict(self, which: str = "master") -> Dict[str, torch.Tensor]:
        return {n: self.view(which, n) for n in self.names}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        missing = [n for n in self.names if n not in sd]
        unexpected = [k for k in sd if k not in self.shapes]
        if strict and (missing or unexpected):
            raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for n in self.names:
                if n in sd:
                    t = sd[n]
                    if tuple(t.shape) != self.shapes[n]:
                        raise ValueError(f"shape mismatch for {n}: {tuple(t.shape)} vs {self.shapes[n]}")
                    self.master_view(n).copy_(t.to(torch.float32))
        self.sync_shadow()
        self.version += 1

    def new_flat(self, dtype=torch.float32, device=None, pin: bool = False) -> torch.Tensor:
        dev = torch.device(device) if device is not None else self.device
        t = torch.zeros(self.numel, dtype=dtype, device=dev)
        if pin and dev.type == "cpu" and torch.cuda.is_available():
            t = t.pin_memory()
        return t

    def nbytes(self, dtype=torch.float32) -> int:
        return self.numel * torch.tensor([], dtype=dtype).element_size()
