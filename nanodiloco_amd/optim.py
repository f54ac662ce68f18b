"""Flat-buffer optimizers.

``FlatAdamW``        == ``torch.optim.AdamW(params, lr)`` (betas 0.9/0.999, eps 1e-8, wd 0.01 on every
                        tensor, like REF/nanodiloco/main.py:100) preceded by
                        ``clip_grad_norm_(max_norm=1.0)`` (REF/nanodiloco/diloco/diloco.py:57).
``FlatOuterNesterov`` == ``torch.optim.SGD(lr=0.7, momentum=0.9, nesterov=True)`` applied to the
                        averaged pseudo-gradient (REF/nanodiloco/main.py:101).

State is one flat fp32 vector per moment; the step is two (inner) / one-per-bucket (outer) HIP
kernels on GPU (ops/optim.py).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import ops
from .models.param_store import ParamStore


class FlatAdamW:
    def __init__(self, store: ParamStore, lr: float = 4e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01, max_grad_norm: Optional[float] = 1.0, skip_nonfinite: bool = False):
        self.store = store
        self.lr = lr
        self.betas = tuple(betas)
        self.eps = eps
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.exp_avg = store.new_flat()
        self.exp_avg_sq = store.new_flat()
        self.step_count = 0
        self.last_grad_norm = torch.zeros(1, dtype=torch.float32, device=store.device)
        self.skip_nonfinite = skip_nonfinite
        self.skipped_steps = torch.zeros(1, dtype=torch.int32, device=store.device)
        # torch-style param_groups so code reading `param_groups[0]["lr"]` keeps working
        self.param_groups = [{"lr": lr, "params": store.names}]

    def step(self, lr: Optional[float] = None):
        lr = self.lr if lr is None else lr
        self.param_groups[0]["lr"] = lr
        self.step_count += 1
        ops.join_wgrad()
        ops.adamw_step(self.store.master, self.store.grad, self.exp_avg, self.exp_avg_sq, self.store.shadow,
                       self.step_count, lr, self.betas, self.eps, self.weight_decay, self.max_grad_norm,
                       norm_out=self.last_grad_norm, skip_nonfinite=self.skip_nonfinite,
                       skipped=self.skipped_steps)
        self.store.version += 1

    def zero_grad(self, set_to_none: bool = False):
        ops.join_wgrad()
        self.store.zero_grad()

    def state_dict(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq, "step": self.step_count,
                "lr": self.lr, "betas": list(self.betas), "eps": self.eps, "weight_decay": self.weight_decay}

    def load_state_dict(self, d):
        self.exp_avg.copy_(d["exp_avg"])
        self.exp_avg_sq.copy_(d["exp_avg_sq"])
        self.step_count = int(d["step"])


class FlatOuterNesterov:
    def __init__(self, store: ParamStore, lr: float = 0.7, momentum: float = 0.9):
        self.store = store
        self.lr = lr
        self.momentum = momentum
        self.momentum_buffer = store.new_flat()
        self.step_count = 0
        self.param_groups = [{"lr": lr, "momentum": momentum, "nesterov": True, "params": store.names}]

    def state_dict(self):
        return {"momentum_buffer": self.momentum_buffer, "step": self.step_count, "lr": self.lr,
                "momentum": self.momentum}

    def load_state_dict(self, d):
        self.momentum_buffer.copy_(d["momentum_buffer"])
        self.step_count = int(d["step"])
