"""HIP-graph capture of the micro-batch forward+backward (``--hip-graph``).

Small models (the reference's default 6-layer / 128-wide Llama) are launch-bound: a micro-batch
is a few hundred short kernels, and the host-side cost of PyTorch dispatch + ctypes launches
exceeds the GPU time.  Everything the model does on the GPU is capture-safe -- static shapes, no
host syncs (the loss scale, token counts and clip coefficients live in device memory), every
kernel launched on the current stream, gradients accumulated in place into the flat grad buffer
-- so after two eager warm-up calls (side stream, as torch.cuda.graphs requires) the forward +
backward is captured once into a HIP graph and each later micro-batch is one ``graph.replay()``
after copying the new token ids into the graph's static input buffers.

Not captured: the optimizer step (its learning rate / bias corrections are host scalars that change
every step), the outer DiLoCo step and its collectives, and the inner-DDP gradient hooks (the
trainer disables graphs with ``--inner-dp > 1``).  fp8 is excluded because its weight casts are
refreshed on a host-side version check.
"""
from __future__ import annotations

from typing import Optional

import torch


class GraphedMicroStep:
    def __init__(self, model, warmup: int = 2):
        if getattr(model, "fp8", None) is not None:
            raise ValueError("HIP-graph capture is not supported with --fp8")
        self.model = model
        self.warmup = warmup
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.ids = self.labels = self.loss = None
        self.loss_scale = None
        self.eager_fallbacks = 0

    def _run(self, ids, labels, loss_scale):
        out = self.model(ids, labels=labels, loss_scale=loss_scale)
        out.loss.backward()
        return out.loss.detach()

    def __call__(self, ids: torch.Tensor, labels: torch.Tensor, loss_scale: float = 1.0) -> torch.Tensor:
        if self.graph is None and self.calls < self.warmup:
            self.calls += 1
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                loss = self._run(ids, labels, loss_scale)
            torch.cuda.current_stream().wait_stream(side)
            return loss
        if self.graph is not None and (ids.shape != self.ids.shape or labels.shape != self.labels.shape):
            self.eager_fallbacks += 1  # e.g. a ragged last batch of a real dataset: run it eagerly
            return self._run(ids, labels, loss_scale)
        if self.graph is None:
            self.ids, self.labels, self.loss_scale = ids.clone(), labels.clone(), loss_scale
            self.model.refresh_transposed()  # nothing stale gets captured as a copy
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):  # records only; the replay below does the work
                self.loss = self._run(self.ids, self.labels, loss_scale)
        if loss_scale != self.loss_scale:
            raise ValueError("loss_scale changed after capture")
        self.model.refresh_transposed()  # W^T copies the captured dgrad GEMMs read
        self.ids.copy_(ids, non_blocking=True)
        self.labels.copy_(labels, non_blocking=True)
        self.graph.replay()
        return self.loss
