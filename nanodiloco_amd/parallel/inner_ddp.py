"""Per-step gradient all-reduce inside one DiLoCo worker (two-level topology, BASELINE config 3).

The reference has no intra-worker data parallelism.  Here a worker may span K
GPUs: their gradients are summed every inner step (the 1/K is folded into the loss scale) with
layer-sized buckets launched from the backward itself -- as soon as layer i's gradients are final
(``LlamaForCausalLM.layer_hook``) its contiguous span of the flat fp32 grad buffer goes to RCCL,
overlapping the backward of layers i-1..0.  The embedding / final-norm / lm_head spans follow when
backward ends.  ``finish()`` makes the compute stream (not the host) wait before the optimizer.
"""
from __future__ import annotations

from typing import List, Tuple

from ..models.llama import LlamaForCausalLM
from .comm import FlatCommunicator


class InnerGradSync:
    def __init__(self, model: LlamaForCausalLM, comm: FlatCommunicator, overlap: bool = True):
        self.model = model
        self.comm = comm
        self.overlap = overlap
        st = model.store
        L = model.config.num_hidden_layers
        self.layer_spans: List[Tuple[int, int]] = [st.span(f"model.layers.{i}.") for i in range(L)]
        lo, hi = self.layer_spans[0][0], self.layer_spans[-1][1]
        self.rest_spans = [(0, lo), (hi, st.numel)]
        self._pending = []
        self._armed = False

    @property
    def enabled(self) -> bool:
        return self.comm.enabled

    def arm(self):
        """Call before the backward of the LAST micro-batch of an inner step."""
        if not self.enabled:
            return
        self._armed = True
        self._pending = []
        if self.overlap:
            self.model.layer_hook = self._on_layer

    def _on_layer(self, i: int):
        a, b = self.layer_spans[i]
        self._pending.append(self.comm.all_reduce_async(self.model.store.grad, [(a, b)]))

    def finish(self):
        if not self.enabled or not self._armed:
            return
        self.model.layer_hook = None
        grad = self.model.store.grad
        if self.overlap:
            spans = [s for s in self.rest_spans if s[1] > s[0]]
        else:
            spans = [(0, grad.numel())]
        self._pending.append(self.comm.all_reduce_async(grad, spans))
        for p in self._pending:
            p.wait_all()
        self._pending = []
        self._armed = False
