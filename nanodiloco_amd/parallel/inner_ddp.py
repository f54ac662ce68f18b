"""Per-step gradient all-reduce inside one DiLoCo worker (two-level topology, BASELINE config 3).

The reference has no intra-worker data parallelism.  Here a worker may span K
GPUs: their gradients are summed every inner step (the 1/K is folded into the loss scale) with
layer-sized buckets launched from the backward itself -- as soon as layer i's gradients are final
(``LlamaForCausalLM.layer_hook``: fired after the backward of the norm that feeds layer i, which is
the last writer of layer i's span; any side-stream weight-gradient GEMMs are joined first) its
contiguous span of the flat fp32 grad buffer goes to RCCL, overlapping the backward of layers
i-1..0.  The embedding / final-norm / lm_head spans follow when
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
        self._hooked = set()
        self.last_hook_count = 0

    @property
    def enabled(self) -> bool:
        return self.comm.enabled

    def arm(self):
        """Call before the backward of the LAST micro-batch of an inner step."""
        if not self.enabled:
            return
        self._armed = True
        self._pending = []
        self._hooked = set()
        if self.overlap:
            self.model.layer_hook = self._on_layer

    def _on_layer(self, i: int):
        if i in self._hooked:
            raise RuntimeError(f"inner-DDP hook for layer {i} fired twice in one backward")
        self._hooked.add(i)
        a, b = self.layer_spans[i]
        self._pending.append(self.comm.all_reduce_async(self.model.store.grad, [(a, b)]))

    def finish(self):
        if not self.enabled or not self._armed:
            return
        self.model.layer_hook = None
        grad = self.model.store.grad
        if self.overlap:
            # any layer whose hook did not fire (e.g. a backward that never reached it) is reduced here
            missed = [self.layer_spans[i] for i in range(len(self.layer_spans)) if i not in self._hooked]
            spans = [s for s in self.rest_spans + missed if s[1] > s[0]]
        else:
            spans = [(0, grad.numel())]
        self._pending.append(self.comm.all_reduce_async(grad, spans))
        for p in self._pending:
            p.wait_all()
        self.comm.check("the inner-DDP gradient is used")
        self.last_hook_count = len(self._hooked)
        self._pending = []
        self._armed = False
