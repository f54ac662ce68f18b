"""Tracing / profiling hooks (the reference has none: SURVEY.md §5.1).

* :class:`PhaseTimer`  -- HIP-event timing of named phases (fwd+bwd, inner optimizer, outer step);
  events are only synchronised when a report is requested, so the training loop stays async.
* :func:`range`        -- roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm builds); shows up
  in ``rocprofv3 --marker-trace`` and in torch.profiler traces.  No-op on CPU.
* :func:`torch_profile` -- context manager around ``torch.profiler`` writing a Chrome trace.
Kernel-level counters come from ``rocprofv3 --kernel-trace --stats`` / ``--pmc`` (see docs/PROFILING.md).
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, List, Tuple

import torch


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:
            pass
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


class PhaseTimer:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending: List[Tuple[str, object, object]] = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            t0 = time.perf_counter()
            yield
            self.totals[name] += (time.perf_counter() - t0) * 1e3
            self.counts[name] += 1
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        with range(name):
            yield
        e.record()
        self._pending.append((name, s, e))

    def flush(self):
        for name, s, e in self._pending:
            e.synchronize()
            self.totals[name] += s.elapsed_time(e)
            self.counts[name] += 1
        self._pending = []

    def report(self, reset: bool = True) -> Dict[str, float]:
        self.flush()
        out = {f"{k}_ms": v / max(1, self.counts[k]) for k, v in self.totals.items()}
        if reset:
            self.totals.clear()
            self.counts.clear()
        return out


@contextlib.contextmanager
def torch_profile(out_dir: str, rank: int = 0):
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts, record_shapes=True) as prof:
        yield prof
    os.makedirs(out_dir, exist_ok=True)
    prof.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
    with open(os.path.join(out_dir, f"summary_rank{rank}.txt"), "w") as f:
        sort = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
        f.write(prof.key_averages().table(sort_by=sort, row_limit=50))
