"""Metrics sinks.

The reference logs to wandb only (REF/nanodiloco/main.py:71-73,118-127,130).  We keep the same key
names (``loss``, ``step``, ``lr``, ``Perplexity``, ``effective_step``, ``total_samples``) and add
throughput / comm keys.  Sinks: JSONL file (always available), stdout, and wandb when importable.
Only global rank 0 logs (fixes SURVEY.md Q6).
"""
import json
import os
import sys
import time
from typing import Any, Dict, List, Optional


class MetricSink:
    def log(self, metrics: Dict[str, Any]) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def finish(self) -> None:
        pass


class JsonlSink(MetricSink):
    def __init__(self, path: str):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._f = open(path, "a", buffering=1)

    def log(self, metrics):
        self._f.write(json.dumps({"time": time.time(), **metrics}) + "\n")

    def finish(self):
        self._f.close()


class StdoutSink(MetricSink):
    def __init__(self, stream=None):
        self.stream = stream or sys.stdout

    def log(self, metrics):
        parts = []
        for k, v in metrics.items():
            parts.append(f"{k}={v:.5g}" if isinstance(v, float) else f"{k}={v}")
        print(" ".join(parts), file=self.stream, flush=True)


class WandbSink(MetricSink):
    def __init__(self, project: str, name: str, config: Dict[str, Any]):
        import wandb  # noqa: F401  (optional dependency)

        self._wandb = wandb
        wandb.init(project=project, name=name, config=config)

    def log(self, metrics):
        self._wandb.log(metrics)

    def finish(self):
        self._wandb.finish()


class MultiSink(MetricSink):
    def __init__(self, sinks: List[MetricSink]):
        self.sinks = sinks

    def log(self, metrics):
        for s in self.sinks:
            s.log(metrics)

    def finish(self):
        for s in self.sinks:
            s.finish()


def make_sink(rank: int, project: str, run_name: str, run_config: Dict[str, Any],
              jsonl_path: Optional[str] = None, stdout: bool = True, use_wandb: str = "auto") -> MetricSink:
    if rank != 0:
        return MultiSink([])
    sinks: List[MetricSink] = []
    if stdout:
        sinks.append(StdoutSink())
    if jsonl_path:
        sinks.append(JsonlSink(jsonl_path))
    if use_wandb in ("auto", "on"):
        try:
            sinks.append(WandbSink(project, run_name, run_config))
        except Exception as e:  # wandb absent or offline
            if use_wandb == "on":
                raise
            print(f"[nanodiloco_amd] wandb unavailable ({type(e).__name__}); logging to JSONL/stdout only",
                  file=sys.stderr)
    return MultiSink(sinks)
