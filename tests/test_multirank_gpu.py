"""Multi-rank rehearsal of the driver's N>1 bench launch on a one-GPU box.

The round-end scaling run launches ``torchrun --nproc-per-node N ... bench.py --gpus N`` on an 8-GPU
node over RCCL.  One GPU cannot host several RCCL ranks, so here two ranks share it over gloo
(``--backend gloo``).  That exercises everything around the collective: torchrun env parsing,
device selection, the initial flat broadcast, outer all-reduces inside the timed window, max-over-
ranks timing and the rank-0-only JSON line.  The HIP kernels, the W^T dgrad copies and the tuned
GEMM table are all active, because each rank runs the real GPU training step.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from ._mp import free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _gpu(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_bench_two_ranks_share_gpu_gloo():
    env = dict(os.environ, OMP_NUM_THREADS="4", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--backend", "gloo",
           "--model", "llama_tiny.json", "--batch-size", "16", "--micro-batch", "8", "--seq-len", "256",
           "--steps", "4", "--warmup", "1", "--inner-steps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["steps"] == 4 and j["warmup"] == 1
    assert j["config"]["parallelism"] == "diloco2" and j["config"]["global_batch"] == 32
    assert j["outer_steps_in_window"] == 2  # H=2 inside a 4-step window
    assert j["ops"] == "hip" and j["dgrad_transposed"] is True
    assert j["value"] > 0 and j["final_loss"] == j["final_loss"]
