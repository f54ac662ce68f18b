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

from ._mp import child_env, free_port

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _gpu(hip_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_bench_two_ranks_share_gpu_gloo():
    env = child_env(OMP_NUM_THREADS="4")
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


def test_trainer_two_workers_share_gpu_overlap_bf16_comm(tmp_path):
    """CLI trainer, 2 DiLoCo workers on one GPU over gloo: overlapped outer step with bf16
    pseudo-gradient transport and debug replica checks (the outer all-reduce result must be
    bit-identical on both workers), plus a checkpoint that HF-style tooling can read."""
    import os as _os
    env = child_env(OMP_NUM_THREADS="4")
    log = tmp_path / "log.jsonl"
    ck = tmp_path / "ckpt"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "nanodiloco_amd",
           "--llama-config-file", "configs/llama_tiny.json", "--batch-size", "8", "--per-device-batch-size", "4",
           "--seq-length", "128", "--total-steps", "8", "--inner-steps", "4", "--warmup-steps", "2",
           "--backend", "gloo", "--overlap-outer", "--comm-dtype", "bf16", "--debug-checks",
           "--wandb", "off", "--log-file", str(log), "--log-every", "1", "--checkpoint-dir", str(ck)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    recs = [json.loads(l) for l in open(log)]
    assert recs and all(rec["loss"] == rec["loss"] for rec in recs if "loss" in rec)
    assert any(rec.get("outer_step", 0) >= 1 for rec in recs)
    files = set(_os.listdir(ck)) if ck.is_dir() else set()
    found = files | {f for d in files if (ck / d).is_dir() for f in _os.listdir(ck / d)}
    assert "model.safetensors" in found and "config.json" in found, found


def test_crash_restart_resume_auto_rccl_one_gpu(tmp_path):
    """The §5.3 fault drill on the GPU path: a one-rank torchrun job on the nccl (RCCL) backend crashes after inner
    step 3 (ND_FAULT_INJECT), ``--max-restarts 1`` restarts it, the restart's c10d store is attempt-prefixed
    (parallel/dist.py) and ``--resume auto`` continues from the step-2 checkpoint to the end."""
    ck = tmp_path / "ck"
    log = tmp_path / "m.jsonl"
    env = child_env(OMP_NUM_THREADS="4", ND_FAULT_INJECT="0:3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "--max-restarts", "1", "-m", "nanodiloco_amd",
           "--llama-config-file", "configs/llama_tiny.json", "--batch-size", "8", "--per-device-batch-size", "4",
           "--seq-length", "128", "--warmup-steps", "2", "--wandb", "off", "--data", "synthetic",
           "--inner-steps", "2", "--total-steps", "6", "--backend", "nccl", "--force-collectives", "true",
           "--checkpoint-dir", str(ck),
           "--checkpoint-every", "1", "--resume", "auto", "--log-file", str(log)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "[fault inject] rank 0 step 3: crash" in out and "[resume auto] from" in out, out[-4000:]
    assert json.load(open(ck / "COMPLETE.json"))["step"] == 6
    steps = [json.loads(l)["step"] for l in open(log)]
    assert steps[-1] == 6 and 3 in steps  # step 3 ran (again) after the restart
