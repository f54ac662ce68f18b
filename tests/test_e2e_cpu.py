"""T5: BASELINE config 1 end-to-end through the CLI: tiny-Llama (2L/128d), 2 DiLoCo workers on
CPU/gloo, H=4 inner steps; plus two-level (inner DDP) and overlapped-outer variants and resume."""
import json
import os
import subprocess
import sys

import pytest

from ._mp import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(nproc, args, tmp_path, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m", "nanodiloco_amd"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r


BASE = ["--llama-config-file", "configs/llama_tiny.json", "--batch-size", "8", "--per-device-batch-size", "4",
        "--seq-length", "64", "--warmup-steps", "2", "--wandb", "off", "--device", "cpu", "--debug-checks"]


def _log(path):
    return [json.loads(l) for l in open(path)]


@pytest.mark.slow
def test_config1_two_workers_gloo(tmp_path):
    log = tmp_path / "m.jsonl"
    r = _torchrun(2, BASE + ["--total-steps", "8", "--inner-steps", "4", "--log-file", str(log),
                             "--checkpoint-dir", str(tmp_path / "ck")], tmp_path)
    assert "Training completed!" in r.stdout
    rows = _log(log)
    assert [x["step"] for x in rows] == list(range(1, 9))
    assert rows[0]["lr"] == 0.0                      # Q4: first inner step at lr 0
    assert rows[-1]["outer_step"] == 2
    assert rows[3]["bytes_outer"] > 0
    assert rows[-1]["effective_step"] == 16 and rows[-1]["total_samples"] == 8 * 8 * 2
    for k in ("loss", "Perplexity", "tokens_per_s", "grad_norm"):
        assert k in rows[-1]
    assert os.path.exists(tmp_path / "ck" / "model.safetensors")


@pytest.mark.slow
def test_two_level_and_overlap(tmp_path):
    _torchrun(4, BASE + ["--total-steps", "8", "--inner-steps", "4", "--inner-dp", "2", "--log-every", "4"], tmp_path)
    _torchrun(2, BASE + ["--total-steps", "8", "--inner-steps", "4", "--overlap-outer", "--comm-dtype", "bf16",
                         "--log-every", "4"], tmp_path)


@pytest.mark.slow
def test_resume_matches_uninterrupted(tmp_path):
    a, b = tmp_path / "a", tmp_path / "b"
    la, lb = tmp_path / "a.jsonl", tmp_path / "b.jsonl"
    common = BASE + ["--inner-steps", "2", "--data", "synthetic"]
    _torchrun(2, common + ["--total-steps", "6", "--checkpoint-dir", str(a), "--log-file", str(la)], tmp_path)
    # interrupted run: 4 steps + checkpoint every outer step, then resume to 6
    _torchrun(2, common + ["--total-steps", "6", "--stop-at-step", "4", "--checkpoint-dir", str(b),
                         "--checkpoint-every", "1"], tmp_path)
    _torchrun(2, common + ["--total-steps", "6", "--resume", str(b), "--log-file", str(lb)], tmp_path)
    ra, rb = _log(la), _log(lb)
    assert [x["step"] for x in rb] == [5, 6]
    assert abs(ra[-1]["loss"] - rb[-1]["loss"]) < 1e-5
