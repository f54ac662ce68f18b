"""T5: BASELINE config 1 end-to-end through the CLI: tiny-Llama (2L/128d), 2 DiLoCo workers on
CPU/gloo, H=4 inner steps; plus two-level (inner DDP) and overlapped-outer variants and resume."""
import json
import os
import subprocess
import sys

import pytest
import torch

from ._mp import child_env, free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(nproc, args, tmp_path, timeout=600):
    env = child_env(OMP_NUM_THREADS="1")
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


def _tensors(path):
    from safetensors.torch import load_file
    return load_file(str(path))


@pytest.mark.slow
@pytest.mark.parametrize("nproc,inner_dp,overlap", [(2, 1, False), (4, 2, False), (2, 1, True)])
def test_resume_matches_uninterrupted(tmp_path, nproc, inner_dp, overlap):
    """Stop after 2 outer steps, resume, finish: bit-identical to the uninterrupted run -- weights,
    theta_sync and (two-level mode) every shard of the outer momentum.  With --overlap-outer the
    checkpoint holds the boundary's outer step still pending and the resumed run applies it one inner
    step late, exactly like the uninterrupted run (checkpointing does not change the trajectory)."""
    a, b = tmp_path / "a", tmp_path / "b"
    la, lb = tmp_path / "a.jsonl", tmp_path / "b.jsonl"
    common = BASE + ["--inner-steps", "2", "--data", "synthetic", "--inner-dp", str(inner_dp)]
    if overlap:
        common += ["--overlap-outer"]
    _torchrun(nproc, common + ["--total-steps", "6", "--checkpoint-dir", str(a), "--log-file", str(la)], tmp_path)
    # interrupted run: 4 steps + checkpoint every outer step, then resume to 6
    _torchrun(nproc, common + ["--total-steps", "6", "--stop-at-step", "4", "--checkpoint-dir", str(b),
                               "--checkpoint-every", "1"], tmp_path)
    _torchrun(nproc, common + ["--total-steps", "6", "--resume", str(b), "--log-file", str(lb),
                               "--checkpoint-dir", str(b)], tmp_path)
    ra, rb = _log(la), _log(lb)
    assert [x["step"] for x in rb] == [5, 6]
    if overlap:
        assert json.load(open(b / "trainer_state.json"))["pending_outer"] is False  # final save: applied
        assert "nanodiloco_pending_outer_step" not in json.load(open(b / "config.json"))  # export-ready
    assert ra[-1]["loss"] == rb[-1]["loss"]
    for f in ("model.safetensors", "diloco_state.safetensors"):
        ta, tb = _tensors(a / f), _tensors(b / f)
        assert ta.keys() == tb.keys()
        for k in ta:
            assert torch.equal(ta[k], tb[k]), (f, k)
    mom = _tensors(a / "diloco_state.safetensors")["outer_momentum"]
    if inner_dp > 1:  # every shard carries momentum, not only shard 0
        n = mom.numel() // inner_dp
        assert all(mom[i * n:(i + 1) * n].abs().sum() > 0 for i in range(inner_dp))


def _torchrun_raw(nproc, args, tmp_path, extra_env=None, run_args=(), timeout=600):
    env = child_env(OMP_NUM_THREADS="1", **(extra_env or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *run_args, "-m", "nanodiloco_amd"] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.slow
def test_crash_restart_resumes_bitwise(tmp_path):
    """SURVEY §5.3 fault drill: rank 1 crashes (exit 17) after inner step 5, one outer step past the checkpoint
    of step 4; ``torchrun --max-restarts 1`` restarts the worker group, ``--resume auto`` picks the newest
    COMPLETE checkpoint and the job finishes bit-identical to an uninterrupted run."""
    a, b = tmp_path / "a", tmp_path / "b"
    common = BASE + ["--inner-steps", "2", "--data", "synthetic", "--total-steps", "8"]
    _torchrun(2, common + ["--checkpoint-dir", str(a)], tmp_path)
    r = _torchrun_raw(2, common + ["--checkpoint-dir", str(b), "--checkpoint-every", "1", "--resume", "auto"],
                      tmp_path, extra_env={"ND_FAULT_INJECT": "1:5"}, run_args=("--max-restarts", "1"))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "[fault inject] rank 1 step 5: crash" in out, out[-4000:]
    assert "[resume auto] from" in out, out[-4000:]  # the restart resumed instead of starting over
    assert json.load(open(b / "COMPLETE.json"))["step"] == 8
    assert not os.path.exists(str(b) + ".tmp") and not os.path.exists(str(b) + ".old")
    for f in ("model.safetensors", "diloco_state.safetensors"):
        ta, tb = _tensors(a / f), _tensors(b / f)
        for k in ta:
            assert torch.equal(ta[k], tb[k]), (f, k)


@pytest.mark.slow
def test_hung_peer_fails_by_collective_timeout(tmp_path):
    """A worker that hangs (ND_FAULT_INJECT ...:hang) makes its peer's next outer all-reduce time out after
    --collective-timeout-s: the job fails with an error within seconds instead of hanging."""
    import time
    t0 = time.time()
    r = _torchrun_raw(2, BASE + ["--inner-steps", "2", "--data", "synthetic", "--total-steps", "6",
                                 "--collective-timeout-s", "20"],
                      tmp_path, extra_env={"ND_FAULT_INJECT": "1:1:hang"}, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-4000:]
    assert "[fault inject] rank 1 step 1: hang" in out, out[-4000:]
    assert time.time() - t0 < 200
    assert "time" in out.lower(), out[-4000:]  # gloo: "Timed out ..." on the waiting rank


@pytest.mark.slow
def test_elastic_resume_changes_worker_count(tmp_path):
    """--elastic-resume: a 2-worker checkpoint resumes on 1 worker (a lost node) and on 3 workers (a new one
    joins); the shared outer state is loaded exactly and training continues.  Without the flag the world-size
    change is refused."""
    ck = tmp_path / "ck"
    common = BASE + ["--inner-steps", "2", "--data", "synthetic"]
    _torchrun(2, common + ["--total-steps", "4", "--checkpoint-dir", str(ck)], tmp_path)
    sync0 = _tensors(ck / "diloco_state.safetensors")["theta_sync"]
    r = _torchrun_raw(1, common + ["--total-steps", "6", "--resume", str(ck)], tmp_path)
    assert r.returncode != 0 and "--elastic-resume" in (r.stdout + r.stderr)
    for n in (1, 3):
        out = tmp_path / f"out{n}"
        log = tmp_path / f"l{n}.jsonl"
        r = _torchrun(n, common + ["--total-steps", "6", "--resume", str(ck), "--elastic-resume", "--log-file",
                                   str(log), "--checkpoint-dir", str(out)], tmp_path)
        assert f"[elastic resume] 2 -> {n} workers" in r.stdout + r.stderr
        rows = _log(log)
        assert [x["step"] for x in rows] == [5, 6] and all(x["loss"] == x["loss"] for x in rows)
        st = json.load(open(out / "trainer_state.json"))
        assert st["world_size"] == n and st["outer_step_count"] == 3
    # the resumed runs started from the checkpoint's theta_sync (the 1-worker run's weights after one more
    # outer step differ from it, but by a training step, not by a re-initialisation)
    w1 = _tensors(tmp_path / "out1" / "diloco_state.safetensors")["theta_sync"]
    assert ((w1 - sync0).norm() / sync0.norm()).item() < 0.05


def test_find_checkpoint_prefers_complete(tmp_path):
    """Crash consistency of the staging scheme: only a directory with COMPLETE.json (or its .old copy while a
    swap was interrupted) is a resume point; a half-written staging directory never is."""
    from nanodiloco_amd.utils.checkpoint import COMPLETE, find_checkpoint
    d = tmp_path / "ck"
    assert find_checkpoint(str(d)) is None
    (tmp_path / "ck.tmp").mkdir()
    (tmp_path / "ck.tmp" / "trainer_state.json").write_text("{}")
    assert find_checkpoint(str(d)) is None  # staging only: nothing complete yet
    (tmp_path / "ck.old").mkdir()
    (tmp_path / "ck.old" / COMPLETE).write_text('{"step": 4}')
    assert find_checkpoint(str(d)) == str(tmp_path / "ck.old")  # interrupted between the two renames
    (tmp_path / "ck.tmp" / COMPLETE).write_text('{"step": 5}')
    assert find_checkpoint(str(d)) == str(tmp_path / "ck.tmp")  # marked complete, swap not begun: newest
    # resumed from ck.old (no ck), the next save's swap must never leave only the staging copy
    # unconsidered -- with no final directory the stage moves in BEFORE the old copy is deleted
    from nanodiloco_amd.utils.checkpoint import _swap_in
    _swap_in(str(tmp_path / "ck.tmp"), str(d))
    assert find_checkpoint(str(d)) == str(d) and not (tmp_path / "ck.old").exists()
    assert (d / COMPLETE).read_text() == '{"step": 5}'
    import shutil
    shutil.rmtree(d)
    d.mkdir()
    (d / COMPLETE).write_text('{"step": 6}')
    assert find_checkpoint(str(d)) == str(d)


def _bench_json(stdout: str) -> dict:
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


BENCH = ["bench.py", "--model", "llama_tiny.json", "--batch-size", "4", "--micro-batch", "2", "--seq-len", "64",
         "--steps", "3", "--warmup", "1", "--inner-steps", "2"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.slow
def test_bench_contract_single_process():
    env = child_env(OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable] + BENCH + ["--gpus", "1"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _bench_json(r.stdout)
    assert KEYS <= set(j)
    assert j["n_gpus"] == 1 and j["steps"] == 3 and j["warmup"] == 1 and j["scaling"] == "weak"
    assert j["higher_is_better"] is True and j["value"] > 0 and j["data"] == "synthetic"
    assert abs(j["value"] - 4 * 64 * 3 / (j["ms_per_step"] * 3 / 1000.0)) / j["value"] < 0.01
    assert j["config"]["global_batch"] == 4 and j["config"]["seq_len"] == 64
    assert j["outer_steps_in_window"] >= 1


@pytest.mark.slow
def test_bench_contract_two_ranks_gloo():
    env = child_env(OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port())] + BENCH + ["--gpus", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _bench_json(r.stdout)  # rank 0 only prints
    assert j["n_gpus"] == 2 and j["config"]["global_batch"] == 8
    assert j["config"]["parallelism"] == "diloco2"
    assert j["bytes_per_outer_step"] > 0
