"""Checkpoint / resume (the reference has none -- SURVEY.md §5.4 -- so the format is defined here).

Directory layout (written only at outer-step boundaries, when all replicas are identical):

  <dir>/config.json              HF LlamaConfig JSON (+ "architectures": ["LlamaForCausalLM"])
  <dir>/model.safetensors        fp32 master weights, HF key names -> ``LlamaForCausalLM.from_pretrained(dir)``
  <dir>/diloco_state.safetensors outer state shared by all workers: theta_sync, outer momentum
  <dir>/rank{r}.safetensors      per-rank inner AdamW m/v + data-generator state
  <dir>/trainer_state.json       step counters, schedule, hyper-params, topology (world size, inner_dp,
                                 flat size -- validated on resume), per-rank scalar state

With ``--overlap-outer`` a checkpoint taken at an outer boundary holds that step still PENDING (its
all-reduce finished, its one-step-late application not yet done): the reduced pseudo-gradient and each
rank's drift base and local weights go into the rank files, and the resumed run applies the step after its first inner
step -- the same trajectory as the uninterrupted run (tests/test_e2e_cpu.py).  Such an INTERMEDIATE checkpoint is
not export-ready: its model.safetensors holds rank 0's local weights (drifted by that worker's inner progress,
without the pending outer update), and config.json says so (``"nanodiloco_pending_outer_step": true``).  For
evaluation / export use a checkpoint without that flag -- the final one (``Diloco.finalize`` applies the
pending step first) or any checkpoint of a run without ``--overlap-outer``.

Crash consistency (round 5): every rank writes into ``<dir>.tmp``; after a barrier rank 0 adds
``COMPLETE.json`` and swaps the staging directory in (``<dir>`` -> ``<dir>.old``, ``<dir>.tmp`` -> ``<dir>``,
then ``<dir>.old`` is removed), so a crash at any point of a save leaves the previous complete checkpoint
readable (``find_checkpoint`` falls back to ``<dir>.old`` when the swap itself was interrupted).  ``--resume
auto`` resumes from the newest complete checkpoint in ``--checkpoint-dir`` if there is one and starts fresh
otherwise -- the restart form for ``torchrun --max-restarts N`` (tests/test_e2e_cpu.py
injects a crash with ``ND_FAULT_INJECT``).

Only safetensors + JSON: nothing executable is ever deserialised.
"""
from __future__ import annotations

import json
import os
import shutil
from typing import Any, Dict, Optional

import torch

from ..parallel.dist import DistEnv, barrier


COMPLETE = "COMPLETE.json"


def _stage_dir(ckpt_dir: str) -> str:
    return os.path.normpath(ckpt_dir) + ".tmp"


def find_checkpoint(ckpt_dir: Optional[str]) -> Optional[str]:
    """The newest COMPLETE checkpoint for ``ckpt_dir``: itself; else the staging ``<dir>.tmp`` when a save was
    interrupted after its COMPLETE marker but before its swap finished (newer than ``<dir>.old``); else
    ``<dir>.old``; else a pre-round-5 checkpoint without the marker; else None."""
    if not ckpt_dir:
        return None
    d = os.path.normpath(ckpt_dir)
    for cand in (d, _stage_dir(d), d + ".old"):
        if os.path.isfile(os.path.join(cand, COMPLETE)):
            return cand
    if os.path.isfile(os.path.join(d, "trainer_state.json")) and not os.path.exists(_stage_dir(d)):
        return d  # written before the staging scheme existed
    return None


def _swap_in(stage: str, final: str) -> None:
    """Make the complete ``stage`` the checkpoint.  At every instant some complete copy is where
    :func:`find_checkpoint` looks: ``final`` (or ``stage``, or ``final.old``) -- a leftover ``.old`` is deleted
    only while a complete ``final`` exists, and with no ``final`` the stage moves in before anything is deleted."""
    old = final + ".old"
    if os.path.isdir(final):
        if os.path.isdir(old):
            shutil.rmtree(old)
        os.replace(final, old)
    os.replace(stage, final)
    shutil.rmtree(old, ignore_errors=True)


def _save_st(path: str, tensors: Dict[str, torch.Tensor]):
    from safetensors.torch import save_file

    save_file({k: v.detach().contiguous().cpu() for k, v in tensors.items()}, path + ".tmp")
    os.replace(path + ".tmp", path)


def _load_st(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    return load_file(path)


def save_checkpoint(ckpt_dir: str, model, diloco, env: DistEnv, step: int, data_state: Optional[Dict[str, Any]] = None,
                    extra: Optional[Dict[str, Any]] = None):
    pending = diloco.pending_outer_state()  # overlapped mode: saved as pending, not applied
    if env.inner_dp > 1:
        # two-level mode: each GPU of a worker updates only its shard of the outer momentum
        # (parallel/diloco.py, sharded outer step); gather the worker's full buffer before rank 0
        # writes it, so a resumed run restores every shard (not just shard 0)
        diloco.inner_comm.all_gather_flat(diloco.outer_optimizer.momentum_buffer, diloco.shards, env.inner_rank)
    final = os.path.normpath(ckpt_dir)
    ckpt_dir = _stage_dir(final)  # every file below goes to the staging directory
    r = env.rank
    if r == 0:
        shutil.rmtree(ckpt_dir, ignore_errors=True)  # leftovers of a save that crashed
        os.makedirs(ckpt_dir)
    barrier(env)
    store = model.store
    # per-rank state (every rank)
    per = {"adamw.exp_avg": diloco.inner_optimizer.exp_avg, "adamw.exp_avg_sq": diloco.inner_optimizer.exp_avg_sq}
    scal: Dict[str, Any] = {"adamw_step": diloco.inner_optimizer.step_count}
    if pending is not None:
        # until the pending step lands, every worker's local weights differ (each carries its own
        # inner progress since the boundary): model.safetensors holds rank 0's, each rank keeps its own
        per["outer.delta"] = pending["delta"]
        per["outer.drift_base"] = pending["drift_base"]
        per["master"] = store.master
    if data_state:
        for k, v in data_state.items():
            if isinstance(v, torch.Tensor):
                per[f"data.{k}"] = v
            else:
                scal[f"data.{k}"] = v
    _save_st(os.path.join(ckpt_dir, f"rank{r}.safetensors"), per)
    with open(os.path.join(ckpt_dir, f"rank{r}.json"), "w") as f:
        json.dump(scal, f)
    if r == 0:
        cfg_json = model.config.to_hf_json()
        if pending is not None:  # see the module doc: weights are rank 0's local ones, not the synced model
            cfg_json["nanodiloco_pending_outer_step"] = True
        with open(os.path.join(ckpt_dir, "config.json"), "w") as f:
            json.dump(cfg_json, f, indent=2)
        _save_st(os.path.join(ckpt_dir, "model.safetensors"), {n: store.master_view(n) for n in store.names})
        sync = diloco.sync.to(store.device) if diloco.sync.device != store.device else diloco.sync
        _save_st(os.path.join(ckpt_dir, "diloco_state.safetensors"),
                 {"theta_sync": sync, "outer_momentum": diloco.outer_optimizer.momentum_buffer})
        state = {"step": step, "local_step": diloco.local_step, "outer_step_count": diloco.outer_step_count,
                 "outer_opt_step": diloco.outer_optimizer.step_count, "scheduler": diloco.scheduler.state_dict(),
                 "world_size": env.world_size, "inner_dp": env.inner_dp, "flat_numel": store.numel,
                 "pending_outer": pending is not None, **(extra or {})}
        with open(os.path.join(ckpt_dir, "trainer_state.json"), "w") as f:
            json.dump(state, f, indent=2)
    barrier(env)  # every rank's files are in the staging directory
    # every tensor above went through a host copy (so every collective it depends on has completed or been
    # aborted, and a watchdog abort sets the sticky error before it releases the collective): a failed own
    # RCCL communicator must not leave a COMPLETE checkpoint of partially reduced state behind
    for comm in (getattr(diloco, "outer_comm", None), getattr(diloco, "inner_comm", None)):
        if comm is not None:
            comm.check("the checkpoint is marked complete")
    if r == 0:
        with open(os.path.join(ckpt_dir, COMPLETE), "w") as f:
            json.dump({"step": step, "world_size": env.world_size}, f)
        _swap_in(ckpt_dir, final)
    barrier(env)


def load_checkpoint(ckpt_dir: str, model, diloco, env: DistEnv, elastic: bool = False) -> Dict[str, Any]:
    """``elastic`` (``--elastic-resume``): the number of DiLoCo workers may differ from the checkpoint's (one GPU
    per worker, a checkpoint without a pending overlapped outer step).  The shared outer state (theta_sync,
    outer momentum, schedule) is exact; worker r keeps its own AdamW state when the checkpoint has rank r, and a
    NEW worker starts from rank 0's AdamW state -- the "average over the survivors" recovery DiLoCo allows
    (SURVEY.md §5.3).  Data: the memmap stream is global (csrc/runtime/token_loader.cpp), so every worker
    restarts it where the old workers stopped together (``data_state_rank0``; nothing repeated or skipped);
    the HF loader's contiguous shards cannot be re-cut exactly and the resume refuses; synthetic workers keep
    their own random stream (new ones draw a fresh one)."""
    found = find_checkpoint(ckpt_dir)
    if found is None:
        raise FileNotFoundError(f"no complete checkpoint at {ckpt_dir}")
    ckpt_dir = found
    with open(os.path.join(ckpt_dir, "trainer_state.json")) as f:
        state = json.load(f)
    store = model.store
    old_world = int(state.get("world_size", env.world_size))
    resized = elastic and old_world != env.world_size
    if resized:
        if env.inner_dp != 1 or int(state.get("inner_dp", 1)) != 1:
            raise ValueError("--elastic-resume needs one GPU per worker (--inner-dp 1) in both runs")
        if state.get("pending_outer"):
            raise ValueError(f"checkpoint {ckpt_dir} holds a pending overlapped outer step (per-worker state): "
                             f"--elastic-resume needs a checkpoint without one")
    # topology: every rank restores its OWN AdamW state and (two-level mode) its shard of the outer
    # step, so a resume on a different layout would silently drop workers' state or mis-shard the
    # outer momentum -- refuse it (unless --elastic-resume, above)
    for key, have in (("world_size", env.world_size), ("inner_dp", env.inner_dp), ("flat_numel", store.numel)):
        if key == "world_size" and resized:
            continue
        if key in state and int(state[key]) != int(have):
            raise ValueError(f"checkpoint {ckpt_dir} was written with {key}={state[key]}, this run has {have}: "
                             f"resume needs the same world size, --inner-dp and model (or --elastic-resume)")
    sd = _load_st(os.path.join(ckpt_dir, "model.safetensors"))
    model.load_state_dict(sd)
    ds = _load_st(os.path.join(ckpt_dir, "diloco_state.safetensors"))
    diloco.load_state_dict({"sync": ds["theta_sync"],
                            "outer": {"momentum_buffer": ds["outer_momentum"], "step": state["outer_opt_step"]},
                            "scheduler": state["scheduler"], "local_step": state["local_step"],
                            "outer_step_count": state["outer_step_count"]})
    rfile = os.path.join(ckpt_dir, f"rank{env.rank}.safetensors")
    data_state: Dict[str, Any] = {}
    own = os.path.exists(rfile)
    if not own and resized:  # a worker the checkpoint did not have: rank 0's AdamW state, fresh data stream
        rfile = os.path.join(ckpt_dir, "rank0.safetensors")
    elif not own and "world_size" in state:
        raise FileNotFoundError(f"{rfile} missing: the checkpoint is incomplete for rank {env.rank}")
    if os.path.exists(rfile):
        per = _load_st(rfile)
        if state.get("pending_outer"):
            store.master.copy_(per["master"].to(store.master.device))
            diloco.restore_pending_outer(per["outer.delta"].to(diloco.delta.device),
                                         per["outer.drift_base"].to(diloco.delta.device))
        diloco.inner_optimizer.exp_avg.copy_(per["adamw.exp_avg"])
        diloco.inner_optimizer.exp_avg_sq.copy_(per["adamw.exp_avg_sq"])
        with open(rfile[:-len(".safetensors")] + ".json") as f:
            scal = json.load(f)
        diloco.inner_optimizer.step_count = int(scal["adamw_step"])
        if own:
            for k, v in per.items():
                if k.startswith("data."):
                    data_state[k[5:]] = v
            for k, v in scal.items():
                if k.startswith("data."):
                    data_state[k[5:]] = v
    state["data_state"] = data_state
    if resized:
        # the data sources whose stream is global (memmap) restart every worker -- survivors and new ones --
        # at the position the old workers reached together; they advance in lockstep, so rank 0's state says
        per0 = _load_st(os.path.join(ckpt_dir, "rank0.safetensors"))
        with open(os.path.join(ckpt_dir, "rank0.json")) as f:
            scal0 = json.load(f)
        ds0 = {k[5:]: v for k, v in list(per0.items()) + list(scal0.items()) if k.startswith("data.")}
        state["data_state_rank0"] = ds0
    state["resized_from"] = old_world if resized else None
    store.sync_shadow()
    return state
