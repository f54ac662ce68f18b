"""Inner DDP (two-level topology, BASELINE config 3): the per-step gradient all-reduce that is
launched from inside the backward must see every layer's FINAL gradient.

Oracle: every rank recomputes, in-process and without any communication, the gradients of every
other rank's micro-batches and sums them; the synced ``store.grad`` after ``InnerGradSync.finish()``
must equal that sum to fp32 rounding, on every rank (so replicas cannot diverge).  Runs with several
micro-batches per inner step and >= 3 layers, with and without the backward-overlapped hooks.
"""
import pytest
import torch

from nanodiloco_amd.config import LlamaConfig
from nanodiloco_amd.models import LlamaForCausalLM

from ._mp import run_ranks

CFG = dict(hidden_size=32, intermediate_size=64, num_attention_heads=2, num_hidden_layers=3, vocab_size=61,
           rms_norm_eps=1e-5)
MICRO, B, T = 3, 2, 16


def _batches(rank, cfg=CFG, device="cpu", t=T):
    g = torch.Generator().manual_seed(1000 + rank)
    return [torch.randint(0, cfg["vocab_size"], (B, t), generator=g).to(device) for _ in range(MICRO)]


def _grad_of(model, batches, scale):
    model.store.zero_grad()
    for ids in batches:
        model(ids, labels=ids, loss_scale=scale).loss.backward()
    return model.store.grad.clone()


def _inner_sync(rank, world, inner_dp, overlap, cfg=CFG, gpu=False, rtol=1e-6, t=T):
    from nanodiloco_amd.parallel.comm import FlatCommunicator
    from nanodiloco_amd.parallel.dist import init_distributed
    from nanodiloco_amd.parallel.inner_ddp import InnerGradSync

    env = init_distributed("gloo", inner_dp=inner_dp, device=None if gpu else "cpu")
    dt = torch.bfloat16 if gpu else torch.float32
    m = LlamaForCausalLM(LlamaConfig.from_dict(cfg), env.device, dt).init_weights(3)
    scale = 1.0 / MICRO / inner_dp
    # oracle: sum over the ranks of MY worker of their (locally recomputed) gradients
    members = range(env.worker * inner_dp, (env.worker + 1) * inner_dp)
    expect = sum(_grad_of(m, _batches(r, cfg, env.device, t), scale) for r in members)
    # the real thing: own micro-batches, hook armed before the last micro-batch's backward
    comm = FlatCommunicator(env.inner_group, inner_dp)
    sync = InnerGradSync(m, comm, overlap=overlap)
    m.store.zero_grad()
    for j, ids in enumerate(_batches(rank, cfg, env.device, t)):
        if j == MICRO - 1:
            sync.arm()
        m(ids, labels=ids, loss_scale=scale).loss.backward()
    sync.finish()
    got = m.store.grad
    err = (got - expect).abs().max().item()
    ref = expect.abs().max().item()
    assert err <= rtol * max(1.0, ref), f"rank {rank}: max|err| {err} vs max|grad| {ref}"
    # every layer's span got reduced exactly once (hooks fired once per layer)
    assert sync.last_hook_count == (cfg["num_hidden_layers"] if overlap else 0)
    return True


@pytest.mark.parametrize("overlap", [True, False])
def test_inner_ddp_two_ranks(overlap):
    assert all(run_ranks(_inner_sync, 2, 2, overlap))


def test_inner_ddp_four_ranks_two_workers():
    assert all(run_ranks(_inner_sync, 4, 2, True))


def test_inner_ddp_four_ranks_one_worker():
    assert all(run_ranks(_inner_sync, 4, 4, True))


def _divergence_detected(rank, world):
    """--debug-checks must catch intra-worker divergence (theta_sync alone cannot: it is all-gathered)."""
    from nanodiloco_amd.optim import FlatAdamW, FlatOuterNesterov
    from nanodiloco_amd.parallel.diloco import Diloco
    from nanodiloco_amd.parallel.dist import init_distributed

    env = init_distributed("gloo", inner_dp=2)
    m = LlamaForCausalLM(LlamaConfig.from_dict(CFG)).init_weights(3)
    dl = Diloco(m, FlatAdamW(m.store, lr=1e-3), FlatOuterNesterov(m.store), 1, 8, 4, env=env, debug_checks=True)
    dl.check_inner_replicas()  # identical after the init broadcast
    if rank == 1:
        m.store.master[5] += 1e-3
    try:
        dl.check_inner_replicas()
    except RuntimeError as e:
        assert "diverged" in str(e)
        return True
    raise AssertionError("intra-worker divergence not detected")


def test_debug_checks_catch_inner_divergence():
    assert all(run_ranks(_divergence_detected, 2))
