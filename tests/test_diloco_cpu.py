"""DiLoCo algorithm on CPU/gloo, incl. the golden values of SURVEY.md §3.4 (measured on the
reference class itself)."""
import torch

from nanodiloco_amd.config import LlamaConfig
from nanodiloco_amd.models import LlamaForCausalLM
from nanodiloco_amd.optim import FlatAdamW, FlatOuterNesterov
from nanodiloco_amd.parallel.diloco import Diloco
from nanodiloco_amd.parallel.dist import init_distributed

from ._mp import run_ranks

TINY = dict(hidden_size=32, intermediate_size=64, num_attention_heads=2, num_hidden_layers=1, vocab_size=50,
            rms_norm_eps=1e-5)


def _mk(rank, overlap=False, comm=torch.float32, inner_dp=1, seed=None):
    env = init_distributed("gloo", inner_dp=inner_dp)
    m = LlamaForCausalLM(LlamaConfig.from_dict(TINY)).init_weights(seed if seed is not None else 100 + rank)
    dl = Diloco(m, FlatAdamW(m.store, lr=1e-3), FlatOuterNesterov(m.store, lr=0.7, momentum=0.9), 2, 8, 4, env=env,
                comm_dtype=comm, overlap=overlap)
    return env, m, dl


def _golden(rank, world):
    env, m, dl = _mk(rank)
    st = m.store
    theta0 = st.master.clone()
    # broadcast made replicas identical even though each rank initialised differently
    sums = [None] * world
    import torch.distributed as dist
    t = theta0.sum().reshape(1)
    gathered = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(gathered, t)
    assert all(torch.equal(g, gathered[0]) for g in gathered)
    # local drift: rank r moves every weight by -(r+1)  -> delta = r+1, avg 1.5
    st.master.sub_(rank + 1.0)
    dl.outer_step()
    step1 = (st.master - theta0)
    assert torch.allclose(step1[: st.num_params], torch.full_like(step1[: st.num_params], -1.995), atol=1e-5), \
        step1[:4]
    assert torch.equal(dl.sync, st.master)
    # second outer step with zero drift: momentum only
    th1 = st.master.clone()
    dl.outer_step()
    step2 = st.master - th1
    assert torch.allclose(step2[: st.num_params], torch.full_like(step2[: st.num_params], -0.8505), atol=1e-5)
    assert dl.avg_sync_time > 0
    return True


def test_golden_values_two_workers():
    assert all(run_ranks(_golden, 2))


def _matches_torch(rank, world):
    """Full outer step == reference math: per-tensor all_reduce(AVG) + SGD-Nesterov on snapshot."""
    import torch.distributed as dist
    env, m, dl = _mk(rank, seed=7)
    st = m.store
    g = torch.Generator().manual_seed(rank)
    drift = 0.01 * torch.randn(st.numel, generator=g)
    base = st.master.clone()
    st.master.add_(drift)
    # reference
    p = torch.nn.Parameter(base.clone())
    sgd = torch.optim.SGD([p], lr=0.7, momentum=0.9, nesterov=True)
    grad = base - (base + drift)
    dist.all_reduce(grad)
    p.grad = grad / world
    sgd.step()
    dl.outer_step()
    assert torch.allclose(st.master, p.detach(), atol=1e-6)
    return True


def test_outer_step_matches_torch_sgd_four_workers():
    assert all(run_ranks(_matches_torch, 4))


def _overlap(rank, world):
    """Overlapped mode: the outer update lands one inner step late, local progress preserved."""
    env, m, dl = _mk(rank, overlap=True, seed=5)
    st = m.store
    base = st.master.clone()
    st.master.sub_(rank + 1.0)          # drift before the boundary
    dl.outer_step()                     # launches the all-reduce; nothing applied yet
    assert torch.equal(st.master, base - (rank + 1.0))
    st.master.add_(0.25)                # "next inner step" progress
    dl.finalize()
    expect = base - 1.995 + 0.25        # outer result + local progress since the boundary
    assert torch.allclose(st.master[: st.num_params], expect[: st.num_params], atol=1e-5)
    assert torch.allclose(dl.sync[: st.num_params], (base - 1.995)[: st.num_params], atol=1e-5)
    return True


def test_overlapped_outer_step():
    assert all(run_ranks(_overlap, 2))


def _bf16_comm(rank, world):
    env, m, dl = _mk(rank, comm=torch.bfloat16, seed=9)
    st = m.store
    base = st.master.clone()
    st.master.sub_(rank + 1.0)
    dl.outer_step()
    assert torch.allclose(st.master[: st.num_params], (base - 1.995)[: st.num_params], atol=2e-2)
    assert dl.bytes_per_outer_step == st.numel * 2
    return True


def test_bf16_pseudograd_transport():
    assert all(run_ranks(_bf16_comm, 2))


def _two_level(rank, world):
    """4 ranks = 2 workers x 2-GPU inner DDP; sharded outer all-reduce + intra-worker all-gather."""
    env, m, dl = _mk(rank, inner_dp=2, seed=11)
    st = m.store
    base = st.master.clone()
    st.master.sub_(env.worker + 1.0)    # both GPUs of a worker drift identically
    dl.outer_step()
    assert torch.allclose(st.master[: st.num_params], (base - 1.995)[: st.num_params], atol=1e-5)
    assert dl.bytes_per_outer_step == st.numel // 2 * 4
    dl.check_replicas()
    return True


def test_two_level_sharded_outer():
    assert all(run_ranks(_two_level, 4))


def test_single_process_no_group():
    import os
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    env, m, dl = _mk(0)
    st = m.store
    base = st.master.clone()
    st.master.sub_(2.0)
    dl.outer_step()  # W=1: avg delta = 2 -> -0.7*(2+1.8) = -2.66
    assert torch.allclose(st.master[: st.num_params], (base - 2.66)[: st.num_params], atol=1e-5)


def test_skip_nonfinite_step():
    from nanodiloco_amd.ops import adamw_step
    n = 128
    master = torch.randn(n)
    before = master.clone()
    m, v = torch.zeros(n), torch.zeros(n)
    g = torch.randn(n)
    g[3] = float("nan")
    skipped = torch.zeros(1, dtype=torch.int32)
    adamw_step(master, g, m, v, None, 1, 1e-3, skip_nonfinite=True, skipped=skipped)
    assert torch.equal(master, before) and int(skipped.item()) == 1
    g[3] = 0.0
    adamw_step(master, g, m, v, None, 1, 1e-3, skip_nonfinite=True, skipped=skipped)
    assert not torch.equal(master, before) and int(skipped.item()) == 1


def _overlap_bf16_exact_drift(rank, world):
    """Overlapped + bf16 transport: the re-applied local progress is exact (fp32 drift base); only
    the averaged pseudo-gradient itself carries bf16 rounding."""
    env, m, dl = _mk(rank, overlap=True, comm=torch.bfloat16, seed=5)
    st = m.store
    base = st.master.clone()
    drift = torch.full_like(base, -(rank + 1.0))
    drift[: st.num_params] += 1e-3 * torch.arange(st.num_params).remainder(13)  # not bf16-representable
    st.master.add_(drift)
    dl.outer_step()
    local_after = st.master.clone()
    st.master.add_(0.25)
    dl.finalize()
    # master - sync_new must equal the local progress since the boundary EXACTLY: (base+drift+0.25) - (base+drift)
    progress = (st.master - dl.sync)[: st.num_params]
    exact = ((local_after + 0.25) - local_after)[: st.num_params]
    assert torch.allclose(progress, exact, atol=1e-6), (progress - exact).abs().max()
    return True


def test_overlapped_bf16_transport_keeps_fp32_drift():
    assert all(run_ranks(_overlap_bf16_exact_drift, 2))
