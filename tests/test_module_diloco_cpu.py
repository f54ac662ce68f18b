"""Generic DiLoCo wrapper (any nn.Module + torch optimizers) against the reference's per-tensor math
(REF/nanodiloco/diloco/diloco.py:35-60), on 2 gloo ranks."""
import torch

from nanodiloco_amd.parallel.diloco import Diloco
from nanodiloco_amd.parallel.module_diloco import ModuleDiloco

from ._mp import run_ranks


def _net(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(12, 16), torch.nn.GELU(), torch.nn.Linear(16, 5))


def _reference_outer(params, snaps, outer, world):
    """Literal reference outer step: per-tensor delta, all_reduce(AVG) (SUM / W on gloo), reset,
    SGD-Nesterov step."""
    import torch.distributed as dist
    for p, s in zip(params, snaps):
        p.grad = s - p.data
        dist.all_reduce(p.grad)
        p.grad /= world
        p.data = s.clone()
    outer.step()
    outer.zero_grad()
    return [p.detach().clone() for p in params]


def _run(rank, world):
    import torch.distributed as dist
    dist.init_process_group("gloo")
    a, b = _net(100 + rank), _net(100 + rank)
    # reference replica: same broadcast init
    for p in b.parameters():
        dist.broadcast(p.data, src=0)
    inner_a = torch.optim.AdamW(a.parameters(), lr=1e-2, weight_decay=0.1)
    outer_a = torch.optim.SGD(a.parameters(), lr=0.7, momentum=0.9, nesterov=True)
    dl = Diloco(a, inner_a, outer_a, warmup_steps=2, total_steps=12, inner_steps=3)
    assert isinstance(dl, ModuleDiloco)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
    inner_b = torch.optim.AdamW(b.parameters(), lr=1e-2, weight_decay=0.1)
    outer_b = torch.optim.SGD(b.parameters(), lr=0.7, momentum=0.9, nesterov=True)
    from transformers import get_cosine_schedule_with_warmup
    sched_b = get_cosine_schedule_with_warmup(inner_b, 2, 12)
    snaps = [p.detach().clone() for p in b.parameters()]
    g = torch.Generator().manual_seed(rank)
    for step in range(12):
        x, y = torch.randn(8, 12, generator=g), torch.randn(8, 5, generator=g)
        torch.nn.functional.mse_loss(dl(x), y).backward()
        dl.inner_step()
        torch.nn.functional.mse_loss(b(x), y).backward()
        torch.nn.utils.clip_grad_norm_(b.parameters(), 1.0)
        inner_b.step()
        sched_b.step()
        inner_b.zero_grad()
        if (step + 1) % 3 == 0:
            dl.outer_step()
            snaps = _reference_outer(list(b.parameters()), snaps, outer_b, world)
        for pa, pb in zip(a.parameters(), b.parameters()):
            assert torch.allclose(pa, pb, atol=1e-6, rtol=1e-5), (step, (pa - pb).abs().max())
        assert abs(dl.current_lr() - sched_b.get_last_lr()[0]) < 1e-12
    assert dl.avg_sync_time > 0
    # replicas agree after every outer step
    flat = torch.cat([p.detach().reshape(-1) for p in a.parameters()])
    ref = flat.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(flat, ref)
    return True


def test_module_diloco_matches_reference_math_two_workers():
    assert all(run_ranks(_run, 2))


def test_module_diloco_single_process_bf16_transport():
    net = _net(0)
    dl = ModuleDiloco(net, torch.optim.SGD(net.parameters(), lr=0.1),
                      torch.optim.SGD(net.parameters(), lr=1.0), 0, 10, comm_dtype=torch.bfloat16)
    before = [p.detach().clone() for p in net.parameters()]
    for p in net.parameters():
        p.data.add_(0.5)
    dl.outer_step()  # W=1, lr 1, no momentum: theta <- sync - (sync - theta) = theta (bf16-rounded delta)
    for p, q in zip(net.parameters(), before):
        assert torch.allclose(p, q + 0.5, atol=1e-2)
    sd = dl.state_dict()
    dl.load_state_dict(sd)
