"""Process-group bootstrap (parallel/dist.py): every group gets its own RCCL Options object and the
collective timeout, and WORLD keeps its settings after the two-level sub-groups are created."""
import datetime

import pytest

from nanodiloco_amd.parallel import dist as D

from ._mp import run_ranks


def test_pg_options_fresh_object_per_call():
    pytest.importorskip("torch.distributed")
    a, b = D._pg_options("nccl", True), D._pg_options("nccl", True)
    if a is None:
        pytest.skip("torch built without ProcessGroupNCCL")
    assert a is not b and a.is_high_priority_stream and b.is_high_priority_stream
    assert D._pg_options("gloo", True) is None and D._pg_options("nccl", False) is None


def _groups_keep_timeout(rank, world):
    import torch
    import torch.distributed as dist

    seen = []
    real_new_group = dist.new_group

    def spy(ranks, **kw):  # record what every sub-group is created with
        seen.append((tuple(ranks), kw.get("timeout"), id(kw.get("pg_options"))))
        return real_new_group(ranks, **kw)

    dist.new_group = spy
    try:
        env = D.init_distributed(backend="gloo", inner_dp=2, device="cpu", timeout_s=77.0)
    finally:
        dist.new_group = real_new_group
    cpu = torch.device("cpu")
    out = {
        "world": env.world_group._get_backend(cpu).options._timeout.total_seconds(),
        "inner": env.inner_group._get_backend(cpu).options._timeout.total_seconds(),
        "outer": env.outer_group._get_backend(cpu).options._timeout.total_seconds(),
        "sub_timeouts": [t.total_seconds() if t else None for _, t, _ in seen],
        "n_groups": len(seen),
        "world_ranks": dist.get_process_group_ranks(env.world_group),
    }
    return out


def test_subgroups_keep_world_timeout_and_ranks():
    res = run_ranks(_groups_keep_timeout, 4)
    for r in res:
        assert r["world"] == 77.0 and r["inner"] == 77.0 and r["outer"] == 77.0, r
        assert r["n_groups"] == 4 and r["sub_timeouts"] == [77.0] * 4, r
        assert r["world_ranks"] == [0, 1, 2, 3], r
    assert datetime.timedelta(seconds=77).total_seconds() == 77.0
