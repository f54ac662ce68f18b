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


def _group_member(rank, world, port, run_id, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TORCHELASTIC_RUN_ID=run_id, TORCHELASTIC_USE_AGENT_STORE="True",
                      TORCHELASTIC_RESTART_COUNT="0")  # a membership change does not move the restart count
    try:
        import torch
        import torch.distributed as dist
        env = D.init_distributed(backend="gloo", device="cpu", timeout_s=60.0)
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t)
        ns = dist.distributed_c10d._get_default_store()
        q.put((rank, "ok", (t.item(), env.world_size)))
        dist.barrier()
        dist.destroy_process_group()
        del ns
    except Exception:
        import traceback
        q.put((rank, "err", traceback.format_exc()))


def _run_group(world, port, run_id):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_group_member, args=(r, world, port, run_id, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, st, res = q.get()
        if st != "ok":
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {r} failed:\n{res}")
        out[r] = res
    for p in procs:
        p.join(60)
    return out


def test_worker_groups_sharing_an_agent_store_get_their_own_namespace():
    """an elastic membership change restarts the worker group on torchrun's SAME agent store
    without moving TORCHELASTIC_RESTART_COUNT.  Three consecutive groups (2, 3, then 2 ranks, count 0 every
    time) on one store: each must rendezvous in a namespace of its own (no stale gloo addresses) and
    all-reduce correctly."""
    import torch.distributed as dist

    from ._mp import free_port
    port = free_port()
    store = dist.TCPStore("127.0.0.1", port, 1, True, timeout=datetime.timedelta(seconds=60))  # the agent's store
    for world in (2, 3, 2):
        out = _run_group(world, port, "elastic-test")
        want = world * (world + 1) / 2
        assert all(v == (want, world) for v in out.values()), out
    # every rank 0 .. 2 drew a fresh incarnation per group it was part of
    assert int(store.add("nd_ns/inc/0", 0)) == 3 and int(store.add("nd_ns/inc/2", 0)) == 1


def test_worker_group_namespace_ignores_stale_keys():
    """A dead group's leftovers (a request pointer and an acknowledgement carrying another nonce) are never
    taken for the new group's handshake; every member of the new group agrees on rank 0's nonce."""
    import threading

    import torch.distributed as dist
    store = dist.HashStore()
    store.set("nd_ns/req/1", "7")              # leftover of a dead rank 1 (incarnation 7 never existed here)
    store.set("nd_ns/ack/1/7", "stale-nonce")
    store.set("nd_ns/ans/2/1", "stale-answer")  # a stale answer under a key the NEW rank 2 will not read
    store.add("nd_ns/inc/2", 1)                 # rank 2 had one incarnation before
    res = {}

    def member(r):
        res[r] = D.worker_group_namespace(store, r, 3, timeout_s=30)

    th = [threading.Thread(target=member, args=(r,)) for r in (1, 2)]
    for t in th:
        t.start()
    res[0] = D.worker_group_namespace(store, 0, 3, timeout_s=30)
    for t in th:
        t.join(30)
    assert res[0] == res[1] == res[2] and "stale" not in res[0], res
