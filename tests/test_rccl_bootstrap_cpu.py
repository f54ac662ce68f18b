"""Bootstrap of the own RCCL communicator (parallel/rccl.py) on CPU: rank 0 of each group publishes its
ncclUniqueId through the c10d store and every member reads the same 128 bytes -- checked with 4 gloo
ranks, overlapping groups (world, two inner pairs, two outer pairs) and a fake library in place of
libnd_comm.so (no GPU here; the real communicator runs in tests/_rccl_check.py on the GPU box)."""
import ctypes

from ._mp import run_ranks


class _FakeFn:
    def __init__(self, fn):
        self.fn = fn

    def __call__(self, *a):
        return self.fn(*a)


class _FakeLib:
    """Stands in for libnd_comm.so: unique ids encode (creating rank, call #); init records what it got."""

    def __init__(self, rank):
        self.rank, self.n, self.inits = rank, 0, []
        self.nd_comm_unique_id_bytes = _FakeFn(lambda: 128)
        self.nd_comm_get_unique_id = _FakeFn(self._uid)
        self.nd_comm_init2 = _FakeFn(self._init)
        self.nd_comm_destroy2 = _FakeFn(lambda h, abort: 0)

    def _uid(self, buf):
        self.n += 1
        raw = f"uid-r{self.rank}-n{self.n}".encode().ljust(128, b"\0")
        ctypes.memmove(buf, raw, 128)
        return 0

    def _init(self, handle, nranks, idbuf, rank, device, hp, timeout, init_timeout):
        self.inits.append((nranks, rank, bytes(idbuf.raw).rstrip(b"\0").decode()))
        handle._obj.value = 1
        return 0


def _bootstrap(rank, world):
    import torch
    import torch.distributed as dist

    from nanodiloco_amd.parallel import rccl

    dist.init_process_group("gloo")
    fake = _FakeLib(rank)
    rccl._lib = fake
    try:
        inner = [dist.new_group([0, 1]), dist.new_group([2, 3])]
        outer = [dist.new_group([0, 2]), dist.new_group([1, 3])]
        dev = torch.device("cpu")
        cw = rccl.communicator_for(None, dev)
        ci = rccl.communicator_for(inner[rank // 2], dev)
        co = rccl.communicator_for(outer[rank % 2], dev)
        again = rccl.communicator_for(None, dev)  # cached: no second init for the same group
        out = {"inits": fake.inits, "ranks": [cw.rank, ci.rank, co.rank], "same": again is cw}
        for c in (cw, ci, co):
            c._h = None  # nothing to destroy in the fake
        rccl._COMMS.clear()
        return out
    finally:
        rccl._lib = None


def test_unique_id_exchange_through_store_4_ranks():
    res = run_ranks(_bootstrap, 4)
    for r, o in enumerate(res):
        assert o["same"] and len(o["inits"]) == 3, o
        assert o["ranks"] == [r, r % 2, r // 2], o
        (nw, rw, uw), (ni, ri, ui), (no, ro, uo) = o["inits"]
        assert (nw, ni, no) == (4, 2, 2) and (rw, ri, ro) == (r, r % 2, r // 2)
        assert uw == "uid-r0-n1"                      # world: created by rank 0
        assert ui == ("uid-r0-n2" if r < 2 else "uid-r2-n1")  # inner pair: its first member
        assert uo.startswith(f"uid-r{r % 2}-")         # outer pair: its first member
    # every member of a group got the same id
    assert res[0]["inits"][1][2] == res[1]["inits"][1][2] and res[2]["inits"][1][2] == res[3]["inits"][1][2]
    assert res[0]["inits"][2][2] == res[2]["inits"][2][2] and res[1]["inits"][2][2] == res[3]["inits"][2][2]


def _fallback(rank, world, fail_rank):
    import torch
    import torch.distributed as dist

    from nanodiloco_amd.parallel import rccl
    from nanodiloco_amd.parallel.comm import FlatCommunicator

    dist.init_process_group("gloo")
    fake = _FakeLib(rank)
    destroyed = []
    fake.nd_comm_destroy2 = _FakeFn(lambda h, abort: destroyed.append(int(abort)) or 0)
    if rank == fail_rank:  # this member's bootstrap fails (e.g. its peers never joined in time)
        fake.nd_comm_init2 = _FakeFn(lambda *a: 7)
        fake.nd_comm_error_string = _FakeFn(lambda rc: b"fake init failure")
    rccl._lib = fake
    try:
        fc = FlatCommunicator(None, world, bucket_mb=1.0, impl="rccl", device=torch.device("cpu"))
        x = torch.full((1000,), float(rank + 1))
        if fc.rccl is None:  # agreed fallback: the bulk traffic really runs on c10d (gloo here)
            fc.all_reduce(x)
        out = {"impl": fc.impl, "has_rccl": fc.rccl is not None, "sum": float(x[0]), "destroyed": destroyed,
               "cached": len(rccl._COMMS)}
        if fc.rccl is not None:
            fc.rccl._h = None
        rccl._COMMS.clear()
        return out
    finally:
        rccl._lib = None


def test_failed_bootstrap_on_one_member_moves_every_member_to_c10d():
    res = run_ranks(_fallback, 3, 1)
    for o in res:
        assert o["impl"] == "c10d" and not o["has_rccl"] and o["cached"] == 0, o
        assert o["sum"] == 6.0, o  # 1 + 2 + 3 through gloo
    assert res[0]["destroyed"] == [1] and res[2]["destroyed"] == [1]  # survivors aborted their communicator
    assert res[1]["destroyed"] == []


def test_successful_bootstrap_keeps_own_communicator():
    res = run_ranks(_fallback, 2, -1)
    assert all(o["impl"] == "rccl" and o["has_rccl"] for o in res), res
