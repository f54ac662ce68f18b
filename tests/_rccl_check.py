"""RCCL path on ONE GPU (run by tests/test_rccl_gpu.py in its own process, under a time limit).

The round-end scaling run is the only place several RCCL ranks meet; a one-GPU box cannot host two.
A one-rank ``nccl`` process group (``init_distributed(force_pg=True)``) with every collective forced
on still runs the real code: the eager communicator init (``device_id``), ``Work.wait()`` stream
semantics of the bucketed async all-reduce, broadcast, ``all_gather_into_tensor`` on a sub-group, the
device barrier, a whole Diloco outer step (pipelined and overlapped) and inner-DDP layer hooks that
launch RCCL collectives from the autograd thread.  With one rank every SUM is the identity, so each
result must equal, bit for bit, the same computation with the collectives off and over gloo.
(Reference collectives: REF/nanodiloco/diloco/diloco.py:21-22,49; backend REF/.../utils.py:42.)
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nanodiloco_amd.models import LlamaForCausalLM  # noqa: E402
from nanodiloco_amd.optim import FlatAdamW, FlatOuterNesterov  # noqa: E402
from nanodiloco_amd.parallel.comm import FlatCommunicator  # noqa: E402
from nanodiloco_amd.parallel.diloco import Diloco  # noqa: E402
from nanodiloco_amd.parallel.dist import DistEnv, barrier, init_distributed  # noqa: E402
from nanodiloco_amd.parallel.inner_ddp import InnerGradSync  # noqa: E402
from nanodiloco_amd.config import LlamaConfig  # noqa: E402

BACKEND = sys.argv[1] if len(sys.argv) > 1 else "nccl"  # "gloo": the same checks on CPU (tests/test_force_pg_cpu.py)
CPU = BACKEND == "gloo"


def sync():
    if not CPU:
        torch.cuda.synchronize()


CFG = dict(hidden_size=256, intermediate_size=512, num_attention_heads=4, num_hidden_layers=3, vocab_size=1000,
           rms_norm_eps=1e-5)


def check(cond, what):
    if not cond:
        raise SystemExit(f"FAIL: {what}")
    print(f"ok: {what}", flush=True)


def train_run(env, overlap, steps=3, H=2, comm_dtype=torch.float32):
    """A few inner steps + outer steps of a small bf16 Llama on the HIP path; returns master, sync."""
    dev = env.device
    model = LlamaForCausalLM(LlamaConfig(**CFG), dev, torch.float32 if CPU else torch.bfloat16).init_weights(7)
    inner = FlatAdamW(model.store, lr=1e-3)
    outer = FlatOuterNesterov(model.store, lr=0.7, momentum=0.9)
    dl = Diloco(model, inner, outer, warmup_steps=1, total_steps=100, inner_steps=H, env=env, comm_dtype=comm_dtype,
                bucket_mb=0.25, overlap=overlap)
    isync = InnerGradSync(model, dl.inner_comm)
    g = torch.Generator(device="cpu").manual_seed(3)
    hooks = []
    for s in range(steps * H):
        ids = torch.randint(0, CFG["vocab_size"], (2, 32 if CPU else 128), generator=g).to(dev)
        isync.arm()
        out = model(ids, labels=ids, loss_scale=1.0)
        out.loss.backward()
        isync.finish()
        hooks.append(isync.last_hook_count)
        dl.inner_step()
        if (s + 1) % H == 0:
            dl.outer_step()
    dl.finalize()
    sync()
    return model.store.master.clone(), dl.sync.clone(), hooks, dl


def gloo_cuda_ok(group, dev) -> bool:
    try:
        t = torch.ones(4, device=dev)
        dist.all_reduce(t, group=group)
        sync()
        return True
    except RuntimeError as e:  # a gloo build without GPU-tensor collectives
        print(f"note: gloo rejects GPU tensors here ({str(e)[:80]}); gloo comparisons use host copies")
        return False


def main():
    from nanodiloco_amd import ops
    ops.set_deterministic(True)  # no float atomics: two runs of the same step are bitwise equal
    env = init_distributed(BACKEND, device="cpu" if CPU else None, force_pg=True)
    env.force_inner_ddp = True  # exercise the inner-DDP hooks on RCCL too (off in the trainer / bench)
    dev = env.device
    check(dist.is_initialized() and dist.get_backend() == BACKEND and env.backend == BACKEND,
          f"one-rank {BACKEND} group")
    check(env.force_collectives and env.is_distributed, "collectives forced on at world size 1")
    if not CPU:
        from nanodiloco_amd.parallel.dist import comm_stream_high_priority
        hp = comm_stream_high_priority()
        check(hp is True, f"RCCL collectives on a high-priority stream (got {hp})")

    # ---- bucketed async all-reduce, per-bucket waits on the compute stream
    comm = FlatCommunicator(None, 1, bucket_mb=1.0, force=True)
    x = torch.randn(3_000_000 // (8 if CPU else 1), device=dev)
    ref = x.clone()
    p = comm.all_reduce_async(x)
    nb = -(-x.numel() * 4 // (1 << 20))
    check(len(p) == nb and comm.stats.calls == nb, f"{nb} buckets of 1 MiB issued async")
    for i in range(len(p)):
        p.wait(i)
    y = x * 2  # consumer on the compute stream, ordered after the waits only
    sync()
    check(torch.equal(x, ref) and torch.equal(y, ref * 2), "all-reduce SUM over one rank is exact")
    gloo = dist.new_group(backend="gloo")
    gpu_gloo = gloo_cuda_ok(gloo, dev)
    xg = ref.clone() if gpu_gloo else ref.cpu()
    dist.all_reduce(xg, group=gloo)
    check(torch.equal(xg.to(dev), x), "nccl result == gloo result")

    # ---- broadcast + all_gather_into_tensor on a sub-group + device barrier
    sub = dist.new_group([0])
    c2 = FlatCommunicator(sub, 1, bucket_mb=0.01, force=True)
    b = torch.arange(40_000, device=dev, dtype=torch.float32)
    b0 = b.clone()
    c2.broadcast(b, 0)
    c2.all_gather_flat(b, [(0, 40_000)], 0)
    barrier(env)
    sync()
    check(torch.equal(b, b0), "bucketed broadcast + sub-group all-gather")

    # ---- the own RCCL communicator (parallel/rccl.py, csrc/comm/nd_comm.cpp): bucketed in-place all-reduce
    # with GPU-side waits, broadcast, in-place all-gather, its high-priority stream, the c10d result
    if not CPU:
        from nanodiloco_amd.parallel import rccl
        check(env.comm_impl == "rccl", f"own RCCL communicator selected by default (got {env.comm_impl})")
        oc = FlatCommunicator(None, 1, bucket_mb=1.0, force=True, impl="rccl", device=dev, timeout_s=120.0)
        check(oc.rccl is not None and oc.rccl.size == 1, "own communicator initialised (ncclCommInitRank via the store)")
        x2 = ref.clone()
        p2 = oc.all_reduce_async(x2)
        for i in range(len(p2)):
            p2.wait(i)
        y2 = x2 * 2
        sync()
        check(len(p2) == nb and torch.equal(x2, ref) and torch.equal(y2, ref * 2), "own RCCL bucketed all-reduce exact")
        st = oc.rccl.stats()
        lo, hi = torch.cuda.Stream.priority_range()
        check(st["calls"] >= nb and st["priority"] == hi, f"own RCCL stream at the highest priority ({st})")
        b2 = torch.arange(40_000, device=dev, dtype=torch.float32)
        oc.broadcast(b2, 0)
        oc.all_gather_flat(b2, [(0, 40_000)], 0)
        sync()
        check(torch.equal(b2, b0) and all(p2.works[i].is_completed() for i in range(len(p2))),
              "own RCCL broadcast + in-place all-gather")
        # the consumer really waits for the collective: a long all-reduce followed at once by a consumer kernel
        big = torch.ones(64 << 20, device=dev)
        t = oc.rccl.all_reduce(big)
        oc.rccl.wait(t)
        s2 = big.sum()
        check(float(s2.item()) == float(64 << 20) and oc.rccl.error() == 0, "consumer ordered after the collective")
        check(rccl.version() is not None and rccl.version() > 0, f"RCCL version {rccl.version()}")
        cc = DistEnv(device=dev, backend="nccl", force_collectives=True, comm_impl="c10d", force_inner_ddp=True)
        m_r, s_r, _, dlr = train_run(env, False)
        m_c, s_c, _, dlc = train_run(cc, False)
        check(dlr.outer_comm.impl == "rccl" and dlc.outer_comm.impl == "c10d", "Diloco on own RCCL vs c10d")
        check(torch.equal(m_r, m_c) and torch.equal(s_r, s_c), "own RCCL == c10d ProcessGroupNCCL, bitwise")

    # ---- Diloco outer steps (pipelined and overlapped) + inner-DDP hooks from the autograd thread
    off = DistEnv(device=dev)  # collectives off: the oracle
    gl = DistEnv(device=dev, backend="gloo", force_collectives=True, force_inner_ddp=True, inner_group=gloo,
                 outer_group=gloo,
                 world_group=gloo)
    for overlap in (False, True):
        m_nc, s_nc, hooks, dl = train_run(env, overlap)
        m_off, s_off, _, _ = train_run(off, overlap)
        m_gl, s_gl, _, _ = train_run(gl, overlap) if gpu_gloo else (m_off, s_off, None, None)
        check(dl.outer_comm.enabled and dl.outer_comm.stats.calls > 0 and dl.inner_comm.stats.calls > 0,
              f"overlap={overlap}: outer and inner collectives issued on RCCL ({dl.outer_comm.impl})")
        check(all(h == CFG["num_hidden_layers"] for h in hooks), f"overlap={overlap}: every layer hook fired")
        check(torch.equal(m_nc, m_off) and torch.equal(s_nc, s_off), f"overlap={overlap}: RCCL == no-comm, bitwise")
        check(torch.equal(m_nc, m_gl) and torch.equal(s_nc, s_gl), f"overlap={overlap}: RCCL == gloo, bitwise")
    # bf16 pseudo-gradient transport
    m_b, _, _, _ = train_run(env, False, comm_dtype=torch.bfloat16)
    m_bo, _, _, _ = train_run(off, False, comm_dtype=torch.bfloat16)
    check(torch.equal(m_b, m_bo), "bf16 transport: RCCL == no-comm, bitwise")

    # ---- phased outer step: per-phase HIP-event spans
    _, _, _, dl = train_run(env, False, steps=1)
    dl.outer_step(phases=True)
    ph = dl.outer_phase_ms()
    check(CPU and ph == {} or set(ph) == {"pseudograd_ms", "allreduce_ms", "outer_update_ms"} and all(v >= 0 for v in ph.values()),
          f"outer phase spans {ph}")
    from nanodiloco_amd.parallel.dist import destroy_distributed
    destroy_distributed()
    print("RCCL_CHECK_PASSED", flush=True)


if __name__ == "__main__":
    main()
