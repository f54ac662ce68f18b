"""Multi-process CPU harness: W gloo ranks on 127.0.0.1 via torch.multiprocessing."""
import os
import socket
import traceback

import torch.multiprocessing as mp


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child_env(**kw):
    """Environment of a test's child process: the repo first on PYTHONPATH, the parent's entries KEPT after
    it (appended, not replaced -- a harness that injects its own path entries, e.g. to observe which native
    libraries the children load, must still see them), plus ``kw``."""
    pp = os.environ.get("PYTHONPATH", "")
    env = dict(os.environ, PYTHONPATH=ROOT + (os.pathsep + pp if pp else ""))
    env.update({k: str(v) for k, v in kw.items()})
    return env


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def run_ranks(fn, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
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
        p.join(timeout)
    return [out[r] for r in range(world)]
