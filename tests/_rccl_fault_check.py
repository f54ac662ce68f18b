"""Failure paths of the own RCCL communicator on ONE GPU (run by tests/test_rccl_gpu.py in its own process,
under a time limit; SURVEY.md §5.3, csrc/comm/nd_comm.cpp).

1. A 2-rank communicator in which only rank 0 ever joins: the non-blocking ``ncclCommInitRankConfig`` must
   return the timeout error within ``init_timeout_s`` + 5 s (the reference's blocking NCCL init,
   REF/nanodiloco/training_utils/utils.py:42, would wait forever), and the process must go on working.
2. A one-rank communicator still works afterwards: bucketed in-place all-reduce, GPU-side wait.
3. ``abort()`` from the host: every later call raises, ``check()`` raises, ``destroy(abort=True)`` returns.
4. A normal destroy of a healthy communicator drains and returns.
The process then exits 0 (no thread of the aborted init keeps it alive).
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nanodiloco_amd.parallel import rccl  # noqa: E402

INIT_TIMEOUT = float(os.environ.get("ND_FAULT_INIT_TIMEOUT", "6"))


def check(cond, what):
    if not cond:
        raise SystemExit(f"FAIL: {what}")
    print(f"ok: {what}", flush=True)


def new_id():
    L = rccl.lib()
    buf = ctypes.create_string_buffer(L.nd_comm_unique_id_bytes())
    rccl._check(L.nd_comm_get_unique_id(buf), "ncclGetUniqueId")
    return buf


def main():
    torch.cuda.init()
    L = rccl.lib()
    dev = torch.device("cuda", 0)

    # 1. peer never joins
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    rc = L.nd_comm_init2(ctypes.byref(h), 2, new_id(), 0, 0, 1, 30.0, INIT_TIMEOUT)
    dt = time.perf_counter() - t0
    print(f"2-rank init with a missing peer: rc={rc} ({L.nd_comm_error_string(rc).decode()}) after {dt:.2f} s",
          flush=True)
    check(rc == -3, "init with a peer that never joins returns the timeout error")
    check(INIT_TIMEOUT - 0.5 <= dt <= INIT_TIMEOUT + 5.0, f"... within init_timeout + 5 s ({dt:.2f} s)")
    check(not h.value, "... and hands back no communicator")

    # 2. a one-rank communicator still works
    uid = new_id()
    h1 = ctypes.c_void_p()
    rccl._check(L.nd_comm_init2(ctypes.byref(h1), 1, uid, 0, 0, 1, 30.0, INIT_TIMEOUT), "one-rank init")
    x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
    ref = x.clone()
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    tk = ctypes.c_int64(-1)
    for a in range(0, x.numel(), 1 << 18):
        seg = x[a:a + (1 << 18)]
        rccl._check(L.nd_comm_all_reduce(h1, ctypes.c_void_p(seg.data_ptr()), ctypes.c_void_p(seg.data_ptr()),
                                         seg.numel(), 7, 0, st, ctypes.byref(tk)), "all_reduce")
    rccl._check(L.nd_comm_wait(h1, tk.value, st), "wait")
    torch.cuda.synchronize()
    check(torch.equal(x, ref), "one-rank bucketed all-reduce after the failed init")

    # 3. host abort: sticky error, calls fail, check raises, abort-destroy returns
    check(L.nd_comm_error(h1) == 0, "healthy before abort")
    rccl._check(L.nd_comm_abort(h1), "abort")
    check(L.nd_comm_error(h1) == -2, "sticky 'aborted' error")
    rc = L.nd_comm_all_reduce(h1, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()), 1024, 7, 0, st,
                              ctypes.byref(tk))
    check(rc == -2, "a collective after abort returns the error instead of running")
    t0 = time.perf_counter()
    L.nd_comm_destroy2(h1, 1)
    check(time.perf_counter() - t0 < 10.0, "destroy(abort) returns promptly")

    # the Python wrapper: check() raises once failed; destroy(abort=True)
    c = rccl.RcclCommunicator.__new__(rccl.RcclCommunicator)
    h2 = ctypes.c_void_p()
    rccl._check(L.nd_comm_init2(ctypes.byref(h2), 1, new_id(), 0, 0, 1, 30.0, INIT_TIMEOUT), "one-rank init (2)")
    c._h, c.key, c.device = h2, "fault-check", dev
    c.check("healthy")
    c.abort()
    try:
        c.check("after abort")
        raise SystemExit("FAIL: check() did not raise after abort")
    except rccl.RcclError as e:
        print(f"ok: check() raises after abort ({e})", flush=True)
    c.destroy(abort=True)

    # 4. healthy normal destroy
    h3 = ctypes.c_void_p()
    rccl._check(L.nd_comm_init2(ctypes.byref(h3), 1, new_id(), 0, 0, 1, 30.0, INIT_TIMEOUT), "one-rank init (3)")
    rccl._check(L.nd_comm_all_reduce(h3, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()), x.numel(), 7,
                                     0, st, ctypes.byref(tk)), "all_reduce (3)")
    t0 = time.perf_counter()
    check(L.nd_comm_destroy2(h3, 0) == 0, "normal destroy drains and returns ok")
    check(time.perf_counter() - t0 < 10.0, "... promptly")
    print("RCCL_FAULT_CHECK_PASSED", flush=True)


if __name__ == "__main__":
    main()
