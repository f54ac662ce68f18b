"""Own RCCL communicator (``_lib/libnd_comm.so``, csrc/comm/nd_comm.cpp), SURVEY.md §5.8.

Reference: ``dist.broadcast`` / ``dist.all_reduce(AVG)`` per parameter tensor on torch's NCCL process
group (REF/nanodiloco/diloco/diloco.py:21-22, 49; REF/nanodiloco/training_utils/utils.py:42).

Here each process group that carries DiLoCo traffic gets its own ``ncclComm_t``:

* bootstrap: rank 0 of the group calls ``ncclGetUniqueId`` and publishes the 128 bytes through the
  c10d store that torchrun's rendezvous already set up (key = the group's global ranks + a per-group
  sequence number, so the keys of two groups never collide); every member then runs
  ``ncclCommInitRank`` -- no extra process group, no torch ProcessGroupNCCL involved;
* collectives run in place on the communicator's own high-priority HIP stream, ordered after the
  producer stream's queued work by an event; ``wait(ticket)`` makes a consumer stream wait on the GPU
  (the host never blocks);
* the communicator is non-blocking: ``ncclCommInitRankConfig`` waits for the other members at most
  ``init_timeout_s`` (a member that never joins -> :class:`RcclError`, not a hang);
* a watchdog thread in the library aborts the communicator when a collective outlives the collective
  timeout or RCCL reports an asynchronous error; every later call raises :class:`RcclError`, and
  :meth:`RcclCommunicator.check` raises it at the step boundaries that KEEP reduced data (the outer
  update, the inner-DDP gradient, a checkpoint): an aborted collective's completion event still fires, so
  without the check a partially reduced buffer could reach the weights or a checkpoint;
* ``destroy(abort=True)`` (an exception is propagating) aborts at once; a normal destroy drains the
  communicator stream within the collective timeout and aborts if that fails.

The torch process group stays for the control plane (barriers, the bench's MAX reduction, the debug
replica checksums); the bulk traffic -- initial broadcast, outer all-reduce buckets, inner-DDP gradient
spans, two-level all-gathers -- goes through this communicator.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_lib", "libnd_comm.so")

_DTYPES = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.float64: 8, torch.int32: 2,
           torch.int64: 4, torch.uint8: 1, torch.int8: 0}
SUM = 0

_lib = None
_lock = threading.Lock()


class RcclError(RuntimeError):
    pass


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RcclError(f"{LIB_PATH} missing: build it with `python -m nanodiloco_amd.csrc.build`")
                l = ctypes.CDLL(LIB_PATH)
                P, I, L64, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
                sig = {
                    "nd_comm_unique_id_bytes": [],
                    "nd_comm_get_unique_id": [P],
                    "nd_comm_init": [ctypes.POINTER(P), I, P, I, I, I, ctypes.c_double],
                    "nd_comm_init2": [ctypes.POINTER(P), I, P, I, I, I, ctypes.c_double, ctypes.c_double],
                    "nd_comm_destroy": [P],
                    "nd_comm_destroy2": [P, I],
                    "nd_comm_abort": [P],
                    "nd_comm_all_reduce": [P, P, P, SZ, I, I, P, ctypes.POINTER(L64)],
                    "nd_comm_broadcast": [P, P, SZ, I, I, P, ctypes.POINTER(L64)],
                    "nd_comm_all_gather": [P, P, SZ, I, P, ctypes.POINTER(L64)],
                    "nd_comm_wait": [P, L64, P],
                    "nd_comm_query": [P, L64],
                    "nd_comm_error": [P],
                    "nd_comm_stats": [P, ctypes.POINTER(L64), ctypes.POINTER(L64), ctypes.POINTER(P),
                                      ctypes.POINTER(I)],
                    "nd_comm_version": [],
                }
                for name, args in sig.items():
                    f = getattr(l, name)
                    f.argtypes = args
                    f.restype = I
                l.nd_comm_error_string.argtypes = [I]
                l.nd_comm_error_string.restype = ctypes.c_char_p
                _lib = l
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        raise RcclError(f"{what}: {lib().nd_comm_error_string(rc).decode()} (code {rc})")


def _stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _group_ranks(group) -> List[int]:
    if group is None or group is dist.group.WORLD:
        return list(range(dist.get_world_size()))
    return dist.get_process_group_ranks(group)


_SEQ: Dict[Tuple[int, ...], int] = {}


class RcclCommunicator:
    """One ``ncclComm_t`` for the members of ``group`` (torch process group or None = WORLD)."""

    def __init__(self, group, device: torch.device, timeout_s: float = 1800.0, high_priority: bool = True,
                 store=None, init_timeout_s: Optional[float] = None):
        L = lib()
        self.device = device
        self.ranks = _group_ranks(group)
        self.size = len(self.ranks)
        self.rank = self.ranks.index(dist.get_rank())
        key_ranks = tuple(self.ranks)
        seq = _SEQ.get(key_ranks, 0)
        _SEQ[key_ranks] = seq + 1
        key = f"nd_rccl/{'-'.join(map(str, key_ranks))}/{seq}"
        st = store if store is not None else dist.distributed_c10d._get_default_store()
        nbytes = L.nd_comm_unique_id_bytes()
        if self.rank == 0:
            buf = ctypes.create_string_buffer(nbytes)
            _check(L.nd_comm_get_unique_id(buf), "ncclGetUniqueId")
            uid = buf.raw
            st.set(key, uid)
        else:
            uid = bytes(st.get(key))  # blocks until the group's rank 0 has published it (store timeout)
        if len(uid) != nbytes:
            raise RcclError(f"bad unique id for {key}: {len(uid)} bytes")
        self._h = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(uid, nbytes)
        dev_index = device.index if device.type == "cuda" and device.index is not None else 0
        if os.environ.get("ND_COMM_PRIORITY", "high") == "normal":  # A/B of the stream priority
            high_priority = False
        self.key = key
        rc = L.nd_comm_init2(ctypes.byref(self._h), self.size, idbuf, self.rank, dev_index, int(high_priority),
                             float(timeout_s), float(init_timeout_s if init_timeout_s is not None else timeout_s))
        if rc != 0:
            self._h = None
            _check(rc, f"ncclCommInitRankConfig({key})")

    # ------------------------------------------------------------------ collectives (in place, async)
    def all_reduce(self, t: torch.Tensor) -> int:
        """SUM over the group into ``t`` (contiguous, in place).  Returns the ticket to ``wait`` on."""
        return self._issue("all_reduce", t, lambda tk: lib().nd_comm_all_reduce(
            self._h, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()), t.numel(), _DTYPES[t.dtype], SUM,
            _stream(self.device), tk))

    def broadcast(self, t: torch.Tensor, root: int = 0) -> int:
        return self._issue("broadcast", t, lambda tk: lib().nd_comm_broadcast(
            self._h, ctypes.c_void_p(t.data_ptr()), t.numel(), _DTYPES[t.dtype], int(root), _stream(self.device), tk))

    def all_gather(self, out: torch.Tensor) -> int:
        """In place: member r's contribution is ``out.view(size, -1)[r]``; afterwards all parts are everywhere."""
        if out.numel() % self.size:
            raise ValueError("all_gather: numel not divisible by the group size")
        return self._issue("all_gather", out, lambda tk: lib().nd_comm_all_gather(
            self._h, ctypes.c_void_p(out.data_ptr()), out.numel() // self.size, _DTYPES[out.dtype], _stream(self.device),
            tk))

    def _issue(self, what, t, fn) -> int:
        if not t.is_contiguous() or t.device != self.device:
            raise ValueError(f"{what}: needs a contiguous tensor on {self.device}")
        if self._h is None:
            raise RcclError(f"{what}: communicator destroyed")
        tk = ctypes.c_int64(-1)
        _check(fn(ctypes.byref(tk)), f"rccl {what} ({self.key})")
        return tk.value

    def wait(self, ticket: int):
        """The CURRENT stream waits (GPU side) for collective ``ticket``."""
        _check(lib().nd_comm_wait(self._h, int(ticket), _stream(self.device)), f"rccl wait ({self.key})")

    def query(self, ticket: int) -> bool:
        rc = lib().nd_comm_query(self._h, int(ticket))
        if rc not in (0, 1):
            _check(rc, f"rccl query ({self.key})")
        return rc == 1

    def stats(self) -> dict:
        calls, nbytes, stream, prio = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_void_p(), ctypes.c_int()
        _check(lib().nd_comm_stats(self._h, ctypes.byref(calls), ctypes.byref(nbytes), ctypes.byref(stream),
                                   ctypes.byref(prio)), "rccl stats")
        return {"calls": calls.value, "bytes": nbytes.value, "stream": stream.value, "priority": prio.value}

    def error(self) -> int:
        return lib().nd_comm_error(self._h) if self._h is not None else 0

    def check(self, what: str = "step boundary"):
        """Raise if the communicator has failed (watchdog timeout, async RCCL error, abort).  Called where
        reduced data is about to be kept: an aborted collective still completes its event, so the GPU-side
        waits alone cannot tell a full reduction from a partial one."""
        rc = self.error()
        if rc != 0:
            raise RcclError(f"rccl communicator {self.key} failed before {what}: "
                            f"{lib().nd_comm_error_string(rc).decode()} (code {rc})")

    def abort(self):
        if self._h is not None:
            lib().nd_comm_abort(self._h)

    def destroy(self, abort: bool = False):
        """``abort``: an exception is propagating (or a peer is known dead): no drain, abort at once."""
        if self._h is not None and self._h.value:
            lib().nd_comm_destroy2(self._h, int(abort))
        self._h = None

    def __del__(self):  # best effort; processes normally call destroy_communicators() first
        try:
            self.destroy()
        except Exception:
            pass


# one communicator per distinct group (outer / inner / world FlatCommunicators may share a group)
_COMMS: Dict[Tuple[int, ...], RcclCommunicator] = {}


def communicator_for(group, device: torch.device, timeout_s: float = 1800.0,
                     high_priority: bool = True) -> RcclCommunicator:
    key = tuple(_group_ranks(group))
    c = _COMMS.get(key)
    if c is None:
        c = RcclCommunicator(group, device, timeout_s, high_priority)
        _COMMS[key] = c
    return c


def init_timeout_s(default: float = 300.0) -> float:
    """How long a communicator's bootstrap may wait for its peers (``ND_COMM_INIT_TIMEOUT``, seconds).
    RCCL's init takes seconds on one node; a bounded wait turns a peer that never joins into an error the
    group can agree on (:func:`communicator_or_fallback`) instead of a job that hangs until its own limit."""
    return float(os.environ.get("ND_COMM_INIT_TIMEOUT", default))


def communicator_or_fallback(group, device: torch.device, timeout_s: float = 1800.0,
                             high_priority: bool = True) -> Optional[RcclCommunicator]:
    """The group's own communicator, or None when ANY member failed to create it -- decided together.

    Every member tries ``communicator_for`` (bounded by :func:`init_timeout_s`), then the members take the
    MIN of their success flags over the torch process group of ``group`` (the control plane, which already
    works: it carried the unique id).  If one member failed, all of them drop the own communicator and the
    caller moves its bulk traffic to c10d, so no member is left issuing RCCL calls its peers never join.
    ``ND_COMM_FALLBACK=0`` makes a failure fatal instead (strict A/B runs)."""
    err: Optional[BaseException] = None
    c: Optional[RcclCommunicator] = None
    key = tuple(_group_ranks(group))
    try:
        c = _COMMS.get(key)
        if c is None:
            c = RcclCommunicator(group, device, timeout_s, high_priority, init_timeout_s=init_timeout_s())
            _COMMS[key] = c
    except (RcclError, OSError) as e:
        err, c = e, None
    if os.environ.get("ND_COMM_FALLBACK", "1") == "0" and err is not None:
        raise err
    flag_dev = device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    ok = torch.tensor([0 if c is None else 1], dtype=torch.int32, device=flag_dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if int(ok.item()) == 1:
        return c
    if c is not None:  # a peer failed: this member's communicator has no partner to talk to
        c.destroy(abort=True)
        _COMMS.pop(key, None)
    import warnings
    warnings.warn(f"own RCCL communicator for ranks {list(key)} unavailable "
                  f"({'here: ' + str(err) if err is not None else 'on a peer'}); bulk traffic falls back to c10d")
    return None


def destroy_communicators(abort: bool = False):
    for c in list(_COMMS.values()):
        c.destroy(abort)
    _COMMS.clear()


def version() -> Optional[int]:
    try:
        return int(lib().nd_comm_version())
    except (RcclError, OSError):
        return None
