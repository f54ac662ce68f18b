// Own RCCL communicator: one ncclComm_t per process group, driven from Python through
// a plain C ABI (parallel/rccl.py), outside torch's ProcessGroupNCCL.
//
// Reference role: the two collective call sites of REF/nanodiloco/diloco/diloco.py -- the initial
// per-tensor dist.broadcast (:21-22) and the outer step's per-tensor dist.all_reduce(AVG) (:49), on the
// NCCL process group of REF/nanodiloco/training_utils/utils.py:42.  Here they become a few large
// in-place collectives on flat buffers (bucketed by the caller).
//
// Stream model (MI355X, RCCL over xGMI):
//   * every communicator owns ONE high-priority HIP stream; a collective is ordered after the work
//     already queued on the caller's (producer) stream by an event, runs on the communicator stream,
//     and records a completion event -- the producer stream is never blocked and the host never waits;
//   * a consumer stream waits for one collective with nd_comm_wait(ticket) (a GPU-side event wait):
//     bucket i's consumer kernel then overlaps the reduction of bucket i + 1;
//   * all collectives are in place (all-gather: send = recv + rank * count), so no temporary buffer
//     is shared between the caching allocator's stream and the communicator stream.
//
// Failure detection (a dead peer must surface as an error on every rank, never a hang):
//   * the communicator is NON-BLOCKING (ncclConfig_t.blocking = 0): ncclCommInitRankConfig and every
//     collective return at once (ncclSuccess or ncclInProgress) and the caller polls
//     ncclCommGetAsyncError against a deadline -- a peer that never joins makes nd_comm_init return
//     ND_E_TIMEOUT after init_timeout_s instead of blocking forever in the bootstrap;
//   * three locks, none held across an unbounded wait:
//       mu      -- issue order (producer event, enqueue, completion event, ticket); issuers only;
//       pend_mu -- the outstanding-collective list (issuers append, the watchdog retires);
//       life_mu -- the ncclComm_t's lifetime: every NCCL call (each returns promptly in non-blocking
//                  mode), ncclCommGetAsyncError, ncclCommAbort, and the pointer swap to nullptr;
//     so the watchdog never waits behind an issuer that is polling an in-progress call, and an issuer
//     polling an in-progress call gives up as soon as the watchdog (or nd_comm_abort) has failed the
//     communicator;
//   * a watchdog thread per communicator retires completed collectives (hipEventQuery, no NCCL call)
//     and polls the asynchronous error state; a collective older than the timeout, or an async error,
//     fails the communicator: the sticky error is set first (issuers stop), then ncclCommAbort releases
//     the kernels spinning on dead / stuck peers, and every later call returns the error, which Python
//     raises (and checks at the outer-step / inner-DDP / checkpoint boundaries, parallel/rccl.py);
//   * nd_comm_destroy waits for the communicator stream with the same timeout, the watchdog still
//     running, and aborts instead of syncing forever when that wait fails (or when asked to abort).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#define ND_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kRing = 1024;  // completion events kept per communicator (tickets older than this are stale)

// error codes returned to Python (>0: ncclResult_t, <0: ours)
enum : int { ND_OK = 0, ND_E_STALE = -1, ND_E_ABORTED = -2, ND_E_TIMEOUT = -3, ND_E_HIP = -4, ND_E_ARG = -5 };

using Clock = std::chrono::steady_clock;

struct Outstanding {
  int64_t ticket;
  Clock::time_point t0;
};

struct Comm {
  ncclComm_t nccl = nullptr;           // guarded by life_mu
  int device = 0, rank = 0, nranks = 1;
  hipStream_t stream = nullptr;
  hipEvent_t in_ev = nullptr;          // producer -> communicator stream ordering
  std::vector<hipEvent_t> done;        // completion event of ticket t: done[t % kRing]
  std::atomic<int64_t> next{0};        // next ticket
  std::mutex mu;                       // issue order (issuers only)
  std::mutex pend_mu;                  // the outstanding list
  std::mutex life_mu;                  // ncclComm_t lifetime: NCCL calls, async-error polls, abort
  std::deque<Outstanding> pending;     // collectives not yet seen complete by the watchdog
  std::atomic<int> err{ND_OK};         // sticky error (abort / timeout / async RCCL error)
  double timeout_s = 1800.0;
  std::thread watchdog;
  std::atomic<bool> stop{false};
  std::condition_variable cv;
  std::mutex cv_mu;
  std::atomic<int64_t> calls{0}, bytes{0};
};

int hip_ok(hipError_t e) { return e == hipSuccess ? ND_OK : ND_E_HIP; }

double secs_since(Clock::time_point t0) { return std::chrono::duration<double>(Clock::now() - t0).count(); }

// Fail the communicator: the first error sticks; issuers see it before the abort runs.  ncclCommAbort
// runs under life_mu only, which an issuer holds for one non-blocking NCCL call at most.
void fail_comm(Comm* c, int code) {
  int expect = ND_OK;
  c->err.compare_exchange_strong(expect, code);
  std::lock_guard<std::mutex> g(c->life_mu);
  if (c->nccl) ncclCommAbort(c->nccl);
  c->nccl = nullptr;
}

// Poll a non-blocking call to completion (ncclCommGetAsyncError != ncclInProgress).  Gives up when the
// communicator has failed meanwhile (watchdog / nd_comm_abort) or the deadline passes (-> timeout).
int poll_in_progress(Comm* c, double timeout_s) {
  const auto t0 = Clock::now();
  for (;;) {
    if (const int e = c->err.load(); e != ND_OK) return e;
    ncclResult_t st = ncclSuccess;
    {
      std::lock_guard<std::mutex> g(c->life_mu);
      if (!c->nccl) return c->err.load() != ND_OK ? c->err.load() : ND_E_ABORTED;
      const ncclResult_t q = ncclCommGetAsyncError(c->nccl, &st);
      if (q != ncclSuccess) st = q;
    }
    if (st == ncclSuccess) return ND_OK;
    if (st != ncclInProgress) return (int)st;
    if (secs_since(t0) > timeout_s) return ND_E_TIMEOUT;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

void watchdog_loop(Comm* c) {
  (void)hipSetDevice(c->device);
  while (!c->stop.load()) {
    {
      std::unique_lock<std::mutex> lk(c->cv_mu);
      c->cv.wait_for(lk, std::chrono::milliseconds(50));
    }
    if (c->stop.load() || c->err.load() != ND_OK) continue;
    int fail = ND_OK;
    {
      std::lock_guard<std::mutex> g(c->pend_mu);
      while (!c->pending.empty()) {
        const Outstanding& o = c->pending.front();
        const hipError_t q = hipEventQuery(c->done[o.ticket % kRing]);
        if (q == hipSuccess || c->next.load() - o.ticket > kRing) {  // done (or its event already reused)
          c->pending.pop_front();
          continue;
        }
        if (q != hipErrorNotReady) fail = ND_E_HIP;
        else if (secs_since(o.t0) > c->timeout_s) fail = ND_E_TIMEOUT;
        break;
      }
    }
    if (fail == ND_OK) {
      std::lock_guard<std::mutex> g(c->life_mu);
      ncclResult_t ae = ncclSuccess;
      if (c->nccl && ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
        fail = (int)ae;
    }
    if (fail != ND_OK) fail_comm(c, fail);
  }
}

// Enqueue one collective: `call` runs under life_mu with the live ncclComm_t; an in-progress result is
// polled (life_mu released between polls) before the completion event is recorded.  Caller holds mu.
template <class F>
int issue(Comm* c, hipStream_t producer, int64_t nbytes, int64_t* ticket, F&& call) {
  if (const int e = c->err.load(); e != ND_OK) return e;
  if (hipEventRecord(c->in_ev, producer) != hipSuccess) return ND_E_HIP;
  if (hipStreamWaitEvent(c->stream, c->in_ev, 0) != hipSuccess) return ND_E_HIP;
  ncclResult_t r;
  {
    std::lock_guard<std::mutex> g(c->life_mu);
    if (!c->nccl) return c->err.load() != ND_OK ? c->err.load() : ND_E_ABORTED;
    r = call(c->nccl);
  }
  if (r == ncclInProgress) {
    const int e = poll_in_progress(c, c->timeout_s);
    if (e != ND_OK) {
      if (e == ND_E_TIMEOUT || e > 0) fail_comm(c, e);
      return c->err.load() != ND_OK ? c->err.load() : e;
    }
  } else if (r != ncclSuccess) {
    return (int)r;
  }
  const int64_t t = c->next.load();
  if (hipEventRecord(c->done[t % kRing], c->stream) != hipSuccess) return ND_E_HIP;
  {
    std::lock_guard<std::mutex> g(c->pend_mu);
    c->pending.push_back({t, Clock::now()});
  }
  c->next.store(t + 1);
  c->calls.fetch_add(1);
  c->bytes.fetch_add(nbytes);
  *ticket = t;
  return ND_OK;
}

size_t dtype_bytes(int dt) {
  switch (dt) {
    case ncclFloat32: return 4;
    case ncclBfloat16: case ncclFloat16: return 2;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    case ncclInt32: case ncclUint32: return 4;
    case ncclInt8: case ncclUint8: return 1;
    default: return 0;
  }
}

void free_hip(Comm* c) {
  for (hipEvent_t e : c->done)
    if (e) (void)hipEventDestroy(e);
  if (c->in_ev) (void)hipEventDestroy(c->in_ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
}

}  // namespace

ND_API int nd_comm_unique_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

ND_API int nd_comm_get_unique_id(void* out) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  std::memcpy(out, &id, sizeof(id));
  return ND_OK;
}

// high_priority: the communicator stream gets the device's greatest stream priority, so its collectives
// are scheduled ahead of the compute queue's kernels when both are ready (the overlapped outer
// all-reduce beside the next inner step, the inner-DDP buckets beside the backward).
// timeout_s: collective timeout (watchdog); init_timeout_s: how long ncclCommInitRankConfig may wait for
// the other members (<= 0: timeout_s).  A member that never joins -> ND_E_TIMEOUT, nothing leaked but the
// aborted NCCL communicator's own threads.
ND_API int nd_comm_init2(void** handle, int nranks, const void* id, int rank, int device, int high_priority,
                         double timeout_s, double init_timeout_s) {
  if (!handle || !id || nranks < 1 || rank < 0 || rank >= nranks) return ND_E_ARG;
  auto* c = new Comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  c->timeout_s = timeout_s > 0 ? timeout_s : 1800.0;
  const double init_to = init_timeout_s > 0 ? init_timeout_s : c->timeout_s;
  int rc = hip_ok(hipSetDevice(device));
  int lo = 0, hi = 0;
  if (rc == ND_OK) rc = hip_ok(hipDeviceGetStreamPriorityRange(&lo, &hi));
  if (rc == ND_OK) rc = hip_ok(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, high_priority ? hi : lo));
  if (rc == ND_OK) rc = hip_ok(hipEventCreateWithFlags(&c->in_ev, hipEventDisableTiming));
  c->done.assign(kRing, nullptr);
  for (int i = 0; rc == ND_OK && i < kRing; ++i) rc = hip_ok(hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming));
  if (rc == ND_OK) {
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r;
    {
      std::lock_guard<std::mutex> g(c->life_mu);
      r = ncclCommInitRankConfig(&c->nccl, nranks, uid, rank, &cfg);
    }
    if (r == ncclInProgress || (r == ncclSuccess && c->nccl)) {
      rc = poll_in_progress(c, init_to);
    } else {
      rc = r == ncclSuccess ? ND_E_HIP : (int)r;
    }
    if (rc != ND_OK) {
      std::lock_guard<std::mutex> g(c->life_mu);
      if (c->nccl) ncclCommAbort(c->nccl);  // also ends the init job still waiting on the missing members
      c->nccl = nullptr;
    }
  }
  if (rc != ND_OK) {
    free_hip(c);
    delete c;
    return rc;
  }
  c->watchdog = std::thread(watchdog_loop, c);
  *handle = c;
  return ND_OK;
}

ND_API int nd_comm_init(void** handle, int nranks, const void* id, int rank, int device, int high_priority,
                        double timeout_s) {
  return nd_comm_init2(handle, nranks, id, rank, device, high_priority, timeout_s, 0.0);
}

// abort != 0 (an exception is propagating, or the caller knows a peer is gone): no drain, abort at once.
// Otherwise the communicator stream is drained with the collective timeout, the watchdog still running;
// a drain that times out (a peer died mid-collective) aborts instead of blocking forever.
ND_API int nd_comm_destroy2(void* handle, int abort) {
  auto* c = static_cast<Comm*>(handle);
  if (!c) return ND_E_ARG;
  (void)hipSetDevice(c->device);
  if (abort) {
    fail_comm(c, ND_E_ABORTED);
  } else {
    const auto t0 = Clock::now();
    for (;;) {
      if (c->err.load() != ND_OK) break;
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) {
        fail_comm(c, ND_E_HIP);
        break;
      }
      if (secs_since(t0) > c->timeout_s) {
        fail_comm(c, ND_E_TIMEOUT);
        break;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
  }
  c->stop.store(true);
  c->cv.notify_all();
  if (c->watchdog.joinable()) c->watchdog.join();
  int rc = ND_OK;
  {
    std::lock_guard<std::mutex> g(c->life_mu);
    if (c->nccl) {
      if (c->err.load() == ND_OK) {
        ncclResult_t r = ncclCommFinalize(c->nccl);
        if (r == ncclInProgress) r = ncclSuccess;  // polled below
        if (r != ncclSuccess) rc = (int)r;
      }
    }
  }
  if (rc == ND_OK && c->err.load() == ND_OK) {
    const int e = poll_in_progress(c, c->timeout_s);  // finalize's flush
    if (e != ND_OK) rc = e;
  }
  {
    std::lock_guard<std::mutex> g(c->life_mu);
    if (c->nccl) {
      if (rc == ND_OK && c->err.load() == ND_OK) {
        const ncclResult_t r = ncclCommDestroy(c->nccl);
        if (r != ncclSuccess) rc = (int)r;
      } else {
        ncclCommAbort(c->nccl);
      }
      c->nccl = nullptr;
    }
  }
  (void)hipStreamSynchronize(c->stream);  // aborted collectives have been released: this returns
  free_hip(c);
  delete c;
  return rc;
}

ND_API int nd_comm_destroy(void* handle) { return nd_comm_destroy2(handle, 0); }

// abort from Python (e.g. a failure elsewhere): releases collectives stuck on peers; sticky error.
// Takes neither the issue lock nor the outstanding list's.
ND_API int nd_comm_abort(void* handle) {
  auto* c = static_cast<Comm*>(handle);
  if (!c) return ND_E_ARG;
  fail_comm(c, ND_E_ABORTED);
  return ND_OK;
}

// recv = op over ranks of send (count elements of dtype; send == recv: in place).  op: ncclSum / ncclAvg / ...
ND_API int nd_comm_all_reduce(void* handle, const void* send, void* recv, size_t count, int dtype, int op,
                              hipStream_t producer, int64_t* ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || !ticket || dtype_bytes(dtype) == 0) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return issue(c, producer, (int64_t)(count * dtype_bytes(dtype)), ticket, [&](ncclComm_t n) {
    return ncclAllReduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, n, c->stream);
  });
}

ND_API int nd_comm_broadcast(void* handle, void* buf, size_t count, int dtype, int root, hipStream_t producer,
                             int64_t* ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || !ticket || dtype_bytes(dtype) == 0 || root < 0 || root >= c->nranks) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  return issue(c, producer, (int64_t)(count * dtype_bytes(dtype)), ticket, [&](ncclComm_t n) {
    return ncclBroadcast(buf, buf, count, (ncclDataType_t)dtype, root, n, c->stream);
  });
}

// in place: rank r contributes recv[r * count, (r + 1) * count)
ND_API int nd_comm_all_gather(void* handle, void* recv, size_t count, int dtype, hipStream_t producer, int64_t* ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || !ticket || dtype_bytes(dtype) == 0) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  const char* send = static_cast<const char*>(recv) + (size_t)c->rank * count * dtype_bytes(dtype);
  return issue(c, producer, (int64_t)(count * dtype_bytes(dtype)), ticket, [&](ncclComm_t n) {
    return ncclAllGather(send, recv, count, (ncclDataType_t)dtype, n, c->stream);
  });
}

// the consumer stream waits (GPU side) for collective `ticket`
ND_API int nd_comm_wait(void* handle, int64_t ticket, hipStream_t consumer) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || ticket < 0) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (const int e = c->err.load(); e != ND_OK) return e;
  const int64_t next = c->next.load();
  if (ticket >= next) return ND_E_ARG;
  if (next - ticket > kRing) return ND_E_STALE;
  return hip_ok(hipStreamWaitEvent(consumer, c->done[ticket % kRing], 0));
}

// host-side: 1 = collective `ticket` complete, 0 = still running, <0 / >0 error
ND_API int nd_comm_query(void* handle, int64_t ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || ticket < 0) return ND_E_ARG;
  if (const int e = c->err.load(); e != ND_OK) return e;
  std::lock_guard<std::mutex> g(c->mu);
  const int64_t next = c->next.load();
  if (ticket >= next) return ND_E_ARG;
  if (next - ticket > kRing) return 1;
  const hipError_t q = hipEventQuery(c->done[ticket % kRing]);
  return q == hipSuccess ? 1 : q == hipErrorNotReady ? 0 : ND_E_HIP;
}

ND_API int nd_comm_error(void* handle) {
  auto* c = static_cast<Comm*>(handle);
  return c ? c->err.load() : ND_E_ARG;
}

ND_API const char* nd_comm_error_string(int code) {
  switch (code) {
    case ND_OK: return "ok";
    case ND_E_STALE: return "ticket older than the completion-event ring";
    case ND_E_ABORTED: return "communicator aborted";
    case ND_E_TIMEOUT: return "timed out (communicator aborted)";
    case ND_E_HIP: return "HIP runtime error";
    case ND_E_ARG: return "invalid argument";
    default: return code > 0 ? ncclGetErrorString((ncclResult_t)code) : "unknown error";
  }
}

ND_API int nd_comm_stats(void* handle, int64_t* calls, int64_t* bytes, void** stream, int* priority) {
  auto* c = static_cast<Comm*>(handle);
  if (!c) return ND_E_ARG;
  if (calls) *calls = c->calls.load();
  if (bytes) *bytes = c->bytes.load();
  if (stream) *stream = c->stream;
  if (priority) (void)hipStreamGetPriority(c->stream, priority);
  return ND_OK;
}

ND_API int nd_comm_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}
