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
// Failure detection: a watchdog thread per communicator polls the completion events of outstanding
// collectives and RCCL's asynchronous error state; a collective older than the timeout, or an async
// error, aborts the communicator (ncclCommAbort releases the kernels spinning on the peers) and every
// later call returns the error, which Python raises -- a dead peer surfaces as an error on every rank
// instead of a hang.
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

struct Outstanding {
  int64_t ticket;
  std::chrono::steady_clock::time_point t0;
};

struct Comm {
  ncclComm_t nccl = nullptr;
  int device = 0, rank = 0, nranks = 1;
  hipStream_t stream = nullptr;
  hipEvent_t in_ev = nullptr;          // producer -> communicator stream ordering
  std::vector<hipEvent_t> done;        // completion event of ticket t: done[t % kRing]
  int64_t next = 0;                    // next ticket
  std::mutex mu;                       // issue order and the outstanding list
  std::deque<Outstanding> pending;     // collectives not yet seen complete by the watchdog
  std::atomic<int> err{ND_OK};         // sticky error (abort / timeout / async RCCL error)
  double timeout_s = 1800.0;
  std::thread watchdog;
  std::atomic<bool> stop{false};
  std::condition_variable cv;
  std::mutex cv_mu;
  int64_t calls = 0, bytes = 0;
};

int hip_ok(hipError_t e) { return e == hipSuccess ? ND_OK : ND_E_HIP; }

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
      std::lock_guard<std::mutex> g(c->mu);
      while (!c->pending.empty()) {
        const Outstanding& o = c->pending.front();
        const hipError_t q = hipEventQuery(c->done[o.ticket % kRing]);
        if (q == hipSuccess || c->next - o.ticket > kRing) {  // done (or its event already reused)
          c->pending.pop_front();
          continue;
        }
        const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() - o.t0).count();
        if (q != hipErrorNotReady) fail = ND_E_HIP;
        else if (age > c->timeout_s) fail = ND_E_TIMEOUT;
        break;
      }
    }
    if (fail == ND_OK) {
      std::lock_guard<std::mutex> g(c->mu);
      ncclResult_t ae = ncclSuccess;
      if (c->nccl && ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress)
        fail = (int)ae;
    }
    if (fail != ND_OK) {
      std::lock_guard<std::mutex> g(c->mu);
      c->err.store(fail);
      if (c->nccl) ncclCommAbort(c->nccl);  // releases the collective kernels waiting on dead / stuck peers
      c->nccl = nullptr;
    }
  }
}

int issue_prologue(Comm* c, hipStream_t producer) {
  if (const int e = c->err.load(); e != ND_OK) return e;
  if (hipEventRecord(c->in_ev, producer) != hipSuccess) return ND_E_HIP;
  return hip_ok(hipStreamWaitEvent(c->stream, c->in_ev, 0));
}

int issue_epilogue(Comm* c, int64_t* ticket) {
  const int64_t t = c->next++;
  if (hipEventRecord(c->done[t % kRing], c->stream) != hipSuccess) return ND_E_HIP;
  c->pending.push_back({t, std::chrono::steady_clock::now()});
  ++c->calls;
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
// all-reduce beside the next inner step, the inner-DDP buckets beside the backward)
ND_API int nd_comm_init(void** handle, int nranks, const void* id, int rank, int device, int high_priority,
                        double timeout_s) {
  if (!handle || !id || nranks < 1 || rank < 0 || rank >= nranks) return ND_E_ARG;
  auto* c = new Comm();
  c->device = device;
  c->rank = rank;
  c->nranks = nranks;
  c->timeout_s = timeout_s > 0 ? timeout_s : 1800.0;
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
    const ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
    if (r != ncclSuccess) rc = (int)r;
  }
  if (rc != ND_OK) {
    for (hipEvent_t e : c->done)
      if (e) (void)hipEventDestroy(e);
    if (c->in_ev) (void)hipEventDestroy(c->in_ev);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return rc;
  }
  c->watchdog = std::thread(watchdog_loop, c);
  *handle = c;
  return ND_OK;
}

ND_API int nd_comm_destroy(void* handle) {
  auto* c = static_cast<Comm*>(handle);
  if (!c) return ND_E_ARG;
  c->stop.store(true);
  c->cv.notify_all();
  if (c->watchdog.joinable()) c->watchdog.join();
  (void)hipSetDevice(c->device);
  int rc = ND_OK;
  if (c->nccl) {
    if (c->err.load() == ND_OK) {
      (void)hipStreamSynchronize(c->stream);
      const ncclResult_t r = ncclCommDestroy(c->nccl);
      if (r != ncclSuccess) rc = (int)r;
    } else {
      ncclCommAbort(c->nccl);
    }
  }
  for (hipEvent_t e : c->done) (void)hipEventDestroy(e);
  (void)hipEventDestroy(c->in_ev);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return rc;
}

// abort from Python (e.g. a failure elsewhere): releases collectives stuck on peers; sticky error
ND_API int nd_comm_abort(void* handle) {
  auto* c = static_cast<Comm*>(handle);
  if (!c) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  c->err.store(ND_E_ABORTED);
  if (c->nccl) ncclCommAbort(c->nccl);
  c->nccl = nullptr;
  return ND_OK;
}

// recv = op over ranks of send (count elements of dtype; send == recv: in place).  op: ncclSum / ncclAvg / ...
ND_API int nd_comm_all_reduce(void* handle, const void* send, void* recv, size_t count, int dtype, int op,
                              hipStream_t producer, int64_t* ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || !ticket || dtype_bytes(dtype) == 0) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (const int e = issue_prologue(c, producer); e != ND_OK) return e;
  const ncclResult_t r = ncclAllReduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, c->nccl, c->stream);
  if (r != ncclSuccess) return (int)r;
  c->bytes += (int64_t)(count * dtype_bytes(dtype));
  return issue_epilogue(c, ticket);
}

ND_API int nd_comm_broadcast(void* handle, void* buf, size_t count, int dtype, int root, hipStream_t producer,
                             int64_t* ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || !ticket || dtype_bytes(dtype) == 0 || root < 0 || root >= c->nranks) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (const int e = issue_prologue(c, producer); e != ND_OK) return e;
  const ncclResult_t r = ncclBroadcast(buf, buf, count, (ncclDataType_t)dtype, root, c->nccl, c->stream);
  if (r != ncclSuccess) return (int)r;
  c->bytes += (int64_t)(count * dtype_bytes(dtype));
  return issue_epilogue(c, ticket);
}

// in place: rank r contributes recv[r * count, (r + 1) * count)
ND_API int nd_comm_all_gather(void* handle, void* recv, size_t count, int dtype, hipStream_t producer, int64_t* ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || !ticket || dtype_bytes(dtype) == 0) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (const int e = issue_prologue(c, producer); e != ND_OK) return e;
  const char* send = static_cast<const char*>(recv) + (size_t)c->rank * count * dtype_bytes(dtype);
  const ncclResult_t r = ncclAllGather(send, recv, count, (ncclDataType_t)dtype, c->nccl, c->stream);
  if (r != ncclSuccess) return (int)r;
  c->bytes += (int64_t)(count * dtype_bytes(dtype));
  return issue_epilogue(c, ticket);
}

// the consumer stream waits (GPU side) for collective `ticket`
ND_API int nd_comm_wait(void* handle, int64_t ticket, hipStream_t consumer) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || ticket < 0) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (const int e = c->err.load(); e != ND_OK) return e;
  if (ticket >= c->next) return ND_E_ARG;
  if (c->next - ticket > kRing) return ND_E_STALE;
  return hip_ok(hipStreamWaitEvent(consumer, c->done[ticket % kRing], 0));
}

// host-side: 1 = collective `ticket` complete, 0 = still running, <0 / >0 error
ND_API int nd_comm_query(void* handle, int64_t ticket) {
  auto* c = static_cast<Comm*>(handle);
  if (!c || ticket < 0) return ND_E_ARG;
  if (const int e = c->err.load(); e != ND_OK) return e;
  std::lock_guard<std::mutex> g(c->mu);
  if (ticket >= c->next) return ND_E_ARG;
  if (c->next - ticket > kRing) return 1;
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
    case ND_E_TIMEOUT: return "collective timed out (watchdog aborted the communicator)";
    case ND_E_HIP: return "HIP runtime error";
    case ND_E_ARG: return "invalid argument";
    default: return code > 0 ? ncclGetErrorString((ncclResult_t)code) : "unknown error";
  }
}

// stats: calls issued, payload bytes issued; stream handle (for tests / profiling)
ND_API int nd_comm_stats(void* handle, int64_t* calls, int64_t* bytes, void** stream, int* priority) {
  auto* c = static_cast<Comm*>(handle);
  if (!c) return ND_E_ARG;
  std::lock_guard<std::mutex> g(c->mu);
  if (calls) *calls = c->calls;
  if (bytes) *bytes = c->bytes;
  if (stream) *stream = c->stream;
  if (priority) (void)hipStreamGetPriority(c->stream, priority);
  return ND_OK;
}

ND_API int nd_comm_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}
