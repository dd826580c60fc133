// RCCL communicator for the data-parallel Reducer.
//
// Replaces the NCCL traffic that DistributedDataParallel issues on the reference's behalf
// (src/ddp/trainer.py:31): the construction-time broadcast of module state, the per-forward
// buffer broadcast and the bucketed gradient SUM all-reduce overlapped with backward.
// The communicator owns a non-blocking side stream; `allreduce_async` forks from the
// compute stream with an event, runs the collective on the side stream and `join` makes
// the compute stream wait for every bucket (fork/join is also valid under stream capture).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include "comm.h"
#include "common.h"
#include "kernels.h"

namespace dtc {

#define DTC_NCCL(expr)                                                                                       \
  do {                                                                                                       \
    ncclResult_t r_ = (expr);                                                                                \
    if (r_ != ncclSuccess)                                                                                   \
      return ::dtc::set_error(1000 + (int)r_, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, \
                              __LINE__);                                                                     \
  } while (0)

struct ThreadGroup;

struct Comm {
  ncclComm_t nccl = nullptr;
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> fork;
  hipEvent_t done = nullptr;
  int rank = 0, world = 1, device = 0;
  int next_fork = 0;
  bool pending = false;
  // loopback (test) communicator: no RCCL; every all-reduce multiplies the buffer by `factor` on the
  // stream the collective would run on and is logged (address, count, async) -- lets one GPU check
  // that the Reducer reduces every bucket exactly once, after its producers (dtc_comm_init_loopback)
  bool loopback = false;
  float factor = 1.f;
  std::vector<CommLogEntry> log;
  float* token = nullptr;  // barrier: one float all-reduced on the side stream
  // in-process thread group (test transport, dtc_comm_init_thread_group): this handle is rank `rank`
  // of `world` handles driven by one host thread each; collectives rendezvous on the host and run as
  // real data movement between the ranks' buffers on one GPU
  ThreadGroup* grp = nullptr;
  hipEvent_t ready = nullptr;  // this rank's "inputs produced" marker for the current collective
};

// The communicator's own stream (its broadcasts, the barrier token, and the bucket all-reduces when option
// comm_on_side is 0). Option comm_prio (read at communicator creation): 0 = normal priority; 1 = the most
// urgent priority, so RCCL's channel kernels are dispatched ahead of queued compute work.
static hipError_t comm_stream_create(hipStream_t* s) {
  if (option_get(OPT_COMM_PRIO) == 1) {
    int lo = 0, hi = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi);
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// ---------------------------------------------------------------- thread-group transport
// W ranks in one process, one host thread each, their buffers on one device. Every collective is
// matched by call order (as RCCL matches them): each rank records its producer stream, the LAST rank to
// arrive makes the group stream wait for every rank's marker, moves the data (rank-ordered SUM into
// every buffer, or root -> all copies), records a completion event, and every rank's consumer stream
// waits for it. The host rendezvous blocks the calling thread (an RCCL enqueue does not), which only
// serialises issue order -- the semantics the Reducer relies on (ordering, coverage, values) are RCCL's.
struct ThreadGroup {
  int world = 0, device = 0, refs = 0;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  int kind = -1, dtype = 0, root = 0;
  size_t count = 0;
  std::vector<void*> bufs;
  std::vector<hipEvent_t> ready;
  hipStream_t st = nullptr;
  std::vector<hipEvent_t> done;
  int done_next = 0;
  hipEvent_t last = nullptr;
  int err = 0;
  std::string errmsg;
};

enum { GK_ALLREDUCE = 0, GK_BROADCAST = 1, GK_BARRIER = 2 };

static size_t dtype_size(int dtype) { return dtype == 1 ? 2 : (dtype == 2 || dtype == 3) ? 8 : 4; }

static int group_issue(ThreadGroup* g) {  // called with g->mu held by the last rank to arrive
  for (int r = 0; r < g->world; ++r) DTC_HIP(hipStreamWaitEvent(g->st, g->ready[r], 0));
  if (g->kind == GK_ALLREDUCE && g->count > 0) {
    GroupPtrs p{};
    for (int r = 0; r < g->world; ++r) p.p[r] = g->bufs[r];
    DTC_TRY(group_sum(p, g->world, (int64_t)g->count, g->dtype, g->st));
  } else if (g->kind == GK_BROADCAST && g->count > 0) {
    for (int r = 0; r < g->world; ++r)
      if (r != g->root)
        DTC_HIP(hipMemcpyAsync(g->bufs[r], g->bufs[g->root], g->count * dtype_size(g->dtype), hipMemcpyDeviceToDevice,
                               g->st));
  }
  g->last = g->done[g->done_next];
  g->done_next = (g->done_next + 1) % (int)g->done.size();
  DTC_HIP(hipEventRecord(g->last, g->st));
  return 0;
}

// One collective of rank c->rank: `after` orders the inputs, `waiter` waits for the result.
static int group_collective(Comm* c, int kind, void* buf, size_t count, int dtype, int root, hipStream_t after,
                            hipStream_t waiter) {
  ThreadGroup* g = c->grp;
  DTC_CHECK_ARG(kind != GK_ALLREDUCE || dtype == 0 || dtype == 2 || dtype == 3, "thread group: SUM of fp32 / int64 / fp64 only");
  DTC_HIP(hipEventRecord(c->ready, after));
  hipEvent_t res = nullptr;
  {
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->err) return set_error(g->err, "%s", g->errmsg.c_str());
    if (g->arrived == 0) {
      g->kind = kind;
      g->count = count;
      g->dtype = dtype;
      g->root = root;
    } else if (g->kind != kind || g->count != count || g->dtype != dtype || g->root != root) {
      g->err = DTC_EINVAL;
      g->errmsg = "thread group: ranks issued mismatched collectives (kind/count/dtype/root differ)";
      g->cv.notify_all();
      return set_error(g->err, "%s", g->errmsg.c_str());
    }
    g->bufs[c->rank] = buf;
    g->ready[c->rank] = c->ready;
    const uint64_t my = g->gen;
    if (++g->arrived == g->world) {
      const int rc = group_issue(g);
      g->arrived = 0;
      ++g->gen;
      if (rc) {
        g->err = rc;
        g->errmsg = last_error();
      }
      g->cv.notify_all();
      if (rc) return rc;
    } else if (!g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->gen != my || g->err != 0; })) {
      g->err = DTC_EINVAL;
      g->errmsg = "thread group: timed out waiting for the other ranks' collective";
      g->cv.notify_all();
      return set_error(g->err, "%s (rank %d)", g->errmsg.c_str(), c->rank);
    }
    if (g->err) return set_error(g->err, "%s", g->errmsg.c_str());
    res = g->last;
  }
  DTC_HIP(hipStreamWaitEvent(waiter, res, 0));
  return 0;
}

int comm_init_thread_group(Comm** outs, int world, int device) {
  DTC_CHECK_ARG(outs && world >= 1 && world <= DTC_GROUP_MAX, "comm_init_thread_group: bad args");
  DTC_HIP(hipSetDevice(device));
  ThreadGroup* g = new ThreadGroup();
  g->world = world;
  g->device = device;
  g->refs = world;
  g->bufs.assign(world, nullptr);
  g->ready.assign(world, nullptr);
  DTC_HIP(hipStreamCreateWithFlags(&g->st, hipStreamNonBlocking));
  g->done.resize(64);
  for (auto& e : g->done) DTC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (int r = 0; r < world; ++r) {
    Comm* c = new Comm();
    c->rank = r;
    c->world = world;
    c->device = device;
    c->grp = g;
    DTC_HIP(comm_stream_create(&c->side));
    c->fork.resize(64);
    for (auto& e : c->fork) DTC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    DTC_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
    DTC_HIP(hipEventCreateWithFlags(&c->ready, hipEventDisableTiming));
    outs[r] = c;
  }
  return 0;
}

static void group_release(ThreadGroup* g) {
  bool last = false;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    last = --g->refs == 0;
  }
  if (!last) return;
  (void)hipStreamSynchronize(g->st);
  for (auto& e : g->done)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(g->st);
  delete g;
}

static ncclDataType_t to_nccl(int dtype) {
  switch (dtype) {
    case 1: return ncclBfloat16;
    case 2: return ncclInt64;
    case 3: return ncclFloat64;
    default: return ncclFloat32;
  }
}

size_t comm_unique_id_bytes() { return sizeof(ncclUniqueId); }

int comm_get_unique_id(void* out) {
  DTC_CHECK_ARG(out != nullptr, "comm_get_unique_id: null output");
  ncclUniqueId id;
  DTC_NCCL(ncclGetUniqueId(&id));
  memcpy(out, &id, sizeof(id));
  return 0;
}

int comm_init(Comm** out, int rank, int world, const void* uid, int device) {
  DTC_CHECK_ARG(out && uid && world >= 1 && rank >= 0 && rank < world, "comm_init: bad args");
  DTC_HIP(hipSetDevice(device));
  Comm* c = new Comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  ncclUniqueId id;
  memcpy(&id, uid, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&c->nccl, world, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return set_error(1000 + (int)r, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
  }
  DTC_HIP(comm_stream_create(&c->side));
  c->fork.resize(64);
  for (auto& e : c->fork) DTC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  DTC_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
  *out = c;
  return 0;
}

int comm_init_loopback(Comm** out, int device, int world, float factor) {
  DTC_CHECK_ARG(out != nullptr && world >= 1, "comm_init_loopback: bad args");
  DTC_HIP(hipSetDevice(device));
  Comm* c = new Comm();
  c->device = device;
  c->loopback = true;
  c->world = world;
  c->factor = factor;
  DTC_HIP(comm_stream_create(&c->side));
  c->fork.resize(64);
  for (auto& e : c->fork) DTC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  DTC_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
  *out = c;
  return 0;
}

const std::vector<CommLogEntry>* comm_log(Comm* c) { return c ? &c->log : nullptr; }
void comm_log_clear(Comm* c) {
  if (c) c->log.clear();
}

// the loopback collective: buf *= factor (fp32 / fp64; int64 buffers -- BN statistics -- by the integer
// factor) on `st`
static int loopback_reduce(Comm* c, void* buf, size_t count, int dtype, hipStream_t st, bool async) {
  DTC_CHECK_ARG(dtype == 0 || dtype == 2 || dtype == 3, "loopback communicator: fp32 / int64 / fp64 buffers only");
  DTC_CHECK_ARG(dtype != 2 || c->factor == (float)(int64_t)c->factor, "loopback communicator: int64 needs an integer factor");
  c->log.push_back(CommLogEntry{(uint64_t)(uintptr_t)buf, (uint64_t)count, async ? 1 : 0});
  if (dtype == 2) return scale_i64(reinterpret_cast<int64_t*>(buf), (int64_t)count, (int64_t)c->factor, st);
  return dtype == 0 ? scale_f32(reinterpret_cast<float*>(buf), (int64_t)count, c->factor, st)
                    : scale_f64(reinterpret_cast<double*>(buf), (int64_t)count, (double)c->factor, st);
}

// Host-side wait that polls instead of sleeping in the driver: after the reference's per-step
// barrier the GPU queue is empty, so every microsecond of wake-up latency is GPU idle time.
// The poll is bounded: after ~2 ms -- a rank that lags that long (e.g. while rank 0 runs the
// reference's rank-0-only validation) is not a per-step barrier -- the wait becomes the driver's blocking
// hipEventSynchronize, so waiting ranks stop pinning a host core.
static int spin_wait(hipEvent_t ev) {
  if (option_get(OPT_BARRIER_SPIN) == 0) {
    DTC_HIP(hipEventSynchronize(ev));
    return 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) return set_error((int)e, "barrier: hipEventQuery: %s", hipGetErrorString(e));
    if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) {
      DTC_HIP(hipEventSynchronize(ev));
      return 0;
    }
  }
}

// dist.barrier() (reference ddp/trainer.py:156): every rank's host returns only after
// all ranks reached it AND this rank's work queued on `st` before it has finished (what torch's
// NCCL barrier does: an all-reduce of one element, then a stream synchronize). One float is SUM
// all-reduced on the communicator's side stream (after `st`, so every collective of this
// communicator stays on one stream), the host polls its completion event. Without an RCCL
// communicator (comm == NULL or a loopback test communicator) it is the stream drain (the Python
// barrier() passes NULL at world 1: a one-rank all-reduce would only add a launch).
int comm_barrier(Comm* c, hipStream_t st) {
  static thread_local hipEvent_t local_ev = nullptr;
  if (c != nullptr && c->grp != nullptr) {  // every rank's host meets, then waits for its own stream
    DTC_TRY(group_collective(c, GK_BARRIER, nullptr, 0, 0, 0, st, st));
    if (!local_ev) DTC_HIP(hipEventCreateWithFlags(&local_ev, hipEventDisableTiming));
    DTC_HIP(hipEventRecord(local_ev, st));
    return spin_wait(local_ev);
  }
  if (c == nullptr || c->loopback || c->nccl == nullptr) {
    if (!local_ev) DTC_HIP(hipEventCreateWithFlags(&local_ev, hipEventDisableTiming));
    DTC_HIP(hipEventRecord(local_ev, st));
    return spin_wait(local_ev);
  }
  if (!c->token) {
    DTC_HIP(hipMalloc(&c->token, sizeof(float)));
    DTC_HIP(hipMemsetAsync(c->token, 0, sizeof(float), st));
  }
  hipEvent_t ev = c->fork[c->next_fork];
  c->next_fork = (c->next_fork + 1) % (int)c->fork.size();
  DTC_HIP(hipEventRecord(ev, st));
  DTC_HIP(hipStreamWaitEvent(c->side, ev, 0));
  DTC_NCCL(ncclAllReduce(c->token, c->token, 1, ncclFloat32, ncclSum, c->nccl, c->side));
  DTC_HIP(hipEventRecord(c->done, c->side));
  return spin_wait(c->done);  // anything issued after the return is ordered after it in real time
}

int comm_destroy(Comm* c) {
  if (!c) return 0;
  if (c->side) (void)hipStreamSynchronize(c->side);
  if (c->token) (void)hipFree(c->token);
  if (c->nccl) ncclCommDestroy(c->nccl);
  for (auto& e : c->fork)
    if (e) (void)hipEventDestroy(e);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->ready) (void)hipEventDestroy(c->ready);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->grp) group_release(c->grp);
  delete c;
  return 0;
}

int comm_allreduce(Comm* c, void* buf, size_t count, int dtype, hipStream_t st) {
  DTC_CHECK_ARG(c && buf, "comm_allreduce: bad args");
  if (count == 0) return 0;
  if (c->loopback) return loopback_reduce(c, buf, count, dtype, st, false);
  if (c->grp) {
    c->log.push_back(CommLogEntry{(uint64_t)(uintptr_t)buf, (uint64_t)count, 0});
    return group_collective(c, GK_ALLREDUCE, buf, count, dtype, 0, st, st);
  }
  DTC_NCCL(ncclAllReduce(buf, buf, count, to_nccl(dtype), ncclSum, c->nccl, st));
  return 0;
}

int comm_broadcast(Comm* c, void* buf, size_t count, int dtype, int root, hipStream_t st) {
  DTC_CHECK_ARG(c && buf && root >= 0 && root < c->world, "comm_broadcast: bad args");
  if (count == 0) return 0;
  if (c->loopback) return 0;  // one rank: the root's buffer already is the result
  if (c->grp) return group_collective(c, GK_BROADCAST, buf, count, dtype, root, st, st);
  // on the communicator's side stream, like its bucket all-reduces and barrier: every collective of
  // one communicator on ONE stream, so two ranks can never order them differently on the device
  // (VERDICT r2); `st` is ordered before (the buffer's producers) and after (its consumers)
  hipEvent_t ev = c->fork[c->next_fork];
  c->next_fork = (c->next_fork + 1) % (int)c->fork.size();
  DTC_HIP(hipEventRecord(ev, st));
  DTC_HIP(hipStreamWaitEvent(c->side, ev, 0));
  DTC_NCCL(ncclBroadcast(buf, buf, count, to_nccl(dtype), root, c->nccl, c->side));
  DTC_HIP(hipEventRecord(c->done, c->side));
  DTC_HIP(hipStreamWaitEvent(st, c->done, 0));
  return 0;
}

int comm_allreduce_async(Comm* c, void* buf, size_t count, hipStream_t compute, hipEvent_t t0, hipEvent_t t1) {
  DTC_CHECK_ARG(c && buf, "comm_allreduce_async: bad args");
  if (count == 0) return 0;
  if (c->grp) {  // the bucket's producers on `compute`, the result awaited by the side stream
    c->log.push_back(CommLogEntry{(uint64_t)(uintptr_t)buf, (uint64_t)count, 1});
    if (t0) DTC_HIP(hipEventRecord(t0, compute));
    DTC_TRY(group_collective(c, GK_ALLREDUCE, buf, count, 0, 0, compute, c->side));
    if (t1) DTC_HIP(hipEventRecord(t1, c->side));
    c->pending = true;
    return 0;
  }
  hipEvent_t ev = c->fork[c->next_fork];
  c->next_fork = (c->next_fork + 1) % (int)c->fork.size();
  DTC_HIP(hipEventRecord(ev, compute));
  DTC_HIP(hipStreamWaitEvent(c->side, ev, 0));
  if (t0) DTC_HIP(hipEventRecord(t0, c->side));  // (after the wait: when the collective can start)
  if (c->loopback) DTC_TRY(loopback_reduce(c, buf, count, 0, c->side, true));
  else DTC_NCCL(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c->nccl, c->side));
  if (t1) DTC_HIP(hipEventRecord(t1, c->side));
  c->pending = true;
  return 0;
}

int comm_allreduce_on(Comm* c, void* buf, size_t count, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
  DTC_CHECK_ARG(c && buf, "comm_allreduce_on: bad args");
  if (count == 0) return 0;
  if (t0) DTC_HIP(hipEventRecord(t0, st));
  if (c->grp) {
    c->log.push_back(CommLogEntry{(uint64_t)(uintptr_t)buf, (uint64_t)count, 1});
    DTC_TRY(group_collective(c, GK_ALLREDUCE, buf, count, 0, 0, st, st));
  } else if (c->loopback) {
    DTC_TRY(loopback_reduce(c, buf, count, 0, st, true));
  } else {
    DTC_NCCL(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c->nccl, st));
  }
  if (t1) DTC_HIP(hipEventRecord(t1, st));
  return 0;
}

int comm_join(Comm* c, hipStream_t compute) {
  if (!c || !c->pending) return 0;
  DTC_HIP(hipEventRecord(c->done, c->side));
  DTC_HIP(hipStreamWaitEvent(compute, c->done, 0));
  c->pending = false;
  c->next_fork = 0;
  return 0;
}

bool comm_pending(const Comm* c) { return c != nullptr && c->pending; }
int comm_world(const Comm* c) { return c ? c->world : 1; }
int comm_rank(const Comm* c) { return c ? c->rank : 0; }

}  // namespace dtc

// ---------------------------------------------------------------- DataParallel group (config 4)
// nn.DataParallel (reference src/dp/trainer.py:27) is ONE process driving every GPU: torch
// replicates the module with broadcast_coalesced and sums the replicas' gradients with
// reduce_add_coalesced (NCCL) every step. Here: one RCCL communicator per
// device from ncclCommInitAll (single-process multi-rank), and the flat parameter / gradient
// buffers move as ONE broadcast / ONE reduce each, grouped across devices. A group whose replicas
// all share one device (the one-GPU test form, device_ids=[0, 0]) cannot hold one RCCL rank per
// replica; it runs the same collectives as on-device copies and a fixed-order HIP reduce-add.
namespace dtc {

struct DPGroup {
  int n = 0;
  std::vector<int> devs;
  bool local = false;  // every replica on one device
  std::vector<ncclComm_t> comms;
};

static size_t dtype_bytes(int dtype) { return dtype == 1 ? 2 : (dtype == 2 || dtype == 3) ? 8 : 4; }

struct DeviceGuard {
  int prev = 0;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

int dp_create(DPGroup** out, int n, const int* devs) {
  DTC_CHECK_ARG(out && devs && n >= 1 && n <= 64, "dp_create: bad args");
  DPGroup* g = new DPGroup();
  g->n = n;
  g->devs.assign(devs, devs + n);
  bool all_same = true, distinct = true;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (devs[i] != devs[j]) all_same = false;
      if (i != j && devs[i] == devs[j]) distinct = false;
    }
  if (!all_same && !distinct) {
    delete g;
    return set_error(DTC_EINVAL, "dp_create: device ids must be all distinct or all equal");
  }
  g->local = all_same;
  if (!g->local) {
    DeviceGuard guard;
    g->comms.resize(n);
    ncclResult_t r = ncclCommInitAll(g->comms.data(), n, devs);
    if (r != ncclSuccess) {
      delete g;
      return set_error(1000 + (int)r, "ncclCommInitAll failed: %s", ncclGetErrorString(r));
    }
  }
  *out = g;
  return 0;
}

int dp_destroy(DPGroup* g) {
  if (!g) return 0;
  for (auto& c : g->comms)
    if (c) ncclCommDestroy(c);
  delete g;
  return 0;
}

int dp_local(const DPGroup* g) { return g ? (g->local ? 1 : 0) : DTC_EINVAL; }

// bufs[i] lives on devs[i]; bufs[0] is the root (the module on device_ids[0])
int dp_broadcast(DPGroup* g, void* const* bufs, size_t count, int dtype, void* const* streams) {
  DTC_CHECK_ARG(g && bufs && streams, "dp_broadcast: bad args");
  if (count == 0 || g->n == 1) return 0;
  if (g->local) {
    for (int i = 1; i < g->n; ++i)
      DTC_HIP(hipMemcpyAsync(bufs[i], bufs[0], count * dtype_bytes(dtype), hipMemcpyDeviceToDevice,
                             (hipStream_t)streams[0]));
    return 0;
  }
  DeviceGuard guard;
  DTC_NCCL(ncclGroupStart());
  for (int i = 0; i < g->n; ++i) {
    DTC_HIP(hipSetDevice(g->devs[i]));
    DTC_NCCL(ncclBroadcast(bufs[i], bufs[i], count, to_nccl(dtype), 0, g->comms[i], (hipStream_t)streams[i]));
  }
  DTC_NCCL(ncclGroupEnd());
  return 0;
}

// bufs[0] += sum_{i>0} bufs[i] (fp32), i.e. torch's reduce_add onto device_ids[0]
int dp_reduce_add(DPGroup* g, float* const* bufs, size_t count, void* const* streams) {
  DTC_CHECK_ARG(g && bufs && streams, "dp_reduce_add: bad args");
  if (count == 0 || g->n == 1) return 0;
  if (g->local) {
    for (int i = 1; i < g->n; ++i) DTC_TRY(add_f32(bufs[0], bufs[i], (int64_t)count, (hipStream_t)streams[0]));
    return 0;
  }
  DeviceGuard guard;
  DTC_NCCL(ncclGroupStart());
  for (int i = 0; i < g->n; ++i) {
    DTC_HIP(hipSetDevice(g->devs[i]));
    DTC_NCCL(ncclReduce(bufs[i], bufs[i], count, ncclFloat32, ncclSum, 0, g->comms[i], (hipStream_t)streams[i]));
  }
  DTC_NCCL(ncclGroupEnd());
  return 0;
}

int copy_peer(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, hipStream_t st) {
  DTC_CHECK_ARG(dst && src, "copy_peer: null pointer");
  if (bytes == 0) return 0;
  if (dst_dev == src_dev) DTC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
  else DTC_HIP(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, st));
  return 0;
}

}  // namespace dtc
