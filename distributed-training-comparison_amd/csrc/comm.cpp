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
#include <cstring>
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
};

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
  DTC_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
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
  DTC_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
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

// the loopback collective: buf *= factor (fp32 / fp64 only) on `st`
static int loopback_reduce(Comm* c, void* buf, size_t count, int dtype, hipStream_t st, bool async) {
  DTC_CHECK_ARG(dtype == 0 || dtype == 3, "loopback communicator: fp32 / fp64 buffers only");
  c->log.push_back(CommLogEntry{(uint64_t)(uintptr_t)buf, (uint64_t)count, async ? 1 : 0});
  return dtype == 0 ? scale_f32(reinterpret_cast<float*>(buf), (int64_t)count, c->factor, st)
                    : scale_f64(reinterpret_cast<double*>(buf), (int64_t)count, (double)c->factor, st);
}

int comm_destroy(Comm* c) {
  if (!c) return 0;
  if (c->side) (void)hipStreamSynchronize(c->side);
  if (c->nccl) ncclCommDestroy(c->nccl);
  for (auto& e : c->fork)
    if (e) (void)hipEventDestroy(e);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->side) (void)hipStreamDestroy(c->side);
  delete c;
  return 0;
}

int comm_allreduce(Comm* c, void* buf, size_t count, int dtype, hipStream_t st) {
  DTC_CHECK_ARG(c && buf, "comm_allreduce: bad args");
  if (count == 0) return 0;
  if (c->loopback) return loopback_reduce(c, buf, count, dtype, st, false);
  DTC_NCCL(ncclAllReduce(buf, buf, count, to_nccl(dtype), ncclSum, c->nccl, st));
  return 0;
}

int comm_broadcast(Comm* c, void* buf, size_t count, int dtype, int root, hipStream_t st) {
  DTC_CHECK_ARG(c && buf && root >= 0 && root < c->world, "comm_broadcast: bad args");
  if (count == 0) return 0;
  if (c->loopback) return 0;  // one rank: the root's buffer already is the result
  DTC_NCCL(ncclBroadcast(buf, buf, count, to_nccl(dtype), root, c->nccl, st));
  return 0;
}

int comm_allreduce_async(Comm* c, void* buf, size_t count, hipStream_t compute) {
  DTC_CHECK_ARG(c && buf, "comm_allreduce_async: bad args");
  if (count == 0) return 0;
  hipEvent_t ev = c->fork[c->next_fork];
  c->next_fork = (c->next_fork + 1) % (int)c->fork.size();
  DTC_HIP(hipEventRecord(ev, compute));
  DTC_HIP(hipStreamWaitEvent(c->side, ev, 0));
  if (c->loopback) DTC_TRY(loopback_reduce(c, buf, count, 0, c->side, true));
  else DTC_NCCL(ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, c->nccl, c->side));
  c->pending = true;
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

int comm_world(const Comm* c) { return c ? c->world : 1; }

}  // namespace dtc
