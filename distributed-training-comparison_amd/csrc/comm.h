// Internal RCCL communicator interface (see comm.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <vector>

namespace dtc {
struct Comm;
struct CommLogEntry {
  uint64_t addr, count;
  int async;  // 1: a Reducer bucket (side stream), 0: an in-stream collective
};
size_t comm_unique_id_bytes();
int comm_get_unique_id(void* out);
int comm_init(Comm** out, int rank, int world, const void* uid, int device);
int comm_destroy(Comm* c);
// blocking-order collectives on the given stream
int comm_allreduce(Comm* c, void* buf, size_t count, int dtype, hipStream_t st);
int comm_broadcast(Comm* c, void* buf, size_t count, int dtype, int root, hipStream_t st);
// Reducer primitives: fp32 SUM all-reduce of a bucket on the side stream after everything
// enqueued so far on `compute`; join orders `compute` after all outstanding buckets.
// t0 / t1 (optional timing events): recorded on the collective's stream right before / after it (t0 after
// the fork wait: when the collective can start) -- the executor's per-bucket timing (dtc_rn18_comm_timing)
int comm_allreduce_async(Comm* c, void* buf, size_t count, hipStream_t compute, hipEvent_t t0 = nullptr,
                         hipEvent_t t1 = nullptr);
int comm_join(Comm* c, hipStream_t compute);
// a bucket all-reduce issued directly on `st` (its producers already ordered before it on `st`): no fork,
// no join -- the executor's weight-gradient stream carries it (one stream fewer in the backward)
int comm_allreduce_on(Comm* c, void* buf, size_t count, hipStream_t st, hipEvent_t t0 = nullptr,
                      hipEvent_t t1 = nullptr);
// true while a comm_allreduce_async collective is not yet joined (comm_join)
bool comm_pending(const Comm* c);
int comm_world(const Comm* c);
int comm_rank(const Comm* c);
// in-process thread group: `world` handles (outs[r] = rank r) on one device, one host thread per rank
int comm_init_thread_group(Comm** outs, int world, int device);
// dist.barrier(): all ranks + this rank's queued work on `st`; the host polls (comm.cpp)
int comm_barrier(Comm* c, hipStream_t st);
// test communicator without RCCL: all-reduce = buf *= factor, logged; reports `world` ranks (comm.cpp)
int comm_init_loopback(Comm** out, int device, int world, float factor);
const std::vector<CommLogEntry>* comm_log(Comm* c);
void comm_log_clear(Comm* c);
// DataParallel group (single process, one replica per device; see comm.cpp)
struct DPGroup;
int dp_create(DPGroup** out, int n, const int* devs);
int dp_destroy(DPGroup* g);
int dp_local(const DPGroup* g);
int dp_broadcast(DPGroup* g, void* const* bufs, size_t count, int dtype, void* const* streams);
int dp_reduce_add(DPGroup* g, float* const* bufs, size_t count, void* const* streams);
int copy_peer(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, hipStream_t st);
}  // namespace dtc
