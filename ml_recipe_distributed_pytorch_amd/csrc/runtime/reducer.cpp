// Flat-bucket gradient reducer over RCCL (native replacement for torch DDP's Reducer).
//
// * Owns its own RCCL communicator (bootstrapped with a unique id that Python ships through the
//   torch.distributed TCPStore) and a normal-priority HIP stream for communication.
// * allreduce(ptr, count, …, compute_stream): records an event on the compute stream, makes the comm
//   stream wait on it, then ncclAllReduce(ncclAvg) in place on a contiguous slice of the fp32 grad
//   arena — the bucket IS the arena slice, so there is no copy-in/copy-out.
// * bf16 mode: cast fp32→bf16 into a scratch slice on the comm stream, all-reduce half the bytes,
//   cast back (the casts run on the comm stream, overlapped with backward compute).
// * wait(compute_stream): compute stream waits for everything issued so far (optimizer boundary).
// RCCL over xGMI: buckets are sized by the caller (default 32 MiB) so that each of the ≥7 RCCL
// channels moves multi-MiB chunks per link.
#include "hq_reducer.h"

#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "hq_kernels.h"

#define NCCL_CHECK(x)                                                                              \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r_)); \
  } while (0)
#define HIP_CHECK_THROW(x)                                                                         \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_)); \
  } while (0)

std::string hq_rccl_unique_id() {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

HqReducer::HqReducer(int rank, int world, const std::string& uid, int device) : rank_(rank), world_(world), device_(device) {
  if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad RCCL unique id size");
  HIP_CHECK_THROW(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  ncclComm_t comm;
  NCCL_CHECK(ncclCommInitRank(&comm, world, id, rank));
  comm_ = comm;
  int lo = 0, hi = 0;
  HIP_CHECK_THROW(hipDeviceGetStreamPriorityRange(&lo, &hi));
  // The comm stream runs at NORMAL priority: measured on MI355X (tools/stream_overlap_bench.py), a
  // high-priority comm queue slows every kernel of the compute stream while an all-reduce is in flight
  // (+1.9 ms per 48 GEMMs against +0.5 ms at normal priority).  HQ_COMM_PRIO=1 restores the high priority.
  const char* pe = getenv("HQ_COMM_PRIO");
  const int prio = (pe && atoi(pe) == 1) ? hi : lo;
  hipStream_t st;
  HIP_CHECK_THROW(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, prio));
  stream_ = st;
  for (int i = 0; i < kEvents; ++i) {
    hipEvent_t e;
    HIP_CHECK_THROW(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    events_[i] = e;
  }
}

HqReducer::~HqReducer() {
  if (stream_) hipStreamSynchronize((hipStream_t)stream_);
  for (int i = 0; i < kEvents; ++i)
    if (events_[i]) hipEventDestroy((hipEvent_t)events_[i]);
  if (comm_) ncclCommDestroy((ncclComm_t)comm_);
  if (stream_) hipStreamDestroy((hipStream_t)stream_);
}

void* HqReducer::next_event() {
  void* e = events_[ev_idx_];
  ev_idx_ = (ev_idx_ + 1) % kEvents;
  return e;
}

void HqReducer::fence_from(int64_t compute_stream) {
  hipEvent_t e = (hipEvent_t)next_event();
  HIP_CHECK_THROW(hipEventRecord(e, (hipStream_t)compute_stream));
  HIP_CHECK_THROW(hipStreamWaitEvent((hipStream_t)stream_, e, 0));
}

void HqReducer::allreduce_f32(int64_t ptr, int64_t count, int64_t compute_stream, int op) {
  fence_from(compute_stream);
  NCCL_CHECK(ncclAllReduce((const void*)ptr, (void*)ptr, (size_t)count, ncclFloat32, op == 1 ? ncclSum : ncclAvg,
                           (ncclComm_t)comm_,
                           (hipStream_t)stream_));
}

void HqReducer::allreduce_bf16(int64_t ptr_f32, int64_t scratch_bf16, int64_t count, int64_t compute_stream) {
  fence_from(compute_stream);
  hipStream_t st = (hipStream_t)stream_;
  hq_cast_f32_bf16((const float*)ptr_f32, (uint16_t*)scratch_bf16, count, 1.f, st);
  NCCL_CHECK(ncclAllReduce((const void*)scratch_bf16, (void*)scratch_bf16, (size_t)count, ncclBfloat16, ncclAvg,
                           (ncclComm_t)comm_, st));
  hq_cast_bf16_f32((const uint16_t*)scratch_bf16, (float*)ptr_f32, count, 1.f, st);
}

void HqReducer::broadcast(int64_t ptr, int64_t count, int dtype, int root, int64_t compute_stream) {
  fence_from(compute_stream);
  ncclDataType_t dt = dtype == 0 ? ncclFloat32 : (dtype == 1 ? ncclBfloat16 : ncclInt64);
  NCCL_CHECK(ncclBroadcast((const void*)ptr, (void*)ptr, (size_t)count, dt, root, (ncclComm_t)comm_, (hipStream_t)stream_));
}

void HqReducer::probe_f32(int64_t ptr, int64_t count, int64_t partials, int nparts, int64_t compute_stream) {
  fence_from(compute_stream);
  hq_sq_norm_partials((const float*)ptr, count, (float*)partials, nparts, (hipStream_t)stream_);
}

void HqReducer::sq_norm_chunks(int64_t grad, int64_t chunks, int c0, int c1, int64_t partials) {
  hq_sq_norm_chunks((const float*)grad, (const int64_t*)chunks, c0, c1, (float*)partials, (hipStream_t)stream_);
}

void HqReducer::wait(int64_t compute_stream) {
  hipEvent_t e = (hipEvent_t)next_event();
  HIP_CHECK_THROW(hipEventRecord(e, (hipStream_t)stream_));
  HIP_CHECK_THROW(hipStreamWaitEvent((hipStream_t)compute_stream, e, 0));
}

int HqReducer::comm_count() const {
  int n = 0;
  NCCL_CHECK(ncclCommCount((ncclComm_t)comm_, &n));
  return n;
}

void HqReducer::synchronize() { HIP_CHECK_THROW(hipStreamSynchronize((hipStream_t)stream_)); }
