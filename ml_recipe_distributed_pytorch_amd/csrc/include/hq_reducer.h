// RCCL flat-bucket gradient reducer (see runtime/reducer.cpp).  No torch / rccl types in the
// interface so bindings.cpp does not need the RCCL headers.
#pragma once
#include <stdint.h>

#include <string>

std::string hq_rccl_unique_id();

class HqReducer {
 public:
  HqReducer(int rank, int world, const std::string& unique_id, int device);
  ~HqReducer();
  HqReducer(const HqReducer&) = delete;
  HqReducer& operator=(const HqReducer&) = delete;

  void allreduce_f32(int64_t ptr, int64_t count, int64_t compute_stream, int op = 0);  // op 0 = avg, 1 = sum
  void allreduce_bf16(int64_t ptr_f32, int64_t scratch_bf16, int64_t count, int64_t compute_stream);
  void broadcast(int64_t ptr, int64_t count, int dtype, int root, int64_t compute_stream);
  void wait(int64_t compute_stream);
  // ordering probe (tests, HQ_REDUCER_VERIFY): after the same fence an all-reduce would take, the comm
  // stream writes deterministic per-block sum-of-squares partials of [ptr, ptr+count) to `partials`
  void probe_f32(int64_t ptr, int64_t count, int64_t partials, int nparts, int64_t compute_stream);
  // grad-norm partials of chunks c0 … c1-1 (hq_sq_norm_chunks), on the comm stream right behind the bucket's
  // all-reduce that produced them (no fence: stream order is the dependency)
  void sq_norm_chunks(int64_t grad, int64_t chunks, int c0, int c1, int64_t partials);
  // comm stream waits for all work issued so far on `stream` (e.g. a side stream computing grads)
  void fence_from(int64_t stream);
  void synchronize();
  int64_t comm_stream() const { return (int64_t)stream_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  // ranks the RCCL communicator actually spans (ncclCommCount) — bench.py reports it as proof of world size
  int comm_count() const;

 private:
  static constexpr int kEvents = 64;
  void* next_event();
  int rank_, world_, device_;
  void* comm_ = nullptr;
  void* stream_ = nullptr;
  void* events_[kEvents] = {};
  int ev_idx_ = 0;
};
