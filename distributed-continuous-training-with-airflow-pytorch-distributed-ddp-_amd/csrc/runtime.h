#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace dct {

enum DType { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2, DT_I32 = 3, DT_I64 = 4, DT_U8 = 5 };
enum ROp { OP_SUM = 0, OP_AVG = 1, OP_MAX = 2, OP_MIN = 3 };

std::string comm_unique_id();

class Comm {
 public:
  Comm(const std::string& uid, int world, int rank, int device);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  void allreduce(uintptr_t buf, int64_t count, int dtype, int op, uintptr_t stream);
  void broadcast(uintptr_t buf, int64_t count, int dtype, int root, uintptr_t stream);
  void reduce_scatter(uintptr_t send, uintptr_t recv, int64_t recv_count, int dtype, int op, uintptr_t stream);
  void all_gather(uintptr_t send, uintptr_t recv, int64_t send_count, int dtype, uintptr_t stream);
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  void* comm_ = nullptr;
  int world_ = 1, rank_ = 0, device_ = 0;
};

class BucketReducer {
 public:
  BucketReducer(Comm* comm, uintptr_t flat_grad, std::vector<int64_t> bucket_offsets,
                std::vector<int64_t> bucket_counts, std::vector<int> param_bucket, int dtype, int op);
  ~BucketReducer();
  void prepare();
  int mark_ready(int param_idx, uintptr_t compute_stream);
  void finalize(uintptr_t compute_stream);
  int num_buckets() const { return (int)offsets_.size(); }
  int launched() const { return n_launched_; }
  uintptr_t comm_stream() const { return reinterpret_cast<uintptr_t>(comm_stream_); }

 private:
  void launch_bucket(int b, uintptr_t compute_stream);
  Comm* comm_;
  uintptr_t flat_;
  std::vector<int64_t> offsets_, counts_;
  std::vector<int> param_bucket_, expected_, pending_, launched_;
  int dtype_, op_;
  size_t dsize_ = 4;
  int next_to_launch_ = 0, n_launched_ = 0;
  hipStream_t comm_stream_ = nullptr;
  std::vector<hipEvent_t> ready_events_;
  hipEvent_t done_event_ = nullptr;
};

class StreamGraph {
 public:
  StreamGraph() = default;
  ~StreamGraph();
  void begin(uintptr_t stream);
  void end(uintptr_t stream);
  void replay(uintptr_t stream);
  void reset();
  size_t num_nodes() const;

 private:
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

}  // namespace dct
