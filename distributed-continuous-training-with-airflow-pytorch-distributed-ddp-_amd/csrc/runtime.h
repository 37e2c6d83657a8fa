#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace dct {

enum DType { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2, DT_I32 = 3, DT_I64 = 4, DT_U8 = 5 };
enum ROp { OP_SUM = 0, OP_AVG = 1, OP_MAX = 2, OP_MIN = 3 };

std::string comm_unique_id();
// a stream restricted to the CUs set in `mask` (32 CUs per word, hipExtStreamCreateWithCUMask), its
// mask read back, and the device's CU count: CU reservation for the bucket reducer's collectives
uintptr_t cu_masked_stream(const std::vector<uint32_t>& mask);
void stream_destroy(uintptr_t stream);
std::vector<uint32_t> stream_cu_mask(uintptr_t stream);
int device_cu_count();

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
  bool is_identity() const { return identity_; }
  int device() const { return device_; }

 private:
  void* comm_ = nullptr;
  int world_ = 1, rank_ = 0, device_ = 0;
  bool identity_ = false;  // one rank: in-place collectives are the identity, RCCL is not called
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
  // buckets the mark_ready hooks launched before finalize() in the last step: > 0 means the
  // all-reduce really overlapped (part of) the backward
  int launched_before_finalize() const { return n_before_finalize_; }
  uintptr_t comm_stream() const { return reinterpret_cast<uintptr_t>(comm_stream_); }
  bool inline_mode() const { return inline_; }
  // device-side instrumentation (also inside captured graphs): span / exposed all-reduce time per
  // step; with `check` a compute-stream kernel after the join verifies the stream ordering
  void enable_timing(bool check);
  // {span_ms, exposed_ms, steps, ordering_violations} accumulated since the last reset
  std::vector<double> read_timing() const;
  void reset_timing();
  // 1 if an eager cross-stream edge's wait expired (its consumer went on without the producer)
  int edge_timeouts() const;
  // throws if an edge wait has expired (no synchronisation; prepare() calls it every step)
  void check_edges() const;
  bool peer_world() const { return peer_world_; }
  // run the collectives on a stream restricted to these CUs (hipExtStreamCreateWithCUMask bit words):
  // with a compute stream whose mask excludes every one of them (cu_masked_stream), no collective
  // kernel ever shares a CU with the backward's kernels (the packed-fp32 / LDS-DMA hazard below), so
  // the comm stream is allowed with real peers too
  void set_comm_cu_mask(const std::vector<uint32_t>& mask);
  std::vector<uint32_t> comm_cu_mask() const { return comm_mask_; }

 private:
  bool disjoint_from_comm(hipStream_t compute);
  void launch_bucket(int b, uintptr_t compute_stream);
  void edge(int slot, hipEvent_t ev, hipStream_t from, hipStream_t to, bool join = false);
  void collective(int b, hipStream_t rs);
  Comm* comm_;
  uintptr_t flat_;
  std::vector<int64_t> offsets_, counts_;
  std::vector<int> param_bucket_, expected_, pending_, launched_;
  int dtype_, op_;
  size_t dsize_ = 4;
  int next_to_launch_ = 0, n_launched_ = 0, n_before_finalize_ = 0;
  hipStream_t comm_stream_ = nullptr;
  std::vector<uint32_t> comm_mask_;         // set_comm_cu_mask (empty: every CU)
  hipStream_t checked_stream_ = nullptr;   // last compute stream tested against comm_mask_
  bool checked_disjoint_ = false;
  bool auto_inline_ = false;  // DCT_REDUCER_INLINE auto (-2) chose the placement
  std::vector<hipEvent_t> ready_events_;
  hipEvent_t done_event_ = nullptr;
  hipEvent_t tail_event_ = nullptr;
  int* dsync_ = nullptr;  // eager edges' device counters (edge())
  int* status_host_ = nullptr;  // edge-wait timeout word, coherent host memory (check_edges())
  int* status_dev_ = nullptr;   // its device address
  bool peer_world_ = false;     // a communicator with real peers (world > 1)
  unsigned long long* stamps_ = nullptr;  // [8], see step_kernels.hip reducer_close_kernel
  bool timing_ = false, check_ = false;
  int inline_knob_ = -1;  // DCT_REDUCER_INLINE resolved (1 / 0 / -1 = inline while the compute stream is capturing)
  int standin_us_ = 0, standin_wgs_ = 16;  // DCT_REDUCER_STANDIN_US / _WGS (test-only stand-in collective)
  int64_t total_count_ = 0;
  bool inline_ = false;   // this step's choice (collectives on the compute stream)
  bool step_inline(void* compute_stream);
};

// Receive buffers of the in-kernel (xGMI) gradient exchange.  Each rank allocates an
// UNCACHED device buffer (remote xGMI writes land in HBM, the local poll must not hit a stale
// L2 line), exports it as an IPC handle, and maps every peer's buffer into its own address
// space; `peers()` is a device array of the W buffer addresses, indexed by rank.
class PeerExchange {
 public:
  PeerExchange(int world, int rank, int64_t bytes);
  ~PeerExchange();
  PeerExchange(const PeerExchange&) = delete;
  PeerExchange& operator=(const PeerExchange&) = delete;
  std::string ipc_handle() const;                          // this rank's buffer
  void open_peers(const std::vector<std::string>& handles);  // all ranks' handles, rank order
  void set_peers(const std::vector<uintptr_t>& ptrs);        // same process (tests): raw addresses
  void reset(uintptr_t stream);                              // zero receive buffer + status
  void barrier(uintptr_t stream, double timeout_s);          // device-side barrier over the peer mappings
  unsigned int read_status() const;                          // synchronous D2H of status[0]
  uintptr_t recv() const { return reinterpret_cast<uintptr_t>(recv_); }
  uintptr_t peers() const { return reinterpret_cast<uintptr_t>(d_peers_); }
  uintptr_t status() const { return reinterpret_cast<uintptr_t>(status_); }
  int64_t bytes() const { return bytes_; }
  int world() const { return world_; }
  int rank() const { return rank_; }

 private:
  void upload(const std::vector<void*>& ptrs);
  int world_, rank_;
  int64_t bytes_;
  void* recv_ = nullptr;
  void** d_peers_ = nullptr;
  unsigned int* status_ = nullptr;
  std::vector<void*> opened_;
  unsigned bar_count_ = 0;
  static constexpr int64_t BARRIER_BYTES = 16 * 64;
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
