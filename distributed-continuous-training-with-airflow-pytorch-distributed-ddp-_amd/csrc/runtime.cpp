// Native distributed runtime: RCCL communicator, gradient bucket reducer, HIP graph capture.
//
// Reference parity: the reference's collectives are all implicit inside
// Lightning/torch DDP over gloo/TCP - Reducer buckets (X5, 2,056 B per step), the
// sync_dist scalar all-reduces (X6/X7), broadcasts of the initial state (X3) and barriers
// (X9).  This file is the MI355X replacement: one RCCL communicator per process (the torch
// "nccl" backend on ROCm is RCCL too; owning the comm directly lets the C++ step executor
// issue collectives with no Python on the path and capture them into hipGraphs), a
// bucketed reducer whose buckets are views of ONE flat gradient buffer (no copy-in/out),
// all-reduced with ncclAvg on a dedicated comm stream as soon as the backward kernels that
// produce each bucket have been enqueued (event-ordered overlap with the rest of backward),
// and a thin stream-capture wrapper used to collapse launch-bound step loops.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.h"
#include "runtime.h"

namespace dct {

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
static void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

static ncclDataType_t to_nccl_dtype(int dt) {
  switch (dt) {
    case DT_F32: return ncclFloat32;
    case DT_BF16: return ncclBfloat16;
    case DT_F16: return ncclFloat16;
    case DT_I32: return ncclInt32;
    case DT_I64: return ncclInt64;
    case DT_U8: return ncclUint8;
    default: throw std::runtime_error("unsupported dtype for RCCL");
  }
}
static ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case OP_SUM: return ncclSum;
    case OP_AVG: return ncclAvg;
    case OP_MAX: return ncclMax;
    case OP_MIN: return ncclMin;
    default: throw std::runtime_error("unsupported reduce op");
  }
}

std::string comm_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

Comm::Comm(const std::string& uid, int world, int rank, int device) : world_(world), rank_(rank), device_(device) {
  if ((int)uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("bad RCCL unique id size");
  hip_check(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c;
  nccl_check(ncclCommInitRank(&c, world, id, rank), "ncclCommInitRank");
  comm_ = c;
  // An in-place all-reduce / broadcast over ONE rank is the identity (x / 1 is exact in fp32), yet
  // RCCL's one-rank path runs a pre-multiply kernel plus ~4 blit copies / fills per call (~13 us on
  // MI355X, profiles/rccl_one_rank_r4.log).  One-rank communicators (a DDP job of world size 1, the
  // DCT_FORCE_DDP=1 rehearsals) skip it; DCT_RCCL_ONE_RANK=1 calls RCCL anyway.
  dct::knobs_reload();
  identity_ = world == 1 && !dct::knobs().rccl_one_rank;
}

Comm::~Comm() {
  if (comm_) ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm_));
}

void Comm::allreduce(uintptr_t buf, int64_t count, int dtype, int op, uintptr_t stream) {
  if (count <= 0 || identity_) return;
  nccl_check(ncclAllReduce(reinterpret_cast<void*>(buf), reinterpret_cast<void*>(buf), (size_t)count,
                           to_nccl_dtype(dtype), to_nccl_op(op), reinterpret_cast<ncclComm_t>(comm_),
                           reinterpret_cast<hipStream_t>(stream)),
             "ncclAllReduce");
}

void Comm::broadcast(uintptr_t buf, int64_t count, int dtype, int root, uintptr_t stream) {
  if (count <= 0 || identity_) return;
  nccl_check(ncclBroadcast(reinterpret_cast<void*>(buf), reinterpret_cast<void*>(buf), (size_t)count,
                           to_nccl_dtype(dtype), root, reinterpret_cast<ncclComm_t>(comm_),
                           reinterpret_cast<hipStream_t>(stream)),
             "ncclBroadcast");
}

void Comm::reduce_scatter(uintptr_t send, uintptr_t recv, int64_t recv_count, int dtype, int op, uintptr_t stream) {
  nccl_check(ncclReduceScatter(reinterpret_cast<void*>(send), reinterpret_cast<void*>(recv), (size_t)recv_count,
                               to_nccl_dtype(dtype), to_nccl_op(op), reinterpret_cast<ncclComm_t>(comm_),
                               reinterpret_cast<hipStream_t>(stream)),
             "ncclReduceScatter");
}

void Comm::all_gather(uintptr_t send, uintptr_t recv, int64_t send_count, int dtype, uintptr_t stream) {
  nccl_check(ncclAllGather(reinterpret_cast<void*>(send), reinterpret_cast<void*>(recv), (size_t)send_count,
                           to_nccl_dtype(dtype), reinterpret_cast<ncclComm_t>(comm_),
                           reinterpret_cast<hipStream_t>(stream)),
             "ncclAllGather");
}

// ------------------------------------------------------------------------- BucketReducer
uintptr_t cu_masked_stream(const std::vector<uint32_t>& mask) {
  hipStream_t s = nullptr;
  hip_check(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
  return reinterpret_cast<uintptr_t>(s);
}

void stream_destroy(uintptr_t stream) { hip_check(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)), "hipStreamDestroy"); }

std::vector<uint32_t> stream_cu_mask(uintptr_t stream) {
  const int n = (device_cu_count() + 31) / 32;
  std::vector<uint32_t> m(n, 0u);
  hip_check(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), (uint32_t)n, m.data()), "hipExtStreamGetCUMask");
  return m;
}

int device_cu_count() {
  int dev = 0, n = 0;
  hip_check(hipGetDevice(&dev), "hipGetDevice");
  hip_check(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  return n;
}

BucketReducer::BucketReducer(Comm* comm, uintptr_t flat_grad, std::vector<int64_t> bucket_offsets,
                             std::vector<int64_t> bucket_counts, std::vector<int> param_bucket, int dtype,
                             int op)
    : comm_(comm),
      flat_(flat_grad),
      offsets_(std::move(bucket_offsets)),
      counts_(std::move(bucket_counts)),
      param_bucket_(std::move(param_bucket)),
      dtype_(dtype),
      op_(op) {
  dct::knobs_reload();  // bind time: DCT_REDUCER_INLINE
  const size_t nb = offsets_.size();
  if (counts_.size() != nb) throw std::runtime_error("bucket offsets/counts mismatch");
  expected_.assign(nb, 0);
  for (int b : param_bucket_) {
    if (b < 0 || (size_t)b >= nb) throw std::runtime_error("param bucket index out of range");
    expected_[b]++;
  }
  pending_.assign(nb, 0);
  launched_.assign(nb, 0);
  // (normal priority: a greatest-priority comm stream made the forced-DDP tabular step with the stand-in
  // collective 0.187 -> 0.705 ms and the TabTransformer one 0.42 -> 1.16 ms, profiles/ddp_reducer_standin_ab_r5.log)
  hip_check(hipStreamCreateWithFlags(&comm_stream_, hipStreamNonBlocking), "hipStreamCreate");
  // Where the collectives run (DCT_REDUCER_INLINE, read once here into this reducer's copy):
  //   -2 (auto, default): on the compute stream for a one-rank communicator (the identity: no
  //      collective runs, and fork / join edges would cost time for nothing); otherwise on the comm
  //      stream in eager steps, so each bucket's all-reduce overlaps the rest of backward (the DDP
  //      Reducer's point, reference jobs/train_lightning_ddp.py:136): forced-DDP tabular step with a
  //      60 us stand-in collective 0.187 ms vs 0.235 inline (profiles/ddp_reducer_standin_ab_r5.log) -
  //      and on the compute stream while a step is captured: the TabTransformer's replayed step lost
  //      with the collectives beside it (0.435-0.437 vs 0.425-0.428 ms inline) - its backward kernels
  //      fill every CU's VGPRs and LDS at exactly one workgroup round, so any co-resident comm wave
  //      pushes a workgroup into a second round;
  //    1 / 0: always the compute / the comm stream (0 with a captured step: the graph's event edges);
  //   -1: inline while the compute stream is capturing.
  // The test-only stand-in collective (DCT_REDUCER_STANDIN_US) counts as a real collective.
  //   With real peers (world > 1) the auto mode keeps the collectives on the compute stream too: RCCL's
  //   fp32 sum / average kernels (runRing / runTreeSplit / runTreeUpDown over FuncSum<float> and
  //   FuncPreMulSum<float> in librccl's gfx950 code object) compute with v_pk_add_f32, and packed fp32
  //   in a kernel whose waves share a CU with LDS-DMA traffic - the operand path of every gemm2 tile
  //   this runtime launches - goes wrong now and then (tools/probes/adam_ride_probe.hip mode 8: an
  //   Adam kernel on a second stream beside GEMM-only launches, 58 of 60 launches with wrong low
  //   halves; profiles/packed_fp32_lds_dma_r6.log).  A collective overlapping the backward GEMMs could
  //   therefore return a wrong gradient sum with no error; inline, nothing runs beside it.
  //   DCT_REDUCER_INLINE=0 / -1 still selects the comm stream (stand-in measurements, or steps whose
  //   kernels use no LDS-DMA).
  const Knobs& k = dct::knobs();
  standin_us_ = k.reducer_standin_us;
  standin_wgs_ = k.reducer_standin_wgs;
  inline_knob_ = k.reducer_inline;
  const bool real_peers = comm_ != nullptr && comm_->world() > 1 && !comm_->is_identity();
  if (inline_knob_ == -2) {
    const bool identity = comm_ == nullptr || (comm_->world() == 1 && comm_->is_identity());
    inline_knob_ = ((identity && standin_us_ == 0) || real_peers) ? 1 : -1;
    auto_inline_ = true;
  }
  inline_ = inline_knob_ == 1;
  for (int64_t c : counts_) total_count_ += c;
  // A communicator with real peers (world > 1, not the one-rank identity): RCCL transports may read
  // the send buffer straight from a peer GPU, so the fork events keep the default system-scope
  // release until a multi-GPU run has confirmed that the device scope suffices; the
  // join is an event wait (unbounded, see edge()).  One-rank / stand-in communicators: fork / join
  // between two streams of ONE device, where a device-scope release is all the collective (and
  // Adam after the join) needs, not the system-scope fence (its cache writeback / invalidate is
  // most of an edge's cost).
  peer_world_ = real_peers;
  const unsigned ev_flags = peer_world_ ? hipEventDisableTiming : (hipEventDisableTiming | hipEventReleaseToDevice);
  ready_events_.resize(nb);
  for (auto& e : ready_events_) hip_check(hipEventCreateWithFlags(&e, ev_flags), "hipEventCreate");
  hip_check(hipEventCreateWithFlags(&done_event_, ev_flags), "hipEventCreate");
  dsize_ = (dtype == DT_BF16 || dtype == DT_F16) ? 2 : 4;
  // eager edges' device counters: [nb + 2] signals (buckets, done, timing tail), [nb + 2] consumed, status
  if ((!inline_ || inline_knob_ != 1) && k.reducer_flag_edges) {
    const size_t bytes = (2 * (nb + 2) + 1) * sizeof(int);
    hip_check(hipMalloc(&dsync_, bytes), "hipMalloc edge counters");
    hip_check(hipMemset(dsync_, 0, bytes), "hipMemset edge counters");
    // the wait kernels' timeout word in coherent host memory: prepare() reads it every step with
    // no synchronisation and throws, so an expired edge can never go unnoticed
    hip_check(hipHostMalloc(reinterpret_cast<void**>(&status_host_), sizeof(int),
                            hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc edge status");
    *status_host_ = 0;
    hip_check(hipHostGetDevicePointer(reinterpret_cast<void**>(&status_dev_), status_host_, 0),
              "hipHostGetDevicePointer edge status");
  }
}

BucketReducer::~BucketReducer() {
  for (auto& e : ready_events_) hipEventDestroy(e);
  if (done_event_) hipEventDestroy(done_event_);
  if (tail_event_) hipEventDestroy(tail_event_);
  if (stamps_) hipFree(stamps_);
  if (dsync_) hipFree(dsync_);
  if (status_host_) hipHostFree(status_host_);
  if (comm_stream_) hipStreamDestroy(comm_stream_);
}

void BucketReducer::prepare() {
  check_edges();
  std::fill(pending_.begin(), pending_.end(), 0);
  std::fill(launched_.begin(), launched_.end(), 0);
  next_to_launch_ = 0;
  n_launched_ = 0;
}

void BucketReducer::enable_timing(bool check) {
  if (!stamps_) {
    hip_check(hipMalloc(&stamps_, 8 * sizeof(unsigned long long)), "hipMalloc stamps");
    hip_check(hipMemset(stamps_, 0, 8 * sizeof(unsigned long long)), "hipMemset stamps");
    hip_check(hipEventCreateWithFlags(&tail_event_, hipEventDisableTiming), "hipEventCreate");
  }
  timing_ = true;
  check_ = check;
}

std::vector<double> BucketReducer::read_timing() const {
  std::vector<double> out(4, 0.0);
  if (!stamps_) return out;
  unsigned long long h[8];
  // the close kernel of the last step runs on the non-blocking comm stream, or inline on the
  // caller's compute stream: a legacy-stream copy is ordered after neither
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  hip_check(hipMemcpy(h, stamps_, sizeof(h), hipMemcpyDeviceToHost), "read reducer stamps");
  out[0] = (double)h[2] / 1e5;  // s_memrealtime ticks at 100 MHz -> ms
  out[1] = (double)h[3] / 1e5;
  out[2] = (double)h[7];
  out[3] = (double)h[6];
  return out;
}

void BucketReducer::reset_timing() {
  if (!stamps_) return;
  hip_check(hipDeviceSynchronize(), "reset_timing sync");
  unsigned long long h[8];
  hip_check(hipMemcpy(h, stamps_, sizeof(h), hipMemcpyDeviceToHost), "read reducer stamps");
  h[2] = h[3] = h[6] = h[7] = 0;  // keep the close / check counters in step with each other
  hip_check(hipMemcpy(stamps_, h, sizeof(h), hipMemcpyHostToDevice), "reset reducer stamps");
}

void BucketReducer::set_comm_cu_mask(const std::vector<uint32_t>& mask) {
  hipStream_t s = nullptr;
  hip_check(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
  hip_check(hipStreamSynchronize(comm_stream_), "hipStreamSynchronize");
  hip_check(hipStreamDestroy(comm_stream_), "hipStreamDestroy");
  comm_stream_ = s;
  comm_mask_ = mask;
  checked_stream_ = nullptr;
}

// true when the compute stream's CU mask shares no CU with the comm stream's (reserved CUs)
bool BucketReducer::disjoint_from_comm(hipStream_t compute) {
  if (comm_mask_.empty()) return false;
  if (compute == checked_stream_) return checked_disjoint_;
  std::vector<uint32_t> cm(comm_mask_.size(), 0u);
  bool ok = compute != nullptr &&
            hipExtStreamGetCUMask(compute, (uint32_t)cm.size(), cm.data()) == hipSuccess;
  if (!ok) (void)hipGetLastError();
  for (size_t i = 0; ok && i < cm.size(); ++i) ok = (cm[i] & comm_mask_[i]) == 0u;
  checked_stream_ = compute;
  checked_disjoint_ = ok;
  return ok;
}

bool BucketReducer::step_inline(void* compute_stream) {
  // real peers, auto placement: inline unless the collectives own CUs the compute stream cannot use
  // (set_comm_cu_mask) - then eager steps overlap them, captured ones keep them inline (-1 below)
  const bool reserved = peer_world_ && auto_inline_ && disjoint_from_comm(reinterpret_cast<hipStream_t>(compute_stream));
  if (inline_knob_ >= 0 && !reserved) return inline_knob_ == 1;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(reinterpret_cast<hipStream_t>(compute_stream), &st) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return st == hipStreamCaptureStatusActive;
}

// One cross-stream edge (from -> to) of a step: eagerly a device counter (dct_flag_signal /
// dct_flag_wait, csrc/step_kernels.hip - a one-wave kernel per side instead of an event record and
// wait, which held the queues 6-13 us each); under stream capture an event (the graph's edge).
// The signal is always enqueued before its wait, so two streams that share one hardware queue
// (more streams than GPU_MAX_HW_QUEUES) serialise but never deadlock.  (A captured step whose
// graph only signalled the buckets, with the collectives enqueued eagerly on the comm stream before
// each replay, did deadlock there until the wait bound: the replay's join sat ahead of its own
// collectives in the shared queue - removed again, profiles/ddp_reducer_standin_ab_r5.log.)
// The flag wait is bounded (a spinning wave must end); an expired wait is recorded in status_host_
// and prepare() throws at the next step.  `join` = the comm -> compute edge at the end of a step:
// with real peers its producer (the collective) waits on OTHER ranks - a peer seconds behind (rank 0
// writing a checkpoint, a validation pass, RCCL's first connections) would expire a bounded wait -
// so that edge is an event wait, unbounded like the reference DDP's own.  The fork
// edges' producers are this rank's backward kernels, which never wait on a peer.
void BucketReducer::edge(int slot, hipEvent_t ev, hipStream_t from, hipStream_t to, bool join) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(from, &cap) != hipSuccess) {
    (void)hipGetLastError();
    cap = hipStreamCaptureStatusNone;
  }
  if (cap == hipStreamCaptureStatusNone && dsync_ && !(join && peer_world_)) {
    const int ns = (int)offsets_.size() + 2;
    hip_check((hipError_t)dct_flag_signal(dsync_ + slot, from), "edge signal");
    hip_check((hipError_t)dct_flag_wait(dsync_ + slot, dsync_ + ns + slot, status_dev_, to), "edge wait");
    return;
  }
  hip_check(hipEventRecord(ev, from), "hipEventRecord");
  hip_check(hipStreamWaitEvent(to, ev, 0), "hipStreamWaitEvent");
}

int BucketReducer::edge_timeouts() const {
  if (!status_host_) return 0;
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return *reinterpret_cast<volatile int*>(status_host_);
}

void BucketReducer::check_edges() const {
  // no synchronisation: the word reflects every wait kernel that has run so far
  if (status_host_ && *reinterpret_cast<volatile int*>(status_host_) != 0)
    throw std::runtime_error(
        "DDP bucket reducer: a cross-stream edge wait expired - a collective or the optimizer ran without "
        "its producer, gradients / parameters of this rank are not trustworthy");
}

void BucketReducer::launch_bucket(int b, uintptr_t compute_stream) {
  hipStream_t cs = reinterpret_cast<hipStream_t>(compute_stream);
  inline_ = step_inline(cs);
  hipStream_t rs = inline_ ? cs : comm_stream_;
  if (!inline_) edge(b, ready_events_[b], cs, comm_stream_);
  if (timing_ && b == 0)
    hip_check((hipError_t)dct_reducer_stamp(stamps_, reinterpret_cast<void*>(rs)), "reducer stamp");
  collective(b, rs);
  launched_[b] = 1;
  n_launched_++;
}

void BucketReducer::collective(int b, hipStream_t rs) {
  if (comm_) {
    comm_->allreduce(flat_ + (uintptr_t)(offsets_[b] * dsize_), counts_[b], dtype_, op_,
                     reinterpret_cast<uintptr_t>(rs));
  }
  if (standin_us_ > 0 && total_count_ > 0) {
    // stand-in collective: busy workgroups for this bucket's share of the per-step time
    const double us = (double)standin_us_ * (double)counts_[b] / (double)total_count_;
    hip_check((hipError_t)dct_busy_spin((long long)(us * 100.0), standin_wgs_, reinterpret_cast<void*>(rs)),
              "stand-in collective");
  }
}

// Buckets are launched strictly in index order (bucket 0 = last layers, filled first by
// backward) so every rank issues the collectives in the same order even when hooks fire in
// a different order on different ranks.
int BucketReducer::mark_ready(int param_idx, uintptr_t compute_stream) {
  if (param_idx < 0 || (size_t)param_idx >= param_bucket_.size()) throw std::runtime_error("param index out of range");
  const int b = param_bucket_[param_idx];
  pending_[b]++;
  if (pending_[b] > expected_[b]) throw std::runtime_error("parameter marked ready twice in one step");
  int launched_now = 0;
  while (next_to_launch_ < (int)offsets_.size() && pending_[next_to_launch_] == expected_[next_to_launch_]) {
    launch_bucket(next_to_launch_, compute_stream);
    next_to_launch_++;
    launched_now++;
  }
  return launched_now;
}

void BucketReducer::finalize(uintptr_t compute_stream) {
  hipStream_t cs = reinterpret_cast<hipStream_t>(compute_stream);
  inline_ = step_inline(cs);
  hipStream_t rs = inline_ ? cs : comm_stream_;
  n_before_finalize_ = n_launched_;
  if (timing_) {  // end of backward on the compute stream, ordered before the comm stream's close
    hip_check((hipError_t)dct_reducer_stamp(stamps_ + 1, reinterpret_cast<void*>(cs)), "reducer stamp");
    if (!inline_) edge((int)offsets_.size() + 1, tail_event_, cs, comm_stream_);
  }
  // buckets whose params did not all receive a gradient (unused params): reduce anyway so
  // the collective sequence matches across ranks (find_unused_parameters=False semantics
  // would error; we zero-fill instead, which is what DDP's static graph does).
  while (next_to_launch_ < (int)offsets_.size()) {
    launch_bucket(next_to_launch_, compute_stream);
    next_to_launch_++;
  }
  if (timing_) hip_check((hipError_t)dct_reducer_close(stamps_, reinterpret_cast<void*>(rs)), "reducer close");
  if (!inline_) edge((int)offsets_.size(), done_event_, comm_stream_, cs, /*join=*/true);
  if (timing_ && check_) hip_check((hipError_t)dct_reducer_check(stamps_, reinterpret_cast<void*>(cs)), "reducer check");
}

// ---------------------------------------------------------------------------- StreamGraph
StreamGraph::~StreamGraph() { reset(); }

void StreamGraph::reset() {
  if (exec_) hipGraphExecDestroy(exec_);
  if (graph_) hipGraphDestroy(graph_);
  exec_ = nullptr;
  graph_ = nullptr;
}

void StreamGraph::begin(uintptr_t stream) {
  reset();
  hip_check(hipStreamBeginCapture(reinterpret_cast<hipStream_t>(stream), hipStreamCaptureModeThreadLocal),
            "hipStreamBeginCapture");
}

void StreamGraph::end(uintptr_t stream) {
  hip_check(hipStreamEndCapture(reinterpret_cast<hipStream_t>(stream), &graph_), "hipStreamEndCapture");
  hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "hipGraphInstantiate");
}

void StreamGraph::replay(uintptr_t stream) {
  if (!exec_) throw std::runtime_error("graph not captured");
  hip_check(hipGraphLaunch(exec_, reinterpret_cast<hipStream_t>(stream)), "hipGraphLaunch");
}

size_t StreamGraph::num_nodes() const {
  if (!graph_) return 0;
  size_t n = 0;
  hipGraphGetNodes(graph_, nullptr, &n);
  return n;
}

// ------------------------------------------------------------------------ PeerExchange
PeerExchange::PeerExchange(int world, int rank, int64_t bytes) : world_(world), rank_(rank), bytes_(bytes) {
  if (world < 1 || rank < 0 || rank >= world || bytes <= 0) throw std::invalid_argument("PeerExchange: bad arguments");
  // exchange slabs, then the barrier region (BARRIER_BYTES: one 16-B slot per source rank)
  hip_check(hipExtMallocWithFlags(&recv_, (size_t)(bytes + BARRIER_BYTES), hipDeviceMallocUncached),
            "hipExtMallocWithFlags(uncached)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&d_peers_), sizeof(void*) * world), "hipMalloc(peers)");
  hip_check(hipMalloc(reinterpret_cast<void**>(&status_), 64), "hipMalloc(status)");
  hip_check(hipMemset(recv_, 0, (size_t)(bytes + BARRIER_BYTES)), "hipMemset(recv)");
  hip_check(hipMemset(status_, 0, 64), "hipMemset(status)");
  std::vector<void*> self(world, nullptr);
  self[rank] = recv_;
  upload(self);
}

PeerExchange::~PeerExchange() {
  hipDeviceSynchronize();
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  if (recv_) hipFree(recv_);
  if (d_peers_) hipFree(d_peers_);
  if (status_) hipFree(status_);
}

void PeerExchange::upload(const std::vector<void*>& ptrs) {
  hip_check(hipMemcpy(d_peers_, ptrs.data(), sizeof(void*) * world_, hipMemcpyHostToDevice), "hipMemcpy(peers)");
}

std::string PeerExchange::ipc_handle() const {
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, recv_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void PeerExchange::open_peers(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::invalid_argument("PeerExchange: need one handle per rank");
  std::vector<void*> ptrs(world_, nullptr);
  for (int q = 0; q < world_; ++q) {
    if (q == rank_) {
      ptrs[q] = recv_;
      continue;
    }
    if (handles[q].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("PeerExchange: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[q].data(), sizeof(h));
    void* p = nullptr;
    hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(p);
    ptrs[q] = p;
  }
  upload(ptrs);
}

void PeerExchange::set_peers(const std::vector<uintptr_t>& addrs) {
  if ((int)addrs.size() != world_) throw std::invalid_argument("PeerExchange: need one address per rank");
  std::vector<void*> ptrs(world_);
  for (int q = 0; q < world_; ++q) ptrs[q] = reinterpret_cast<void*>(addrs[q]);
  upload(ptrs);
}

void PeerExchange::barrier(uintptr_t stream, double timeout_s) {
  // every rank calls barrier() the same number of times (a collective), so the call count is a
  // tag no earlier barrier wrote; reset() zeroes the region and tags keep counting from here
  const unsigned tag = ++bar_count_;
  const long long ticks = (long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  hip_check((hipError_t)dct_xg_barrier(recv_, reinterpret_cast<void* const*>(d_peers_), bytes_, status_, world_, rank_,
                                       tag, ticks, reinterpret_cast<void*>(stream)),
            "xg_barrier");
}

unsigned int PeerExchange::read_status() const {
  unsigned int v = 0;
  hip_check(hipMemcpy(&v, status_, sizeof(v), hipMemcpyDeviceToHost), "hipMemcpy(status)");
  return v;
}

void PeerExchange::reset(uintptr_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hip_check(hipMemsetAsync(recv_, 0, (size_t)(bytes_ + BARRIER_BYTES), st), "hipMemsetAsync(recv)");
  hip_check(hipMemsetAsync(status_, 0, 64, st), "hipMemsetAsync(status)");
}

}  // namespace dct
