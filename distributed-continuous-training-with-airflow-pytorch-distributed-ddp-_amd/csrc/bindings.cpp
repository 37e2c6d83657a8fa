// pybind11 module `_dct_native`: the Python face of the HIP kernels and the C++ runtime.
// Tensors cross the boundary as raw device pointers (validated for shape/dtype/device by
// the Python wrappers in ops/ before any launch) and streams as hipStream_t handles, so the
// module has no libtorch dependency and builds in seconds with hipcc.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels.h"
#include "mlp_fused.h"
#include "runtime.h"
#include "mlp_executor.h"

namespace py = pybind11;

static void check(int err, const char* what) {
  if (err != 0) {
    throw std::runtime_error(std::string(what) + " failed: " + hipGetErrorString((hipError_t)err));
  }
}

template <class T>
static T* P(uintptr_t x) {
  return reinterpret_cast<T*>(x);
}

struct MlpPlan {
  std::vector<char> shape;
  int nt = 0, maxblk = 0, supported = 0;
  int use_wave = 0;  // single-wave register-resident kernel (narrow MLPs), see mlp_wave.hip
  MlpPlan(const std::vector<int>& dims, int bmax) {
    if (dims.size() < 2 || dims.size() > 5) throw std::invalid_argument("MLP needs 1..4 linear layers");
    for (int d : dims)
      if (d < 1 || d > 4096) throw std::invalid_argument("MLP layer width out of range");
    shape.resize(dct_mlp_shape_size());
    if (dct_mlp_make_shape(shape.data(), dims.data(), (int)dims.size() - 1, bmax) != 0)
      throw std::invalid_argument("bad MLP shape");
    supported = dct_mlp_select(sh(), &nt, &maxblk);
    dct::knobs_reload();  // plan time: the DCT_* knobs of this process's launches
    reinterpret_cast<dct::MlpShape*>(shape.data())->mlp_block = dct::knobs().mlp_block;
    const bool force_lds = dct::knobs().mlp_force_lds != 0;
    use_wave = (!force_lds && dct_mlp_wave_supported(dims.data(), (int)dims.size() - 1, 1)) ? 1 : 0;
    if (use_wave) supported = 1;
  }
  const dct::MlpShape* sh() const { return reinterpret_cast<const dct::MlpShape*>(shape.data()); }
};


// Validated MlpArgs of a training launch (the kernels trust their arguments).
static dct::MlpArgs make_train_args(const MlpPlan& plan, uintptr_t p, uintptr_t mo, uintptr_t vo, uintptr_t grad_out,
                                    uintptr_t X, int ldx, uintptr_t Y, uintptr_t idx, int n_items, int B, int steps,
                                    int t0, float lr, float b1, float b2, float eps, float wd, float dropout,
                                    uint32_t seed, uint32_t step_base, uintptr_t loss_out, int mode, int loss_kind,
                                    uintptr_t step_counter, uintptr_t cursor, uintptr_t prof, uintptr_t pending,
                                    uintptr_t stage, uintptr_t xg_recv, uintptr_t xg_peers, int xg_world, int xg_rank,
                                    uintptr_t xg_status, int64_t xg_timeout, int xg_poll) {
  if (!plan.supported) throw std::runtime_error("MLP too large for the fused kernel");
  if (steps < 1 || n_items < 1 || B < 1) throw std::invalid_argument("empty launch");
  if (!cursor && (int64_t)(steps - 1) * B >= n_items) throw std::invalid_argument("more steps than batches");
  dct::MlpArgs a{};
  a.p = P<float>(p);
  a.m = P<float>(mo);
  a.v = P<float>(vo);
  a.grad_out = P<float>(grad_out);
  a.X = P<const float>(X);
  a.ldx = ldx;
  a.Y = P<const int>(Y);
  a.idx = P<const int>(idx);
  a.n_items = n_items;
  a.B = B;
  a.steps = steps;
  a.t0 = t0;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd;
  a.dropout = dropout;
  // float arithmetic as the kernels' own derivation (same roundings on host and device)
  a.k_drop_scale = dropout > 0.f ? 1.0f / (1.0f - dropout) : 1.0f;
  a.k_l2b1 = std::log2(b1);
  a.k_l2b2 = std::log2(b2);
  a.k_rc1 = 1.f / (1.f - b1);
  a.k_rc2 = 1.f / (1.f - b2);
  a.k_sqc2 = std::sqrt(1.f - b2);
  a.seed = seed;
  a.step_base = step_base;
  a.loss_out = P<float>(loss_out);
  a.mode = mode;
  a.loss_kind = loss_kind;
  a.step_counter = P<int>(step_counter);
  a.cursor = P<int>(cursor);
  a.prof = P<unsigned long long>(prof);
  a.pending = P<int>(pending);
  a.stage = P<uint32_t>(stage);
  a.xg_recv = P<unsigned long long>(xg_recv);
  a.xg_peers = P<unsigned long long* const>(xg_peers);
  a.xg_world = xg_world;
  a.xg_rank = xg_rank;
  a.xg_status = P<unsigned int>(xg_status);
  a.xg_timeout = xg_timeout;
  a.xg_poll = xg_poll;
  if (xg_world > 1) {
    const dct::MlpShape* sh = plan.sh();
    const bool wave = plan.use_wave && dct_mlp_wave_supported(sh->dims, sh->L, B);
    const bool blk5 = !plan.use_wave && mode == 0 && dct::mlp_block5_shape_ok(sh->dims, sh->L, B) &&
                      dct::mlp_block5_xg_bytes(xg_world) > 0;
    if (!wave && !blk5)
      throw std::invalid_argument("in-kernel all-reduce needs the single-wave kernel or the 3x128 block kernel "
                                  "(train mode, 2 / 4 / 8 ranks)");
    if (!xg_recv || !xg_peers || !xg_status || xg_rank < 0 || xg_rank >= xg_world)
      throw std::invalid_argument("in-kernel all-reduce: exchange buffers / rank missing");
  }
  if (pending && (mode != 1 || !plan.use_wave || !mo || !vo))
    throw std::invalid_argument("update-then-grad needs grad mode, m/v and the single-wave kernel");
  if (cursor && mode != 1) throw std::invalid_argument("cursor is only valid in grad mode");
  if (mode == 1 && !grad_out) throw std::invalid_argument("grad mode needs grad_out");
  if (mode == 1 && steps != 1) throw std::invalid_argument("grad mode runs exactly one step");
  return a;
}

static void launch_train(const MlpPlan& plan, const dct::MlpArgs& a, uintptr_t stream) {
  const dct::MlpShape* sh = plan.sh();
  if (plan.use_wave && dct_mlp_wave_supported(sh->dims, sh->L, a.B))
    check(dct_mlp_wave_train(sh->dims, sh->L, &a, reinterpret_cast<void*>(stream)), "mlp_wave_train");
  else
    check(dct_mlp_train(plan.shape.data(), &a, reinterpret_cast<void*>(stream)), "mlp_train");
}

// A training launch with every operand bound once (FusedMLPKernel.prepare_train validates
// them in Python): run(first_step, steps, stream) only offsets the index list and the loss
// slots, so a persistent epoch launch costs one short positional call instead of ~35
// keyword arguments and the Python-side operand checks.
struct MlpLaunch {
  MlpPlan plan;
  dct::MlpArgs base{};
  int64_t n_items = 0;   // index entries bound at base.idx
  int64_t loss_len = 0;  // loss slots bound at base.loss_out (0 = none)
  void run(int first_step, int steps, uintptr_t stream) const {
    if (first_step < 0 || steps < 1) throw std::invalid_argument("MlpLaunch.run: bad step range");
    const int64_t off = (int64_t)first_step * base.B;
    if (off + (int64_t)(steps - 1) * base.B >= n_items) throw std::invalid_argument("MlpLaunch.run: past the index list");
    if (base.loss_out && first_step + steps > loss_len) throw std::invalid_argument("MlpLaunch.run: past the loss buffer");
    dct::MlpArgs a = base;
    a.idx = base.idx + off;
    a.n_items = (int)(n_items - off);
    a.steps = steps;
    if (base.loss_out) a.loss_out = base.loss_out + first_step;
    launch_train(plan, a, stream);
  }
};

PYBIND11_MODULE(_dct_native, m) {
  m.doc() = "MI355X-native kernels and runtime for dct_amd";

  // ------------------------------------------------------------------ device info
  m.def("device_count", []() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    return e == hipSuccess ? n : 0;
  });
  m.def("arch_name", [](int dev) {
    hipDeviceProp_t p;
    check((int)hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
    return std::string(p.gcnArchName);
  });
  m.def("synchronize", []() { check((int)hipDeviceSynchronize(), "hipDeviceSynchronize"); });
  // re-read the DCT_* knobs (csrc/knobs.h) - plan / bind time only, never per launch
  m.def("reload_knobs", []() { dct::knobs_reload(); });
  // the struct the launchers read (introspection / tests)
  m.def("knobs", []() {
    const dct::Knobs& k = dct::knobs();
    py::dict d;
    d["mlp_force_lds"] = k.mlp_force_lds; d["mlp_block"] = k.mlp_block; d["fused_head"] = k.fused_head;
    d["dw_into_adam"] = k.dw_into_adam; d["reducer_inline"] = k.reducer_inline; d["rccl_one_rank"] = k.rccl_one_rank;
    d["reducer_standin_us"] = k.reducer_standin_us; d["reducer_standin_wgs"] = k.reducer_standin_wgs;
    d["reducer_flag_edges"] = k.reducer_flag_edges;
    return d;
  });
  // PCI bus id of a device: identifies the physical GPU behind a rank (ranks sharing one GPU in a
  // rehearsal report the same id)
  m.def("pci_bus_id", [](int dev) {
    char buf[64] = {0};
    check((int)hipDeviceGetPCIBusId(buf, (int)sizeof(buf), dev), "hipDeviceGetPCIBusId");
    return std::string(buf);
  });
  // hipDeviceCanAccessPeer over every ordered pair of visible devices (1 on the diagonal): the
  // xGMI peer matrix the in-kernel exchange depends on
  m.def("peer_matrix", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    std::vector<std::vector<int>> mat(n, std::vector<int>(n, 0));
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        int ok = (i == j) ? 1 : 0;
        if (i != j && hipDeviceCanAccessPeer(&ok, i, j) != hipSuccess) ok = 0;
        mat[i][j] = ok;
      }
    return mat;
  });

  // ------------------------------------------------------------------ fused MLP
  py::class_<MlpLaunch>(m, "MlpLaunch")
      .def("run", &MlpLaunch::run, py::arg("first_step"), py::arg("steps"), py::arg("stream"))
      .def_readonly("n_items", &MlpLaunch::n_items)
      .def_readonly("loss_len", &MlpLaunch::loss_len);
  py::class_<MlpPlan>(m, "MlpPlan")
      .def(py::init<const std::vector<int>&, int>(), py::arg("dims"), py::arg("bmax"))
      .def_readonly("supported", &MlpPlan::supported)
      .def_readonly("threads", &MlpPlan::nt)
      .def_readonly("max_blocks_per_thread", &MlpPlan::maxblk)
      .def_readonly("use_wave", &MlpPlan::use_wave)
      .def_property_readonly("num_params", [](const MlpPlan& p) { return p.sh()->P; })
      .def_property_readonly("lds_bytes", [](const MlpPlan& p) { return p.sh()->lds_floats * 4; })
      .def_property_readonly("bmax", [](const MlpPlan& p) { return p.sh()->bmax; })
      .def_property_readonly("mlp_block", [](const MlpPlan& p) { return p.sh()->mlp_block; })
      .def(
          "train",
          [](const MlpPlan& plan, uintptr_t p, uintptr_t mo, uintptr_t vo, uintptr_t grad_out, uintptr_t X, int ldx,
             uintptr_t Y, uintptr_t idx, int n_items, int B, int steps, int t0, float lr, float b1, float b2,
             float eps, float wd, float dropout, uint32_t seed, uint32_t step_base, uintptr_t loss_out, int mode,
             int loss_kind, uintptr_t step_counter, uintptr_t cursor, uintptr_t prof, uintptr_t pending,
             uintptr_t stage, uintptr_t stream, uintptr_t xg_recv, uintptr_t xg_peers, int xg_world, int xg_rank,
             uintptr_t xg_status, int64_t xg_timeout, int xg_poll) {
            const dct::MlpArgs a = make_train_args(plan, p, mo, vo, grad_out, X, ldx, Y, idx, n_items, B, steps, t0, lr,
                                                   b1, b2, eps, wd, dropout, seed, step_base, loss_out, mode,
                                                   loss_kind, step_counter, cursor, prof, pending, stage, xg_recv,
                                                   xg_peers, xg_world, xg_rank, xg_status, xg_timeout, xg_poll);
            launch_train(plan, a, stream);
          },
          py::arg("p"), py::arg("m"), py::arg("v"), py::arg("grad_out"), py::arg("X"), py::arg("ldx"), py::arg("Y"),
          py::arg("idx"), py::arg("n_items"), py::arg("B"), py::arg("steps"), py::arg("t0"), py::arg("lr"),
          py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("dropout"), py::arg("seed"),
          py::arg("step_base"), py::arg("loss_out"), py::arg("mode"), py::arg("loss_kind"), py::arg("step_counter"),
          py::arg("cursor"), py::arg("prof") = 0, py::arg("pending") = 0, py::arg("stage") = 0,
          py::arg("stream") = 0, py::arg("xg_recv") = 0, py::arg("xg_peers") = 0, py::arg("xg_world") = 0,
          py::arg("xg_rank") = 0, py::arg("xg_status") = 0, py::arg("xg_timeout") = 200000000LL, py::arg("xg_poll") = 0)
      .def(
          "prepare_train",
          [](const MlpPlan& plan, uintptr_t p, uintptr_t mo, uintptr_t vo, uintptr_t X, int ldx, uintptr_t Y,
             uintptr_t idx, int n_items, int B, float lr, float b1, float b2, float eps, float wd, float dropout,
             uint32_t seed, uintptr_t loss_out, int64_t loss_len, int loss_kind, uintptr_t step_counter,
             uintptr_t xg_recv, uintptr_t xg_peers, int xg_world, int xg_rank, uintptr_t xg_status,
             int64_t xg_timeout, int xg_poll, uintptr_t xg_ticks) {
            auto l = std::make_unique<MlpLaunch>(MlpLaunch{plan});
            l->base = make_train_args(plan, p, mo, vo, 0, X, ldx, Y, idx, n_items, B, 1, 0, lr, b1, b2, eps, wd,
                                      dropout, seed, 0, loss_out, 0, loss_kind, step_counter, 0, 0, 0, 0, xg_recv,
                                      xg_peers, xg_world, xg_rank, xg_status, xg_timeout, xg_poll);
            l->base.xg_ticks = P<unsigned long long>(xg_ticks);
            l->n_items = n_items;
            l->loss_len = loss_out ? loss_len : 0;
            return l;
          },
          py::arg("p"), py::arg("m"), py::arg("v"), py::arg("X"), py::arg("ldx"), py::arg("Y"), py::arg("idx"),
          py::arg("n_items"), py::arg("B"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"),
          py::arg("dropout"), py::arg("seed"), py::arg("loss_out"), py::arg("loss_len"), py::arg("loss_kind"),
          py::arg("step_counter"), py::arg("xg_recv") = 0, py::arg("xg_peers") = 0, py::arg("xg_world") = 0,
          py::arg("xg_rank") = 0, py::arg("xg_status") = 0, py::arg("xg_timeout") = 200000000LL,
          py::arg("xg_poll") = 0, py::arg("xg_ticks") = 0)
      .def(
          "eval",
          [](const MlpPlan& plan, uintptr_t p, uintptr_t X, int ldx, uintptr_t Y, uintptr_t idx, int n_items,
             int loss_kind, uintptr_t acc_out, uintptr_t logits_out, int grid, uintptr_t stream) {
            dct::MlpArgs a{};
            a.p = P<float>(p);
            a.X = P<const float>(X);
            a.ldx = ldx;
            a.Y = P<const int>(Y);
            a.idx = P<const int>(idx);
            a.n_items = n_items;
            a.B = plan.sh()->bmax;
            a.loss_kind = loss_kind;
            a.eval_acc = P<float>(acc_out);
            a.logits_out = P<float>(logits_out);
            check(dct_mlp_eval(plan.shape.data(), &a, grid, reinterpret_cast<void*>(stream)), "mlp_eval");
          },
          py::arg("p"), py::arg("X"), py::arg("ldx"), py::arg("Y"), py::arg("idx"), py::arg("n_items"),
          py::arg("loss_kind"), py::arg("acc_out"), py::arg("logits_out"), py::arg("grid"), py::arg("stream"));

  // ------------------------------------------------------------------ optimizer
  m.def(
      "adam_flat",
      [](uintptr_t p, uintptr_t g, uintptr_t mo, uintptr_t vo, uintptr_t p_bf16, int64_t n, float lr, float b1,
         float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled, uintptr_t step_counter,
         uintptr_t stream) {
        check(dct_adam_flat(P<float>(p), P<const float>(g), P<float>(mo), P<float>(vo), P<uint16_t>(p_bf16), n, lr,
                            b1, b2, eps, wd, t, grad_scale, decoupled, P<const int>(step_counter),
                            reinterpret_cast<void*>(stream)),
              "adam_flat");
      },
      py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("p_bf16"), py::arg("n"), py::arg("lr"),
      py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("t"), py::arg("grad_scale"),
      py::arg("decoupled"), py::arg("step_counter"), py::arg("stream"));
  m.def("xg_adam_buffer_bytes", &dct_xg_adam_buffer_bytes, py::arg("n"), py::arg("world"));
  m.def(
      "xg_allreduce_adam",
      [](uintptr_t g, uintptr_t p, uintptr_t mo, uintptr_t vo, int64_t n, int64_t np, uintptr_t step_counter,
         float lr, float b1, float b2, float eps, float wd, const dct::PeerExchange& xg, double timeout_s,
         uintptr_t stream) {
        if (xg.bytes() < dct_xg_adam_buffer_bytes(n, xg.world()))
          throw std::invalid_argument("xg_allreduce_adam: exchange buffer too small for n");
        check(dct_xg_allreduce_adam(P<float>(g), P<float>(p), P<float>(mo), P<float>(vo), n, np,
                                    P<const int>(step_counter), lr, b1, b2, eps, wd, P<void>(xg.recv()),
                                    P<void* const>(xg.peers()), P<unsigned>(xg.status()), xg.world(), xg.rank(),
                                    (long long)(timeout_s * 1e8), reinterpret_cast<void*>(stream)),
              "xg_allreduce_adam");
      },
      py::arg("g"), py::arg("p"), py::arg("m"), py::arg("v"), py::arg("n"), py::arg("P"), py::arg("step_counter"),
      py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("xg"),
      py::arg("timeout_s"), py::arg("stream"));
  m.def("adam_flat_step",
        [](uintptr_t p, uintptr_t g, uintptr_t mo, uintptr_t vo, uintptr_t p_bf16, int64_t n, float lr, float b1,
           float b2, float eps, float wd, int64_t t, float grad_scale, int decoupled, uintptr_t step_counter,
           uintptr_t cursor, uintptr_t loss_slot, uintptr_t loss_out, int loss_cap, uintptr_t stream) {
          check(dct_adam_flat_step(P<float>(p), P<const float>(g), P<float>(mo), P<float>(vo), P<uint16_t>(p_bf16), n,
                                   lr, b1, b2, eps, wd, t, grad_scale, decoupled, P<const int>(step_counter),
                                   P<int>(cursor), P<const float>(loss_slot), P<float>(loss_out), loss_cap,
                                   reinterpret_cast<void*>(stream)),
                "adam_flat_step");
        });
  // Adam over [0, n) of p / g / m / v (step t read from step_counter): riding in a split-K dW launch
  // of dZ^T X (mode 0: one element per thread - the executor's body; 1: the float4 body) or as its own
  // launch (mode 2, dct_adam_range) - tests/test_packed_fp32_gpu.py compares them bit for bit
  m.def("adam_ride_check",
        [](int mode, uintptr_t dz, uintptr_t x, uintptr_t part, uintptr_t colsum, int M, int N, int K, int splits,
           uintptr_t p, uintptr_t g, uintptr_t mo, uintptr_t vo, int64_t n, float lr, float b1, float b2, float eps,
           uintptr_t step_counter, uintptr_t stream) {
          dct::AdamRange r{};
          r.p = P<float>(p); r.g = P<const float>(g); r.m = P<float>(mo); r.v = P<float>(vo); r.n = n;
          r.lr = lr; r.b1 = b1; r.b2 = b2; r.eps = eps; r.wd = 0.f; r.grad_scale = 1.f;
          r.step_counter = P<const int>(step_counter); r.nparts = 0; r.lo = 0; r.hi = n;
          if (mode == 2) {
            check(dct_adam_range(&r, nullptr, nullptr, nullptr, 0, reinterpret_cast<void*>(stream)), "adam_range");
            return;
          }
          check(dct_gemm_bf16_dw_partials_adam_ex(P<const uint16_t>(dz), P<const uint16_t>(x), P<float>(part),
                                                  P<float>(colsum), M, N, K, splits, &r, mode == 1 ? 1 : 0,
                                                  reinterpret_cast<void*>(stream)),
                "gemm_bf16_dw_partials_adam");
        });
  m.def("ag_step_prologue",
        [](uintptr_t X, int row_bytes, uintptr_t Y, uintptr_t idx, uintptr_t cursor, int B, int64_t n_items,
           uintptr_t xdst, uintptr_t ydst, uintptr_t step_counter, uintptr_t zero, int64_t zero_n, uintptr_t stream) {
          check(dct_ag_step_prologue(P<const void>(X), row_bytes, P<const int64_t>(Y), P<const int64_t>(idx),
                                     P<const int>(cursor), B, n_items, P<void>(xdst), P<int64_t>(ydst),
                                     P<int>(step_counter), P<float>(zero), zero_n, reinterpret_cast<void*>(stream)),
                "ag_step_prologue");
        });
  // device timestamps (s_memrealtime, 100 MHz) of step phases: graph-capturable one-thread kernels
  m.def("phase_stamp", [](uintptr_t buf, int index, uintptr_t stream) {
    check(dct_reducer_stamp(P<unsigned long long>(buf) + index, reinterpret_cast<void*>(stream)), "phase_stamp");
  });
  m.def("phase_accum", [](uintptr_t buf, int n, uintptr_t stream) {
    check(dct_phase_accum(P<unsigned long long>(buf), n, reinterpret_cast<void*>(stream)), "phase_accum");
  });
  m.def("zero_f32", [](uintptr_t p, int64_t n, uintptr_t stream) {
    check(dct_zero_f32(P<float>(p), n, reinterpret_cast<void*>(stream)), "zero_f32");
  });
  m.def("f32_to_bf16", [](uintptr_t in, uintptr_t out, int64_t n, uintptr_t stream) {
    check(dct_f32_to_bf16(P<const float>(in), P<uint16_t>(out), n, reinterpret_cast<void*>(stream)), "f32_to_bf16");
  });

  // ------------------------------------------------------------------ GEMM / NN ops
  m.def(
      "gemm_bf16",
      [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, int M, int N, int K, int lda, int ldb, int ldc,
         int trans_a, int trans_b, int epilogue, int out_f32, int accumulate, uintptr_t aux, uintptr_t stream) {
        check(dct_gemm_bf16(P<const uint16_t>(A), P<const uint16_t>(B), P<void>(C), P<const float>(bias), M, N, K,
                            lda, ldb, ldc, trans_a, trans_b, epilogue, out_f32, accumulate, P<void>(aux),
                            reinterpret_cast<void*>(stream)),
              "gemm_bf16");
      },
      py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("trans_a"), py::arg("trans_b"), py::arg("epilogue"),
      py::arg("out_f32"), py::arg("accumulate"), py::arg("aux"), py::arg("stream"));
  m.def("gemm_bf16_bt",
        [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, int M, int N, int K, int lda, int ldb, int ldc,
           int epilogue, int out_f32, uintptr_t aux, uintptr_t bt_out, int bt_ld, uintptr_t stream) {
          check(dct_gemm_bf16_bt(P<const uint16_t>(A), P<const uint16_t>(B), P<void>(C), P<const float>(bias), M, N,
                                 K, lda, ldb, ldc, epilogue, out_f32, P<void>(aux), P<uint16_t>(bt_out), bt_ld,
                                 reinterpret_cast<void*>(stream)),
                "gemm_bf16_bt");
        });
  m.def(
      "gemm_bf16_ex",
      [](uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias, int M, int N, int K, int lda, int ldb, int ldc,
         int trans_a, int trans_b, int epilogue, int out_f32, int accumulate, uintptr_t aux, uintptr_t colsum,
         uintptr_t stream) {
        check(dct_gemm_bf16_ex(P<const uint16_t>(A), P<const uint16_t>(B), P<void>(C), P<const float>(bias), M, N, K,
                               lda, ldb, ldc, trans_a, trans_b, epilogue, out_f32, accumulate, P<void>(aux),
                               P<float>(colsum), reinterpret_cast<void*>(stream)),
              "gemm_bf16_ex");
      },
      py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("M"), py::arg("N"), py::arg("K"),
      py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("trans_a"), py::arg("trans_b"), py::arg("epilogue"),
      py::arg("out_f32"), py::arg("accumulate"), py::arg("aux"), py::arg("colsum"), py::arg("stream"));
  m.def("gemm_bf16_residual", [](uintptr_t A, uintptr_t W, uintptr_t C, uintptr_t bias, uintptr_t residual, int M, int N,
                                  int K, uintptr_t stream) {
    check(dct_gemm_bf16_residual(P<const uint16_t>(A), P<const uint16_t>(W), P<float>(C), P<const float>(bias),
                                 P<const float>(residual), M, N, K, reinterpret_cast<void*>(stream)),
          "gemm_bf16_residual");
  });
  m.def("skinny_fwd", [](uintptr_t X, uintptr_t W, uintptr_t bias, uintptr_t Y, int B, int K, int C, uintptr_t stream) {
    check(dct_skinny_fwd(P<const uint16_t>(X), P<const uint16_t>(W), P<const float>(bias), P<uint16_t>(Y), B, K, C,
                         reinterpret_cast<void*>(stream)),
          "skinny_fwd");
  });
  m.def("skinny_dx", [](uintptr_t dZ, uintptr_t W, uintptr_t aux, uintptr_t dX, int B, int K, int C, uintptr_t stream) {
    check(dct_skinny_dx(P<const uint16_t>(dZ), P<const uint16_t>(W), P<const uint16_t>(aux), P<uint16_t>(dX), B, K, C,
                        reinterpret_cast<void*>(stream)),
          "skinny_dx");
  });
  m.def("skinny_dw", [](uintptr_t dZ, uintptr_t X, uintptr_t dW, uintptr_t db, int B, int K, int C, uintptr_t stream) {
    check(dct_skinny_dw(P<const uint16_t>(dZ), P<const uint16_t>(X), P<float>(dW), P<float>(db), B, K, C,
                        reinterpret_cast<void*>(stream)),
          "skinny_dw");
  });
  m.def("skinny_head_supported", [](int K, int C) { return dct_skinny_head_supported(K, C) != 0; });
  m.def("skinny_head", [](uintptr_t H, uintptr_t W, uintptr_t bias, uintptr_t labels, uintptr_t dH, uintptr_t dW,
                          uintptr_t db, uintptr_t loss_sum, int B, int K, int C, float grad_scale, int loss_kind,
                          float loss_scale, int relu_mask, uintptr_t stream) {
    check(dct_skinny_head(P<const uint16_t>(H), P<const uint16_t>(W), P<const float>(bias), P<const int>(labels),
                          P<uint16_t>(dH), P<float>(dW), P<float>(db), P<float>(loss_sum), B, K, C, grad_scale,
                          loss_kind, loss_scale, relu_mask, reinterpret_cast<void*>(stream)),
          "skinny_head");
  });
  m.attr("EPI_NONE") = 0;
  m.attr("EPI_BIAS") = 1;
  m.attr("EPI_BIAS_RELU") = 2;
  m.attr("EPI_BIAS_GELU") = 3;
  m.attr("EPI_RELU_MASK") = 4;
  m.attr("EPI_GELU_GRAD") = 5;
  m.def(
      "bias_act_bwd",
      [](uintptr_t dY, uintptr_t act_aux, uintptr_t dZ_bf16, uintptr_t dbias, int M, int N, int ldy, int act,
         int accumulate_bias, uintptr_t stream) {
        check(dct_bias_act_bwd(P<const void>(dY), P<const void>(act_aux), P<uint16_t>(dZ_bf16), P<float>(dbias), M, N,
                               ldy, act, accumulate_bias, reinterpret_cast<void*>(stream)),
              "bias_act_bwd");
      },
      py::arg("dY"), py::arg("act_aux"), py::arg("dZ_bf16"), py::arg("dbias"), py::arg("M"), py::arg("N"),
      py::arg("ldy"), py::arg("act"), py::arg("accumulate_bias"), py::arg("stream"));
  m.def(
      "cross_entropy_fwd_bwd",
      [](uintptr_t logits, int logits_bf16, uintptr_t labels, uintptr_t dlogits, uintptr_t loss_sum,
         uintptr_t correct_sum, int M, int C, float grad_scale, int loss_kind, uintptr_t stream) {
        check(dct_loss_fwd_bwd(P<const void>(logits), logits_bf16, P<const int>(labels), P<void>(dlogits),
                               P<float>(loss_sum), P<float>(correct_sum), M, C, grad_scale, loss_kind,
                               reinterpret_cast<void*>(stream)),
              "loss_fwd_bwd");
      },
      py::arg("logits"), py::arg("logits_bf16"), py::arg("labels"), py::arg("dlogits"), py::arg("loss_sum"),
      py::arg("correct_sum"), py::arg("M"), py::arg("C"), py::arg("grad_scale"), py::arg("loss_kind"),
      py::arg("stream"));
  m.def(
      "layernorm_fwd",
      [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t y, uintptr_t mean, uintptr_t rstd, int M, int N, float eps,
         int in_bf16, int out_bf16, uintptr_t stream) {
        check(dct_layernorm_fwd(P<const void>(x), P<const float>(w), P<const float>(b), P<void>(y), P<float>(mean),
                                P<float>(rstd), M, N, eps, in_bf16, out_bf16, reinterpret_cast<void*>(stream)),
              "layernorm_fwd");
      });
  m.def(
      "layernorm_bwd",
      [](uintptr_t dy, uintptr_t x, uintptr_t w, uintptr_t mean, uintptr_t rstd, uintptr_t dx, uintptr_t dw,
         uintptr_t db, int M, int N, int bf16_io, uintptr_t stream) {
        check(dct_layernorm_bwd(P<const void>(dy), P<const void>(x), P<const float>(w), P<const float>(mean),
                                P<const float>(rstd), P<void>(dx), P<float>(dw), P<float>(db), M, N, bf16_io,
                                reinterpret_cast<void*>(stream)),
              "layernorm_bwd");
      });
  m.def(
      "layernorm_bwd_ex",
      [](uintptr_t dy, int dy_bf16, uintptr_t x, int x_bf16, uintptr_t w, uintptr_t mean, uintptr_t rstd, uintptr_t dx,
         int dx_bf16, uintptr_t dx2, uintptr_t dres, uintptr_t dw, uintptr_t db, uintptr_t ws, int M, int N,
         uintptr_t stream) {
        check(dct_layernorm_bwd_ex(P<const void>(dy), dy_bf16, P<const void>(x), x_bf16, P<const float>(w),
                                   P<const float>(mean), P<const float>(rstd), P<void>(dx), dx_bf16, P<uint16_t>(dx2),
                                   P<const float>(dres), P<float>(dw), P<float>(db), P<float>(ws), M, N,
                                   reinterpret_cast<void*>(stream)),
              "layernorm_bwd_ex");
      },
      py::arg("dy"), py::arg("dy_bf16"), py::arg("x"), py::arg("x_bf16"), py::arg("w"), py::arg("mean"),
      py::arg("rstd"), py::arg("dx"), py::arg("dx_bf16"), py::arg("dx2"), py::arg("dres"), py::arg("dw"),
      py::arg("db"), py::arg("ws"), py::arg("M"), py::arg("N"), py::arg("stream"));
  m.def("layernorm_bwd_ws_floats", &dct_layernorm_bwd_ws_floats);
  m.def(
      "attention_fwd",
      [](uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t lse, int Bsz, int H, int T, int D, int ldq,
         int ldo, float scale, uintptr_t stream) {
        check(dct_attention_fwd(P<const uint16_t>(q), P<const uint16_t>(k), P<const uint16_t>(v), P<uint16_t>(o),
                                P<float>(lse), Bsz, H, T, D, ldq, ldo, scale, reinterpret_cast<void*>(stream)),
              "attention_fwd");
      });
  m.def(
      "tt_block_fwd",
      [](std::vector<uintptr_t> ptrs, int Bsz, int T, int DM, int H, int FF, float eps, float scale, uintptr_t stream) {
        check(dct_tt_block_fwd(ptrs.data(), (int)ptrs.size(), Bsz, T, DM, H, FF, eps, scale,
                               reinterpret_cast<void*>(stream)),
              "tt_block_fwd");
      });
  m.def(
      "tt_block_bwd",
      [](std::vector<uintptr_t> ptrs, int Bsz, int T, int DM, int H, int FF, float scale, uintptr_t stream) {
        check(dct_tt_block_bwd(ptrs.data(), (int)ptrs.size(), Bsz, T, DM, H, FF, scale,
                               reinterpret_cast<void*>(stream)),
              "tt_block_bwd");
      });
  m.def(
      "tt_block_fwd_ex",
      [](std::vector<uintptr_t> ptrs, int Bsz, int T, int DM, int H, int FF, float eps, float scale, uintptr_t pool,
         uintptr_t ex, uintptr_t eE, uintptr_t ec, uintptr_t stream) {
        check(dct_tt_block_fwd_ex(ptrs.data(), (int)ptrs.size(), Bsz, T, DM, H, FF, eps, scale, P<float>(pool),
                                  P<const float>(ex), P<const float>(eE), P<const float>(ec),
                                  reinterpret_cast<void*>(stream)),
              "tt_block_fwd_ex");
      });
  m.def(
      "tt_block_fwd_gx",
      [](std::vector<uintptr_t> ptrs, int Bsz, int T, int DM, int H, int FF, float eps, float scale, uintptr_t pool,
         uintptr_t ex, uintptr_t eE, uintptr_t ec, std::vector<uintptr_t> gx, uintptr_t stream) {
        check(dct_tt_block_fwd_gx(ptrs.data(), (int)ptrs.size(), Bsz, T, DM, H, FF, eps, scale, P<float>(pool),
                                  P<const float>(ex), P<const float>(eE), P<const float>(ec), gx.data(),
                                  (int)gx.size(), reinterpret_cast<void*>(stream)),
              "tt_block_fwd_gx");
      });
  m.def(
      "tt_block_bwd_ex",
      [](std::vector<uintptr_t> ptrs, int Bsz, int T, int DM, int H, int FF, float scale, uintptr_t dpool,
         uintptr_t dout16, uintptr_t ex, uintptr_t eE, uintptr_t ec, uintptr_t lnrep, uintptr_t ticket,
         uintptr_t a1, uintptr_t wqkv, uintptr_t bqkv, uintptr_t stream) {
        check(dct_tt_block_bwd_ex(ptrs.data(), (int)ptrs.size(), Bsz, T, DM, H, FF, scale, P<const float>(dpool),
                                  P<uint16_t>(dout16), P<const float>(ex), P<const float>(eE), P<const float>(ec),
                                  P<float>(lnrep), P<unsigned>(ticket), P<const uint16_t>(a1),
                                  P<const uint16_t>(wqkv), P<const float>(bqkv), reinterpret_cast<void*>(stream)),
              "tt_block_bwd_ex");
      });
  m.def("tt_embed_fwd", [](uintptr_t x, uintptr_t E, uintptr_t c, uintptr_t h, int B, int F, int D, uintptr_t st) {
    check(dct_tt_embed_fwd(P<const float>(x), P<const float>(E), P<const float>(c), P<float>(h), B, F, D,
                           reinterpret_cast<void*>(st)), "tt_embed_fwd");
  });
  m.def("tt_embed_bwd", [](uintptr_t x, uintptr_t dh, uintptr_t dE, uintptr_t dc, int B, int F, int D, uintptr_t st) {
    check(dct_tt_embed_bwd(P<const float>(x), P<const float>(dh), P<float>(dE), P<float>(dc), B, F, D,
                           reinterpret_cast<void*>(st)), "tt_embed_bwd");
  });
  m.def("tt_head_fwd", [](std::vector<uintptr_t> p, int B, int T, int D, int C, float eps, uintptr_t st) {
    check(dct_tt_head_fwd(p.data(), (int)p.size(), B, T, D, C, eps, reinterpret_cast<void*>(st)), "tt_head_fwd");
  });
  m.def("tt_head_bwd", [](std::vector<uintptr_t> p, int B, int T, int D, int C, float eps, uintptr_t st) {
    check(dct_tt_head_bwd(p.data(), (int)p.size(), B, T, D, C, eps, reinterpret_cast<void*>(st)), "tt_head_bwd");
  });
  m.def("tt_head_fused", [](std::vector<uintptr_t> p, int B, int T, int D, int C, float eps, uintptr_t st) {
    check(dct_tt_head_fused(p.data(), (int)p.size(), B, T, D, C, eps, reinterpret_cast<void*>(st)), "tt_head_fused");
  });
  m.def("gemm_bf16_dw_grouped",
        [](std::vector<uintptr_t> dz, std::vector<uintptr_t> x, std::vector<uintptr_t> c, std::vector<int> M,
           std::vector<int> N, int K, std::vector<uintptr_t> colsum, int accumulate, uintptr_t stream) {
          const size_t n = dz.size();
          if (x.size() != n || c.size() != n || M.size() != n || N.size() != n || (colsum.size() && colsum.size() != n))
            throw std::invalid_argument("gemm_bf16_dw_grouped: list lengths differ");
          std::vector<const uint16_t*> pz(n), px(n);
          std::vector<float*> pc(n), pcs(n);
          for (size_t i = 0; i < n; ++i) {
            pz[i] = P<const uint16_t>(dz[i]); px[i] = P<const uint16_t>(x[i]); pc[i] = P<float>(c[i]);
            pcs[i] = colsum.size() ? P<float>(colsum[i]) : nullptr;
          }
          check(dct_gemm_bf16_dw_grouped((int)n, pz.data(), px.data(), pc.data(), M.data(), N.data(), K,
                                         colsum.size() ? pcs.data() : nullptr, accumulate,
                                         reinterpret_cast<void*>(stream)),
                "gemm_bf16_dw_grouped");
        });
  m.def("gemm_bf16_dw_grouped_embed",
        [](std::vector<uintptr_t> dz, std::vector<uintptr_t> x, std::vector<uintptr_t> c, std::vector<int> M,
           std::vector<int> N, int K, std::vector<uintptr_t> colsum, int accumulate, uintptr_t ex, uintptr_t edh,
           uintptr_t edE, uintptr_t edc, int eB, int eF, uintptr_t stream) {
          const size_t n = dz.size();
          if (x.size() != n || c.size() != n || M.size() != n || N.size() != n || colsum.size() != n)
            throw std::invalid_argument("gemm_bf16_dw_grouped_embed: list lengths differ");
          std::vector<const uint16_t*> pz(n), px(n);
          std::vector<float*> pc(n), pcs(n);
          for (size_t i = 0; i < n; ++i) {
            pz[i] = P<const uint16_t>(dz[i]); px[i] = P<const uint16_t>(x[i]); pc[i] = P<float>(c[i]);
            pcs[i] = P<float>(colsum[i]);
          }
          const int r = dct_gemm_bf16_dw_grouped_embed((int)n, pz.data(), px.data(), pc.data(), M.data(), N.data(), K,
                                                       pcs.data(), accumulate, P<const float>(ex),
                                                       P<const float>(edh), P<float>(edE), P<float>(edc), eB, eF,
                                                       reinterpret_cast<void*>(stream));
          if (r != 0 && r != 1) check(r, "gemm_bf16_dw_grouped_embed");
          return r == 0;  // True: the embedding gradients rode in the launch
        });
  m.def(
      "attention_bwd",
      [](uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t dout, uintptr_t lse, uintptr_t dq, uintptr_t dk,
         uintptr_t dv, int Bsz, int H, int T, int D, int ldq, int ldo, float scale, uintptr_t stream) {
        check(dct_attention_bwd(P<const uint16_t>(q), P<const uint16_t>(k), P<const uint16_t>(v), P<const uint16_t>(o),
                                P<const uint16_t>(dout), P<const float>(lse), P<uint16_t>(dq), P<uint16_t>(dk),
                                P<uint16_t>(dv), Bsz, H, T, D, ldq, ldo, scale, reinterpret_cast<void*>(stream)),
              "attention_bwd");
      });
  m.def("gather_rows", [](uintptr_t src, uintptr_t idx, uintptr_t dst, int64_t n_rows, int row_bytes,
                          uintptr_t stream) {
    check(dct_gather_rows(P<const void>(src), P<const int>(idx), P<void>(dst), n_rows, row_bytes,
                          reinterpret_cast<void*>(stream)),
          "gather_rows");
  });

  // ------------------------------------------------------------------ runtime
  m.def("comm_unique_id", []() { return py::bytes(dct::comm_unique_id()); });
  py::class_<dct::Comm>(m, "Comm")
      .def(py::init([](py::bytes uid, int world, int rank, int device) {
             return new dct::Comm(std::string(uid), world, rank, device);
           }),
           py::arg("uid"), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def("allreduce", &dct::Comm::allreduce, py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("op"),
           py::arg("stream"))
      .def("broadcast", &dct::Comm::broadcast, py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("root"),
           py::arg("stream"))
      .def("reduce_scatter", &dct::Comm::reduce_scatter)
      .def("all_gather", &dct::Comm::all_gather)
      .def_property_readonly("rank", &dct::Comm::rank)
      .def_property_readonly("world", &dct::Comm::world);
  py::class_<dct::BucketReducer>(m, "BucketReducer")
      .def(py::init([](dct::Comm* comm, uintptr_t flat, std::vector<int64_t> offs, std::vector<int64_t> counts,
                       std::vector<int> pb, int dtype, int op) {
             return new dct::BucketReducer(comm, flat, std::move(offs), std::move(counts), std::move(pb), dtype, op);
           }),
           py::arg("comm"), py::arg("flat_grad"), py::arg("bucket_offsets"), py::arg("bucket_counts"),
           py::arg("param_bucket"), py::arg("dtype"), py::arg("op"), py::keep_alive<1, 2>())
      .def("prepare", &dct::BucketReducer::prepare)
      .def("mark_ready", &dct::BucketReducer::mark_ready)
      .def("finalize", &dct::BucketReducer::finalize)
      .def_property_readonly("num_buckets", &dct::BucketReducer::num_buckets)
      .def_property_readonly("launched", &dct::BucketReducer::launched)
      .def_property_readonly("launched_before_finalize", &dct::BucketReducer::launched_before_finalize)
      .def("edge_timeouts", &dct::BucketReducer::edge_timeouts)
      .def("check_edges", &dct::BucketReducer::check_edges)
      .def_property_readonly("peer_world", &dct::BucketReducer::peer_world)
      .def_property_readonly("comm_stream", &dct::BucketReducer::comm_stream)
      .def_property_readonly("inline_mode", &dct::BucketReducer::inline_mode)
      .def("enable_timing", &dct::BucketReducer::enable_timing, py::arg("check") = false)
      .def("read_timing", &dct::BucketReducer::read_timing)
      .def("reset_timing", &dct::BucketReducer::reset_timing)
      .def("set_comm_cu_mask", &dct::BucketReducer::set_comm_cu_mask, py::arg("mask"))
      .def_property_readonly("comm_cu_mask", &dct::BucketReducer::comm_cu_mask);
  m.def("cu_masked_stream", &dct::cu_masked_stream, py::arg("mask"));
  m.def("stream_destroy", &dct::stream_destroy, py::arg("stream"));
  m.def("stream_cu_mask", &dct::stream_cu_mask, py::arg("stream"));
  m.def("device_cu_count", &dct::device_cu_count);
  py::class_<dct::PeerExchange>(m, "PeerExchange")
      .def(py::init<int, int, int64_t>(), py::arg("world"), py::arg("rank"), py::arg("bytes"))
      .def("ipc_handle", [](const dct::PeerExchange& x) { return py::bytes(x.ipc_handle()); })
      .def("open_peers",
           [](dct::PeerExchange& x, const std::vector<py::bytes>& hs) {
             std::vector<std::string> v;
             for (const auto& h : hs) v.emplace_back(std::string(h));
             x.open_peers(v);
           })
      .def("set_peers", &dct::PeerExchange::set_peers)
      .def("reset", &dct::PeerExchange::reset, py::arg("stream") = 0)
      .def("barrier", &dct::PeerExchange::barrier, py::arg("stream"), py::arg("timeout_s") = 20.0)
      .def("read_status", &dct::PeerExchange::read_status)
      .def_property_readonly("recv", &dct::PeerExchange::recv)
      .def_property_readonly("peers", &dct::PeerExchange::peers)
      .def_property_readonly("status", &dct::PeerExchange::status)
      .def_property_readonly("bytes", &dct::PeerExchange::bytes)
      .def_property_readonly("world", &dct::PeerExchange::world)
      .def_property_readonly("rank", &dct::PeerExchange::rank);
  // exchange buffer bytes of the 3x128 block kernel's in-kernel data-parallel launches (0: no such
  // launch for this shape / batch / world size)
  m.def("mlp_block5_xg_bytes", [](const std::vector<int>& dims, int B, int world) -> int64_t {
    if (dims.size() != 4 || !dct::mlp_block5_shape_ok(dims.data(), 3, B)) return 0;
    return (int64_t)dct::mlp_block5_xg_bytes(world);
  }, py::arg("dims"), py::arg("batch"), py::arg("world"));
  m.def("mlp_xg_slab_granules", [](const std::vector<int>& dims) {
    return (int64_t)dct_mlp_xg_slab_granules(dims.data(), (int)dims.size() - 1);
  });
  py::class_<dct::MlpStepExecutor>(m, "MlpStepExecutor")
      .def(py::init<const std::vector<int>&, int, int, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                    const std::vector<uintptr_t>&, const std::vector<uintptr_t>&, uintptr_t, uintptr_t, uintptr_t,
                    uintptr_t, dct::BucketReducer*>(),
           py::arg("dims"), py::arg("batch"), py::arg("act"), py::arg("loss_kind"), py::arg("p"), py::arg("p_bf16"),
           py::arg("g"), py::arg("m"), py::arg("v"), py::arg("acts"), py::arg("pre"), py::arg("dz0"), py::arg("dz1"),
           py::arg("ybuf"), py::arg("stats"), py::arg("reducer") = nullptr, py::keep_alive<1, 17>())
      .def("set_adam", &dct::MlpStepExecutor::set_adam, py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"),
           py::arg("wd"), py::arg("decoupled") = 0)
      .def("step", &dct::MlpStepExecutor::step, py::arg("X"), py::arg("row_bytes"), py::arg("Y"), py::arg("idx"),
           py::arg("n_items"), py::arg("cursor"), py::arg("step_counter"), py::arg("loss_out"), py::arg("loss_cap"),
           py::arg("rows"), py::arg("stream"))
      .def("eval_batch", &dct::MlpStepExecutor::eval_batch, py::arg("X"), py::arg("row_bytes"), py::arg("Y"),
           py::arg("idx"), py::arg("n_items"), py::arg("cursor"), py::arg("rows"), py::arg("stats"),
           py::arg("stream"))
      .def_property("adam_ride", &dct::MlpStepExecutor::adam_ride, &dct::MlpStepExecutor::set_adam_ride)
      .def("set_gather_fuse", &dct::MlpStepExecutor::set_gather_fuse)
      .def_property_readonly("gather_fused_steps", &dct::MlpStepExecutor::gather_fused_steps)
      .def_property_readonly("num_params", &dct::MlpStepExecutor::num_params)
      .def_property_readonly("part_fallbacks", &dct::MlpStepExecutor::part_fallbacks)
      .def_property_readonly("partial_layers", &dct::MlpStepExecutor::partial_layers);
  py::class_<dct::StreamGraph>(m, "StreamGraph")
      .def(py::init<>())
      .def("begin", &dct::StreamGraph::begin)
      .def("end", &dct::StreamGraph::end)
      .def("replay", &dct::StreamGraph::replay)
      .def("reset", &dct::StreamGraph::reset)
      .def_property_readonly("num_nodes", &dct::StreamGraph::num_nodes);

  m.attr("DT_F32") = (int)dct::DT_F32;
  m.attr("DT_BF16") = (int)dct::DT_BF16;
  m.attr("DT_F16") = (int)dct::DT_F16;
  m.attr("DT_I32") = (int)dct::DT_I32;
  m.attr("DT_I64") = (int)dct::DT_I64;
  m.attr("DT_U8") = (int)dct::DT_U8;
  m.attr("OP_SUM") = (int)dct::OP_SUM;
  m.attr("OP_AVG") = (int)dct::OP_AVG;
  m.attr("OP_MAX") = (int)dct::OP_MAX;
  m.attr("OP_MIN") = (int)dct::OP_MIN;
}
