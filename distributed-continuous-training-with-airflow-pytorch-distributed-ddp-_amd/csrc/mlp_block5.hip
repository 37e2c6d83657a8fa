// One-rank launches (train mode, the one-step grad mode of the DDP step path, profiling) and the
// host-side checks of the 3x128 weather trainer; device code in mlp_block5_impl.h.  Compiled with
// the max-ILP machine scheduler (_build.py FILE_FLAGS): 3.90 -> 3.80 us/step at one rank
// (profiles/b5_sched_strategy_ab_r4.log).
#include "mlp_block5_impl.h"

namespace dct {

void mlp_launch_block5_xg(int world, size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a);
void mlp_launch_block5_b8(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a);

// in-kernel data-parallel launches of this kernel: 2 .. 8 ranks (one node), train mode; the profiling
// instantiations exist for 2 / 4 / 8
static bool b5_xg_world_ok(int w) { return w >= 2 && w <= 8; }

bool mlp_block5_ok(const MlpShape& sh, const MlpArgs& a) {
  const bool aligned = (sh.woff[1] % 4) == 0 && ((uintptr_t)a.p & 15) == 0 && (((uintptr_t)a.m | (uintptr_t)a.v) & 15) == 0;
  const bool xg_ok = a.xg_world <= 1 ||
                     (a.mode == 0 && b5_xg_world_ok(a.xg_world) && a.xg_rank >= 0 && a.xg_rank < a.xg_world &&
                      a.xg_recv != nullptr && a.xg_peers != nullptr && a.xg_status != nullptr &&
                      (a.prof == nullptr || a.xg_world == 2 || a.xg_world == 4 || a.xg_world == 8));
  // per-rank batch 5..8 (two micro-batches per step, mlp_block5_b8.hip): no profiling instantiation
  const bool b8_ok = (a.B <= blk5::B && sh.mlp_block != 8) || a.prof == nullptr;
  return aligned && b8_ok && mlp_block5_shape_ok(sh.dims, sh.L, a.B) &&
         // train mode, or grad mode for ONE step (the DDP step path: grads + loss to grad_out, device cursor)
         ((a.mode == 0 && a.cursor == nullptr) || (a.mode == 1 && a.steps == 1 && a.grad_out != nullptr)) &&
         (a.loss_kind == 0 || a.loss_kind == 1) && a.pending == nullptr && (a.stage == nullptr || a.mode == 1) && xg_ok;
}

bool mlp_block5_shape_ok(const int* dims, int L, int B) {
  return L == 3 && dims[1] == blk5::H && dims[2] == blk5::H && dims[0] >= 1 && dims[0] <= blk5::DMAX &&
         dims[3] == blk5::C && B >= 1 && B <= blk5::BMAX;
}

size_t mlp_block5_xg_bytes(int world) {
  switch (world) {
    case 2: return (size_t)b5x::Lay<2>::BYTES;
    case 4: return (size_t)b5x::Lay<4>::BYTES;
    case 8: return (size_t)b5x::Lay<8>::BYTES;
    case 3: return (size_t)b5x::Lay<3>::BYTES;
    case 5: return (size_t)b5x::Lay<5>::BYTES;
    case 6: return (size_t)b5x::Lay<6>::BYTES;
    case 7: return (size_t)b5x::Lay<7>::BYTES;
    default: return 0;
  }
}

hipError_t mlp_launch_block5(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  const size_t bytes = (size_t)blk5::LDS_FLOATS * sizeof(float);
  const bool wd = a.wd != 0.f;
  if (a.B > blk5::B || sh.mlp_block == 8) {
    mlp_launch_block5_b8(bytes, st, sh, a);  // two micro-batches per step, every world size
  } else if (a.xg_world > 1) {
    mlp_launch_block5_xg(a.xg_world, bytes, st, sh, a);  // mlp_block5_xg.hip
  } else if (a.mode == 1) {  // grad mode: no Adam, no moments
    if (a.loss_kind == 0) b5_launch<false, 0, false, true, false>(bytes, st, sh, a);
    else b5_launch<false, 1, false, true, false>(bytes, st, sh, a);
  } else if (a.prof) {  // per-phase cycle stamps (tools/prof_block.py)
    if (a.loss_kind == 0) b5_launch<true, 0, true>(bytes, st, sh, a);
    else b5_launch<true, 1, true>(bytes, st, sh, a);
  } else if (a.loss_kind == 0) {
    if (wd) b5_launch<true, 0>(bytes, st, sh, a);
    else b5_launch<false, 0>(bytes, st, sh, a);
  } else {
    if (wd) b5_launch<true, 1>(bytes, st, sh, a);
    else b5_launch<false, 1>(bytes, st, sh, a);
  }
  return hipGetLastError();
}

}  // namespace dct
