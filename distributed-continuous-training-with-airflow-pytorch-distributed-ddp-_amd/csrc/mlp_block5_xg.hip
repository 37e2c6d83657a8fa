// Data-parallel launches of the 3x128 weather trainer (mlp_block5_impl.h, XW = 2 .. 8 ranks):
// the per-rank compile-time-rank kernels of the reference configuration (CE, no weight decay) and
// the runtime-rank kernels of every other one.  Compiled with the default scheduler: the
// max-ILP strategy of the one-rank unit measured slower here (profiles/b5_sched_strategy_ab_r4.log).
#include "mlp_block5_impl.h"

namespace dct {

template <int XW>
static void b5_launch_xg(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  const bool wd = a.wd != 0.f;
  if (a.loss_kind == 0 && !wd) {
    // the reference's configuration (cross-entropy, Adam without weight decay): one kernel per rank
    b5x::static_for<XW>([&](auto rc) {
      constexpr int R = decltype(rc)::value;
      if (a.xg_rank == R) b5_launch<false, 0, false, true, true, XW, R>(bytes, st, sh, a);
    });
  } else if (a.loss_kind == 0) {
    b5_launch<true, 0, false, true, true, XW>(bytes, st, sh, a);
  } else {
    if (wd) b5_launch<true, 1, false, true, true, XW>(bytes, st, sh, a);
    else b5_launch<false, 1, false, true, true, XW>(bytes, st, sh, a);
  }
}

void mlp_launch_block5_xg_static(int world, size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a);

// world sizes that do not divide the 16 W1 pairs per lane (3, 5, 6, 7 ranks; pair XW t + rank, the last
// slots of some ranks empty): the reference configuration on per-rank kernels (mlp_block5_xgs.hip),
// every other one on runtime-rank kernels with the weight-decay term compiled in (wd = 0 adds
// fmaf(0, p, g) = g exactly) - two kernels per world size instead of one per rank
template <int XW>
static void b5_launch_xg_rt(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  if (a.loss_kind == 0 && a.wd == 0.f) mlp_launch_block5_xg_static(XW, bytes, st, sh, a);
  else if (a.loss_kind == 0) b5_launch<true, 0, false, true, true, XW>(bytes, st, sh, a);
  else b5_launch<true, 1, false, true, true, XW>(bytes, st, sh, a);
}

void mlp_launch_block5_xg_prof(int world, size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a);

void mlp_launch_block5_xg(int world, size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  if (a.prof) return mlp_launch_block5_xg_prof(world, bytes, st, sh, a);  // mlp_block5_xgprof.hip
  if (world == 2) {
    b5_launch_xg<2>(bytes, st, sh, a);
  } else if (world == 4) {
    b5_launch_xg<4>(bytes, st, sh, a);
  } else if (world == 8) {
    b5_launch_xg<8>(bytes, st, sh, a);
  } else if (world == 3) {
    b5_launch_xg_rt<3>(bytes, st, sh, a);
  } else if (world == 5) {
    b5_launch_xg_rt<5>(bytes, st, sh, a);
  } else if (world == 6) {
    b5_launch_xg_rt<6>(bytes, st, sh, a);
  } else {
    b5_launch_xg_rt<7>(bytes, st, sh, a);
  }
}

}  // namespace dct
