// Profiling launches of the data-parallel 3x128 trainer (mlp_block5_impl.h with PROF, XW = 2 / 4 / 8):
// the production kernels plus s_memtime stamps per phase and wave, exchange phases included
// (slots 15..20: dW1 + reduce-scatter pushes, reduce-scatter poll wait, owned Adam + all-gather
// pushes, small pairs, all-gather poll wait, unpack).  tools/prof_b5x.py reads them; a unit of its
// own so the extra instantiations compile in parallel with the production ones.
#include "mlp_block5_impl.h"

namespace dct {

template <int XW>
static void b5_launch_xg_prof(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  if (a.loss_kind == 0 && a.wd == 0.f) {  // the reference configuration: the compile-time-rank kernels
    b5x::static_for<XW>([&](auto rc) {
      constexpr int R = decltype(rc)::value;
      if (a.xg_rank == R) b5_launch<false, 0, true, true, true, XW, R>(bytes, st, sh, a);
    });
  } else {
    b5_launch<true, 0, true, true, true, XW>(bytes, st, sh, a);  // (profiling: CE only)
  }
}

void mlp_launch_block5_xg_prof(int world, size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  if (world == 2) b5_launch_xg_prof<2>(bytes, st, sh, a);
  else if (world == 4) b5_launch_xg_prof<4>(bytes, st, sh, a);
  else if (world == 8) b5_launch_xg_prof<8>(bytes, st, sh, a);  // (3 / 5 / 6 / 7 ranks: no profiling instantiation; mlp_block5_ok refuses prof there)
}

}  // namespace dct
