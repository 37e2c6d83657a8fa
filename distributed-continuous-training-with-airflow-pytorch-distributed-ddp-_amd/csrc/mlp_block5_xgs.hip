// Compile-time-rank kernels of the data-parallel 3x128 trainer at the world sizes that do not divide
// the 16 W1 pairs per lane (3, 5, 6, 7 ranks), for the reference configuration (cross-entropy, Adam
// without weight decay): every ownership test folds, as for 2 / 4 / 8 ranks (mlp_block5_xg.hip).  The
// runtime-rank kernels made 6 ranks slower per step than 8 (13.0 vs 11.5 us in the shared-GPU
// rehearsal, profiles/b5x_dp_rehearsal_r5.log).  Own unit: compiled in parallel with the others.
#include "mlp_block5_impl.h"

namespace dct {

template <int XW>
static void b5_launch_xgs(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  b5x::static_for<XW>([&](auto rc) {
    constexpr int R = decltype(rc)::value;
    if (a.xg_rank == R) b5_launch<false, 0, false, true, true, XW, R>(bytes, st, sh, a);
  });
}

void mlp_launch_block5_xg_static(int world, size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  switch (world) {
    case 3: b5_launch_xgs<3>(bytes, st, sh, a); break;
    case 5: b5_launch_xgs<5>(bytes, st, sh, a); break;
    case 6: b5_launch_xgs<6>(bytes, st, sh, a); break;
    default: b5_launch_xgs<7>(bytes, st, sh, a); break;
  }
}

}  // namespace dct
