// Per-rank batch 5..8 on the 3x128 weather trainer (mlp_block5_impl.h with MB = 2: two micro-batches
// of four rows per step, gradients summed in registers, one Adam): one-rank train / grad mode, and
// the data-parallel launches at 2..8 ranks (runtime-rank kernels, weight-decay term compiled in:
// wd = 0 adds fmaf(0, p, g) = g exactly).  The reference trains at batch 4 per rank
// (jobs/train_lightning_ddp.py:122); these keep a doubled batch on the same kernel instead of the
// slower generic trainers.  Its own unit: compiled in parallel with the batch <= 4 ones.
#include "mlp_block5_impl.h"

namespace dct {

template <int XW>
static void b8_xg(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  if (a.loss_kind == 0) b5_launch<true, 0, false, true, true, XW, -1, 2>(bytes, st, sh, a);
  else b5_launch<true, 1, false, true, true, XW, -1, 2>(bytes, st, sh, a);
}

void mlp_launch_block5_b8(size_t bytes, hipStream_t st, const MlpShape& sh, const MlpArgs& a) {
  const bool wd = a.wd != 0.f;
  switch (a.xg_world > 1 ? a.xg_world : 1) {
    case 2: b8_xg<2>(bytes, st, sh, a); return;
    case 3: b8_xg<3>(bytes, st, sh, a); return;
    case 4: b8_xg<4>(bytes, st, sh, a); return;
    case 5: b8_xg<5>(bytes, st, sh, a); return;
    case 6: b8_xg<6>(bytes, st, sh, a); return;
    case 7: b8_xg<7>(bytes, st, sh, a); return;
    case 8: b8_xg<8>(bytes, st, sh, a); return;
    default: break;
  }
  if (a.mode == 1) {  // grad mode (the DDP step path): no Adam, no moments
    if (a.loss_kind == 0) b5_launch<false, 0, false, true, false, 1, -1, 2>(bytes, st, sh, a);
    else b5_launch<false, 1, false, true, false, 1, -1, 2>(bytes, st, sh, a);
  } else if (a.loss_kind == 0) {
    if (wd) b5_launch<true, 0, false, true, true, 1, -1, 2>(bytes, st, sh, a);
    else b5_launch<false, 0, false, true, true, 1, -1, 2>(bytes, st, sh, a);
  } else {
    if (wd) b5_launch<true, 1, false, true, true, 1, -1, 2>(bytes, st, sh, a);
    else b5_launch<false, 1, false, true, true, 1, -1, 2>(bytes, st, sh, a);
  }
}

}  // namespace dct
