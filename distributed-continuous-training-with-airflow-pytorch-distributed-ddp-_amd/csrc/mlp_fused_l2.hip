// Instantiation unit: fused MLP kernels with 2 linear layers (see mlp_fused_impl.h).
#include "mlp_fused_impl.h"

namespace dct {
hipError_t mlp_launch_train_L2(const MlpShape& sh, const MlpArgs& a, hipStream_t st) {
  return launch_train_L<2>(sh, a, st);
}
hipError_t mlp_launch_eval_L2(const MlpShape& sh, const MlpArgs& a, int grid, hipStream_t st) {
  return launch_eval_L<2>(sh, a, grid, st);
}
}  // namespace dct
