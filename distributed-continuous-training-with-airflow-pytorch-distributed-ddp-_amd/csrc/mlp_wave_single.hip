// Single-wave MLP trainer instantiations without the in-kernel exchange (see mlp_wave_impl.h).
#include "mlp_wave_impl.h"

namespace dct {
hipError_t wave_single_launch(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  if (sh.L == 2) return a.B <= 4 ? launch_wave_d0<2, 4, 0>(sh, a, st) : launch_wave_d0<2, 8, 0>(sh, a, st);
  return a.B <= 4 ? launch_wave_d0<3, 4, 0>(sh, a, st) : launch_wave_d0<3, 8, 0>(sh, a, st);
}
}  // namespace dct
