// Single-wave MLP trainer instantiations with the in-kernel exchange (see mlp_wave_impl.h).
#include "mlp_wave_impl.h"

namespace dct {
hipError_t wave_single_launch_xg(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  return a.B <= 4 ? launch_wave_xg<4>(sh, a, st) : launch_wave_xg<8>(sh, a, st);
}
}  // namespace dct
