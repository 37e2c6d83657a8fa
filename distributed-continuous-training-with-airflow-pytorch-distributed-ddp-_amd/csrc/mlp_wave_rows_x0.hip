// Row-parallel weather-MLP trainer instantiations, exchange width 0 (see mlp_wave_impl.h).
#include "mlp_wave_impl.h"

namespace dct {
hipError_t wave_rows_launch_x0(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  return launch_rows_d0<0>(sh, a, st);
}
}  // namespace dct
