// Row-parallel weather-MLP trainer instantiations, exchange width 2 (see mlp_wave_impl.h).
#include "mlp_wave_impl.h"

namespace dct {
hipError_t wave_rows_launch_x2(const WaveShape& sh, const MlpArgs& a, hipStream_t st) {
  return launch_rows_d0<2>(sh, a, st);
}
}  // namespace dct
