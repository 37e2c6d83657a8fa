// Entry points of the narrow-MLP trainers (kernels: mlp_wave_impl.h; the template instantiations
// live in mlp_wave_rows_x*.hip / mlp_wave_single*.hip so they compile in parallel).
#include "mlp_wave_impl.h"

extern "C" {

// 1 if dims fit the single-wave kernel: 2 or 3 layers, hidden <= 64, d0 <= 16, classes <= 4
int dct_mlp_wave_supported(const int* dims, int L, int B) {
  if (L != 2 && L != 3) return 0;
  if (dims[0] > 16 || dims[L] > 4 || B < 1 || B > 8) return 0;
  for (int l = 1; l < L; ++l)
    if (dims[l] > 64) return 0;
  return 1;
}

// receive-buffer granules per rank per parity for the in-kernel all-reduce (0 = unsupported)
size_t dct_mlp_xg_slab_granules(const int* dims, int L) {
  if (L != 2 || !dct_mlp_wave_supported(dims, L, 1)) return 0;
  const int D0 = (dims[0] == 5 && dims[2] == 2) ? 5 : (dims[0] <= 8 ? 8 : 16);
  const int CM = (dims[0] == 5 && dims[2] == 2) ? 2 : 4;
  // the single-wave kernel's [KX][64] layout or the row-parallel kernel's per-wave regions
  const size_t wave_kernel = (size_t)(D0 + CM + 2 + ((D0 + CM) & 1)) * 64;
  return wave_kernel > (size_t)dct::XG_ROWS_GRANULES ? wave_kernel : (size_t)dct::XG_ROWS_GRANULES;
}

int dct_mlp_wave_train(const int* dims, int L, const dct::MlpArgs* a, void* stream) {
  if (!dct_mlp_wave_supported(dims, L, a->B)) return (int)hipErrorInvalidValue;
  WaveShape sh{};
  sh.L = L;
  sh.d0 = dims[0];
  sh.h1 = dims[1];
  sh.h2 = L == 3 ? dims[2] : dims[1];
  sh.C = dims[L];
  int flat = 0;
  for (int l = 0; l < L; ++l) {
    sh.woff[l] = flat;
    flat += dims[l] * dims[l + 1];
    sh.boff[l] = flat;
    flat += dims[l + 1];
  }
  sh.P = flat;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool xg = a->xg_world > 1;
  if (xg) {
    if (L != 2 || a->mode != 0 || !a->xg_recv || !a->xg_peers || !a->xg_status || a->xg_world > dct::XG_MAXW ||
        a->xg_rank < 0 || a->xg_rank >= a->xg_world || a->cursor || a->pending)
      return (int)hipErrorInvalidValue;
    if (rows_eligible(L, *a)) {
      if (a->xg_world <= 2) return (int)dct::wave_rows_launch_x2(sh, *a, st);
      if (a->xg_world <= 4) return (int)dct::wave_rows_launch_x4(sh, *a, st);
      return (int)dct::wave_rows_launch_x8(sh, *a, st);
    }
    return (int)dct::wave_single_launch_xg(sh, *a, st);
  }
  if (rows_eligible(L, *a)) return (int)dct::wave_rows_launch_x0(sh, *a, st);
  return (int)dct::wave_single_launch(sh, *a, st);
}

}  // extern "C"
