// Fused tabular-MLP kernels: host-side planning and the C launch API.
// Device code: mlp_fused_impl.h; one instantiation unit per layer count
// (mlp_fused_l2/l3/l4.hip) so hipcc compiles them in parallel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mlp_fused.h"

namespace dct {

static inline int r4(int x) { return (x + 3) & ~3; }

// largest split s in {16, 4, 2, 1} with s <= limit and groups * s <= nt (at least 1)
static inline int pick_split_log2(int limit, int groups, int nt) {
  const int cand[4] = {4, 2, 1, 0};
  for (int c : cand) {
    const int s = 1 << c;
    if (s <= limit && groups * s <= nt) return c;
  }
  return 0;
}

int mlp_make_shape(MlpShape* sh, const int* dims, int L, int bmax) {
  if (L < 2 || L > MLP_MAXL) return -1;
  *sh = MlpShape{};
  sh->L = L;
  sh->bmax = bmax;
  for (int i = 0; i <= L; ++i) sh->dims[i] = dims[i];
  int flat = 0, nblk4 = 0, nblk1 = 0, nbias = 0;
  for (int l = 0; l < L; ++l) {
    const int in = dims[l], out = dims[l + 1];
    sh->rows4[l] = r4(out);
    sh->cols4[l] = r4(in);
    sh->blk_cols[l] = sh->cols4[l] / 4;
    sh->woff[l] = flat;
    flat += in * out;
    sh->boff[l] = flat;
    flat += out;
    nblk4 += (sh->rows4[l] / 4) * sh->blk_cols[l];
    nblk1 += out * sh->blk_cols[l];
    sh->bias_start[l] = nbias;
    nbias += out;
  }
  sh->P = flat;
  sh->nbias = nbias;
  for (int l = L; l <= MLP_MAXL; ++l) sh->bias_start[l] = nbias;

  // threads / ownership: 1x4 blocks when they spread over <= 2 per thread of 256, else 4x4
  int nt = 0, maxq = 0, br = 0;
  if (nblk1 <= 256) { nt = 256; maxq = 1; br = 1; }
  else if (nblk1 <= 512) { nt = 256; maxq = 2; br = 1; }
  else if (nblk4 <= 256) { nt = 256; maxq = 1; br = 4; }
  else if (nblk4 <= 512) { nt = 256; maxq = 2; br = 4; }
  else if (nblk4 <= 1024) { nt = 256; maxq = 4; br = 4; }
  else if (nblk4 <= 1536) { nt = 512; maxq = 3; br = 4; }
  else if (nblk4 <= 2048) { nt = 512; maxq = 4; br = 4; }
  sh->nt = nt;
  sh->maxq = maxq;
  sh->br = br;
  int nb = 0;
  for (int l = 0; l < L; ++l) {
    sh->blk_start[l] = nb;
    nb += (br == 4 ? sh->rows4[l] / 4 : dims[l + 1]) * sh->blk_cols[l];
  }
  for (int l = L; l <= MLP_MAXL; ++l) sh->blk_start[l] = nb;
  sh->nblk = nb;

  // per-layer work splits for the chosen thread count
  const int ntw = nt > 0 ? nt : 256;
  for (int l = 0; l < L; ++l) {
    const int K4 = sh->cols4[l] / 4, NG = sh->rows4[l] / 4;
    const int ksl = pick_split_log2(K4, NG, ntw);
    sh->f_ksl[l] = ksl;
    sh->f_kc[l] = (K4 + (1 << ksl) - 1) >> ksl;
    sh->f_items[l] = NG << ksl;
    const int CG = sh->cols4[l] / 4, O4 = sh->rows4[l] / 4;
    const int osl = pick_split_log2(O4, CG, ntw);
    sh->d_osl[l] = osl;
    sh->d_oc[l] = (O4 + (1 << osl) - 1) >> osl;
    sh->d_items[l] = CG << osl;
  }
  sh->fuse_loss = (sh->rows4[L - 1] == 4) ? 1 : 0;

  // LDS layout (floats, every region 16-B aligned)
  int off = 0;
  for (int l = 0; l < L; ++l) {
    int ldw = sh->cols4[l];
    if (ldw % 8 == 0) ldw += 4;  // 16 rows of a ds_read_b128 column slice -> 16 distinct slots
    sh->ldw[l] = ldw;
    sh->w_lds[l] = off;
    off += sh->rows4[l] * ldw;
    sh->b_lds[l] = off;
    off += sh->rows4[l];
  }
  for (int l = 0; l <= L; ++l) sh->lda[l] = r4(dims[l]);
  for (int b = 0; b < 2; ++b) {
    sh->a0_lds[b] = off;
    off += bmax * sh->lda[0];
  }
  sh->a_lds[0] = sh->a0_lds[0];
  for (int l = 1; l <= L; ++l) {
    sh->a_lds[l] = off;
    off += bmax * sh->lda[l];
  }
  for (int l = 0; l < L; ++l) {
    sh->dz_lds[l] = off;
    off += bmax * sh->rows4[l];
  }
  for (int b = 0; b < 2; ++b) {
    sh->lab_lds[b] = off;
    off += r4(bmax);
  }
  sh->red_lds = off;
  off += r4(2 * bmax);
  sh->lds_floats = off;
  sh->supported = (nt > 0) && (nbias <= 2 * nt) && ((size_t)off * 4 <= 160 * 1024) ? 1 : 0;
  sh->mlp_block = -1;  // auto until the plan stamps its knob copy
  return 0;
}

}  // namespace dct

using dct::MlpArgs;
using dct::MlpShape;

extern "C" {

int dct_mlp_shape_size() { return (int)sizeof(MlpShape); }

int dct_mlp_make_shape(void* out, const int* dims, int L, int bmax) {
  return dct::mlp_make_shape(reinterpret_cast<MlpShape*>(out), dims, L, bmax);
}

int dct_mlp_select(const MlpShape* sh, int* nt, int* maxblk) {
  *nt = sh->nt;
  *maxblk = sh->maxq;
  return sh->supported;
}

int dct_mlp_train(const void* shape, const MlpArgs* a, void* stream) {
  const MlpShape& sh = *reinterpret_cast<const MlpShape*>(shape);
  if (!sh.supported) return (int)hipErrorInvalidValue;
  if (a->B < 1 || a->B > sh.bmax) return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->stage && !dct::mlp_block5_ok(sh, *a)) {  // only mlp_block5's grad mode stages batches here
    MlpArgs b = *a;
    b.stage = nullptr;
    return dct_mlp_train(shape, &b, stream);
  }
  if (a->xg_world > 1) {  // in-kernel data parallelism: only the 3x128 block kernel has it here
    if (!dct::mlp_block5_ok(sh, *a)) return (int)hipErrorInvalidValue;
    return (int)dct::mlp_launch_block5(sh, *a, st);
  }
  const int blk = sh.mlp_block;  // plan-time DCT_MLP_BLOCK: -1 auto, 3 mlp_block3, 0 the generic LDS trainer
  if ((blk < 0 || blk == 8) && dct::mlp_block5_ok(sh, *a)) return (int)dct::mlp_launch_block5(sh, *a, st);
  if (blk != 0 && dct::mlp_block3_ok(sh, *a)) return (int)dct::mlp_launch_block3(sh, *a, st);
  switch (sh.L) {
    case 2: return (int)dct::mlp_launch_train_L2(sh, *a, st);
    case 3: return (int)dct::mlp_launch_train_L3(sh, *a, st);
    case 4: return (int)dct::mlp_launch_train_L4(sh, *a, st);
    default: return (int)hipErrorInvalidValue;
  }
}

int dct_mlp_eval(const void* shape, const MlpArgs* a, int grid, void* stream) {
  const MlpShape& sh = *reinterpret_cast<const MlpShape*>(shape);
  if ((size_t)sh.lds_floats * 4 > 160 * 1024) return (int)hipErrorInvalidValue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (sh.L) {
    case 2: return (int)dct::mlp_launch_eval_L2(sh, *a, grid, st);
    case 3: return (int)dct::mlp_launch_eval_L3(sh, *a, grid, st);
    case 4: return (int)dct::mlp_launch_eval_L4(sh, *a, grid, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // extern "C"
