// The one place the native side reads DCT_* environment knobs (see knobs.h).
#include "knobs.h"

#include <cstdlib>
#include <cstring>

namespace dct {

namespace {
Knobs g_knobs;
bool g_loaded = false;

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e && *e) ? std::atoi(e) : dflt;
}
bool env_set(const char* name) { return std::getenv(name) != nullptr; }
}  // namespace

void knobs_reload() {
  Knobs k;
  const char* mk = std::getenv("DCT_MLP_KERNEL");
  k.mlp_force_lds = (mk && std::strcmp(mk, "lds") == 0) ? 1 : 0;
  if (const char* b = std::getenv("DCT_MLP_BLOCK")) k.mlp_block = (b[0] == '0') ? 0 : (b[0] == '3' ? 3 : -1);
  k.mlp_block_mf = env_int("DCT_MLP_BLOCK_MF", 1) != 0;
  k.b3_prio = env_int("DCT_B3_PRIO", -1);
  k.mlp_rows = env_int("DCT_MLP_ROWS", 1) != 0;
  k.gemm_v1 = env_set("DCT_GEMM_V1");
  k.gemm_split_ws = env_set("DCT_GEMM_SPLIT_WS");
  k.gemm_two_pass = env_int("DCT_GEMM_SPLIT_TWO_PASS", -1);
  k.gemm_stages = env_int("DCT_GEMM_STAGES", 0);
  k.gemm_split_wg = env_int("DCT_GEMM_SPLIT_WG", 0);
  k.gemm_splits = env_int("DCT_GEMM_SPLITS", 0);
  k.gemm_8w = env_int("DCT_GEMM_8W", -1);  // -1 auto, 0 off
  k.gemm_split_8w = env_int("DCT_GEMM_SPLIT_8W", 1) != 0;
  k.gemm_bm128 = env_set("DCT_GEMM_BM128");
  k.gemm_bm64_nk = env_int("DCT_GEMM_BM64_NK", 4);
  k.gemm_no_group = env_set("DCT_GEMM_NO_GROUP");
  k.gemm_dw_mink = env_int("DCT_GEMM_DW_MINK", 0);
  k.skinny_head_rpw = env_int("DCT_SKINNY_HEAD_RPW", 0);
  k.skinny_head_waves = env_int("DCT_SKINNY_HEAD_WAVES", 0);
  k.skinny_dw_splits = env_int("DCT_SKINNY_DW_SPLITS", 0);
  k.tt_head_spb = env_int("DCT_TT_HEAD_SPB", 4) == 16 ? 16 : 4;
  k.attn_scalar = env_set("DCT_ATTN_SCALAR");
  k.fused_head = env_int("DCT_FUSED_HEAD", 1) != 0;
  k.dw_into_adam = env_int("DCT_DW_INTO_ADAM", 1) != 0;
  k.reducer_inline = env_int("DCT_REDUCER_INLINE", -2);
  k.rccl_one_rank = env_int("DCT_RCCL_ONE_RANK", 0) == 1;
  if (k.reducer_inline > 1 || k.reducer_inline < -2) k.reducer_inline = -2;
  k.reducer_standin_us = env_int("DCT_REDUCER_STANDIN_US", 0);
  k.reducer_standin_wgs = env_int("DCT_REDUCER_STANDIN_WGS", 16);
  if (k.reducer_standin_us < 0) k.reducer_standin_us = 0;
  if (k.reducer_standin_wgs < 1) k.reducer_standin_wgs = 1;
  if (k.reducer_standin_wgs > 1024) k.reducer_standin_wgs = 1024;
  g_knobs = k;
  g_loaded = true;
}

const Knobs& knobs() {
  if (!g_loaded) knobs_reload();  // first use in a process that never called the reload
  return g_knobs;
}

}  // namespace dct

extern "C" void dct_knobs_reload() { dct::knobs_reload(); }
