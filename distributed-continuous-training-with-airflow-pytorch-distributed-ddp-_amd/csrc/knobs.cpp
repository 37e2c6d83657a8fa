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
}  // namespace

void knobs_reload() {
  Knobs k;
  const char* mk = std::getenv("DCT_MLP_KERNEL");
  k.mlp_force_lds = (mk && std::strcmp(mk, "lds") == 0) ? 1 : 0;
  if (const char* b = std::getenv("DCT_MLP_BLOCK")) k.mlp_block = (b[0] == '0') ? 0 : (b[0] == '3' ? 3 : (b[0] == '8' ? 8 : -1));
  k.fused_head = env_int("DCT_FUSED_HEAD", 1) != 0;
  k.dw_into_adam = env_int("DCT_DW_INTO_ADAM", 1) != 0;
  k.reducer_inline = env_int("DCT_REDUCER_INLINE", -2);
  if (k.reducer_inline > 1 || k.reducer_inline < -2) k.reducer_inline = -2;
  k.rccl_one_rank = env_int("DCT_RCCL_ONE_RANK", 0) == 1;
  k.reducer_standin_us = env_int("DCT_REDUCER_STANDIN_US", 0);
  k.reducer_standin_wgs = env_int("DCT_REDUCER_STANDIN_WGS", 16);
  k.reducer_flag_edges = env_int("DCT_REDUCER_FLAG_EDGES", 1) != 0;
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
