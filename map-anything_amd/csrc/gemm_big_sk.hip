// Stream-K launch of the 256-row bf16 / fp16 GEMM (gemm_big_kernels.h gemm_sk_kernel): persistent grid, contiguous
// K-iteration ranges, last-arriver fix-up (see the kernel's comment).
#include "gemm_big_kernels.h"

namespace mapa_gemm_impl {

// Stream-K variants: 0 = 256x128 / 64-B rows / 3 stages / setprio / 2 per CU, 1 = 256x256 / 64-B rows / 3 stages
// / setprio / 1 per CU.  Workspace: [tickets: 64 Ki words][slabs: G * 2 * 256 * BN * 4].
static int sk_cus() { return gemm_device_cus(); }

static void sk_shape(int variant, int& bn, int& per_cu) {
  bn = variant == 1 ? 256 : 128;
  per_cu = variant == 1 ? 1 : 2;
}

int gemm_streamk_slots(int variant) {
  int bn, per_cu;
  sk_shape(variant, bn, per_cu);
  return sk_cus() * per_cu;
}

// Ticket words live in a fixed-size head shared by every shape (a shape-dependent split would let one shape's slabs
// overwrite another's tickets, which must stay zero between calls); shapes with more tiles use the DP schedule.
// the top LN_TICKET_WORDS words of the head belong to the LayerNorm-fused GEMM (launch_gemm_big_ln)
constexpr int64_t SK_MAX_TILES = GEMM_TICKET_BYTES / 4 - LN_TICKET_WORDS, SK_TICKET_BYTES = GEMM_TICKET_BYTES;

int64_t streamk_workspace_bytes(int M, int N, int variant) {
  if (variant < 0 || variant > 2) return 0;
  int bn, per_cu;
  sk_shape(variant, bn, per_cu);
  const int64_t tiles = (int64_t)((M + BBM - 1) / BBM) * ((N + bn - 1) / bn);
  if (tiles > SK_MAX_TILES) return 0;
  const int64_t G = (int64_t)sk_cus() * per_cu;
  return SK_TICKET_BYTES + G * 2 * BBM * bn * 4;
}

bool launch_gemm_streamk(const GemmArgs& a, bool conv, int variant, void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (variant < 0 || variant > 2 || !ws || (conv && variant != 1)) return false;  // convs: 256x256 only
  const int64_t need = streamk_workspace_bytes(a.M, a.N, variant);
  if (need == 0 || ws_bytes < need) return false;
  int bn, per_cu;
  sk_shape(variant, bn, per_cu);
  const int bk = 32;  // 64-B LDS rows
  const int64_t tiles = (int64_t)((a.M + BBM - 1) / BBM) * ((a.N + bn - 1) / bn);
  const int64_t nk = (a.K + bk - 1) / bk;
  if (tiles * nk >= (int64_t(1) << 31)) return false;
  SkArgs s;
  const int g = sk_cus() * per_cu;
  static const int dp_env = getenv("MAPA_SK_DP") ? atoi(getenv("MAPA_SK_DP")) : 1;   // tuning: 0 = pure stream-K
  static const int per_env = getenv("MAPA_SK_PER") ? atoi(getenv("MAPA_SK_PER")) : 0;  // tuning: iterations/block
  // kbench, 8 views: the tenth-of-a-tile floor took rn4@19 80 -> 55 us, layer4_rn 119 -> 87 (mapa_idx::sk_make_plan)
  const int G = mapa_idx::sk_make_plan(tiles, (int)nk, g, variant == 2, dp_env != 0, per_env, s);
  s.tickets = reinterpret_cast<int*>(ws);
  s.slabs = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + SK_TICKET_BYTES);
  void (*k)(GemmArgs, SkArgs);
  if (a.lp_f16) {  // the TF32-equivalent head convs / linears (MAPA_F16X2 operands)
    if (variant != 1) k = gemm_sk_kernel<0, 128, 64, 3, 1, 4, true>;
    else k = conv ? gemm_sk_kernel<1, 256, 64, 3, 1, 1, true> : gemm_sk_kernel<0, 256, 64, 3, 1, 1, true>;
  } else if (variant != 1) {
    k = gemm_sk_kernel<0, 128, 64, 3, 1, 4>;
  } else {
    k = conv ? gemm_sk_kernel<1, 256, 64, 3, 1, 1> : gemm_sk_kernel<0, 256, 64, 3, 1, 1>;
  }
  hipLaunchKernelGGL(k, dim3(G), dim3(BTHREADS), 0, stream, a, s);
  return true;
}

}  // namespace mapa_gemm_impl
