// Timing diagnostics and main-loop experiments of the 256-row tile kernels (gemm_big_kernels.h; wrong results by
// design except 12 / 13; launch: gemm_big.hip): 6 = 256x256 without K-tile reloads (compute only), 7 = loads only;
// 12 / 13 = ping-pong wave groups, 32-deep K tiles in a ring of 4 / 5 buffers; 16..18 = variant 10 (256x128, 2 per
// CU) compute-only / loads-only / no epilogue, 19..21 = variant 14 (192x256) the same (tools/gemm_breakdown.py).
#include "gemm_big_kernels.h"

namespace mapa_gemm_impl {

GemmKernel big_kernel_diag(int variant, bool conv) {
  switch (variant) {
    case 6: return conv ? nullptr : gemm_big_kernel<0, 256, 128, 2, 1>;
    case 7: return conv ? nullptr : gemm_big_kernel<0, 256, 128, 2, 2>;
    case 12: return conv ? gemm_pp_kernel<1, 4> : gemm_pp_kernel<0, 4>;
    case 13: return conv ? gemm_pp_kernel<1, 5> : gemm_pp_kernel<0, 5>;
    case 16: return conv ? nullptr : gemm_big_kernel<0, 128, 64, 3, 1, 0, 2>;
    case 17: return conv ? nullptr : gemm_big_kernel<0, 128, 64, 3, 2, 0, 2>;
    case 18: return conv ? nullptr : gemm_big_kernel<0, 128, 64, 3, 3, 0, 2>;
    case 19: return conv ? nullptr : gemm_big_kernel<0, 256, 128, 2, 1, 1, 1, 192>;
    case 20: return conv ? nullptr : gemm_big_kernel<0, 256, 128, 2, 2, 1, 1, 192>;
    case 21: return conv ? nullptr : gemm_big_kernel<0, 256, 128, 2, 3, 1, 1, 192>;
    default: return nullptr;
  }
}

}  // namespace mapa_gemm_impl
