// bf16 dense-A instantiations of the 256-row tile kernels (gemm_big_kernels.h; launch: gemm_big.hip).
#include "gemm_big_kernels.h"

namespace mapa_gemm_impl {

GemmKernel big_kernel_bf16_dense(int variant) {
  switch (variant) {
    case 0: return gemm_big_kernel<0, 256, 128, 2>;
    case 1: return gemm_big_kernel<0, 128, 128, 2>;
    case 2: return gemm_big_kernel<0, 256, 64, 4>;
    case 3: return gemm_big_kernel<0, 128, 64, 4>;
    case 4: return gemm_big_kernel<0, 128, 64, 6>;
    case 5: return gemm_big_kernel<0, 128, 128, 3>;
    case 8: return gemm_big_kernel<0, 256, 128, 2, 0, 1>;
    case 9: return gemm_big_kernel<0, 128, 128, 3, 0, 1>;
    // two workgroups per CU (72 KiB LDS, <= 128 VGPRs): one tile's epilogue overlaps the other's main loop
    case 10: return gemm_big_kernel<0, 128, 64, 3, 0, 0, 2>;
    case 11: return gemm_big_kernel<0, 128, 64, 3, 0, 1, 2>;
    // 192-row tiles: 10960 rows -> 58 row tiles, so N = 1024 gives 232 tiles for 256 CUs (256-row: 172)
    case 14: return gemm_big_kernel<0, 256, 128, 2, 0, 1, 1, 192>;
    // 192x192 tiles (wave tile 96x48): N = 768 at 8 views -> 232 tiles, one wave on the CUs (192x256: 174 tiles)
    case 15: return gemm_big_kernel<0, 192, 128, 2, 0, 1, 1, 192>;
    default: return nullptr;
  }
}

// LayerNorm-fused residual linears (launch_gemm_big_ln): 14 = 192x256 tiles, 15 = 192x192
GemmKernel big_kernel_lnf(int variant) {
  return variant == 14 ? gemm_big_kernel<0, 256, 128, 2, 0, 1, 1, 192, false, true>
                       : gemm_big_kernel<0, 192, 128, 2, 0, 1, 1, 192, false, true>;
}

}  // namespace mapa_gemm_impl
