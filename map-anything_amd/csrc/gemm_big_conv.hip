// bf16 implicit-3x3-conv instantiations of the 256-row tile kernels (gemm_big_kernels.h; launch: gemm_big.hip).
#include "gemm_big_kernels.h"

namespace mapa_gemm_impl {

GemmKernel big_kernel_bf16_conv(int variant) {
  switch (variant) {
    case 0: return gemm_big_kernel<1, 256, 128, 2>;
    case 1: return gemm_big_kernel<1, 128, 128, 2>;
    case 2: return gemm_big_kernel<1, 256, 64, 4>;
    case 3: return gemm_big_kernel<1, 128, 64, 4>;
    case 4: return gemm_big_kernel<1, 128, 64, 6>;
    case 5: return gemm_big_kernel<1, 128, 128, 3>;
    case 8: return gemm_big_kernel<1, 256, 128, 2, 0, 1>;
    case 9: return gemm_big_kernel<1, 128, 128, 3, 0, 1>;
    case 10: return gemm_big_kernel<1, 128, 64, 3, 0, 0, 2>;
    case 11: return gemm_big_kernel<1, 128, 64, 3, 0, 1, 2>;
    case 14: return gemm_big_kernel<1, 256, 128, 2, 0, 1, 1, 192>;
    case 15: return gemm_big_kernel<1, 192, 128, 2, 0, 1, 1, 192>;
    default: return nullptr;
  }
}

}  // namespace mapa_gemm_impl
