// fp16-operand instantiations of the 256-row tile kernels (gemm_big_kernels.h; launch: gemm_big.hip): the tiles the
// automatic choice uses for the fp16 recipe's dense linears and for the TF32-equivalent head convs (MAPA_F16 /
// MAPA_F16X2 operands).
#include "gemm_big_kernels.h"

namespace mapa_gemm_impl {

GemmKernel big_kernel_f16(int variant, bool conv) {
  switch (variant) {
    case 8: return conv ? gemm_big_kernel<1, 256, 128, 2, 0, 1, 1, BBM, true> : gemm_big_kernel<0, 256, 128, 2, 0, 1, 1, BBM, true>;
    case 10: return conv ? nullptr : gemm_big_kernel<0, 128, 64, 3, 0, 0, 2, BBM, true>;
    case 11: return conv ? gemm_big_kernel<1, 128, 64, 3, 0, 1, 2, BBM, true> : gemm_big_kernel<0, 128, 64, 3, 0, 1, 2, BBM, true>;
    case 14: return conv ? gemm_big_kernel<1, 256, 128, 2, 0, 1, 1, 192, true> : gemm_big_kernel<0, 256, 128, 2, 0, 1, 1, 192, true>;
    case 15: return conv ? nullptr : gemm_big_kernel<0, 192, 128, 2, 0, 1, 1, 192, true>;
    default: return nullptr;
  }
}

}  // namespace mapa_gemm_impl
