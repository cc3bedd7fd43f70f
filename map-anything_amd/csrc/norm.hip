// LayerNorm (nn.LayerNorm, eps 1e-6) over rows of an fp32 residual stream, one wave per row.
// Replaces norm1/norm2/final norms of DINOv2 (layers/block.py:93-118, vision_transformer.py:304),
// AAT (transformer_blocks.py:452-469, alternating_attention_transformer.py:706-747) and the fusion LayerNorm
// (model.py:1422-1431).  The row is held in registers (dim/64 floats per lane), two-pass mean/variance like
// ATen, and written as fp32 and/or the GEMM operand dtype (bf16 or fp32) in the same pass.
#include "mapa_common.h"

namespace {

template <int NV>  // NV float4 per lane: dim = 256 * NV
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ x, int64_t ldx, int rows,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float eps, float* __restrict__ yf, void* __restrict__ ylp,
                                                        int lp_bf16, int64_t ldy, int group, int64_t gstride,
                                                        int row_off) {
  constexpr int DIM = 256 * NV;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t in_row = (group > 0 ? (int64_t)(row / group) * gstride + row % group : (int64_t)row) + row_off;
  const float* xr = x + in_row * ldx;
  f32x4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = *reinterpret_cast<const f32x4*>(xr + (i * 64 + lane) * 4);
    s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
  }
  const float mean = wave_sum(s) * (1.f / DIM);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = v[i][j] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / DIM) + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 4;
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(b + c);
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = (v[i][j] - mean) * rstd * wv[j] + bv[j];
    if (yf) *reinterpret_cast<f32x4*>(yf + (int64_t)row * ldy + c) = y;
    if (ylp) {
      if (lp_bf16 == 2) {  // split operand row: [hi | lo], 2*ldy wide
        store_split3(reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * 2 * ldy + c, ldy, y);
      } else if (lp_bf16) {
        uint2 pk;
        pk.x = pack_bf16x2(y[0], y[1]);
        pk.y = pack_bf16x2(y[2], y[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * ldy + c) = pk;
      } else {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(ylp) + (int64_t)row * ldy + c) = y;
      }
    }
  }
}

}  // namespace

extern "C" int mapa_layernorm(const float* x, int64_t ldx, int rows, int dim, const float* w, const float* b,
                              float eps, float* y_f32, void* y_lp, int lp_dtype, int64_t ldy, int in_group,
                              int64_t in_group_stride, int in_row_off, hipStream_t stream) {
  MAPA_CHECK_ARG(x && w && b && rows > 0, "mapa_layernorm: bad args");
  MAPA_CHECK_ARG(y_f32 || y_lp, "mapa_layernorm: no output");
  MAPA_CHECK_ARG(dim == 768 || dim == 1024 || dim == 512 || dim == 256, "mapa_layernorm: dim %d unsupported", dim);
  MAPA_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0, "mapa_layernorm: strides must be multiples of 4");
  const dim3 grid((rows + 3) / 4), blk(256);
  MAPA_CHECK_ARG(lp_dtype == MAPA_F32 || lp_dtype == MAPA_BF16 || lp_dtype == MAPA_BF16X3, "mapa_layernorm: bad lp_dtype");
  const int bf = lp_dtype == MAPA_BF16X3 ? 2 : lp_dtype == MAPA_BF16 ? 1 : 0;
  switch (dim / 256) {
    case 1: hipLaunchKernelGGL(layernorm_kernel<1>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off); break;
    case 2: hipLaunchKernelGGL(layernorm_kernel<2>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off); break;
    case 3: hipLaunchKernelGGL(layernorm_kernel<3>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off); break;
    default: hipLaunchKernelGGL(layernorm_kernel<4>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off); break;
  }
  MAPA_CHECK_LAUNCH("mapa_layernorm");
  return 0;
}
