// LayerNorm (nn.LayerNorm, eps 1e-6) over rows of an fp32 residual stream, one wave per row.
// Replaces norm1/norm2/final norms of DINOv2 (layers/block.py:93-118, vision_transformer.py:304),
// AAT (transformer_blocks.py:452-469, alternating_attention_transformer.py:706-747) and the fusion LayerNorm
// (model.py:1422-1431).  The row is held in registers (dim/64 floats per lane), two-pass mean/variance like
// ATen, and written as fp32 and/or the GEMM operand dtype (bf16, fp16, a split bf16 pair, or fp32) in the same pass.
#include <stdlib.h>

#include "mapa_common.h"

namespace {

template <int NV>  // NV float4 per lane: dim = 256 * NV
__global__ void __launch_bounds__(256) layernorm_kernel(const float* __restrict__ x, int64_t ldx, int rows,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float eps, float* __restrict__ yf, void* __restrict__ ylp,
                                                        int lp_bf16, int64_t ldy, int group, int64_t gstride,
                                                        int row_off, unsigned* fault) {
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
      } else if (lp_bf16 == 4) {  // MAPA_F16X2 split row
        store_split2h(reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * 2 * ldy + c, ldy, y, fault);
      } else if (lp_bf16) {  // 1 = bf16, 3 = fp16
        if (lp_bf16 == 3) f16_check4(fault, y);
        uint2 pk;
        pk.x = pack_lp2(lp_bf16 == 3, y[0], y[1]);
        pk.y = pack_lp2(lp_bf16 == 3, y[2], y[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * ldy + c) = pk;
      } else {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(ylp) + (int64_t)row * ldy + c) = y;
      }
    }
  }
}


// 1024 wide rows: lane owns whole 8-channel groups (g*64 + lane), so a bf16 output group is one 16-B store
// and a split output one 16-B hi + one 16-B lo store (the float4-per-lane mapping above stores 8 B per lane).
template <int NG>  // 8-channel groups per lane (dim <= 512 * NG)
__global__ void __launch_bounds__(256) layernorm8_kernel(const float* __restrict__ x, int64_t ldx, int rows, int dim,
                                                         const float* __restrict__ w, const float* __restrict__ b,
                                                         float eps, float* __restrict__ yf, void* __restrict__ ylp,
                                                         int lp_bf16, int64_t ldy, int group, int64_t gstride,
                                                         int row_off, unsigned* fault) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int ng = dim / 8;
  const int64_t in_row = (group > 0 ? (int64_t)(row / group) * gstride + row % group : (int64_t)row) + row_off;
  const float* xr = x + in_row * ldx;
  f32x4 v[NG][2];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    const int c = (i * 64 + lane) * 8;
    if (i * 64 + lane < ng) {
      v[i][0] = *reinterpret_cast<const f32x4*>(xr + c);
      v[i][1] = *reinterpret_cast<const f32x4*>(xr + c + 4);
    } else {
      v[i][0] = v[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    s += (v[i][0][0] + v[i][0][1] + v[i][0][2] + v[i][0][3]) + (v[i][1][0] + v[i][1][1] + v[i][1][2] + v[i][1][3]);
  }
  const float mean = wave_sum(s) / (float)dim;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NG; ++i)
    if (i * 64 + lane < ng)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = v[i][h][j] - mean;
          q += d * d;
        }
  const float rstd = rsqrtf(wave_sum(q) / (float)dim + eps);
#pragma unroll
  for (int i = 0; i < NG; ++i) {
    if (i * 64 + lane >= ng) continue;
    const int c = (i * 64 + lane) * 8;
    f32x4 y[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c + 4 * h);
      const f32x4 bv = *reinterpret_cast<const f32x4*>(b + c + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) y[h][j] = (v[i][h][j] - mean) * rstd * wv[j] + bv[j];
    }
    if (yf) {
      *reinterpret_cast<f32x4*>(yf + (int64_t)row * ldy + c) = y[0];
      *reinterpret_cast<f32x4*>(yf + (int64_t)row * ldy + c + 4) = y[1];
    }
    if (ylp) {
      if (lp_bf16 == 2) {  // split operand row: [hi | lo], 2*ldy wide
        uint4 hv, lv;
        uint32_t* hp = &hv.x;
        uint32_t* lq = &lv.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float a0 = y[k >> 1][(k & 1) * 2], a1 = y[k >> 1][(k & 1) * 2 + 1];
          const bf16_t h0 = f32_to_bf16(a0), h1 = f32_to_bf16(a1);
          hp[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
          lq[k] = pack_bf16x2(a0 - bf16_to_f32(h0), a1 - bf16_to_f32(h1));
        }
        bf16_t* dst = reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * 2 * ldy + c;
        *reinterpret_cast<uint4*>(dst) = hv;
        *reinterpret_cast<uint4*>(dst + ldy) = lv;
      } else if (lp_bf16 == 4) {  // MAPA_F16X2 split row
        store_split2h_x8(reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * 2 * ldy + c, ldy, y[0], y[1], fault);
      } else if (lp_bf16) {  // 1 = bf16, 3 = fp16
        const bool h = lp_bf16 == 3;
        if (h) {
          f16_check4(fault, y[0]);
          f16_check4(fault, y[1]);
        }
        uint4 pk;
        pk.x = pack_lp2(h, y[0][0], y[0][1]);
        pk.y = pack_lp2(h, y[0][2], y[0][3]);
        pk.z = pack_lp2(h, y[1][0], y[1][1]);
        pk.w = pack_lp2(h, y[1][2], y[1][3]);
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(ylp) + (int64_t)row * ldy + c) = pk;
      } else {
        float* dst = reinterpret_cast<float*>(ylp) + (int64_t)row * ldy + c;
        *reinterpret_cast<f32x4*>(dst) = y[0];
        *reinterpret_cast<f32x4*>(dst + 4) = y[1];
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
  MAPA_CHECK_ARG(lp_dtype == MAPA_F32 || lp_dtype == MAPA_BF16 || lp_dtype == MAPA_BF16X3 || lp_dtype == MAPA_F16 ||
                     lp_dtype == MAPA_F16X2,
                 "mapa_layernorm: bad lp_dtype");
  const int bf = lp_dtype == MAPA_BF16X3 ? 2 : lp_dtype == MAPA_BF16 ? 1 : lp_dtype == MAPA_F16 ? 3
                 : lp_dtype == MAPA_F16X2 ? 4 : 0;
  unsigned* fault = mapa_gemm_impl::fault_word();
  static const bool f4_only = getenv("MAPA_LN_F4") != nullptr;  // A/B: the float4-per-lane kernel for every width
  // 1024 wide: 8-channel groups (kbench 13.2 -> 12.4 us); 768 wide keeps float4 lanes (10.0 vs 10.5: half the
  // lanes would idle in the second group)
  if (dim == 1024 && ldx % 8 == 0 && ldy % 8 == 0 && !f4_only) {
    hipLaunchKernelGGL(layernorm8_kernel<2>, grid, blk, 0, stream, x, ldx, rows, dim, w, b, eps, y_f32, y_lp, bf, ldy,
                       in_group, in_group_stride, in_row_off, fault);
    MAPA_CHECK_LAUNCH("mapa_layernorm");
    return 0;
  }
  switch (dim / 256) {
    case 1: hipLaunchKernelGGL(layernorm_kernel<1>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off, fault); break;
    case 2: hipLaunchKernelGGL(layernorm_kernel<2>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off, fault); break;
    case 3: hipLaunchKernelGGL(layernorm_kernel<3>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off, fault); break;
    default: hipLaunchKernelGGL(layernorm_kernel<4>, grid, blk, 0, stream, x, ldx, rows, w, b, eps, y_f32, y_lp, bf, ldy, in_group, in_group_stride, in_row_off, fault); break;
  }
  MAPA_CHECK_LAUNCH("mapa_layernorm");
  return 0;
}
