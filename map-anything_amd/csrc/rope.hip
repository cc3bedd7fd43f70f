// RoPE-2D (uniception croco RoPE2D / cuRoPE2D: pos_embed.py:101-155, curope/kernels.cu:17-82), in place.
// tokens (B, H, N, D) with element strides (sb, sh, sn) and contiguous head dim; positions int64 (B, N, 2) = (y, x).
// Head dim layout [u_y | v_y | u_x | v_x], quarters of Q = D/4: the y half rotates pairs (u_y[j], v_y[j]) by
// pos_y * f_j, the x half (u_x[j], v_x[j]) by pos_x * f_j, f_j = F0 / base^(j/Q); u' = u cos - v sin,
// v' = v cos + u sin.  fp32 math (sincos of the fp32 angle, as kernels.cu), one rounding at the store for bf16.
// The frequencies are the reference's fp32 values exactly (below); cos/sin of the same fp32 angle differ from
// torch's CPU ones by at most an ulp or two.
// One thread per (token, head, half, 4 consecutive j): consecutive threads walk j, so a wave reads and writes
// contiguous 16-B (fp32) / 8-B (bf16) segments of each head's row.
#include "mapa_common.h"

namespace {

constexpr int TPB = 256;
inline int grid_for(int64_t n) { return (int)std::min<int64_t>((n + TPB - 1) / TPB, 65536); }

template <typename T>
__device__ __forceinline__ f32x4 ld4(const T* p) {
  if constexpr (sizeof(T) == 2) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return f32x4{bf16_to_f32(u.x & 0xffff), bf16_to_f32(u.x >> 16), bf16_to_f32(u.y & 0xffff), bf16_to_f32(u.y >> 16)};
  } else {
    return *reinterpret_cast<const f32x4*>(p);
  }
}

template <typename T>
__device__ __forceinline__ void st4(T* p, f32x4 v) {
  if constexpr (sizeof(T) == 2) {
    uint2 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = u;
  } else {
    *reinterpret_cast<f32x4*>(p) = v;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) rope2d_kernel(T* __restrict__ tok, const int64_t* __restrict__ pos, int B, int H,
                                                     int N, int D, int64_t sb, int64_t sh, int64_t sn, float base,
                                                     float f0) {
  const int Q = D / 4, g4 = Q / 4;        // 4-wide j groups per half
  const int per_tok = H * 2 * g4;         // threads per token
  const int64_t total = (int64_t)B * N * per_tok;
  // inv_freq[j] = F0 / fp32(base^(j/Q)): pow correctly rounded to fp32 then an fp32 division, which is what the
  // reference's fp32 torch ops produce (1.0 / (base ** (arange(0, D/2, 2) / (D/2))), pos_embed.py:117)
  __shared__ float inv_freq[64];
  for (int j = threadIdx.x; j < Q; j += blockDim.x) inv_freq[j] = f0 / (float)pow((double)base, (double)j / (double)Q);
  __syncthreads();
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int jg = (int)(e % g4);
    int64_t r = e / g4;
    const int X = (int)(r % 2);
    r /= 2;
    const int h = (int)(r % H);
    r /= H;
    const int n = (int)(r % N);
    const int b = (int)(r / N);
    const float p = (float)pos[((int64_t)b * N + n) * 2 + X];
    T* base_ptr = tok + b * sb + h * sh + (int64_t)n * sn + X * (D / 2) + jg * 4;
    const f32x4 u = ld4(base_ptr), v = ld4(base_ptr + Q);
    f32x4 uo, vo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float ang = p * inv_freq[jg * 4 + k];
      const float c = cosf(ang), s = sinf(ang);
      uo[k] = u[k] * c - v[k] * s;
      vo[k] = v[k] * c + u[k] * s;
    }
    st4(base_ptr, uo);
    st4(base_ptr + Q, vo);
  }
}

}  // namespace

extern "C" int mapa_rope2d(void* tokens, int dtype, int B, int H, int N, int D, int64_t sb, int64_t sh, int64_t sn,
                           const int64_t* positions, float base, float f0, hipStream_t stream) {
  MAPA_CHECK_ARG(tokens && positions && B > 0 && H > 0 && N > 0, "mapa_rope2d: bad args");
  MAPA_CHECK_ARG(D > 0 && D % 16 == 0 && D <= 256, "mapa_rope2d: head dim %d must be a multiple of 16, <= 256", D);
  MAPA_CHECK_ARG(dtype == MAPA_F32 || dtype == MAPA_BF16, "mapa_rope2d: dtype must be f32 or bf16");
  MAPA_CHECK_ARG(sb % 4 == 0 && sh % 4 == 0 && sn % 4 == 0, "mapa_rope2d: strides must keep 4-element alignment");
  // the kernel moves 4 elements per vector access (16 B fp32 / 8 B bf16): the base must be aligned to that too
  MAPA_CHECK_ARG(((uintptr_t)tokens % (dtype == MAPA_BF16 ? 8 : 16)) == 0,
                 "mapa_rope2d: tokens base pointer must be %d-byte aligned", dtype == MAPA_BF16 ? 8 : 16);
  const int64_t total = (int64_t)B * N * H * 2 * (D / 16);
  const dim3 g(grid_for(total)), b(TPB);
  if (dtype == MAPA_BF16)
    hipLaunchKernelGGL(rope2d_kernel<bf16_t>, g, b, 0, stream, (bf16_t*)tokens, positions, B, H, N, D, sb, sh, sn, base, f0);
  else
    hipLaunchKernelGGL(rope2d_kernel<float>, g, b, 0, stream, (float*)tokens, positions, B, H, N, D, sb, sh, sn, base, f0);
  MAPA_CHECK_LAUNCH("mapa_rope2d");
  return 0;
}
