// Optional geometric inputs of MapAnything: the layout / normalisation kernels around
// the dense ray / depth encoders (whose convolutions are mapa_gemm implicit GEMMs) and the per-view global
// features (camera rotation / translation / scale, depth scale) broadcast into the fused encoder tokens.
// All HBM-bound or tiny; fp32 throughout (the reference runs this block with autocast disabled, model.py:1377).
#include "mapa_common.h"

namespace {

constexpr int TPB = 256;
constexpr int DEPTH_CHUNKS = 64;  // per-view partial sums of the depth normaliser (deterministic two-pass)

inline int grid_for(int64_t n) {
  int64_t g = (n + TPB - 1) / TPB;
  if (g > 65536) g = 65536;
  return (int)(g < 1 ? 1 : g);
}

// nn.PixelUnshuffle(r) (dense_rep_encoder.py:279) from NHWC input to token rows:
//   out[(v*h + py)*w + px][c*r*r + i*r + j] = f(in[v][py*r + i][px*r + j][c])
// f = identity, or for the depth encoder input (model.py:1120-1132, geometry.py:1594-1626 / 1737-1750):
//   x' = x / view_div[v];  f = x' / max(|x'|, 1e-8) * log1p(|x'|)
template <typename T>
__global__ void unshuffle_kernel(const float* __restrict__ in, int n, int H, int W, int C, int r,
                                 const float* __restrict__ view_div, int lognorm, T* __restrict__ out, int64_t ldo) {
  const int h = H / r, w = W / r;
  const int K = C * r * r;
  const int64_t total = (int64_t)n * h * w * K;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % K);
    const int64_t row = e / K;
    const int px = (int)(row % w);
    const int64_t r2 = row / w;
    const int py = (int)(r2 % h);
    const int v = (int)(r2 / h);
    const int c = k / (r * r), rem = k - c * r * r, i = rem / r, j = rem - i * r;
    float x = in[(((int64_t)v * H + py * r + i) * W + px * r + j) * C + c];
    if (lognorm) {
      x = x / view_div[v];
      const float a = fabsf(x);
      x = x / fmaxf(a, 1e-8f) * log1pf(a);
    }
    if constexpr (sizeof(T) == 2) out[row * ldo + k] = f32_to_bf16(x);
    else out[row * ldo + k] = x;
  }
}

// normalize_depth_using_non_zero_pixels (geometry.py:1594-1626): per view the sum and count of d > 0.
__global__ void depth_partial_kernel(const float* __restrict__ d, int HW, float* __restrict__ part) {
  const int v = blockIdx.y, chunk = blockIdx.x;
  const int i0 = (int)((int64_t)HW * chunk / DEPTH_CHUNKS), i1 = (int)((int64_t)HW * (chunk + 1) / DEPTH_CHUNKS);
  const float* p = d + (int64_t)v * HW;
  float s = 0.f, c = 0.f;
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const float x = p[i];
    if (x > 0.f) {
      s += x;
      c += 1.f;
    }
  }
  __shared__ float ss[TPB / 64], sc[TPB / 64];
  s = wave_sum(s);
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) {
    ss[threadIdx.x >> 6] = s;
    sc[threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ts = 0.f, tc = 0.f;
    for (int k = 0; k < TPB / 64; ++k) {
      ts += ss[k];
      tc += sc[k];
    }
    part[((int64_t)v * DEPTH_CHUNKS + chunk) * 2] = ts;
    part[((int64_t)v * DEPTH_CHUNKS + chunk) * 2 + 1] = tc;
  }
}

// norm factor nf = clip(sum / (count + 1e-8), 1e-8); log_nf = log(nf + 1e-8) (model.py:1151).
__global__ void depth_final_kernel(const float* __restrict__ part, int n, float* __restrict__ nf,
                                   float* __restrict__ log_nf) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  float s = 0.f, c = 0.f;
  for (int k = 0; k < DEPTH_CHUNKS; ++k) {
    s += part[((int64_t)v * DEPTH_CHUNKS + k) * 2];
    c += part[((int64_t)v * DEPTH_CHUNKS + k) * 2 + 1];
  }
  const float f = fmaxf(s / (c + 1e-8f), 1e-8f);
  nf[v] = f;
  if (log_nf) log_nf[v] = logf(f + 1e-8f);
}

__device__ void quat_to_rot3(const float* q_in, float R[9]) {
  // geometry.py:601-652 (normalises q first)
  const float nq = sqrtf(q_in[0] * q_in[0] + q_in[1] * q_in[1] + q_in[2] * q_in[2] + q_in[3] * q_in[3]);
  const float x = q_in[0] / nq, y = q_in[1] / nq, z = q_in[2] / nq, w = q_in[3] / nq;
  R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - w * z);       R[2] = 2.f * (x * z + w * y);
  R[3] = 2.f * (x * y + w * z);       R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - w * x);
  R[6] = 2.f * (x * z - w * y);       R[7] = 2.f * (y * z + w * x);       R[8] = 1.f - 2.f * (x * x + y * y);
}

// Camera inputs of all views in the frame of view 0 (model.py:792-896 with
// transform_pose_using_quats_and_trans_2_to_1, geometry.py:745-852), then normalize_pose_translations
// (geometry.py:1629-1666) across views; identity / zero pose where cam_mask[v] == 0.  One thread (V is small).
__global__ void pose_inputs_kernel(const float* __restrict__ quats, const float* __restrict__ trans,
                                   const uint8_t* __restrict__ cam_mask, int V, float* __restrict__ out_q,
                                   float* __restrict__ out_t, float* __restrict__ out_log_nf) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const float* q1 = quats;
  const float* t1 = trans;
  const float n1 = q1[0] * q1[0] + q1[1] * q1[1] + q1[2] * q1[2] + q1[3] * q1[3];
  const float inv[4] = {-q1[0] / n1, -q1[1] / n1, -q1[2] / n1, q1[3] / n1};
  float R[9];
  quat_to_rot3(inv, R);
  float tinv[3];
  for (int i = 0; i < 3; ++i) tinv[i] = -(R[i * 3] * t1[0] + R[i * 3 + 1] * t1[1] + R[i * 3 + 2] * t1[2]);
  float dsum = 0.f, dcnt = 0.f;
  for (int v = 0; v < V; ++v) {
    float* q = out_q + v * 4;
    float* t = out_t + v * 3;
    if (cam_mask[v]) {
      const float* q2 = quats + v * 4;
      const float* t2 = trans + v * 3;
      const float x1 = inv[0], y1 = inv[1], z1 = inv[2], w1 = inv[3];
      const float x2 = q2[0], y2 = q2[1], z2 = q2[2], w2 = q2[3];
      q[0] = w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2;
      q[1] = w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2;
      q[2] = w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2;
      q[3] = w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2;
      for (int i = 0; i < 3; ++i) t[i] = (R[i * 3] * t2[0] + R[i * 3 + 1] * t2[1] + R[i * 3 + 2] * t2[2]) + tinv[i];
    } else {
      q[0] = q[1] = q[2] = 0.f;
      q[3] = 1.f;
      t[0] = t[1] = t[2] = 0.f;
    }
    const float dis = sqrtf(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
    dsum += dis;
    dcnt += dis > 0.f ? 1.f : 0.f;
  }
  const float nf = fmaxf(dsum / (dcnt + 1e-8f), 1e-8f);
  for (int v = 0; v < V; ++v) {
    for (int i = 0; i < 3; ++i) out_t[v * 3 + i] /= nf;
    out_log_nf[v] = logf(nf + 1e-8f);
  }
}

// x[v*T + t][c] += sum_j scales[j][v] * vecs[j][v][c]   (per-view global features, model.py:1155-1168, 1280-1287)
__global__ void add_view_vectors_kernel(float* __restrict__ x, int T, int C, int nviews,
                                        const float* __restrict__ vecs, const float* __restrict__ scales, int nvec) {
  const int c4 = C / 4;
  const int64_t total = (int64_t)nviews * T * c4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % c4) * 4;
    const int64_t r = e / c4;
    const int v = (int)(r / T);
    f32x4 acc = *reinterpret_cast<const f32x4*>(x + r * C + c);
    for (int j = 0; j < nvec; ++j) {
      const float s = scales[j * nviews + v];
      const f32x4 g = *reinterpret_cast<const f32x4*>(vecs + ((int64_t)j * nviews + v) * C + c);
      acc += s * g;
    }
    *reinterpret_cast<f32x4*>(x + r * C + c) = acc;
  }
}

__global__ void add_f32_kernel(float* __restrict__ dst, const float* __restrict__ src, int64_t n4) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
    f32x4 a = reinterpret_cast<f32x4*>(dst)[e];
    a += reinterpret_cast<const f32x4*>(src)[e];
    reinterpret_cast<f32x4*>(dst)[e] = a;
  }
}

// preprocess_input_views_for_inference (inference.py:222-311) per pixel: unit rays from pinhole intrinsics
// (get_rays_in_camera_frame, geometry.py:186-241) or renormalised given rays, and depth_z -> depth along the ray.
// Compiled without FMA contraction: same operation order as the reference's tensor expressions.
__global__ void view_rays_kernel(const float* __restrict__ K, const float* __restrict__ rays_in,
                                 const float* __restrict__ depth_z, int n, int H, int W, float* __restrict__ rays,
                                 float* __restrict__ depth_ray) {
  const int64_t total = (int64_t)n * H * W;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(e % W);
    const int64_t r2 = e / W;
    const int y = (int)(r2 % H);
    const int v = (int)(r2 / H);
    float d0, d1, d2;
    if (K) {
      const float* k = K + v * 9;
      const float xx = ((float)x - k[2]) / k[0];
      const float yy = ((float)y - k[5]) / k[4];
      const float nrm = sqrtf(xx * xx + yy * yy + 1.f);
      d0 = xx / nrm;
      d1 = yy / nrm;
      d2 = 1.f / nrm;
    } else {
      const float* r = rays_in + e * 3;
      const float nrm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]) + 1e-8f;
      d0 = r[0] / nrm;
      d1 = r[1] / nrm;
      d2 = r[2] / nrm;
    }
    rays[e * 3 + 0] = d0;
    rays[e * 3 + 1] = d1;
    rays[e * 3 + 2] = d2;
    if (depth_z) {
      const float dz = depth_z[e];
      const float p0 = dz * (d0 / d2), p1 = dz * (d1 / d2), p2 = dz * (d2 / d2);
      depth_ray[e] = sqrtf(p0 * p0 + p1 * p1 + p2 * p2);
    }
  }
}

}  // namespace

extern "C" int mapa_view_rays(const float* K, const float* rays_in, const float* depth_z, int n, int H, int W,
                              float* rays, float* depth_along_ray, hipStream_t stream) {
  MAPA_CHECK_ARG((K != nullptr) != (rays_in != nullptr), "mapa_view_rays: exactly one of K / rays_in");
  MAPA_CHECK_ARG(rays && n > 0 && H > 0 && W > 0, "mapa_view_rays: bad args");
  MAPA_CHECK_ARG(!depth_z || depth_along_ray, "mapa_view_rays: depth_z needs depth_along_ray");
  const int64_t total = (int64_t)n * H * W;
  hipLaunchKernelGGL(view_rays_kernel, dim3(grid_for(total)), dim3(TPB), 0, stream, K, rays_in, depth_z, n, H, W, rays,
                     depth_along_ray);
  MAPA_CHECK_LAUNCH("mapa_view_rays");
  return 0;
}

extern "C" int mapa_pixel_unshuffle(const float* in, int n, int H, int W, int C, int r, const float* view_div,
                                    int lognorm, void* out, int out_dtype, int64_t ldo, hipStream_t stream) {
  MAPA_CHECK_ARG(in && out && n > 0 && C > 0 && r > 0 && H % r == 0 && W % r == 0,
                 "mapa_pixel_unshuffle: bad args (H, W must be multiples of r)");
  MAPA_CHECK_ARG(ldo >= (int64_t)C * r * r, "mapa_pixel_unshuffle: ldo < C*r*r");
  MAPA_CHECK_ARG(!lognorm || view_div, "mapa_pixel_unshuffle: lognorm needs view_div");
  const int64_t total = (int64_t)n * (H / r) * (W / r) * C * r * r;
  if (out_dtype == MAPA_BF16)
    hipLaunchKernelGGL(unshuffle_kernel<bf16_t>, dim3(grid_for(total)), dim3(TPB), 0, stream, in, n, H, W, C, r,
                       view_div, lognorm, reinterpret_cast<bf16_t*>(out), ldo);
  else
    hipLaunchKernelGGL(unshuffle_kernel<float>, dim3(grid_for(total)), dim3(TPB), 0, stream, in, n, H, W, C, r,
                       view_div, lognorm, reinterpret_cast<float*>(out), ldo);
  MAPA_CHECK_LAUNCH("mapa_pixel_unshuffle");
  return 0;
}

extern "C" int mapa_depth_norm_factors(const float* depth, int n, int HW, float* nf, float* log_nf, void* work,
                                       hipStream_t stream) {
  MAPA_CHECK_ARG(depth && nf && work && n > 0 && HW > 0, "mapa_depth_norm_factors: bad args");
  float* part = reinterpret_cast<float*>(work);
  hipLaunchKernelGGL(depth_partial_kernel, dim3(DEPTH_CHUNKS, n), dim3(TPB), 0, stream, depth, HW, part);
  hipLaunchKernelGGL(depth_final_kernel, dim3((n + 63) / 64), dim3(64), 0, stream, part, n, nf, log_nf);
  MAPA_CHECK_LAUNCH("mapa_depth_norm_factors");
  return 0;
}

extern "C" int mapa_pose_inputs(const float* quats, const float* trans, const uint8_t* cam_mask, int V, float* out_q,
                                float* out_t, float* out_log_nf, hipStream_t stream) {
  MAPA_CHECK_ARG(quats && trans && cam_mask && out_q && out_t && out_log_nf && V > 0, "mapa_pose_inputs: bad args");
  hipLaunchKernelGGL(pose_inputs_kernel, dim3(1), dim3(64), 0, stream, quats, trans, cam_mask, V, out_q, out_t,
                     out_log_nf);
  MAPA_CHECK_LAUNCH("mapa_pose_inputs");
  return 0;
}

extern "C" int mapa_add_view_vectors(float* x, int T, int C, int nviews, const float* vecs, const float* scales,
                                     int nvec, hipStream_t stream) {
  MAPA_CHECK_ARG(x && vecs && scales && T > 0 && C % 4 == 0 && nviews > 0 && nvec > 0,
                 "mapa_add_view_vectors: bad args (C %% 4 == 0)");
  const int64_t total = (int64_t)nviews * T * (C / 4);
  hipLaunchKernelGGL(add_view_vectors_kernel, dim3(grid_for(total)), dim3(TPB), 0, stream, x, T, C, nviews, vecs,
                     scales, nvec);
  MAPA_CHECK_LAUNCH("mapa_add_view_vectors");
  return 0;
}

extern "C" int mapa_add_f32(float* dst, const float* src, int64_t n, hipStream_t stream) {
  MAPA_CHECK_ARG(dst && src && n >= 0 && n % 4 == 0, "mapa_add_f32: bad args (n %% 4 == 0)");
  if (n == 0) return 0;
  hipLaunchKernelGGL(add_f32_kernel, dim3(grid_for(n / 4)), dim3(TPB), 0, stream, dst, src, n / 4);
  MAPA_CHECK_LAUNCH("mapa_add_f32");
  return 0;
}
