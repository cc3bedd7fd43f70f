// infer() post-processing on the device (the reference does this in CPU numpy at
// ~230 ms/view): edge-aware output mask (inference.py:407-480 with geometry.py:1788-1853 points_to_normals,
// :2200-2258 normals_edge, :2102-2145 depth_edge), pinhole intrinsics recovery (geometry.py:304-447) and
// image de-normalisation (image.py:93-131).
//
// The mask is three 3x3-stencil passes over each view (NHWC, one thread per pixel):
//   K1 normals + normal validity (points_to_normals with mask), K2 per-pixel window state of the normal angles
//   (NaN-propagating like numpy's .max, edge-replicated padding like np.pad mode="edge", transposed mask
//   window), K3 3x3 nan-max pool of the angles (max_pool_2d uses np.nanmax with NaN padding) + depth edge +
//   final combine.  Float operations follow numpy's order (no fma contraction, -ffp-contract=off) so equal
//   inputs give equal bits; the angle threshold is applied on the dot product (arccos is monotone).
#include "mapa_common.h"
#include "index_math.h"

#include <math.h>
#include <string.h>

namespace {

__device__ __forceinline__ bool ldm(const uint8_t* m, int H, int W, int y, int x) {
  return (y >= 0 && y < H && x >= 0 && x < W) ? m[y * W + x] != 0 : false;
}

__device__ __forceinline__ void ldp(const float* p, int H, int W, int y, int x, float v[3]) {
  if (y >= 0 && y < H && x >= 0 && x < W) {
    const float* q = p + ((int64_t)y * W + x) * 3;
    v[0] = q[0]; v[1] = q[1]; v[2] = q[2];
  } else {
    v[0] = v[1] = v[2] = 0.f;
  }
}

__device__ __forceinline__ void cross3(const float a[3], const float b[3], float c[3]) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ float norm3(const float a[3]) {
  return sqrtf(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
}

// K1: points_to_normals(point, mask) -> normal (H,W,3) and normal_mask (H,W).  Stored already renormalised
// (n / (|n| + 1e-12), normals_edge's first step, geometry.py:2216): K2 reads every normal 9 times, and the same
// float operations applied once per pixel give the same bits.  32-bit pixel indices (the host checks n*H*W).
// Grid-stride step in 64-bit, clamped to `total` (mapa_idx::grid_step): a 32-bit `e += stride` overflows when total
// is within one grid of 2^31; the index stays 32-bit inside the loop bodies.
__device__ __forceinline__ int grid_next(int e, int total) {
  return mapa_idx::grid_step(e, total, (int64_t)gridDim.x * blockDim.x);
}

__global__ void normals_kernel(const float* __restrict__ pts, const uint8_t* __restrict__ mask, int n, int H, int W,
                               float* __restrict__ nrm, uint8_t* __restrict__ nmask) {
  const int total = n * H * W, HW = H * W;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e = grid_next(e, total)) {
    const int im = e / HW;
    const int rem = e - im * HW;
    const int y = rem / W, x = rem - y * W;
    const float* P = pts + (int64_t)im * H * W * 3;
    const uint8_t* M = mask + (int64_t)im * H * W;
    float c[3], u[3], l[3], d[3], r[3];
    ldp(P, H, W, y, x, c);
    ldp(P, H, W, y - 1, x, u);
    ldp(P, H, W, y, x - 1, l);
    ldp(P, H, W, y + 1, x, d);
    ldp(P, H, W, y, x + 1, r);
    for (int k = 0; k < 3; ++k) { u[k] -= c[k]; l[k] -= c[k]; d[k] -= c[k]; r[k] -= c[k]; }
    float nn[4][3];
    cross3(u, l, nn[0]);
    cross3(l, d, nn[1]);
    cross3(d, r, nn[2]);
    cross3(r, u, nn[3]);
    const bool mc = ldm(M, H, W, y, x);
    const bool mu = ldm(M, H, W, y - 1, x), ml = ldm(M, H, W, y, x - 1);
    const bool md = ldm(M, H, W, y + 1, x), mr = ldm(M, H, W, y, x + 1);
    const bool valid[4] = {mu && ml && mc, ml && md && mc, md && mr && mc, mr && mu && mc};
    // (normal * valid).sum(axis=0): numpy starts from the first slice and adds the others in order
    float s[3];
    bool any = false;
    for (int i = 0; i < 4; ++i) {
      const float inv = norm3(nn[i]) + 1e-12f;
      const float vf = valid[i] ? 1.f : 0.f;
      any |= valid[i];
      for (int k = 0; k < 3; ++k) {
        const float t = (nn[i][k] / inv) * vf;
        s[k] = i == 0 ? t : s[k] + t;
      }
    }
    const float ns = norm3(s) + 1e-12f;
    float o[3];
    for (int k = 0; k < 3; ++k) o[k] = any ? s[k] / ns : 0.f;
    const float no = norm3(o) + 1e-12f;
    float* un = nrm + (int64_t)e * 3;
    for (int k = 0; k < 3; ++k) un[k] = o[k] / no;
    nmask[e] = any ? 1 : 0;
  }
}

// K2: normals_edge before its max-pool.  Per pixel the reference takes A = max over the 3x3 window (edge
// padding) of where(mask_window, arccos(n_c . n_w), 0) with NaN propagating, then compares the pooled max with
// deg2rad(tol).  arccos is monotone, so "arccos(d) > tol" is "d < cos_thr" for the float32 boundary cos_thr the
// host derives from the same arccos (mapa_normal_cos_threshold / the Python host); a masked-out entry is the
// value 0 = arccos(1).  State per pixel: 2 = A is NaN (some masked-in |d| > 1 or NaN), 1 = A > tol, 0 = A <= tol.
// The mask window is the TRANSPOSE of the normals window: sliding_window_2d(mask, axis=(-3, -2)) on the 2-D mask
// wraps the axes to (1, 0) (geometry.py:1933, 2239-2247), so the normal at (y+dy, x+dx) is gated by the mask at
// (y+dx, x+dy), both clamped to the image (np.pad mode="edge").
__global__ void normal_state_kernel(const float* __restrict__ nrm, const uint8_t* __restrict__ nmask, int n, int H,
                                    int W, float cos_thr, uint8_t* __restrict__ state) {
  const int total = n * H * W, HW = H * W;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e = grid_next(e, total)) {
    const int im = e / HW;
    const int rem = e - im * HW;
    const int y = rem / W, x = rem - y * W;
    const float* N = nrm + (int64_t)im * HW * 3;  // unit normals (K1)
    const uint8_t* Mk = nmask + (int64_t)im * HW;
    float c[3];
    {
      const float* q = N + (y * W + x) * 3;
      for (int k = 0; k < 3; ++k) c[k] = q[k];
    }
    bool nan = false, edge = false;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int ny = min(max(y + dy, 0), H - 1), nx = min(max(x + dx, 0), W - 1);
        const int my = min(max(y + dx, 0), H - 1), mx = min(max(x + dy, 0), W - 1);
        float d = 1.f;  // masked out: angle 0 = arccos(1)
        if (Mk[my * W + mx]) {
          const float* q = N + (ny * W + nx) * 3;
          d = c[0] * q[0] + c[1] * q[1] + c[2] * q[2];
          if (!(fabsf(d) <= 1.f)) nan = true;  // arccos -> NaN (also for NaN d)
        }
        edge |= d < cos_thr;
      }
    state[e] = nan ? 2 : (edge ? 1 : 0);
  }
}

// K3: nan-max pool of the angles (max_pool_2d pads with NaN and takes np.nanmax: the pooled max exceeds tol iff
// some in-image, non-NaN neighbour does), depth edge, final mask
__global__ void mask_combine_kernel(const uint8_t* __restrict__ state, const float* __restrict__ depth_z,
                                    int64_t dz_stride, const uint8_t* __restrict__ m_in, int n, int H, int W,
                                    float rtol, int use_edges, uint8_t* __restrict__ m_out) {
  const int total = n * H * W, HW = H * W;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e = grid_next(e, total)) {
    const bool mc = m_in[e] != 0;
    bool keep = mc;
    if (use_edges && mc) {
      const int im = e / HW;
      const int rem = e - im * HW;
      const int y = rem / W, x = rem - y * W;
      const uint8_t* S = state + (int64_t)im * H * W;
      const uint8_t* M = m_in + (int64_t)im * H * W;
      const float* D = depth_z + (int64_t)im * H * W * dz_stride;
      float dmax = -INFINITY, ndmax = -INFINITY;
      bool nedge = false;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int yy = y + dy, xx = x + dx;
          if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;  // NaN padding: ignored by nanmax
          const int64_t k = (int64_t)yy * W + xx;
          nedge |= S[k] == 1;
          const float d = M[k] ? D[k * dz_stride] : -INFINITY;
          const float nd = M[k] ? -D[k * dz_stride] : -INFINITY;
          if (d == d) dmax = fmaxf(dmax, d);
          if (nd == nd) ndmax = fmaxf(ndmax, nd);
        }
      const float diff = dmax + ndmax;
      const float dc = D[(int64_t)rem * dz_stride];
      const bool dedge = (diff / dc) > rtol;
      keep = !(dedge && nedge);
    }
    m_out[e] = keep ? 1 : 0;
  }
}

// recover_pinhole_intrinsics_from_ray_directions, regression branch (<= 1 MPix): one block per view,
// normal equations of x = cx + fx * dx/dz (and y) over the strided sample grid, fp64 sums.
__global__ void recover_intrinsics_kernel(const float* __restrict__ rays, int H, int W, float* __restrict__ K) {
  const int im = blockIdx.x;
  const int sh = max(1, H / 50), sw = max(1, W / 50);
  const int nh = (H + sh - 1) / sh, nw = (W + sw - 1) / sw;
  double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // n, Sx_r, Sx_rr, Sx_b, Sx_rb, Sy_r, Sy_rr, Sy_b ... (+Sy_rb below)
  double yb = 0.0;
  const float* R = rays + (int64_t)im * H * W * 3;
  for (int s = threadIdx.x; s < nh * nw; s += blockDim.x) {
    const int y = (s / nw) * sh, x = (s % nw) * sw;
    const float* r = R + ((int64_t)y * W + x) * 3;
    const double rx = (double)(r[0] / r[2]), ry = (double)(r[1] / r[2]);
    a[0] += 1.0;
    a[1] += rx; a[2] += rx * rx; a[3] += x; a[4] += rx * x;
    a[5] += ry; a[6] += ry * ry; a[7] += y; yb += ry * y;
  }
  __shared__ double red[9][256];
  for (int i = 0; i < 8; ++i) red[i][threadIdx.x] = a[i];
  red[8][threadIdx.x] = yb;
  __syncthreads();
  for (int st = blockDim.x / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st)
      for (int i = 0; i < 9; ++i) red[i][threadIdx.x] += red[i][threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double N = red[0][0];
    const double detx = N * red[2][0] - red[1][0] * red[1][0];
    const double cx = (red[2][0] * red[3][0] - red[1][0] * red[4][0]) / detx;
    const double fx = (N * red[4][0] - red[1][0] * red[3][0]) / detx;
    const double dety = N * red[6][0] - red[5][0] * red[5][0];
    const double cy = (red[6][0] * red[7][0] - red[5][0] * red[8][0]) / dety;
    const double fy = (N * red[8][0] - red[5][0] * red[7][0]) / dety;
    float* k = K + im * 9;
    k[0] = (float)fx; k[1] = 0.f; k[2] = (float)cx;
    k[3] = 0.f; k[4] = (float)fy; k[5] = (float)cy;
    k[6] = 0.f; k[7] = 0.f; k[8] = 1.f;
  }
}

__global__ void denorm_image_kernel(const float* __restrict__ img, int n, int H, int W, const float* __restrict__ mean,
                                    const float* __restrict__ stdv, float* __restrict__ out) {
  const int64_t total = (int64_t)n * H * W;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int im = (int)(e / ((int64_t)H * W));
    const int64_t p = e - (int64_t)im * H * W;
    for (int c = 0; c < 3; ++c) {
      const float v = img[((int64_t)im * 3 + c) * H * W + p] * stdv[c] + mean[c];
      out[e * 3 + c] = fminf(fmaxf(v, 0.f), 1.f);
    }
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

// Geometry zeroing of infer (inference.py:486-500): pts3d / pts3d_cam / depth_along_ray *= mask (as float, so
// masked values become +-0 and NaN stays NaN, exactly like the reference's multiply).
__global__ void apply_mask_kernel(float* __restrict__ pts3d, float* __restrict__ pts_cam, float* __restrict__ depth,
                                  const uint8_t* __restrict__ mask, int64_t npix) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix; i += (int64_t)gridDim.x * blockDim.x) {
    const float m = mask[i] ? 1.f : 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      pts3d[i * 3 + c] *= m;
      pts_cam[i * 3 + c] *= m;
    }
    depth[i] *= m;
  }
}

// apply_confidence_mask (inference.py:455-470): thr = torch.quantile(conf_view, q) (linear interpolation between
// the floor / ceil order statistics of q*(N-1)), mask_out = mask_in & (conf > thr).  One workgroup per view; the
// two order statistics by 4-pass 8-bit radix select on order-preserving keys of the fp32 bits.
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unkey(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ uint32_t radix_select(const float* __restrict__ x, int64_t N, int64_t k, uint32_t* hist, uint32_t* shared) {
  uint32_t prefix = 0, mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
      const uint32_t key = fkey(x[i]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t kk = (int64_t)shared[1] | ((int64_t)shared[2] << 32);
      if (shift == 24) kk = k;
      uint32_t b = 0;
      for (; b < 255; ++b) {
        if ((int64_t)hist[b] > kk) break;
        kk -= hist[b];
      }
      shared[0] = prefix | (b << shift);
      shared[1] = (uint32_t)(kk & 0xffffffff);
      shared[2] = (uint32_t)(kk >> 32);
    }
    __syncthreads();
    prefix = shared[0];
    mask |= 255u << shift;
    __syncthreads();
  }
  return prefix;
}

__global__ void confidence_mask_kernel(const float* __restrict__ conf, const uint8_t* __restrict__ mask_in,
                                       uint8_t* __restrict__ mask_out, int64_t N, float q) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t shared[3];
  const float* x = conf + (int64_t)blockIdx.x * N;
  const double pos = (double)q * (double)(N - 1);
  const int64_t lo = (int64_t)floor(pos), hi = (int64_t)ceil(pos);
  const float vlo = unkey(radix_select(x, N, lo, hist, shared));
  const float vhi = hi == lo ? vlo : unkey(radix_select(x, N, hi, hist, shared));
  const float thr = vlo + (vhi - vlo) * (float)(pos - (double)lo);
  const uint8_t* mi = mask_in + (int64_t)blockIdx.x * N;
  uint8_t* mo = mask_out + (int64_t)blockIdx.x * N;
  for (int64_t i = threadIdx.x; i < N; i += blockDim.x) mo[i] = (mi[i] && x[i] > thr) ? 1 : 0;
}

}  // namespace

extern "C" int mapa_confidence_mask(const float* conf, const uint8_t* mask_in, uint8_t* mask_out, int n, int64_t HW,
                                    float q, hipStream_t stream) {
  MAPA_CHECK_ARG(conf && mask_in && mask_out && n > 0 && HW > 0 && q >= 0.f && q <= 1.f,
                 "mapa_confidence_mask: bad args");
  hipLaunchKernelGGL(confidence_mask_kernel, dim3(n), dim3(1024), 0, stream, conf, mask_in, mask_out, HW, q);
  MAPA_CHECK_LAUNCH("mapa_confidence_mask");
  return 0;
}

extern "C" int mapa_apply_mask(float* pts3d, float* pts3d_cam, float* depth_along_ray, const uint8_t* mask,
                               int64_t npix, hipStream_t stream) {
  MAPA_CHECK_ARG(pts3d && pts3d_cam && depth_along_ray && mask && npix > 0, "mapa_apply_mask: bad args");
  int64_t g = (npix + 255) / 256;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(apply_mask_kernel, dim3((unsigned)g), dim3(256), 0, stream, pts3d, pts3d_cam, depth_along_ray,
                     mask, npix);
  MAPA_CHECK_LAUNCH("mapa_apply_mask");
  return 0;
}

// mask_in: non-ambiguous (& confidence) mask u8 [n][H][W]; pts3d [n][H][W][3]; depth_z = pts3d_cam (z at +2,
// stride 3); scratch carved from `work`: normals (12 B/pixel), normal mask and edge state (1 B/pixel each).
extern "C" int mapa_postprocess_mask(const float* pts3d, const float* pts3d_cam, const uint8_t* mask_in,
                                     uint8_t* mask_out, int n, int H, int W, float normal_cos_thr, float depth_rtol,
                                     int use_edges, void* work, hipStream_t stream) {
  MAPA_CHECK_ARG(pts3d && pts3d_cam && mask_in && mask_out && n > 0 && H > 0 && W > 0,
                 "mapa_postprocess_mask: bad args");
  MAPA_CHECK_ARG(!use_edges || work, "mapa_postprocess_mask: edges need a work buffer");
  const int64_t P = (int64_t)n * H * W;
  MAPA_CHECK_ARG(P < (1LL << 31), "mapa_postprocess_mask: more than 2^31 pixels in one call");
  float* nrm = reinterpret_cast<float*>(work);
  uint8_t* nmask = reinterpret_cast<uint8_t*>(nrm + P * 3);
  uint8_t* state = nmask + P;
  if (use_edges) {
    hipLaunchKernelGGL(normals_kernel, dim3(grid_for(P)), dim3(256), 0, stream, pts3d, mask_in, n, H, W, nrm, nmask);
    hipLaunchKernelGGL(normal_state_kernel, dim3(grid_for(P)), dim3(256), 0, stream, nrm, nmask, n, H, W,
                       normal_cos_thr, state);
  }
  hipLaunchKernelGGL(mask_combine_kernel, dim3(grid_for(P)), dim3(256), 0, stream, state, pts3d_cam + 2, (int64_t)3,
                     mask_in, n, H, W, depth_rtol, use_edges, mask_out);
  MAPA_CHECK_LAUNCH("mapa_postprocess_mask");
  return 0;
}

// Host: the float32 boundary of normals_edge's "arccos(d) > deg2rad(tol)" (numpy compares the float32 arccos with
// the float64 threshold): the smallest float32 c with arccos(d) > tol <=> d < c for every float32 d in [-1, 1].
// arccos is taken in double and rounded to float32 (numpy's float32 arccos is within an ulp of that; near any
// threshold adjacent float32 inputs are ~90 ulps of angle apart).  Bisection over the ordered float32 bit patterns.
static inline int32_t f32_order(float f) {
  int32_t i;
  memcpy(&i, &f, 4);
  return i < 0 ? (int32_t)(0x80000000u - (uint32_t)i) : i;
}
static inline float f32_unorder(int32_t k) {
  const int32_t i = k < 0 ? (int32_t)(0x80000000u - (uint32_t)k) : k;
  float f;
  memcpy(&f, &i, 4);
  return f;
}
extern "C" float mapa_normal_cos_threshold(double tol_deg) {
  const double tol = tol_deg * (3.141592653589793 / 180.0);
  auto is_edge = [&](float d) { return (double)(float)acos((double)d) > tol; };
  if (!is_edge(-1.f)) return -1.f;                      // nothing exceeds tol
  if (is_edge(1.f)) return 2.f;                         // everything (also the masked-out 0) exceeds it
  int32_t lo = f32_order(-1.f), hi = f32_order(1.f);    // is_edge(lo) true, is_edge(hi) false
  while (hi - lo > 1) {
    const int32_t mid = lo + (hi - lo) / 2;
    if (is_edge(f32_unorder(mid))) lo = mid; else hi = mid;
  }
  return f32_unorder(hi);
}

extern "C" int mapa_recover_intrinsics(const float* rays, int n, int H, int W, float* K, hipStream_t stream) {
  MAPA_CHECK_ARG(rays && K && n > 0 && H > 0 && W > 0 && (int64_t)H * W <= 1000000,
                 "mapa_recover_intrinsics: bad args (high-res geometric branch not implemented)");
  hipLaunchKernelGGL(recover_intrinsics_kernel, dim3(n), dim3(256), 0, stream, rays, H, W, K);
  MAPA_CHECK_LAUNCH("mapa_recover_intrinsics");
  return 0;
}

extern "C" int mapa_denorm_image(const float* img, int n, int H, int W, const float* mean, const float* stdv,
                                 float* out, hipStream_t stream) {
  MAPA_CHECK_ARG(img && mean && stdv && out, "mapa_denorm_image: bad args");
  hipLaunchKernelGGL(denorm_image_kernel, dim3(grid_for((int64_t)n * H * W)), dim3(256), 0, stream, img, n, H, W,
                     mean, stdv, out);
  MAPA_CHECK_LAUNCH("mapa_denorm_image");
  return 0;
}
