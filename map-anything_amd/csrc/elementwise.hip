// Memory-bound layout / elementwise kernels of the MapAnything hot path (gfx950).
// Each is HBM-bound; loads/stores are 16-B vectorised where the layout allows.
#include "mapa_common.h"

namespace {

constexpr int TPB = 256;

inline int grid_for(int64_t n, int per_block = TPB) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g > 65536) g = 65536;
  return (int)(g < 1 ? 1 : g);
}

// ---------------------------------------------------------------------------------------------- patchify
// PatchEmbed (vision_transformer.py:244-249, Conv2d 3->1024 k14 s14) as im2col rows for the GEMM.
template <typename T>
__global__ void patchify_kernel(const float* __restrict__ img, int n, int H, int W, T* __restrict__ out, int kpad,
                                int f16) {
  const int hp = H / 14, wp = W / 14;
  const int64_t total = (int64_t)n * hp * wp * kpad;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % kpad);
    const int64_t row = e / kpad;
    float v = 0.f;
    if (k < 588) {
      const int px = (int)(row % wp);
      const int64_t r2 = row / wp;
      const int py = (int)(r2 % hp);
      const int im = (int)(r2 / hp);
      const int c = k / 196, rem = k - c * 196, ky = rem / 14, kx = rem - ky * 14;
      v = img[(((int64_t)im * 3 + c) * H + py * 14 + ky) * W + px * 14 + kx];
    }
    if constexpr (sizeof(T) == 2) out[e] = f32_to_lp(f16, v);
    else out[e] = v;
  }
}

// ------------------------------------------------------------------------------------- token assembly
__global__ void assemble_tokens_kernel(const float* __restrict__ patch, const float* __restrict__ cls,
                                       const float* __restrict__ pos, int n, int T, int dim, float* __restrict__ x) {
  const int d4 = dim / 4;
  const int64_t total = (int64_t)n * (T + 1) * d4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % d4) * 4;
    const int64_t r = e / d4;
    const int t = (int)(r % (T + 1));
    const int im = (int)(r / (T + 1));
    f32x4 base = t == 0 ? *reinterpret_cast<const f32x4*>(cls + c)
                        : *reinterpret_cast<const f32x4*>(patch + ((int64_t)im * T + t - 1) * dim + c);
    base += *reinterpret_cast<const f32x4*>(pos + (int64_t)t * dim + c);
    *reinterpret_cast<f32x4*>(x + r * dim + c) = base;
  }
}

__global__ void add_rowvec_kernel(float* __restrict__ x, int64_t ldx, int r0, int r1, int dim,
                                  const float* __restrict__ vec) {
  const int64_t total = (int64_t)(r1 - r0) * dim;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % dim);
    const int64_t r = r0 + e / dim;
    x[r * ldx + c] += vec[c];
  }
}

// -------------------------------------------------------------------------- bilinear, align_corners=True
template <typename T>
__device__ __forceinline__ f32x4 load4(const T* p) {
  if constexpr (sizeof(T) == 2) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return f32x4{bf16_to_f32(u.x & 0xffff), bf16_to_f32(u.x >> 16), bf16_to_f32(u.y & 0xffff), bf16_to_f32(u.y >> 16)};
  } else {
    return *reinterpret_cast<const f32x4*>(p);
  }
}
template <typename T>
__device__ __forceinline__ void load8(const T* p, f32x4& lo, f32x4& hi) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    lo = f32x4{bf16_to_f32(u.x & 0xffff), bf16_to_f32(u.x >> 16), bf16_to_f32(u.y & 0xffff), bf16_to_f32(u.y >> 16)};
    hi = f32x4{bf16_to_f32(u.z & 0xffff), bf16_to_f32(u.z >> 16), bf16_to_f32(u.w & 0xffff), bf16_to_f32(u.w >> 16)};
  } else {
    lo = *reinterpret_cast<const f32x4*>(p);
    hi = *reinterpret_cast<const f32x4*>(p + 4);
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* p, f32x4 lo, f32x4 hi) {
  if constexpr (sizeof(T) == 2) {
    uint4 u;
    u.x = pack_bf16x2(lo[0], lo[1]);
    u.y = pack_bf16x2(lo[2], lo[3]);
    u.z = pack_bf16x2(hi[0], hi[1]);
    u.w = pack_bf16x2(hi[2], hi[3]);
    *reinterpret_cast<uint4*>(p) = u;
  } else {
    *reinterpret_cast<f32x4*>(p) = lo;
    *reinterpret_cast<f32x4*>(p + 4) = hi;
  }
}
template <typename T>
__device__ __forceinline__ void store4(T* p, f32x4 v) {
  if constexpr (sizeof(T) == 2) {
    uint2 u;
    u.x = pack_bf16x2(v[0], v[1]);
    u.y = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = u;
  } else {
    *reinterpret_cast<f32x4*>(p) = v;
  }
}

// F.interpolate(mode="bilinear", align_corners=True) as ATen computes it (scale = (in-1)/(out-1) in fp32,
// h1 = h0 + (h0 < in-1), lambdas 1-l / l), NHWC, 4 channels per thread.
// One thread = 8 channels of one output pixel (16-B bf16 accesses); consecutive threads walk the channels of a
// pixel, so a wave reads each of the 4 source taps and writes the output as contiguous row segments.  Grid: x over
// one output row's (pixel, channel-group) pairs, y over output rows (strided past 65535 rows), so the row's source
// rows and weights are block-uniform and a thread splits its index with one shift (c8 a power of two) — the
// grid-stride form spent more on 64-bit index division than on its memory traffic.
// BIL_ROWS: output rows per thread (8 for the x2 upsamples: 74 -> 148 60.3 -> 42.3 us, 148 -> 296 split 222 -> 161;
// 4 for 296 -> 518: 339 -> 254, 264 with 8; kbench 'bil', 8 views, interleaved against the one-row kernel)
// S3: split operand rows [hi | lo] (2C wide): 1 = bf16 (MAPA_BF16X3), 2 = binary16 (MAPA_F16X2; range faults -> fault);
// 3 = plain binary16 rows (MAPA_F16, the TF32-equivalent heads' operand; range faults -> fault)
template <typename TI, typename TO, int S3 = 0, int BIL_ROWS = 4>
__global__ void bilinear_ac_kernel(const TI* __restrict__ in, int n, int IH, int IW, int C, int OHf, int OWf, int OH,
                                   int OW, int c8_shift, TO* __restrict__ out, unsigned* fault) {
  const int c8 = C / 8;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= OW * c8) return;
  const int ox = c8_shift >= 0 ? idx >> c8_shift : idx / c8;
  const int c = (idx - ox * c8) * 8;
  const float sh = OHf > 1 ? (float)(IH - 1) / (float)(OHf - 1) : 0.f;
  const float sw = OWf > 1 ? (float)(IW - 1) / (float)(OWf - 1) : 0.f;
  const float fx = sw * ox;
  const int x0 = (int)fx;
  const int x1 = x0 + (x0 < IW - 1 ? 1 : 0);
  const float lx1 = fx - x0, lx0 = 1.f - lx1;
  // blockIdx.y walks groups of BIL_ROWS output rows: each row re-uses the previous row's source rows when they
  // coincide (align_corners upsampling: rows oy and oy+1 share y0, or the previous row's y1 is this row's y0), so
  // the 296 -> 518 resize loads ~1.2 instead of 2 source rows per output row through L2
  const int rows = n * OH;
  for (int r = BIL_ROWS * blockIdx.y; r < rows; r += BIL_ROWS * gridDim.y) {
    f32x4 a0, a1, b0, b1, c0, c1, d0, d1;  // taps (y0, x0), (y0, x1), (y1, x0), (y1, x1) of the current row
    int pim = -1, py0 = -1, py1 = -1;
#pragma unroll
    for (int h = 0; h < BIL_ROWS; ++h) {
      const int rr = r + h;
      if (rr >= rows) break;
      const int im = rr / OH, oy = rr - im * OH;
      const float fy = sh * oy;
      const int y0 = (int)fy;
      const int y1 = y0 + (y0 < IH - 1 ? 1 : 0);
      const float ly1 = fy - y0, ly0 = 1.f - ly1;
      const TI* base = in + (size_t)im * IH * IW * C + c;
      const size_t o00 = ((size_t)y0 * IW + x0) * C, o01 = ((size_t)y0 * IW + x1) * C;
      const size_t o10 = ((size_t)y1 * IW + x0) * C, o11 = ((size_t)y1 * IW + x1) * C;
      if (im == pim && y0 == py0 && y1 == py1) {
        // same source rows as the previous row
      } else if (im == pim && y0 == py1) {
        a0 = c0; a1 = c1; b0 = d0; b1 = d1;  // the previous row's bottom taps are this row's top taps
        load8(base + o10, c0, c1);
        load8(base + o11, d0, d1);
      } else {
        load8(base + o00, a0, a1);
        load8(base + o01, b0, b1);
        load8(base + o10, c0, c1);
        load8(base + o11, d0, d1);
      }
      pim = im; py0 = y0; py1 = y1;
      TO* op = out + ((size_t)rr * OW + ox) * (S3 == 1 || S3 == 2 ? 2 * C : C) + c;
      const f32x4 r0 = ly0 * (lx0 * a0 + lx1 * b0) + ly1 * (lx0 * c0 + lx1 * d0);
      const f32x4 r1 = ly0 * (lx0 * a1 + lx1 * b1) + ly1 * (lx0 * c1 + lx1 * d1);
      if constexpr (S3 != 0) {  // 8 channels: one 16-B store of hi and one of lo
        uint4 hv, lv;
        uint32_t* hp = &hv.x;
        uint32_t* lp = &lv.x;
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v0 = k < 2 ? r0[2 * k] : r1[2 * k - 4], v1 = k < 2 ? r0[2 * k + 1] : r1[2 * k - 3];
          if constexpr (S3 >= 2) {
            uint32_t h0, l0, h1, l1;
            ok &= split_f16(v0, h0, l0);
            ok &= split_f16(v1, h1, l1);
            hp[k] = h0 | (h1 << 16);
            lp[k] = l0 | (l1 << 16);
          } else {
            const bf16_t h0 = f32_to_bf16(v0), h1 = f32_to_bf16(v1);
            hp[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
            lp[k] = pack_bf16x2(v0 - bf16_to_f32(h0), v1 - bf16_to_f32(h1));
          }
        }
        if constexpr (S3 >= 2) f16_range_fault(fault, !ok);
        if constexpr (S3 == 3) {  // the hi words are the plain binary16 rows
          typedef uint32_t nt3 __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(nt3{hv.x, hv.y, hv.z, hv.w}, reinterpret_cast<nt3*>(op));
          continue;
        }
        typedef uint32_t nt4 __attribute__((ext_vector_type(4)));
        // 1.1 GB at 518^2: streamed past the caches
        __builtin_nontemporal_store(nt4{hv.x, hv.y, hv.z, hv.w}, reinterpret_cast<nt4*>(op));
        __builtin_nontemporal_store(nt4{lv.x, lv.y, lv.z, lv.w}, reinterpret_cast<nt4*>(op + C));
      } else {
        store8(op, r0, r1);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ mean over T
// Two deterministic passes: partial sums over token chunks (coalesced rows), then the chunk sum in fixed order.
constexpr int MEAN_CHUNKS = 32;
__global__ void mean_tokens_partial_kernel(const float* __restrict__ x, int n, int T, int C,
                                           float* __restrict__ part) {
  const int cblk = blockIdx.x, chunk = blockIdx.y, im = blockIdx.z;
  const int c = cblk * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int t0 = (int)((int64_t)T * chunk / MEAN_CHUNKS), t1 = (int)((int64_t)T * (chunk + 1) / MEAN_CHUNKS);
  const float* p = x + (int64_t)im * T * C + c;
  float s = 0.f;
  for (int t = t0; t < t1; ++t) s += p[(int64_t)t * C];
  part[((int64_t)im * MEAN_CHUNKS + chunk) * C + c] = s;
}

__global__ void mean_tokens_final_kernel(const float* __restrict__ part, int n, int T, int C, float* __restrict__ y) {
  const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (e >= (int64_t)n * C) return;
  const int c = (int)(e % C), im = (int)(e / C);
  float s = 0.f;
  for (int k = 0; k < MEAN_CHUNKS; ++k) s += part[((int64_t)im * MEAN_CHUNKS + k) * C + c];
  y[e] = s / (float)T;
}

// -------------------------------------------------------------------------------------- small linear
__global__ void linear_small_kernel(const float* __restrict__ x, int M, int K, const float* __restrict__ w,
                                    const float* __restrict__ b, int N, int act, float* __restrict__ y) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= M * N) return;
  const int m = wave / N, n = wave % N;
  const float* xr = x + (int64_t)m * K;
  const float* wr = w + (int64_t)n * K;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += xr[k] * wr[k];
  s = wave_sum(s);
  if (lane == 0) {
    float v = s + (b ? b[n] : 0.f);
    if (act == MAPA_ACT_RELU) v = fmaxf(v, 0.f);
    else if (act == MAPA_ACT_GELU) v = gelu_erf(v);
    y[(int64_t)m * N + n] = v;
  }
}

// --------------------------------------------------------------------- pose / scale adaptors (per view)
// pose_out[v] = { cam_trans*s (3), quat (4), R row-major (9), t (3) } (19 floats); poses44[v] = 4x4 with
// [:3,:3] = R(q), [:3,3] = cam_trans*s (inference.py:376-390); scale_out[b] = clip(exp(raw), 1e-8).
__global__ void pose_scale_finalize_kernel(const float* __restrict__ pose_raw, const float* __restrict__ scale_raw,
                                           int nviews, int batch, float* __restrict__ pose_out,
                                           float* __restrict__ scale_out, float* __restrict__ poses44) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v < batch) scale_out[v] = fmaxf(expf(scale_raw[v]), 1e-8f);
  if (v >= nviews) return;
  const float s = fmaxf(expf(scale_raw[v % batch]), 1e-8f);
  const float* pr = pose_raw + v * 7;
  float q[4] = {pr[3], pr[4], pr[5], pr[6]};
  float nq = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  nq = fmaxf(nq, 1e-8f);
  for (int i = 0; i < 4; ++i) q[i] /= nq;
  // quaternion_to_rotation_matrix normalises again (geometry.py:619)
  const float n2 = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const float x = q[0] / n2, y = q[1] / n2, z = q[2] / n2, w = q[3] / n2;
  const float R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                      2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                      2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)};
  float* po = pose_out + v * 19;
  for (int i = 0; i < 3; ++i) po[i] = pr[i] * s;
  for (int i = 0; i < 4; ++i) po[3 + i] = q[i];
  for (int i = 0; i < 9; ++i) po[7 + i] = R[i];
  for (int i = 0; i < 3; ++i) po[16 + i] = pr[i];
  if (poses44) {
    float* P = poses44 + v * 16;
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) P[r * 4 + c] = R[r * 3 + c];
      P[r * 4 + 3] = pr[r] * s;
    }
    P[12] = 0.f; P[13] = 0.f; P[14] = 0.f; P[15] = 1.f;
  }
}

// ---------------------------------------------------------------------------- dense head tail (fused)
template <typename T>
__global__ void __launch_bounds__(256) dense_head_out_kernel(
    const T* __restrict__ hidden, int n, int HW, const float* __restrict__ w6, const float* __restrict__ b6,
    const float* __restrict__ pose_out, const float* __restrict__ scale, int batch, float* __restrict__ pts3d,
    float* __restrict__ pts3d_cam, float* __restrict__ rays, float* __restrict__ depth, float* __restrict__ conf,
    float* __restrict__ logits, uint8_t* __restrict__ mask) {
  __shared__ float sw[6 * 128 + 6];
  for (int i = threadIdx.x; i < 6 * 128; i += blockDim.x) sw[i] = w6[i];
  if (threadIdx.x < 6) sw[768 + threadIdx.x] = b6[threadIdx.x];
  __syncthreads();
  const int64_t total = (int64_t)n * HW;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const T* h = hidden + p * 128;
    float acc[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) acc[c] = sw[768 + c];
#pragma unroll 4
    for (int k = 0; k < 128; k += 4) {
      const f32x4 hv = load4(h + k);
#pragma unroll
      for (int c = 0; c < 6; ++c)
        acc[c] += hv[0] * sw[c * 128 + k] + hv[1] * sw[c * 128 + k + 1] + hv[2] * sw[c * 128 + k + 2] +
                  hv[3] * sw[c * 128 + k + 3];
    }
    const int v = (int)(p / HW);
    const float sc = scale[v % batch];  // rows are view-major: v = view * batch + b
    dense_head_pixel(acc, pose_out + v * 19, sc, p, pts3d, pts3d_cam, rays, depth, conf, logits, mask);
  }
}

// Dense adaptor alone (module-level API): raw conv1x1 rows [n][HW][6] -> NCHW planes value [n][4][HW] (unit ray,
// exp depth), conf [n][HW] = 1 + exp, logits [n][HW], mask [n][HW] = sigmoid (the probability, as MaskAdaptor).
__global__ void __launch_bounds__(256) dense_adaptor_kernel(const float* __restrict__ raw, int n, int64_t HW,
                                                            float* __restrict__ value, float* __restrict__ conf,
                                                            float* __restrict__ logits, float* __restrict__ mask) {
  const int64_t total = (int64_t)n * HW;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += (int64_t)gridDim.x * blockDim.x) {
    const float* r = raw + p * 6;
    const int64_t v = p / HW, i = p - v * HW;
    const float rx = r[0], ry = r[1], rz = r[2];
    const float nr = fmaxf(sqrtf(rx * rx + ry * ry + rz * rz), 1e-8f);
    float* val = value + v * 4 * HW + i;
    val[0] = rx / nr;
    val[HW] = ry / nr;
    val[2 * HW] = rz / nr;
    val[3 * HW] = expf(r[3]);
    conf[p] = 1.f + expf(r[4]);
    logits[p] = r[5];
    mask[p] = 1.f / (1.f + expf(-r[5]));
  }
}

// ToTensor + Normalize (torchvision, image.py:270-275): out[v][c][y][x] = (u8 / 255 - mean_c) / std_c, the same
// two IEEE float32 operations in the same order (bit-identical to torch on the CPU).
__global__ void __launch_bounds__(256) normalize_image_kernel(const uint8_t* __restrict__ hwc, int64_t npix,
                                                              int64_t HW, float m0, float m1, float m2, float s0,
                                                              float s1, float s2, float* __restrict__ out) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = p / HW, i = p - v * HW;
    const uint8_t* px = hwc + p * 3;
    float* o = out + v * 3 * HW + i;
    o[0] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)px[0], 255.f), m0), s0);
    o[HW] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)px[1], 255.f), m1), s1);
    o[2 * HW] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)px[2], 255.f), m2), s2);
  }
}

__global__ void convert_rows_kernel(const float* __restrict__ src, int64_t lds, int rows, int cols, void* dst,
                                    int bf, int64_t ldd, unsigned* fault) {
  const int64_t total = (int64_t)rows * cols;
  bool ok = true;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % cols);
    const int64_t r = e / cols;
    const float v = src[r * lds + c];
    if (bf == 2) ok &= f16_ok(v);
    if (bf) reinterpret_cast<bf16_t*>(dst)[r * ldd + c] = f32_to_lp(bf == 2, v);  // 1 bf16, 2 fp16
    else reinterpret_cast<float*>(dst)[r * ldd + c] = v;
  }
  f16_range_fault(fault, !ok);
}

// fp32 rows -> [hi | lo] bf16 column blocks of width cp (zero-padded past cols), hi = bf16(x), lo = bf16(x - hi):
// read by a bf16 GEMM as the logical K blocks [hi | hi | lo] (mapa_gemm_desc.a_split) against weights packed
// [hi | lo | hi], it accumulates x_hi*w_hi + x_hi*w_lo + x_lo*w_hi (the split form of an fp32 product, ~2^-16).
// f16: the TF32-equivalent form instead (MAPA_F16X2: hi = f16(x), lo = f16(x - hi), read as a plain 2C-wide f16
// operand against weights [w | w]); values outside binary16's range set MAPA_FAULT_F16_RANGE.
__global__ void split_bf16x3_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int cols, int cp,
                                    bf16_t* __restrict__ y, int f16, unsigned* fault) {
  const int g4 = cp / 4;
  const int64_t total = rows * g4;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / g4;
    const int c = (int)(e - r * g4) * 4;
    const f32x4 v = c < cols ? *reinterpret_cast<const f32x4*>(x + r * ldx + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (f16) store_split2h(y + r * 2 * cp + c, cp, v, fault);
    else store_split3(y + r * 2 * cp + c, cp, v);
  }
}

__global__ void fill_splitmix_kernel(float* __restrict__ out, int64_t n, uint64_t seed, float half, float mid) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    const float u = (float)(uint32_t)(x >> 40) * 5.9604644775390625e-08f;  // 2^-24, exact
    const float t = __fsub_rn(__fmul_rn(u, 2.0f), 1.0f);
    out[i] = __fadd_rn(__fmul_rn(t, half), mid);
  }
}

}  // namespace

extern "C" int mapa_patchify(const float* img, int n, int H, int W, void* out, int dtype, int kpad,
                             hipStream_t stream) {
  MAPA_CHECK_ARG(img && out && n > 0 && H % 14 == 0 && W % 14 == 0 && kpad >= 588, "mapa_patchify: bad args");
  const int64_t total = (int64_t)n * (H / 14) * (W / 14) * kpad;
  MAPA_CHECK_ARG(dtype == MAPA_BF16 || dtype == MAPA_F16 || dtype == MAPA_F32, "mapa_patchify: bad dtype");
  if (dtype != MAPA_F32)
    hipLaunchKernelGGL(patchify_kernel<bf16_t>, dim3(grid_for(total)), dim3(TPB), 0, stream, img, n, H, W,
                       reinterpret_cast<bf16_t*>(out), kpad, dtype == MAPA_F16 ? 1 : 0);
  else
    hipLaunchKernelGGL(patchify_kernel<float>, dim3(grid_for(total)), dim3(TPB), 0, stream, img, n, H, W,
                       reinterpret_cast<float*>(out), kpad, 0);
  MAPA_CHECK_LAUNCH("mapa_patchify");
  return 0;
}

extern "C" int mapa_assemble_tokens(const float* patch, const float* cls, const float* pos, int n, int T, int dim,
                                    float* x, hipStream_t stream) {
  MAPA_CHECK_ARG(patch && cls && pos && x && dim % 4 == 0, "mapa_assemble_tokens: bad args");
  const int64_t total = (int64_t)n * (T + 1) * (dim / 4);
  hipLaunchKernelGGL(assemble_tokens_kernel, dim3(grid_for(total)), dim3(TPB), 0, stream, patch, cls, pos, n, T, dim,
                     x);
  MAPA_CHECK_LAUNCH("mapa_assemble_tokens");
  return 0;
}

extern "C" int mapa_add_rowvec(float* x, int64_t ldx, int r0, int r1, int dim, const float* vec, hipStream_t stream) {
  MAPA_CHECK_ARG(x && vec && r1 >= r0, "mapa_add_rowvec: bad args");
  if (r1 == r0) return 0;
  hipLaunchKernelGGL(add_rowvec_kernel, dim3(grid_for((int64_t)(r1 - r0) * dim)), dim3(TPB), 0, stream, x, ldx, r0,
                     r1, dim, vec);
  MAPA_CHECK_LAUNCH("mapa_add_rowvec");
  return 0;
}

template <int RW>
static void bilinear_launch(const void* in, int in_dtype, int n, int IH, int IW, int C, int OHf, int OWf, int OH, int OW,
                            int c8_shift, void* out, int out_dtype, hipStream_t stream) {
  const int64_t groups = ((int64_t)n * OH + RW - 1) / RW;
  const dim3 g((unsigned)((OW * (C / 8) + TPB - 1) / TPB), (unsigned)std::min<int64_t>(groups, 65535)), b(TPB);
  unsigned* fault = mapa_gemm_impl::fault_word();
#define MAPA_BIL(TI, TO, S)                                                                                          \
  hipLaunchKernelGGL((bilinear_ac_kernel<TI, TO, S, RW>), g, b, 0, stream, (const TI*)in, n, IH, IW, C, OHf, OWf, OH, \
                     OW, c8_shift, (TO*)out, fault)
  if (out_dtype == MAPA_F16X2 && in_dtype == MAPA_F32) MAPA_BIL(float, bf16_t, 2);
  else if (out_dtype == MAPA_F16 && in_dtype == MAPA_F32) MAPA_BIL(float, bf16_t, 3);
  else if (out_dtype == MAPA_BF16X3 && in_dtype == MAPA_F32) MAPA_BIL(float, bf16_t, 1);
  else if (out_dtype == MAPA_BF16X3) MAPA_BIL(bf16_t, bf16_t, 1);
  else if (in_dtype == MAPA_BF16 && out_dtype == MAPA_BF16) MAPA_BIL(bf16_t, bf16_t, 0);
  else if (in_dtype == MAPA_F32 && out_dtype == MAPA_BF16) MAPA_BIL(float, bf16_t, 0);
  else if (in_dtype == MAPA_BF16 && out_dtype == MAPA_F32) MAPA_BIL(bf16_t, float, 0);
  else MAPA_BIL(float, float, 0);
#undef MAPA_BIL
}

extern "C" int mapa_bilinear_ac(const void* in, int in_dtype, int n, int IH, int IW, int C, int OHf, int OWf, int OH,
                                int OW, void* out, int out_dtype, hipStream_t stream) {
  MAPA_CHECK_ARG(in && out && C % 8 == 0 && OH <= OHf && OW <= OWf, "mapa_bilinear_ac: bad args (C %% 8 == 0)");
  const int c8 = C / 8, c8_shift = (c8 & (c8 - 1)) == 0 ? __builtin_ctz(c8) : -1;
  MAPA_CHECK_ARG((int64_t)OW * c8 < (1LL << 31) && (int64_t)n * OH + 8 * 65536 < (1LL << 31),
                 "mapa_bilinear_ac: too large");
  MAPA_CHECK_ARG((in_dtype == MAPA_F32 || in_dtype == MAPA_BF16) &&
                     (out_dtype == MAPA_F32 || out_dtype == MAPA_BF16 || out_dtype == MAPA_BF16X3 ||
                      ((out_dtype == MAPA_F16X2 || out_dtype == MAPA_F16) && in_dtype == MAPA_F32)),
                 "mapa_bilinear_ac: bad dtypes");
  if (OH >= 2 * IH - 1)
    bilinear_launch<8>(in, in_dtype, n, IH, IW, C, OHf, OWf, OH, OW, c8_shift, out, out_dtype, stream);
  else
    bilinear_launch<4>(in, in_dtype, n, IH, IW, C, OHf, OWf, OH, OW, c8_shift, out, out_dtype, stream);
  MAPA_CHECK_LAUNCH("mapa_bilinear_ac");
  return 0;
}

extern "C" int mapa_mean_tokens(const float* x, int n, int tokens, int C, float* y, void* work, hipStream_t stream) {
  MAPA_CHECK_ARG(x && y && work && n > 0 && tokens > 0 && C > 0, "mapa_mean_tokens: bad args");
  float* part = reinterpret_cast<float*>(work);
  hipLaunchKernelGGL(mean_tokens_partial_kernel, dim3((C + 255) / 256, MEAN_CHUNKS, n), dim3(256), 0, stream, x, n,
                     tokens, C, part);
  hipLaunchKernelGGL(mean_tokens_final_kernel, dim3((unsigned)(((int64_t)n * C + 255) / 256)), dim3(256), 0, stream,
                     part, n, tokens, C, y);
  MAPA_CHECK_LAUNCH("mapa_mean_tokens");
  return 0;
}

extern "C" int mapa_linear_small(const float* x, int M, int K, const float* w, const float* b, int N, int act,
                                 float* y, hipStream_t stream) {
  MAPA_CHECK_ARG(x && w && y && M > 0 && N > 0 && K > 0, "mapa_linear_small: bad args");
  const int64_t waves = (int64_t)M * N;
  hipLaunchKernelGGL(linear_small_kernel, dim3((unsigned)((waves * 64 + TPB - 1) / TPB)), dim3(TPB), 0, stream, x, M,
                     K, w, b, N, act, y);
  MAPA_CHECK_LAUNCH("mapa_linear_small");
  return 0;
}

extern "C" int mapa_pose_scale_finalize(const float* pose_raw, const float* scale_raw, int nviews, int batch,
                                        float* pose_out, float* scale_out, float* poses44, hipStream_t stream) {
  MAPA_CHECK_ARG(pose_raw && scale_raw && pose_out && scale_out && nviews > 0 && batch > 0,
                 "mapa_pose_scale_finalize: bad args");
  const int m = nviews > batch ? nviews : batch;
  hipLaunchKernelGGL(pose_scale_finalize_kernel, dim3((m + 63) / 64), dim3(64), 0, stream, pose_raw, scale_raw,
                     nviews, batch, pose_out, scale_out, poses44);
  MAPA_CHECK_LAUNCH("mapa_pose_scale_finalize");
  return 0;
}

extern "C" int mapa_dense_head_out(const void* hidden, int dtype, int n, int HW, const float* w6, const float* b6,
                                   const float* pose_out, const float* scale, int batch, float* pts3d,
                                   float* pts3d_cam, float* rays, float* depth, float* conf, float* logits,
                                   uint8_t* mask, hipStream_t stream) {
  MAPA_CHECK_ARG(hidden && w6 && b6 && pose_out && scale && pts3d && pts3d_cam && rays && depth && conf && logits &&
                     mask && n > 0 && HW > 0 && batch > 0 && n % batch == 0,
                 "mapa_dense_head_out: bad args");
  const int64_t total = (int64_t)n * HW;
  const dim3 g(grid_for(total)), b(TPB);
  if (dtype == MAPA_BF16)
    hipLaunchKernelGGL(dense_head_out_kernel<bf16_t>, g, b, 0, stream, (const bf16_t*)hidden, n, HW, w6, b6, pose_out,
                       scale, batch, pts3d, pts3d_cam, rays, depth, conf, logits, mask);
  else
    hipLaunchKernelGGL(dense_head_out_kernel<float>, g, b, 0, stream, (const float*)hidden, n, HW, w6, b6, pose_out,
                       scale, batch, pts3d, pts3d_cam, rays, depth, conf, logits, mask);
  MAPA_CHECK_LAUNCH("mapa_dense_head_out");
  return 0;
}

extern "C" int mapa_dense_adaptor(const float* raw, int n, int64_t HW, float* value, float* conf, float* logits,
                                  float* mask, hipStream_t stream) {
  MAPA_CHECK_ARG(raw && value && conf && logits && mask && n > 0 && HW > 0, "mapa_dense_adaptor: bad args");
  const int64_t total = (int64_t)n * HW;
  hipLaunchKernelGGL(dense_adaptor_kernel, dim3(grid_for(total)), dim3(TPB), 0, stream, raw, n, HW, value, conf,
                     logits, mask);
  MAPA_CHECK_LAUNCH("mapa_dense_adaptor");
  return 0;
}

extern "C" int mapa_normalize_image(const uint8_t* hwc, int n, int H, int W, const float* mean3, const float* std3,
                                    float* out, hipStream_t stream) {
  MAPA_CHECK_ARG(hwc && out && mean3 && std3 && n > 0 && H > 0 && W > 0, "mapa_normalize_image: bad args");
  MAPA_CHECK_ARG(std3[0] != 0.f && std3[1] != 0.f && std3[2] != 0.f, "mapa_normalize_image: zero std");
  const int64_t HW = (int64_t)H * W, npix = (int64_t)n * HW;
  hipLaunchKernelGGL(normalize_image_kernel, dim3(grid_for(npix)), dim3(TPB), 0, stream, hwc, npix, HW, mean3[0],
                     mean3[1], mean3[2], std3[0], std3[1], std3[2], out);
  MAPA_CHECK_LAUNCH("mapa_normalize_image");
  return 0;
}

extern "C" int mapa_convert_rows(const float* src, int64_t lds, int rows, int cols, void* dst, int dst_dtype,
                                 int64_t ldd, hipStream_t stream) {
  MAPA_CHECK_ARG(src && dst && rows > 0 && cols > 0, "mapa_convert_rows: bad args");
  hipLaunchKernelGGL(convert_rows_kernel, dim3(grid_for((int64_t)rows * cols)), dim3(TPB), 0, stream, src, lds, rows,
                     cols, dst, dst_dtype == MAPA_BF16 ? 1 : dst_dtype == MAPA_F16 ? 2 : 0, ldd,
                     mapa_gemm_impl::fault_word());
  MAPA_CHECK_LAUNCH("mapa_convert_rows");
  return 0;
}

extern "C" int mapa_split_bf16x3(const float* x, int64_t ldx, int64_t rows, int cols, int cols_padded, void* y,
                                 hipStream_t stream) {
  MAPA_CHECK_ARG(x && y && rows > 0 && cols > 0 && cols % 4 == 0 && cols_padded % 8 == 0 && cols_padded >= cols &&
                     ldx >= cols && ldx % 4 == 0,
                 "mapa_split_bf16x3: bad args (cols %% 4, cols_padded %% 8, ldx %% 4)");
  hipLaunchKernelGGL(split_bf16x3_kernel, dim3(grid_for(rows * (cols_padded / 4))), dim3(TPB), 0, stream, x, ldx,
                     rows, cols, cols_padded, (bf16_t*)y, 0, nullptr);
  MAPA_CHECK_LAUNCH("mapa_split_bf16x3");
  return 0;
}

extern "C" int mapa_split_rows(const float* x, int64_t ldx, int64_t rows, int cols, int cols_padded, void* y,
                               int dtype, hipStream_t stream) {
  MAPA_CHECK_ARG(dtype == MAPA_BF16X3 || dtype == MAPA_F16X2, "mapa_split_rows: dtype must be MAPA_BF16X3 or MAPA_F16X2");
  if (dtype == MAPA_BF16X3) return mapa_split_bf16x3(x, ldx, rows, cols, cols_padded, y, stream);
  MAPA_CHECK_ARG(x && y && rows > 0 && cols > 0 && cols % 4 == 0 && cols_padded % 8 == 0 && cols_padded >= cols &&
                     ldx >= cols && ldx % 4 == 0,
                 "mapa_split_rows: bad args (cols %% 4, cols_padded %% 8, ldx %% 4)");
  hipLaunchKernelGGL(split_bf16x3_kernel, dim3(grid_for(rows * (cols_padded / 4))), dim3(TPB), 0, stream, x, ldx,
                     rows, cols, cols_padded, (bf16_t*)y, 1, mapa_gemm_impl::fault_word());
  MAPA_CHECK_LAUNCH("mapa_split_rows");
  return 0;
}

extern "C" int mapa_fill_splitmix(float* out, int64_t n, uint64_t seed, float half, float mid, hipStream_t stream) {
  MAPA_CHECK_ARG(out && n > 0, "mapa_fill_splitmix: bad args");
  hipLaunchKernelGGL(fill_splitmix_kernel, dim3(grid_for(n)), dim3(TPB), 0, stream, out, n, seed, half, mid);
  MAPA_CHECK_LAUNCH("mapa_fill_splitmix");
  return 0;
}
