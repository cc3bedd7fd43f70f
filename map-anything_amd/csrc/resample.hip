// GPU image resize of the input pipeline, bit-exact with PIL's Image.resize for 8-bit RGB,
// fused with the crop and with ToTensor + Normalize.
//
// Replaces the host resampling of the reference's loader: crop_resize_if_necessary -> Image.resize(LANCZOS when
// shrinking, BICUBIC when growing) -> crop -> ToTensor + Normalize (mapanything/utils/image.py:283-303,
// mapanything/utils/cropping.py:188-280 / 385-465).  The reference's resize is Pillow's (third-party, not vendored
// in /root/reference; this image ships Pillow 12.2.0).  Its published algorithm (src/libImaging/Resample.c) is
// restated here:
//   * precompute_coeffs: per output pixel a window [xmin, xmin + count) of the input and float64 filter weights
//     filter((x + xmin - center + 0.5) / filterscale), normalised to sum 1 (center = in0 + (xx + 0.5) * scale,
//     filterscale = max(scale, 1), support = filter support * filterscale);
//   * normalize_coeffs_8bpc: weights -> int32 fixed point with 22 fraction bits (round half away from zero);
//   * two separable passes, horizontal first, over 8-bit channels: acc = 2^21 + sum(u8 * w) in int32,
//     clip8(acc >> 22) (arithmetic shift, clamped to [0, 255]) after EACH pass (the intermediate image is 8-bit);
//   * a pass runs only when its size changes (need_horizontal / need_vertical); the horizontal pass covers only the
//     input rows the vertical windows touch.
// The weights are computed on the HOST (mapa_resize_plan_build: the same float64 operations on the same libm `sin`
// as Pillow's C, so the fixed-point weights are identical), the passes on the GPU: one thread per output pixel,
// integer MACs.  The crop is folded in (only the kept output pixels are computed: a resized pixel depends on its
// own window only) and the vertical pass writes the normalised float32 planes directly
// ((u8 / 255 - mean) / std in torchvision's order, as mapa_normalize_image).
//
// Built with -ffp-contract=off (Makefile): the host weight arithmetic must not be contracted into FMAs.
#include <math.h>
#include <string.h>

#include "mapa_common.h"

namespace {

constexpr int PREC = 22;  // Resample.c PRECISION_BITS = 32 - 8 - 2

// ---- Pillow's filters (Resample.c), float64
double sinc_filter(double x) {
  if (x == 0.0) return 1.0;
  x = x * M_PI;
  return sin(x) / x;
}
double lanczos_filter(double x) { return (-3.0 <= x && x < 3.0) ? sinc_filter(x) * sinc_filter(x / 3) : 0.0; }
double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}
double bilinear_filter(double x) {
  if (x < 0.0) x = -x;
  if (x < 1.0) return 1.0 - x;
  return 0.0;
}

bool filter_of(int filter, double (**f)(double), double* support) {
  switch (filter) {
    case MAPA_RESAMPLE_LANCZOS: *f = lanczos_filter; *support = 3.0; return true;
    case MAPA_RESAMPLE_BILINEAR: *f = bilinear_filter; *support = 1.0; return true;
    case MAPA_RESAMPLE_BICUBIC: *f = bicubic_filter; *support = 2.0; return true;
    default: return false;
  }
}

int ksize_of(int in_size, int out_size, double support) {
  double filterscale = (double)in_size / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  return (int)ceil(support * filterscale) * 2 + 1;
}

// precompute_coeffs + normalize_coeffs_8bpc over the whole input (box = (0, in_size)): bounds[2 * xx] = xmin,
// bounds[2 * xx + 1] = count, kk[xx * ksize + x] = fixed-point weight (zero past count).
void coeffs(int in_size, int out_size, double (*filter)(double), double support_1, int ksize, int32_t* bounds,
            int32_t* kk) {
  const double in0 = 0.0, in1 = in_size;
  double filterscale, scale;
  filterscale = scale = (double)(in1 - in0) / out_size;
  if (filterscale < 1.0) filterscale = 1.0;
  const double support = support_1 * filterscale;
  double k[1024];
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    for (int x = 0; x < xmax; ++x) {
      const double w = filter((x + xmin - center + 0.5) * ss);
      k[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) k[x] /= ww;
    int32_t* o = kk + (int64_t)xx * ksize;
    for (int x = 0; x < ksize; ++x) {
      const double v = x < xmax ? k[x] : 0.0;
      o[x] = v < 0 ? (int32_t)(-0.5 + v * (1 << PREC)) : (int32_t)(0.5 + v * (1 << PREC));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
}

__device__ __forceinline__ int clip8(int acc) {
  const int v = acc >> PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Horizontal pass: tmp[r][x] (RGBX) for input rows row0 + r (r < nrows), output columns crop_left + x (x < out_w).
__global__ void __launch_bounds__(256) resize_h_kernel(const uint8_t* __restrict__ src, int64_t src_ld, int row0,
                                                       int nrows, int out_w, int crop_left, int ksize,
                                                       const int32_t* __restrict__ bounds,
                                                       const int32_t* __restrict__ kk, uchar4* __restrict__ tmp) {
  const int64_t total = (int64_t)nrows * out_w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / out_w), x = (int)(i - (int64_t)r * out_w);
    const int xx = crop_left + x;
    const int xmin = bounds[2 * xx], cnt = bounds[2 * xx + 1];
    const int32_t* k = kk + (int64_t)xx * ksize;
    const uint8_t* p = src + (int64_t)(row0 + r) * src_ld + (int64_t)xmin * 3;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < cnt; ++t) {
      const int w = k[t];
      s0 += (int)p[3 * t] * w;
      s1 += (int)p[3 * t + 1] * w;
      s2 += (int)p[3 * t + 2] * w;
    }
    tmp[i] = make_uchar4((unsigned char)clip8(s0), (unsigned char)clip8(s1), (unsigned char)clip8(s2), 0);
  }
}

// Vertical pass (or the plain crop when the height is unchanged) + ToTensor / Normalize.  `in` holds rows
// row_base.. of the horizontally resampled image (PS = 4, RGBX, columns already cropped: col0 = 0) or of the
// source (PS = 3, col0 = crop_left).
template <int PS>
__global__ void __launch_bounds__(256) resize_v_kernel(const uint8_t* __restrict__ in, int64_t in_ld, int col0,
                                                       int row_base, int out_h, int out_w, int crop_top, int need_v,
                                                       int ksize, const int32_t* __restrict__ bounds,
                                                       const int32_t* __restrict__ kk, float m0, float m1, float m2,
                                                       float d0, float d1, float d2, float* __restrict__ out,
                                                       uint8_t* __restrict__ out_u8) {
  const int64_t HW = (int64_t)out_h * out_w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < HW; i += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(i / out_w), x = (int)(i - (int64_t)y * out_w);
    const int yy = crop_top + y;
    const uint8_t* col = in + (int64_t)(col0 + x) * PS;
    int v0, v1, v2;
    if (need_v) {
      const int ymin = bounds[2 * yy] - row_base, cnt = bounds[2 * yy + 1];
      const int32_t* k = kk + (int64_t)yy * ksize;
      int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
      for (int t = 0; t < cnt; ++t) {
        const uint8_t* p = col + (int64_t)(ymin + t) * in_ld;
        const int w = k[t];
        s0 += (int)p[0] * w;
        s1 += (int)p[1] * w;
        s2 += (int)p[2] * w;
      }
      v0 = clip8(s0);
      v1 = clip8(s1);
      v2 = clip8(s2);
    } else {
      const uint8_t* p = col + (int64_t)(yy - row_base) * in_ld;
      v0 = p[0];
      v1 = p[1];
      v2 = p[2];
    }
    if (out) {
      out[i] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)v0, 255.f), m0), d0);
      out[HW + i] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)v1, 255.f), m1), d1);
      out[2 * HW + i] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)v2, 255.f), m2), d2);
    }
    if (out_u8) {
      out_u8[3 * i] = (uint8_t)v0;
      out_u8[3 * i + 1] = (uint8_t)v1;
      out_u8[3 * i + 2] = (uint8_t)v2;
    }
  }
}

unsigned grid_of(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

int64_t plan_int32s(const mapa_resize_plan& h) {
  return (int64_t)(sizeof(mapa_resize_plan) / 4) + (h.need_h ? 2LL * h.rs_w + (int64_t)h.rs_w * h.kh : 0) +
         (h.need_v ? 2LL * h.rs_h + (int64_t)h.rs_h * h.kv : 0);
}

}  // namespace

extern "C" int64_t mapa_resize_plan_bytes(int in_w, int in_h, int rs_w, int rs_h, int filter) {
  double (*f)(double);
  double support;
  if (in_w <= 0 || in_h <= 0 || rs_w <= 0 || rs_h <= 0 || !filter_of(filter, &f, &support)) {
    mapa_set_error("mapa_resize_plan_bytes: bad sizes or filter %d", filter);
    return -1;
  }
  mapa_resize_plan h = {};
  h.rs_w = rs_w;
  h.rs_h = rs_h;
  h.need_h = rs_w != in_w;
  h.need_v = rs_h != in_h;
  h.kh = h.need_h ? ksize_of(in_w, rs_w, support) : 0;
  h.kv = h.need_v ? ksize_of(in_h, rs_h, support) : 0;
  return 4 * plan_int32s(h);
}

extern "C" int mapa_resize_plan_build(int in_w, int in_h, int rs_w, int rs_h, int crop_left, int crop_top, int out_w,
                                      int out_h, int filter, void* plan, int64_t plan_bytes) {
  double (*f)(double);
  double support;
  MAPA_CHECK_ARG(plan && in_w > 0 && in_h > 0 && rs_w > 0 && rs_h > 0 && out_w > 0 && out_h > 0,
                 "mapa_resize_plan_build: bad sizes");
  MAPA_CHECK_ARG(filter_of(filter, &f, &support), "mapa_resize_plan_build: filter %d (1 LANCZOS, 2 BILINEAR, 3 BICUBIC)",
                 filter);
  MAPA_CHECK_ARG(crop_left >= 0 && crop_top >= 0 && crop_left + out_w <= rs_w && crop_top + out_h <= rs_h,
                 "mapa_resize_plan_build: crop box (%d, %d, %d, %d) outside the %dx%d resized image", crop_left,
                 crop_top, crop_left + out_w, crop_top + out_h, rs_w, rs_h);
  mapa_resize_plan h = {};
  h.in_w = in_w;
  h.in_h = in_h;
  h.rs_w = rs_w;
  h.rs_h = rs_h;
  h.crop_left = crop_left;
  h.crop_top = crop_top;
  h.out_w = out_w;
  h.out_h = out_h;
  h.filter = filter;
  h.need_h = rs_w != in_w;
  h.need_v = rs_h != in_h;
  h.kh = h.need_h ? ksize_of(in_w, rs_w, support) : 0;
  h.kv = h.need_v ? ksize_of(in_h, rs_h, support) : 0;
  MAPA_CHECK_ARG(h.kh <= 1024 && h.kv <= 1024, "mapa_resize_plan_build: downscale factor above 170 (window > 1024)");
  const int64_t n = plan_int32s(h);
  MAPA_CHECK_ARG(plan_bytes >= 4 * n, "mapa_resize_plan_build: plan buffer %lld bytes < %lld", (long long)plan_bytes,
                 (long long)(4 * n));
  int32_t* body = reinterpret_cast<int32_t*>(plan) + sizeof(mapa_resize_plan) / 4;
  int64_t off = sizeof(mapa_resize_plan) / 4;
  if (h.need_h) {
    h.off_hb = (int32_t)off;
    h.off_hk = (int32_t)(off + 2LL * rs_w);
    coeffs(in_w, rs_w, f, support, h.kh, body, body + 2LL * rs_w);
    body += 2LL * rs_w + (int64_t)rs_w * h.kh;
    off += 2LL * rs_w + (int64_t)rs_w * h.kh;
  }
  if (h.need_v) {
    h.off_vb = (int32_t)off;
    h.off_vk = (int32_t)(off + 2LL * rs_h);
    coeffs(in_h, rs_h, f, support, h.kv, body, body + 2LL * rs_h);
    const int32_t* vb = body;
    // input rows the kept output rows read (the horizontal pass computes only these)
    h.row0 = vb[2 * crop_top];
    h.nrows = vb[2 * (crop_top + out_h - 1)] + vb[2 * (crop_top + out_h - 1) + 1] - h.row0;
  } else {
    h.row0 = crop_top;
    h.nrows = out_h;
  }
  h.int32s = (int32_t)n;
  memcpy(plan, &h, sizeof(h));
  return 0;
}

extern "C" int64_t mapa_resize_workspace_bytes(const void* plan_host) {
  if (!plan_host) return 0;
  const mapa_resize_plan& h = *reinterpret_cast<const mapa_resize_plan*>(plan_host);
  return h.need_h ? 4LL * h.nrows * h.out_w : 0;
}

extern "C" int mapa_resize_normalize(const uint8_t* src, int64_t src_row_bytes, const void* plan_host,
                                     const void* plan_dev, const float* mean3, const float* std3, float* out,
                                     uint8_t* out_u8, void* workspace, int64_t workspace_bytes, mapa_stream_t stream) {
  MAPA_CHECK_ARG(src && plan_host && plan_dev && (out || out_u8), "mapa_resize_normalize: null argument");
  const mapa_resize_plan& h = *reinterpret_cast<const mapa_resize_plan*>(plan_host);
  MAPA_CHECK_ARG(h.int32s > 0 && h.in_w > 0 && h.out_w > 0 && src_row_bytes >= 3LL * h.in_w,
                 "mapa_resize_normalize: plan not built or src_row_bytes %lld < 3 * %d", (long long)src_row_bytes,
                 h.in_w);
  MAPA_CHECK_ARG(!out || (mean3 && std3 && std3[0] != 0.f && std3[1] != 0.f && std3[2] != 0.f),
                 "mapa_resize_normalize: mean3 / std3 (host, nonzero std) needed for the float output");
  const int64_t ws = mapa_resize_workspace_bytes(plan_host);
  MAPA_CHECK_ARG(workspace_bytes >= ws && (ws == 0 || workspace), "mapa_resize_normalize: workspace %lld < %lld bytes",
                 (long long)workspace_bytes, (long long)ws);
  const int32_t* pd = reinterpret_cast<const int32_t*>(plan_dev);
  const hipStream_t st = (hipStream_t)stream;
  const float m0 = out ? mean3[0] : 0.f, m1 = out ? mean3[1] : 0.f, m2 = out ? mean3[2] : 0.f;
  const float d0 = out ? std3[0] : 1.f, d1 = out ? std3[1] : 1.f, d2 = out ? std3[2] : 1.f;
  const int64_t npix = (int64_t)h.out_h * h.out_w;
  const int32_t* vb = h.need_v ? pd + h.off_vb : nullptr;
  const int32_t* vk = h.need_v ? pd + h.off_vk : nullptr;
  if (h.need_h) {
    uchar4* tmp = reinterpret_cast<uchar4*>(workspace);
    hipLaunchKernelGGL(resize_h_kernel, dim3(grid_of((int64_t)h.nrows * h.out_w)), dim3(256), 0, st, src,
                       src_row_bytes, h.row0, h.nrows, h.out_w, h.crop_left, h.kh, pd + h.off_hb, pd + h.off_hk, tmp);
    hipLaunchKernelGGL(resize_v_kernel<4>, dim3(grid_of(npix)), dim3(256), 0, st, (const uint8_t*)tmp,
                       (int64_t)4 * h.out_w, 0, h.row0, h.out_h, h.out_w, h.crop_top, h.need_v, h.kv, vb, vk, m0, m1,
                       m2, d0, d1, d2, out, out_u8);
  } else {
    hipLaunchKernelGGL(resize_v_kernel<3>, dim3(grid_of(npix)), dim3(256), 0, st, src, src_row_bytes, h.crop_left, 0,
                       h.out_h, h.out_w, h.crop_top, h.need_v, h.kv, vb, vk, m0, m1, m2, d0, d1, d2, out, out_u8);
  }
  MAPA_CHECK_LAUNCH("mapa_resize_normalize");
  return 0;
}
