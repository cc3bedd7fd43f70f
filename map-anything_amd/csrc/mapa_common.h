// Shared helpers for the gfx950 (CDNA4) MapAnything kernels.  Wave = 64 lanes, LDS = 160 KiB per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mapa.h"

#define MAPA_WAVE 64

typedef uint16_t bf16_t;  // raw bf16 bits (row-major tensors in HBM)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------------------
// error reporting (thread-local last error, mapa_last_error())
// ---------------------------------------------------------------------------------------------------------
int mapa_set_error(const char* fmt, ...);

#define MAPA_CHECK_ARG(cond, ...)                 \
  do {                                            \
    if (!(cond)) return mapa_set_error(__VA_ARGS__); \
  } while (0)

#define MAPA_CHECK_LAUNCH(what)                                                         \
  do {                                                                                  \
    hipError_t _e = hipGetLastError();                                                  \
    if (_e != hipSuccess) return mapa_set_error("%s: %s", what, hipGetErrorString(_e)); \
  } while (0)

// ---------------------------------------------------------------------------------------------------------
// bf16 <-> f32 (round-to-nearest-even, NaN kept quiet)
// ---------------------------------------------------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Hardware round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950; keeps NaN a NaN).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// IEEE binary16 storage (MAPA_F16: the operand dtype of the reference's fp16 autocast recipe, model.py:2287-2291),
// kept as raw 16-bit words like bf16; conversions round to nearest even (v_cvt_f16_f32).
__device__ __forceinline__ uint16_t f32_to_f16(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ __forceinline__ float f16_to_f32(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ uint32_t pack_f16x2(float lo, float hi) {
  return (uint32_t)f32_to_f16(lo) | ((uint32_t)f32_to_f16(hi) << 16);
}
// 16-bit operand dtype chosen at run time (uniform branch): fp16 or bf16
__device__ __forceinline__ uint32_t pack_lp2(bool f16, float lo, float hi) {
  return f16 ? pack_f16x2(lo, hi) : pack_bf16x2(lo, hi);
}
__device__ __forceinline__ uint16_t f32_to_lp(bool f16, float f) { return f16 ? f32_to_f16(f) : f32_to_bf16(f); }
__device__ __forceinline__ float lp_to_f32(bool f16, uint16_t v) { return f16 ? f16_to_f32(v) : bf16_to_f32(v); }

// MFMA on raw 16-bit operand words: bf16 or fp16 arithmetic by template flag (same shapes and rates on gfx950)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
template <bool F16>
__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}
template <bool F16>
__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                   c, 0, 0, 0);
}

// Split-precision operand of 4 consecutive values, stored compact: hi = bf16(v) at [0, ld), lo = bf16(v - hi) at
// [ld, 2ld).  A bf16 GEMM reads it as the logical K blocks [hi | hi | lo] (the A loader maps the second hi block back
// onto the first) against weights packed [hi | lo | hi]: v_hi*w_hi + v_hi*w_lo + v_lo*w_hi, the fp32 product to
// ~2^-16 (mapa_split_bf16x3's layout).
__device__ __forceinline__ void store_split3(bf16_t* p, int64_t ld, f32x4 v) {
  uint2 h, l;
  const bf16_t h0 = f32_to_bf16(v[0]), h1 = f32_to_bf16(v[1]), h2 = f32_to_bf16(v[2]), h3 = f32_to_bf16(v[3]);
  h.x = (uint32_t)h0 | ((uint32_t)h1 << 16);
  h.y = (uint32_t)h2 | ((uint32_t)h3 << 16);
  l.x = pack_bf16x2(v[0] - bf16_to_f32(h0), v[1] - bf16_to_f32(h1));
  l.y = pack_bf16x2(v[2] - bf16_to_f32(h2), v[3] - bf16_to_f32(h3));
  *reinterpret_cast<uint2*>(p) = h;
  *reinterpret_cast<uint2*>(p + ld) = l;
}
// 8 consecutive values (16-B aligned): one 16-B store of hi, one of lo
__device__ __forceinline__ void store_split3x8(bf16_t* p, int64_t ld, f32x4 a, f32x4 b) {
  uint4 h, l;
  uint32_t* hp = &h.x;
  uint32_t* lp = &l.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x0 = k < 2 ? a[2 * k] : b[2 * k - 4], x1 = k < 2 ? a[2 * k + 1] : b[2 * k - 3];
    const bf16_t h0 = f32_to_bf16(x0), h1 = f32_to_bf16(x1);
    hp[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    lp[k] = pack_bf16x2(x0 - bf16_to_f32(h0), x1 - bf16_to_f32(h1));
  }
  *reinterpret_cast<uint4*>(p) = h;
  *reinterpret_cast<uint4*>(p + ld) = l;
}
__device__ __forceinline__ void store_split1(bf16_t* p, int64_t ld, float x) {
  const bf16_t h = f32_to_bf16(x);
  p[0] = h;
  p[ld] = f32_to_bf16(x - bf16_to_f32(h));
}

// TF32-equivalent head operands (MAPA_F16X2): v = hi + lo with hi = f16(v), lo = f16(v - hi) (22 significant bits,
// stored [hi | lo] like the bf16 split), multiplied against f16 weights [w | w] — the reference's TF32 heads on its own
// hardware round both operands to 11 significant bits; here only the weights are.  binary16 spans |v| <= 65504: a
// larger (or non-finite) value sets MAPA_FAULT_F16_RANGE in the library's fault word (`fault`; the host raises).
namespace mapa_gemm_impl {
unsigned* fault_word();  // device address of the library's fault word on the current device (gemm_big.hip)
}
constexpr float F16_MAX = 65504.f;
constexpr unsigned FAULT_F16_RANGE = 2u;  // MAPA_FAULT_F16_RANGE
__device__ __forceinline__ void f16_range_fault(unsigned* fault, bool bad) {
  if (bad && fault) __hip_atomic_fetch_or(fault, FAULT_F16_RANGE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// hi / lo halves of one value: (hi, lo) 16-bit words; returns whether |x| fits binary16
__device__ __forceinline__ bool split_f16(float x, uint32_t& h, uint32_t& l) {
  const _Float16 hh = (_Float16)x;
  h = __builtin_bit_cast(uint16_t, hh);
  l = f32_to_f16(x - (float)hh);
  return fabsf(x) <= F16_MAX;
}
// binary16 outputs (TF32-equivalent head operands, MAPA_F16; also the fp16 recipe's transformer operands): values
// outside binary16's range raise MAPA_FAULT_F16_RANGE (NaN compares false and raises too)
__device__ __forceinline__ bool f16_ok(float x) { return fabsf(x) <= F16_MAX; }
__device__ __forceinline__ void f16_check4(unsigned* fault, f32x4 v) {
  f16_range_fault(fault, !(f16_ok(v[0]) && f16_ok(v[1]) && f16_ok(v[2]) && f16_ok(v[3])));
}
__device__ __forceinline__ void store_split2h(bf16_t* p, int64_t ld, f32x4 v, unsigned* fault) {
  uint32_t h[4], l[4];
  bool ok = true;
#pragma unroll
  for (int e = 0; e < 4; ++e) ok &= split_f16(v[e], h[e], l[e]);
  *reinterpret_cast<uint2*>(p) = uint2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
  *reinterpret_cast<uint2*>(p + ld) = uint2{l[0] | (l[1] << 16), l[2] | (l[3] << 16)};
  f16_range_fault(fault, !ok);
}
__device__ __forceinline__ void store_split2h_x8(bf16_t* p, int64_t ld, f32x4 a, f32x4 b, unsigned* fault) {
  uint32_t h[8], l[8];
  bool ok = true;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ok &= split_f16(a[e], h[e], l[e]);
    ok &= split_f16(b[e], h[e + 4], l[e + 4]);
  }
  *reinterpret_cast<uint4*>(p) = uint4{h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), h[6] | (h[7] << 16)};
  *reinterpret_cast<uint4*>(p + ld) =
      uint4{l[0] | (l[1] << 16), l[2] | (l[3] << 16), l[4] | (l[5] << 16), l[6] | (l[7] << 16)};
  f16_range_fault(fault, !ok);
}
__device__ __forceinline__ void store_split2h1(bf16_t* p, int64_t ld, float x, unsigned* fault) {
  uint32_t h, l;
  const bool ok = split_f16(x, h, l);
  p[0] = (bf16_t)h;
  p[ld] = (bf16_t)l;
  f16_range_fault(fault, !ok);
}

// erf for the GELU epilogues, faithful to fp32 erff (≤ 1.2 ulp over the whole range, tools/erf_check.py; the
// reference's GELU is exact-erf, dinov2 layers/mlp.py:29-39 / nn.GELU): two minimax pieces evaluated branch-free
// and selected per lane —
//   |x| ≤ 0.9277:  erf = x + x·P(x²), P of degree 5 (odd, degree 11 overall)
//   |x| > 0.9277:  erf = sign(x)·(1 − exp(R(|x|))), R a degree-7 polynomial fit of log(erfc)
// (coefficients: the well-known single-precision erff minimax pair).  One exp2 and 13 FMAs; the device libm erff is
// ~36 instructions with a divergent two-path branch, and the fc1 GEMMs evaluate it on 1.9 G outputs per 8-view step.
// Round 2 used Abramowitz & Stegun 7.1.26 (5e-7 absolute, large relative error in GELU's negative tail); that moved a
// scalar bf16 output measurably, so the epilogue is held to erff accuracy.
__device__ __forceinline__ float erf_fast(float x) {
  const float t = fabsf(x);
  const float s = x * x;
  // large |x|: 1 - exp(R(t))
  float r = __builtin_fmaf(-1.72853470e-5f, t, 3.83197126e-4f);
  const float u = __builtin_fmaf(-3.88396438e-3f, t, 2.42546219e-2f);
  r = __builtin_fmaf(r, s, u);
  r = __builtin_fmaf(r, t, -1.06777877e-1f);
  r = __builtin_fmaf(r, t, -6.34846687e-1f);
  r = __builtin_fmaf(r, t, -1.28717512e-1f);
  r = __builtin_fmaf(r, t, -t);
  const float big = copysignf(1.0f - __builtin_amdgcn_exp2f(r * 1.4426950408889634f), x);
  // small |x|: x + x * P(s)
  float q = __builtin_fmaf(-5.96761703e-4f, s, 4.99119423e-3f);
  q = __builtin_fmaf(q, s, -2.67681349e-2f);
  q = __builtin_fmaf(q, s, 1.12819925e-1f);
  q = __builtin_fmaf(q, s, -3.76125336e-1f);
  q = __builtin_fmaf(q, s, 1.28379166e-1f);
  q = __builtin_fmaf(q, x, x);
  return t > 0.927734375f ? big : q;
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}
// GELU for a bf16-rounded output (the transformer fc1 epilogues, epi_mode 1): x * Phi(x) with the normal tail
// Q(t) = Phi(-t) = exp2(P(t)), t = min(|x|, 12), P a degree-9 fit of log2 Q on [0, 12] in powers of t
// (tools/gelu_fit.py): GELU = max(x, 0) - |x| Q (x >= 0: x - x Q; x < 0: x Q).  Within 3.2e-5 relative of the
// exact-erf GELU (fp64) wherever |GELU| > 1e-30, and within 1e-30 absolute below: far under a bf16 ulp (2^-8) — the
// rounded output differs from the exactly rounded one in 0.06 % of the elements (the reference's own GELU, evaluated on
// the bf16-rounded linear output, differs in ~33 %).  fmin + 9 FMA + exp2 + max + FMA (|x| is a source modifier)
// instead of erf_fast's ~24 (the fp32-output and fp16 epilogues keep gelu_erf).
__device__ __forceinline__ float gelu_bf16out(float x) {
  const float t = fminf(fabsf(x), 12.0f);
  float r = __builtin_fmaf(-2.5161930317096903e-09f, t, 1.7224749626620905e-07f);
  r = __builtin_fmaf(r, t, -5.2183268053340726e-06f);
  r = __builtin_fmaf(r, t, 9.275929915020242e-05f);
  r = __builtin_fmaf(r, t, -0.0010851839324459434f);
  r = __builtin_fmaf(r, t, 0.008933933451771736f);
  r = __builtin_fmaf(r, t, -0.05458483099937439f);
  r = __builtin_fmaf(r, t, -0.45803743600845337f);
  r = __builtin_fmaf(r, t, -1.1513458490371704f);
  r = __builtin_fmaf(r, t, -0.9999959468841553f);
  return __builtin_fmaf(-fabsf(x), __builtin_amdgcn_exp2f(r), fmaxf(x, 0.f));
}

template <typename T>
__device__ __forceinline__ T ceil_div(T a, T b) {
  return (a + b - 1) / b;
}

// Dense-head tail for one pixel (model.py:1865-2150 via the adaptors): raw = conv1x1 128->6 output; po = the view's
// pose_out row (19 floats: cam_trans, cam_quats, R (row-major 3x3) at 7, t at 16); sc = metric scale.  Unit ray, exp
// depth, pts3d_cam = ray * depth, pts3d = R pts3d_cam + t, both scaled; conf = 1 + exp; mask = sigmoid(logit) > 0.5.
__device__ __forceinline__ void dense_head_pixel(const float* raw, const float* po, float sc, int64_t p,
                                                 float* pts3d, float* pts3d_cam, float* rays, float* depth,
                                                 float* conf, float* logits, uint8_t* mask) {
  float rx = raw[0], ry = raw[1], rz = raw[2];
  const float nr = fmaxf(sqrtf(rx * rx + ry * ry + rz * rz), 1e-8f);
  rx /= nr; ry /= nr; rz /= nr;
  const float d = expf(raw[3]);
  const float cx = rx * d, cy = ry * d, cz = rz * d;
  const float* R = po + 7;
  const float* t = po + 16;
  const float wx = R[0] * cx + R[1] * cy + R[2] * cz + t[0];
  const float wy = R[3] * cx + R[4] * cy + R[5] * cz + t[1];
  const float wz = R[6] * cx + R[7] * cy + R[8] * cz + t[2];
  pts3d[p * 3 + 0] = wx * sc; pts3d[p * 3 + 1] = wy * sc; pts3d[p * 3 + 2] = wz * sc;
  pts3d_cam[p * 3 + 0] = cx * sc; pts3d_cam[p * 3 + 1] = cy * sc; pts3d_cam[p * 3 + 2] = cz * sc;
  rays[p * 3 + 0] = rx; rays[p * 3 + 1] = ry; rays[p * 3 + 2] = rz;
  depth[p] = d * sc;
  conf[p] = 1.f + expf(raw[4]);
  logits[p] = raw[5];
  mask[p] = (1.f / (1.f + expf(-raw[5]))) > 0.5f ? 1 : 0;
}

// Wave-level reductions (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 16 zero bytes that out-of-range LDS-DMA lanes read (halo taps, M/N/K tails).
static __device__ __attribute__((aligned(256))) uint32_t g_mapa_zero_page[64];  // one copy per code object TU
