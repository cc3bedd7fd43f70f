// Internal to the GEMM translation units (gemm.hip: 128x128 tiles, all dtypes; gemm_big.hip: 256-row bf16
// tiles): launch arguments and the shared fused epilogue.
#pragma once
#include "mapa_common.h"
#include "index_math.h"

namespace mapa_gemm_impl {

struct GemmArgs {
  const void* A;
  int64_t lda;
  const void* W;
  int64_t ldw;
  int M, N, K;
  int cv_C, cv_IH, cv_IW, cv_OH, cv_OW, cv_stride;
  // split-precision A operand stored compact: logical K layout [hi | hi | lo] (blocks of sp_half per row or per
  // conv tap), physical [hi | lo] (2 * sp_half per row / pixel, cv_Cp); sp_half = INT_MAX when A is plain
  int sp_half;
  int cv_Cp;  // physical elements per input pixel (conv): cv_C, or 2 * sp_half for a compact split operand
  int cv_kb;  // conv K order: 0 tap-major, else channel blocks of cv_kb (mapa_gemm_desc.conv_kblock)
  const float* bias;
  int bias_mod;
  const float* gamma;
  int act;  // MAPA_ACT_*
  const float* resid1;
  const float* resid2;
  float* out_f32;
  void* out_lp;
  void* out_lp_relu;
  void* out_s3;       // split-precision operand outputs (bf16 kernels): [hi | lo] of v, row stride 2*ld
  void* out_s3_relu;
  int64_t ldo;
  int out_mode;  // 0 row-major, 1 pixel shuffle
  int ps_s, ps_h, ps_w, ps_cout;
  int vec_ok;    // N % 4 == 0, ldo % 4 == 0, ps_cout % 4 == 0: 4-wide epilogue
  int lp_f16;    // 16-bit operands (A, W) and out_lp / out_lp_relu are fp16 (MAPA_F16) instead of bf16
  int tile_gm;   // gemm_big_kernel tile order: groups of tile_gm tile rows per XCD range (mapa_idx::tile_coords_rt)
  // fused LayerNorm of the output rows (mapa_gemm_desc.ln_*; launch_gemm_big_ln): weight / bias over N, bf16 output
  const float* ln_w;
  const float* ln_b;
  float ln_eps;
  void* ln_out;
  int64_t ln_ldo;
  int* ln_ctr;                   // [bands] {generation, departure counter} words (zeroed once)
  unsigned* ln_stats;            // [bands][LN_MAX_NTN][BM] 16-B granules {epoch, sum, M2, ~epoch} (scratch)
  int ln_band0, ln_nbands;       // this launch's bands [ln_band0, ln_band0 + ln_nbands) (co-resident by construction)
  unsigned ln_spin;              // bounded wait: polls before the band barrier gives up and raises the fault word
  int ln_skip;                   // bit 0, test hook: tile (band 0, column 0) skips its publish (mapa_gemm_tune
                                 // LN_TEST_SKIP); bits 1-3: env MAPA_LN_DIAG timing diagnostics (ln_diag_bits)
  unsigned* fault;               // the library's device fault word (f16 split outputs out of binary16 range)
  int stagger;                   // gemm_pers_kernel: 100-MHz ticks the workgroups with one tile fewer start late
};

// Device address of the library's fault word on the current device (gemm_big.hip; other translation units pass it
// to their kernels, as device globals are per translation unit without relocatable device code).
unsigned* fault_word();

using mapa_idx::group_coords;
using mapa_idx::tile_coords;
using mapa_idx::xcd_remap;

// Logical A column (within a row, or within a conv tap) -> physical column of a compact split operand: the
// logical blocks [hi | hi | lo] map onto the stored [hi | lo] (the second hi block re-reads the first).
__device__ __forceinline__ int split_col(const GemmArgs& p, int c) { return c - (c >= p.sp_half ? p.sp_half : 0); }
// Byte correction of a dense A row address for logical column kc (0 for plain operands).
__device__ __forceinline__ int64_t split_koff(const GemmArgs& p, int kc, int esz) {
  return kc >= p.sp_half ? (int64_t)p.sp_half * esz : 0;
}

// Logical K column kc of a 3x3 conv -> tap (0..8) and physical input column (split-aware), in the K order of
// mapa_gemm_desc.conv_kblock.
__device__ __forceinline__ void conv_kmap(const GemmArgs& p, int kc, int& tap, int& ci) {
  int c;
  mapa_idx::conv_kmap_logical(kc, p.cv_kb, p.cv_C, tap, c);
  ci = split_col(p, c);
}

// Implicit 3x3 conv (pad 1) staging state of one A row, two ints: the input pixel index of its (ky, kx) = (0, 0)
// tap, and the tap window's top-left corner + 1 packed as y | x << 16 (both >= 0, images < 65535 pixels a side).
__device__ __forceinline__ void conv_row_setup(const GemmArgs& p, int img, int oy, int ox, int& pix, int& yx) {
  const int iy0 = oy * p.cv_stride - 1, ix0 = ox * p.cv_stride - 1;
  pix = img * p.cv_IH * p.cv_IW + iy0 * p.cv_IW + ix0;
  yx = (iy0 + 1) | ((ix0 + 1) << 16);
}
// tap (ky, kx) of that row inside the image (false = a padding tap, read from the zero page)
__device__ __forceinline__ bool conv_tap_in(const GemmArgs& p, int yx, int ky, int kx) {
  return (unsigned)((yx & 0xffff) + ky - 1) < (unsigned)p.cv_IH && (unsigned)((yx >> 16) + kx - 1) < (unsigned)p.cv_IW;
}

// Per-thread column state of the epilogue: 4 consecutive output columns n0..n0+3.
struct EpiCol {
  int n0;
  float bv[4], gv[4];
  int64_t col_off;  // column inside an output row (the pixel's channel in PIXSHUF mode)
  int ps_ky, ps_kx;
  bool vec;
};

__device__ __forceinline__ EpiCol epi_col_setup(const GemmArgs& p, int n0) {
  EpiCol c;
  c.n0 = n0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int n = min(n0 + e, p.N - 1);
    c.bv[e] = p.bias ? p.bias[n % p.bias_mod] : 0.f;
    c.gv[e] = p.gamma ? p.gamma[n] : 1.f;
  }
  c.col_off = n0;
  c.ps_ky = c.ps_kx = 0;
  if (p.out_mode == 1) {
    const int co = n0 % p.ps_cout, t = n0 / p.ps_cout;
    c.ps_ky = t / p.ps_s;
    c.ps_kx = t - c.ps_ky * p.ps_s;
    c.col_off = co;
  }
  c.vec = p.vec_ok && (n0 + 3 < p.N);
  return c;
}

// out = resid1 + resid2 + gamma * act(acc + bias)   (GELU_POST: gelu(acc + bias + resid1 + resid2))
// for row m, columns c.n0..c.n0+3 (caller guarantees m < M and n0 < N).
template <typename T>
__device__ __forceinline__ void epi_store_row(const GemmArgs& p, const EpiCol& c, int m, f32x4 a) {
  int64_t orow, ld;  // output row (pixel in PIXSHUF mode) and its stride
  if (p.out_mode == 0) {
    orow = m;
    ld = p.ldo;
  } else {
    const int hw = p.ps_h * p.ps_w;
    const int img = m / hw, rem = m - img * hw;
    const int y = rem / p.ps_w, x = rem - y * p.ps_w;
    const int64_t W2 = (int64_t)p.ps_w * p.ps_s, H2 = (int64_t)p.ps_h * p.ps_s;
    orow = ((int64_t)img * H2 + y * p.ps_s + c.ps_ky) * W2 + x * p.ps_s + c.ps_kx;
    ld = p.ps_cout;
  }
  const int64_t off = orow * ld + c.col_off;
  const int64_t off3 = orow * 2 * ld + c.col_off;  // split-operand rows are stored [hi | lo], 2*ld wide
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = a[e] + c.bv[e];
  // activation and gamma once per call (uniform branches), not per element
  if (p.act == MAPA_ACT_GELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
  } else if (p.act == MAPA_ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  if (p.gamma) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] *= c.gv[e];
  }
  if (c.vec) {
    if (p.resid1) v += *reinterpret_cast<const f32x4*>(p.resid1 + off);
    if (p.resid2) v += *reinterpret_cast<const f32x4*>(p.resid2 + off);
    if (p.act == MAPA_ACT_GELU_POST) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
    }
    if (p.out_f32) *reinterpret_cast<f32x4*>(p.out_f32 + off) = v;
    if constexpr (sizeof(T) == 2) {
      if (p.lp_f16 && (p.out_lp || p.out_lp_relu)) f16_check4(p.fault, v);
      if (p.out_lp) {
        uint2 u;
        u.x = pack_lp2(p.lp_f16, v[0], v[1]);
        u.y = pack_lp2(p.lp_f16, v[2], v[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out_lp) + off) = u;
      }
      if (p.out_lp_relu) {
        uint2 u;
        u.x = pack_lp2(p.lp_f16, fmaxf(v[0], 0.f), fmaxf(v[1], 0.f));
        u.y = pack_lp2(p.lp_f16, fmaxf(v[2], 0.f), fmaxf(v[3], 0.f));
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out_lp_relu) + off) = u;
      }
      if (p.out_s3) {
        if (p.lp_f16) store_split2h(reinterpret_cast<bf16_t*>(p.out_s3) + off3, ld, v, p.fault);
        else store_split3(reinterpret_cast<bf16_t*>(p.out_s3) + off3, ld, v);
      }
      if (p.out_s3_relu) {
        const f32x4 rr = {fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
        if (p.lp_f16) store_split2h(reinterpret_cast<bf16_t*>(p.out_s3_relu) + off3, ld, rr, p.fault);
        else store_split3(reinterpret_cast<bf16_t*>(p.out_s3_relu) + off3, ld, rr);
      }
    } else {
      if (p.out_lp) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out_lp) + off) = v;
      if (p.out_lp_relu) {
        f32x4 rr = {fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out_lp_relu) + off) = rr;
      }
    }
  } else {
    // scalar tail (N % 4 != 0 or the last partial column group); row-major only
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (c.n0 + e >= p.N) break;
      const int64_t o = off + e;
      float x = v[e];
      if (p.resid1) x += p.resid1[o];
      if (p.resid2) x += p.resid2[o];
      if (p.act == MAPA_ACT_GELU_POST) x = gelu_erf(x);
      if (p.out_f32) p.out_f32[o] = x;
      if constexpr (sizeof(T) == 2) {
        if (p.lp_f16 && (p.out_lp || p.out_lp_relu)) f16_range_fault(p.fault, !f16_ok(x));
        if (p.out_lp) reinterpret_cast<bf16_t*>(p.out_lp)[o] = f32_to_lp(p.lp_f16, x);
        if (p.out_lp_relu) reinterpret_cast<bf16_t*>(p.out_lp_relu)[o] = f32_to_lp(p.lp_f16, fmaxf(x, 0.f));
        if (p.out_s3) {
          if (p.lp_f16) store_split2h1(reinterpret_cast<bf16_t*>(p.out_s3) + off3 + e, ld, x, p.fault);
          else store_split1(reinterpret_cast<bf16_t*>(p.out_s3) + off3 + e, ld, x);
        }
        if (p.out_s3_relu) {
          if (p.lp_f16) store_split2h1(reinterpret_cast<bf16_t*>(p.out_s3_relu) + off3 + e, ld, fmaxf(x, 0.f), p.fault);
          else store_split1(reinterpret_cast<bf16_t*>(p.out_s3_relu) + off3 + e, ld, fmaxf(x, 0.f));
        }
      } else {
        if (p.out_lp) reinterpret_cast<float*>(p.out_lp)[o] = x;
        if (p.out_lp_relu) reinterpret_cast<float*>(p.out_lp_relu)[o] = fmaxf(x, 0.f);
      }
    }
  }
}

// 8 consecutive columns n0..n0+7 of row m: one 16-B store per bf16 output row segment (the 4-column form stores 8 B)
// for row-major outputs with n0 % 8 == 0 and ldo % 8 == 0; otherwise two 4-column calls.
struct EpiCol8 {
  EpiCol a, b;
  bool vec8;
};

__device__ __forceinline__ EpiCol8 epi_col_setup8(const GemmArgs& p, int n0) {
  EpiCol8 c;
  c.a = epi_col_setup(p, n0);
  c.b = epi_col_setup(p, n0 + 4);
  c.vec8 = p.out_mode == 0 && p.vec_ok && p.ldo % 8 == 0 && n0 + 7 < p.N;
  return c;
}

template <typename T>
__device__ __forceinline__ void epi_store_row8(const GemmArgs& p, const EpiCol8& c, int m, f32x4 lo, f32x4 hi) {
  if (!c.vec8) {
    epi_store_row<T>(p, c.a, m, lo);
    if (c.b.n0 < p.N) epi_store_row<T>(p, c.b, m, hi);
    return;
  }
  const int64_t ld = p.ldo;
  const int64_t off = (int64_t)m * ld + c.a.n0;
  const int64_t off3 = (int64_t)m * 2 * ld + c.a.n0;
  f32x4 v0, v1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v0[e] = lo[e] + c.a.bv[e];
    v1[e] = hi[e] + c.b.bv[e];
  }
  // activation and gamma once per call (uniform branches), not per element
  if (p.act == MAPA_ACT_GELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = gelu_erf(v0[e]);
      v1[e] = gelu_erf(v1[e]);
    }
  } else if (p.act == MAPA_ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = fmaxf(v0[e], 0.f);
      v1[e] = fmaxf(v1[e], 0.f);
    }
  }
  if (p.gamma) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] *= c.a.gv[e];
      v1[e] *= c.b.gv[e];
    }
  }
  if (p.resid1) {
    v0 += *reinterpret_cast<const f32x4*>(p.resid1 + off);
    v1 += *reinterpret_cast<const f32x4*>(p.resid1 + off + 4);
  }
  if (p.resid2) {
    v0 += *reinterpret_cast<const f32x4*>(p.resid2 + off);
    v1 += *reinterpret_cast<const f32x4*>(p.resid2 + off + 4);
  }
  if (p.act == MAPA_ACT_GELU_POST) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v0[e] = gelu_erf(v0[e]);
      v1[e] = gelu_erf(v1[e]);
    }
  }
  if (p.out_f32) {
    *reinterpret_cast<f32x4*>(p.out_f32 + off) = v0;
    *reinterpret_cast<f32x4*>(p.out_f32 + off + 4) = v1;
  }
  if constexpr (sizeof(T) == 2) {
    if (p.lp_f16 && (p.out_lp || p.out_lp_relu)) {
      f16_check4(p.fault, v0);
      f16_check4(p.fault, v1);
    }
    if (p.out_lp) {
      const bool h = p.lp_f16;
      const uint4 u = {pack_lp2(h, v0[0], v0[1]), pack_lp2(h, v0[2], v0[3]), pack_lp2(h, v1[0], v1[1]),
                       pack_lp2(h, v1[2], v1[3])};
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.out_lp) + off) = u;
    }
    if (p.out_lp_relu) {
      const bool h = p.lp_f16;
      const uint4 u = {pack_lp2(h, fmaxf(v0[0], 0.f), fmaxf(v0[1], 0.f)), pack_lp2(h, fmaxf(v0[2], 0.f), fmaxf(v0[3], 0.f)),
                       pack_lp2(h, fmaxf(v1[0], 0.f), fmaxf(v1[1], 0.f)), pack_lp2(h, fmaxf(v1[2], 0.f), fmaxf(v1[3], 0.f))};
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.out_lp_relu) + off) = u;
    }
    if (p.out_s3) {
      if (p.lp_f16) store_split2h_x8(reinterpret_cast<bf16_t*>(p.out_s3) + off3, ld, v0, v1, p.fault);
      else store_split3x8(reinterpret_cast<bf16_t*>(p.out_s3) + off3, ld, v0, v1);
    }
    if (p.out_s3_relu) {
      const f32x4 r0 = {fmaxf(v0[0], 0.f), fmaxf(v0[1], 0.f), fmaxf(v0[2], 0.f), fmaxf(v0[3], 0.f)};
      const f32x4 r1 = {fmaxf(v1[0], 0.f), fmaxf(v1[1], 0.f), fmaxf(v1[2], 0.f), fmaxf(v1[3], 0.f)};
      if (p.lp_f16) store_split2h_x8(reinterpret_cast<bf16_t*>(p.out_s3_relu) + off3, ld, r0, r1, p.fault);
      else store_split3x8(reinterpret_cast<bf16_t*>(p.out_s3_relu) + off3, ld, r0, r1);
    }
  } else {
    if (p.out_lp) {
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out_lp) + off) = v0;
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out_lp) + off + 4) = v1;
    }
    if (p.out_lp_relu) {
      const f32x4 r0 = {fmaxf(v0[0], 0.f), fmaxf(v0[1], 0.f), fmaxf(v0[2], 0.f), fmaxf(v0[3], 0.f)};
      const f32x4 r1 = {fmaxf(v1[0], 0.f), fmaxf(v1[1], 0.f), fmaxf(v1[2], 0.f), fmaxf(v1[3], 0.f)};
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out_lp_relu) + off) = r0;
      *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out_lp_relu) + off + 4) = r1;
    }
  }
}

// Epilogue patterns of the transformer blocks, fixed once per tile so the per-row calls carry no output-set checks:
// 1 = act(acc + bias) -> 16-bit out_lp only (qkv, fc1 + GELU); 2 = resid1 + gamma * (acc + bias) -> out_f32 only, in
// place (attn proj, fc2); 0 = anything else (epi_store_row8).
__host__ __device__ __forceinline__ int epi_mode(const GemmArgs& p) {
  const bool lp_outs = p.out_lp_relu || p.out_s3 || p.out_s3_relu;
  if (p.out_mode != 0 || p.resid2 || lp_outs || p.ldo % 8 != 0 || !p.vec_ok) return 0;
  if (p.out_lp && !p.out_f32 && !p.resid1 && !p.gamma && (p.act == MAPA_ACT_NONE || p.act == MAPA_ACT_GELU)) return 1;
  if (p.out_f32 && !p.out_lp && p.resid1 && p.act == MAPA_ACT_NONE) return 2;
  return 0;
}

template <int MODE>
__device__ __forceinline__ void epi_store_row8_mode(const GemmArgs& p, const EpiCol8& c, int m, f32x4 lo, f32x4 hi) {
  if (MODE == 0 || !c.vec8) {
    epi_store_row8<bf16_t>(p, c, m, lo, hi);
    return;
  }
  const int64_t off = (int64_t)m * p.ldo + c.a.n0;
  f32x4 v0, v1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v0[e] = lo[e] + c.a.bv[e];
    v1[e] = hi[e] + c.b.bv[e];
  }
  if constexpr (MODE == 1) {
    if (p.act == MAPA_ACT_GELU) {
      if (p.lp_f16) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[e] = gelu_erf(v0[e]);
          v1[e] = gelu_erf(v1[e]);
        }
      } else {  // bf16 output only: the cheaper tail fit, 1/256 of the output's ulp (mapa_common.h)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[e] = gelu_bf16out(v0[e]);
          v1[e] = gelu_bf16out(v1[e]);
        }
      }
    }
    uint4 u;
    if (p.lp_f16) {
      f16_check4(p.fault, v0);
      f16_check4(p.fault, v1);
      u = uint4{pack_f16x2(v0[0], v0[1]), pack_f16x2(v0[2], v0[3]), pack_f16x2(v1[0], v1[1]), pack_f16x2(v1[2], v1[3])};
    }
    else {
      u = uint4{pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                pack_bf16x2(v1[2], v1[3])};
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.out_lp) + off) = u;
  } else {
    if (p.gamma) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] *= c.a.gv[e];
        v1[e] *= c.b.gv[e];
      }
    }
    v0 += *reinterpret_cast<const f32x4*>(p.resid1 + off);
    v1 += *reinterpret_cast<const f32x4*>(p.resid1 + off + 4);
    *reinterpret_cast<f32x4*>(p.out_f32 + off) = v0;
    *reinterpret_cast<f32x4*>(p.out_f32 + off + 4) = v1;
  }
}

// 256-row bf16 kernel (gemm_big.hip): variant 0 = 256x256 tile, 1 = 256x128 tile.  Returns false if it does not
// take this shape.
bool launch_gemm_big(const GemmArgs& a, bool conv, int variant, hipStream_t stream);
// The 256-row tile kernels' instantiations, one translation unit each (parallel build): nullptr = no such variant.
using GemmKernel = void (*)(GemmArgs);
GemmKernel big_kernel_bf16_dense(int variant);       // gemm_big_dense.hip
GemmKernel big_kernel_lnf(int variant);              // gemm_big_dense.hip (LayerNorm-fused: 14 / 15)
GemmKernel big_kernel_bf16_conv(int variant);        // gemm_big_conv.hip
GemmKernel big_kernel_f16(int variant, bool conv);   // gemm_big_f16.hip
GemmKernel big_kernel_diag(int variant, bool conv);  // gemm_big_diag.hip
int gemm_device_cus();                               // CUs of the current device (cached per device)
void diag_set_grid(int blocks);  // timing diagnostic: launch only the first `blocks` tiles (0 = all)

// Persistent data-parallel kernel for the transformer linears (gemm_pers.hip): dense 16-bit A, epi_mode 1 or 2,
// register epilogue, the next tile's DMA prologue under the epilogue.  shape: 0 = 256x128 (2 / CU), 1 = 192x256,
// 2 = 256x256, 3 = 192x128 (2 / CU); -1 = pers_pick_shape.  cus: the device's CU count.  false if the problem or its
// epilogue does not qualify.
bool launch_gemm_pers(const GemmArgs& a, int shape, int cus, hipStream_t stream);
int pers_pick_shape(int M, int N, int K, int cus);
void pers_set_stagger(int ticks);  // MAPA_TUNE_PERS_STAGGER (100-MHz ticks, 0 = off)

// The in-place residual linear (epi_mode 2: out_f32 = resid1 + gamma * (acc + bias)) with the LayerNorm of its output
// rows fused (gemm_big.hip, LNF): the row statistics combine across a band's column tiles inside the launch (band
// barrier through the workspace), then every tile normalises its own rows into a.ln_out (bf16).
// variant: 14 (192x256 tiles) or 15 (192x192).  Returns false if the shape / epilogue / workspace does not qualify.
// Workspace: the GEMM ticket head (its top LN_TICKET_WORDS words: per-band generation / departure counters) +
// ln_stats_bytes of per-tile row statistics.  Problems with more bands than the device holds at once run as several
// launches of co-resident bands (the barrier's progress never depends on dispatch order).  A band that does not
// complete within its bounded wait sets MAPA_FAULT_LN_BARRIER in the library's fault word (mapa_fault_status).
constexpr int LN_TICKET_WORDS = 16384;
int64_t ln_stats_bytes(int M, int N, int variant);
bool launch_gemm_big_ln(const GemmArgs& a, int variant, void* ws, int64_t ws_bytes, hipStream_t stream);
// Tuning / test state of the LayerNorm-fused launches (mapa_gemm_tune MAPA_TUNE_LN_SPIN / MAPA_TUNE_LN_TEST_SKIP).
void ln_set_spin(unsigned spins);
void ln_arm_test_skip(int n);
int ln_take_test_skip();    // 1 if an armed test skip is consumed by this launch
int ln_diag_bits();         // MAPA_LN_DIAG: 2 no band wait, 4 no LN stores, 8 no residual stores (timing only)
unsigned ln_spin_value();   // the band barrier's poll bound
// The LayerNorm-fused residual linear on the persistent register-epilogue kernel (gemm_pers.hip): 192x128 tiles at 2
// workgroups per CU, N = 768 / 1024, the workspace of launch_gemm_big_ln.  false if it does not qualify.
bool launch_gemm_pers_ln(const GemmArgs& a, void* ws, int64_t ws_bytes, int cus, hipStream_t stream);

// Stride-1 3x3 conv with its A operand read from an LDS halo window (conv_halo.hip); bn = 256 / 128 / 0 (auto).
// Returns false unless the conv is in the 32-channel-slice K order (conv_kblock == 32).
bool launch_conv_halo(const GemmArgs& a, int bn, hipStream_t stream, int bh = 16);

// The halo conv with the regressor tail fused into its epilogue (conv_halo.hip): conv3x3 128->128 + ReLU, 1x1 128->6,
// adaptors and output assembly.  false unless the conv qualifies (bf16, stride 1, conv_kblock 32, N 128, ReLU, bias).
bool launch_conv_halo_headout(const GemmArgs& a, const float* w6, const float* b6, const float* pose,
                              const float* scale, int vps, float* pts3d, float* pts3d_cam, float* rays, float* depth,
                              float* conf, float* logits, uint8_t* mask, hipStream_t stream);
// The halo conv on flat-raster blocks with the 32-channel slices split over nsplit workgroups per tile (maps up to
// 62 pixels wide; conv_halo.hip).  conv_halo_flat_split: the part count for `slots` resident workgroups (force > 0:
// that many, capped at the slice count), 0 if the conv does not qualify.  Workspace: the ticket head of the GEMM
// workspace (GEMM_TICKET_BYTES, shared with stream-K) + the parts' fp32 slabs; none for nsplit = 1.  The launch
// returns false if the conv does not qualify or the workspace is missing / too small.
constexpr int64_t GEMM_TICKET_BYTES = 65536 * 4;
int conv_halo_flat_split(const GemmArgs& a, int slots, int force);
int64_t conv_halo_flat_workspace_bytes(const GemmArgs& a, int nsplit, int64_t ticket_bytes);
bool launch_conv_halo_flat(const GemmArgs& a, int nsplit, void* ws, int64_t ws_bytes, int64_t ticket_bytes,
                           hipStream_t stream);
// Stream-K bf16 kernel (gemm_big.hip): variant 0 = 256x128 tiles, 2 workgroups per CU; 1 = 256x256, 1 per CU.
// streamk_workspace_bytes: bytes the launch needs (ticket words + partial-sum slabs); launch returns false if
// the workspace is missing or too small.
int64_t streamk_workspace_bytes(int M, int N, int variant);
int gemm_streamk_slots(int variant);  // persistent workgroups of a stream-K variant on this device
bool launch_gemm_streamk(const GemmArgs& a, bool conv, int variant, void* ws, int64_t ws_bytes, hipStream_t stream);

}  // namespace mapa_gemm_impl
