// 256-row bf16 MFMA GEMM / implicit-GEMM convolution for gfx950 (the large linears and 3x3 convs of the path): the
// kernel templates, instantiated over several translation units (gemm_big*.hip) so the library builds in parallel.
//
//   C[M,N] = A[M,K] * W[N,K]^T, bf16 operands, fp32 accumulate, the shared fused epilogue (gemm_internal.h).
//
// Why a second tile: a 128x128 tile moves 64 B of operands per 2*128*128*32/... -> 64 flop per staged byte, which
// the L2 / Infinity-cache path cannot feed at the MFMA rate; 256 x 256 doubles the flops per staged byte.
//  * 512 threads = 8 waves, 1 workgroup per CU (128 KiB of LDS for two K stages of 256x64 A + BNx64 B).
//  * BN = 256: waves 2 (M) x 4 (N), wave tile 128x64 = 8x4 MFMA 16x16x32 tiles (128 accumulators / lane).
//    BN = 128: waves 4 (M) x 2 (N), wave tile 64x64 = 4x4 tiles.
//  * HBM/L2 -> LDS with global_load_lds_dwordx4 (lane-linear LDS image, 16-B chunk XOR swizzle chunk ^ (row & 7)
//    applied on the per-lane SOURCE address -> conflict-free ds_read_b128 fragment reads).
//  * K tile t+1 is DMA'd into the other stage while tile t is multiplied; one barrier per K tile.
//  * Epilogue: each wave stages 32 x 64 fp32 of its accumulators through LDS and stores 16-B row segments.
#pragma once
#include <string.h>

#include <algorithm>
#include <type_traits>

#include "gemm_internal.h"

namespace mapa_gemm_impl {
namespace {

constexpr int BBM = 256, BTHREADS = 512, BBK = 64, ROWB = 128;  // ROWB: LDS bytes per row of a K tile
constexpr int ELD = 68;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));                                           // epilogue fp32 row stride (TN = 64 + 4 pad)

template <int BN, int RB, int BM = BBM>
struct Cfg {
  static constexpr int WM = (BN == 256 || BN == 192) ? 2 : 4;
  static constexpr int WN = 8 / WM;
  static constexpr int TM = BM / WM, TN = BN / WN;  // TN = 64 (256-wide) or 32..64
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int CPR = RB / 16;                // 16-B chunks per LDS row
  static constexpr int BK = CPR * 8;                 // K per tile (bf16)
  static constexpr int KG = CPR / 4;                 // 32-deep MFMA k-groups per tile
  static constexpr int RPI = 1024 / RB;              // rows per 1-KiB wave instruction
  static constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int NLA = BM / (8 * RPI), NLB = BN / (8 * RPI);  // wave instructions per thread per tile
  static_assert(BM % (8 * RPI) == 0 && BN % (8 * RPI) == 0, "whole 1-KiB wave instructions per operand");
  static_assert(TN <= 64 && TN % 16 == 0 && FM % 2 == 0, "epilogue: <= 64-column wave tiles, 32-row passes");
  static constexpr int EPI = 8 * 32 * ELD * 4;
};

// 16-B chunk swizzle of an LDS row (applied on the DMA source address, undone on read): conflict-free
// ds_read_b128 of the 16x16x32 fragment pattern for both row sizes.
template <int RB>
__device__ __forceinline__ int swz(int row) {
  if constexpr (RB == 128) return row & 7;
  else return (0x1320 >> (((row >> 2) & 3) * 4)) & 3;  // [0, 2, 3, 1][(row >> 2) & 3]
}

// LDS-DMA of K tile kt into stage buf: NLA 1-KiB wave instructions of A rows, NLB of W rows per wave.
// fast (dense plain A, whole K tiles, both operands under 2 GiB: big_fast_staging): buffer loads from per-lane 32-bit
// row offsets a_o / w_o with the tile's K offset in soffset — no 64-bit pointer per piece in registers, no zero-page
// select.  Otherwise the general form: row pointers recomputed from (bm, bn) per tile (the empty asm keeps them out of
// the loop-invariant code motion that would pin them in registers), K-tail chunks and conv padding from the zero page.
template <int AMODE, int BN, int RB, int BM = BBM>
__device__ __forceinline__ void stage_big(const GemmArgs& p, char* lds, int buf, int kt, int lds_wave, bool k_exact,
                                          const uint32_t* a_o, const int* a_sc, const int* cv_pix,
                                          const int* cv_yx, const uint32_t* w_o, const int* w_sc, bool fast, int bm,
                                          int bn, int wave, int lane) {
  using C = Cfg<BN, RB, BM>;
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  char* As = lds + buf * C::STAGE;
  char* Bs = As + C::A_BYTES;
  if (AMODE == 0 && fast) {
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, 0, 0x7fffffff, 0x00020000);
    const int koff = kt * C::BK * 2;
#pragma unroll
    for (int i = 0; i < C::NLA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(As + lds_wave + i * 8192), 16, (int)a_o[i], koff, 0, 0);
#pragma unroll
    for (int i = 0; i < C::NLB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(Bs + lds_wave + i * 8192), 16, (int)w_o[i], koff, 0, 0);
    return;
  }
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  const int64_t koff = (int64_t)kt * C::BK * 2;
  const int lrow = lane / C::CPR;
#pragma unroll
  for (int i = 0; i < C::NLA; ++i) {
    const int kc = kt * C::BK + a_sc[i] * 8;
    const bool kin = k_exact || kc < p.K;
    const char* src;
    if constexpr (AMODE == 0) {
      int m = min(bm + (i * 8 + wave) * C::RPI + lrow, p.M - 1);
      asm volatile("" : "+v"(m));
      src = kin ? reinterpret_cast<const char*>(p.A) + ((int64_t)m * p.lda + a_sc[i] * 8) * 2 + koff -
                      split_koff(p, kc, 2)
                : zero;
    } else {
      int tap, ci;
      conv_kmap(p, kc, tap, ci);
      const int ky = tap / 3, kx = tap - ky * 3;
      const bool ok = kin && conv_tap_in(p, cv_yx[i], ky, kx);
      src = ok ? reinterpret_cast<const char*>(p.A) + ((int64_t)(cv_pix[i] + ky * p.cv_IW + kx) * p.cv_Cp + ci) * 2
               : zero;
    }
    __builtin_amdgcn_global_load_lds(src, As + lds_wave + i * 8192, 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < C::NLB; ++i) {
    const int kc = kt * C::BK + w_sc[i] * 8;
    const bool kin = k_exact || kc < p.K;
    int n = min(bn + (i * 8 + wave) * C::RPI + lrow, p.N - 1);
    asm volatile("" : "+v"(n));
    const char* src = reinterpret_cast<const char*>(p.W) + ((int64_t)n * p.ldw + w_sc[i] * 8) * 2 + koff;
    __builtin_amdgcn_global_load_lds(kin ? src : zero, Bs + lds_wave + i * 8192, 16, 0, 0);
  }
}

// stage_big's fast form applies to this launch (dense plain A, K a multiple of BK, 32-bit offsets reach every byte)
template <int AMODE, int BK>
__device__ __forceinline__ bool big_fast_staging(const GemmArgs& p) {
  return AMODE == 0 && p.K % BK == 0 && p.sp_half == 0x7fffffff &&
         (int64_t)p.M * p.lda * 2 + (int64_t)p.K * 2 + 256 < 0x7fffffff &&
         (int64_t)p.N * p.ldw * 2 + (int64_t)p.K * 2 + 256 < 0x7fffffff;
}

// ---- epilogue: 32 rows x 64 fp32 per wave per pass through LDS; 8 columns per lane (16-B bf16 stores) -------
// The output pattern (epi_mode) selects one of three copies of the whole epilogue, so each keeps its part loop
// fully unrolled (a runtime part index would move the accumulators to scratch).  LDS must be free (every wave past
// its last main-loop read) before the call.
template <int FM, int FN, int TM, int TN>
__device__ __forceinline__ void big_epilogue(const GemmArgs& p, f32x4 (&acc)[FM][FN], char* lds, int bm, int bn,
                                             int wave, int wm, int wn, int lane) {
  const int g = lane >> 4, r16 = lane & 15;
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * ELD;
  const int c8 = (lane & 7) * 8;
  const int n0 = bn + wn * TN + c8;
  const EpiCol8 ec = epi_col_setup8(p, n0);
  auto epilogue = [&](auto mode_tag) __attribute__((always_inline)) {
    constexpr int MODE = decltype(mode_tag)::value;
#pragma unroll
    for (int part = 0; part < FM / 2; ++part) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ep[(i * 16 + g * 4 + r) * ELD + j * 16 + r16] = acc[part * 2 + i][j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (n0 < p.N && c8 < TN) {
#pragma unroll 2
        for (int pass = 0; pass < 4; ++pass) {
          const int rloc = pass * 8 + (lane >> 3);
          const int m = bm + wm * TM + part * 32 + rloc;
          if (m >= p.M) break;
          epi_store_row8_mode<MODE>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * ELD + c8),
                                    *reinterpret_cast<const f32x4*>(ep + rloc * ELD + c8 + 4));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  };
  const int emode = epi_mode(p);
  if (emode == 1) epilogue(std::integral_constant<int, 1>());
  else if (emode == 2) epilogue(std::integral_constant<int, 2>());
  else epilogue(std::integral_constant<int, 0>());
}

// ---- LayerNorm-fused residual epilogue (LNF) ---------------------------------------------------------------------
// The in-place residual pattern of epi_mode 2 (out_f32 = resid1 + gamma * (acc + bias): the arithmetic of
// epi_store_row8_mode<2>), then nn.LayerNorm over each output row, whose N columns are the band's ntn tiles
// (dinov2 layers/block.py:93-118 norm1 / norm2, transformer_blocks.py:452-469):
//  1. every lane computes its 8-column row segments of the new residual and keeps them in registers (FM/2 parts x
//     4 passes);
//  2. per tile row: the sum over the tile's columns (8-lane butterfly, then the WN column waves' partials in LDS in
//     wave order), the tile mean, then M2 = sum (v - mean_t)^2 the same way (two-pass inside the tile);
//  3. {epoch, sum, M2, ~epoch} of every row published as one 16-byte write-through granule per tile (the data is
//     its own flag: the guide's R2 hand-off, no drain, no arrival counter; epoch = the band's generation word + 1);
//     the new residual rows are stored to out_f32 only now, so they drain while the band gathers;
//  4. per row, the band's ntn granules polled with write-through loads until every one carries this launch's epoch
//     (bounded: past p.ln_spin polls the library's fault word gets MAPA_FAULT_LN_BARRIER and the block proceeds —
//     the host raises on it, mapa_fault_publish / mapa_fault_status), then merged in column order
//     (the same value in every tile of the band): mean = sum / N, M2 = sum_t (M2_t + n_t (mean_t - mean)^2) (Chan's
//     merge, exact up to rounding), rstd = rsqrt(M2 / N + eps);
//  5. the band's last departing block re-arms the departure counter and bumps the generation word; every tile
//     writes y = (v - mean) * rstd * w + b as bf16 for its own columns.
// Equal to the standalone two-pass LayerNorm (norm.hip) up to the fp32 rounding of the statistics.  The launch needs
// N % BN == 0 (every tile holds BN columns of a row) and the row-major in-place residual outputs (epi_mode 2).
// Progress: launch_gemm_big_ln never launches more workgroups than the device holds at once (occupancy x CUs), so
// every tile a waiting tile needs is resident or waits only for a slot held by another kernel — nothing assumes an
// order of dispatch.  The granule hand-off assumes a 16-byte aligned dwordx4 store reaches L2 as one piece (the
// guide's R2 hand-off); a torn granule would fail the {epoch, ~epoch} check and be re-polled, not merged.
constexpr unsigned LN_SPIN_DEFAULT = 1u << 22;  // ~1 us per poll round: seconds before a band gives up
constexpr int LN_MAX_NTN = 8;  // column tiles per band the merge holds in registers (launch_gemm_big_ln checks)
typedef __attribute__((address_space(1))) int gi32;


template <int FM, int FN, int TM, int TN, int WN, int BM>
__device__ __forceinline__ void big_epilogue_ln(const GemmArgs& p, f32x4 (&acc)[FM][FN], char* lds, int tm, int tn,
                                                int ntn, int wave, int wm, int wn, int lane, int tid) {
  constexpr int NP = FM / 2, BN = TN * WN;
  const int g = lane >> 4, r16 = lane & 15;
  const int bm = tm * BM, bn = tn * BN;
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * ELD;
  float* red = reinterpret_cast<float*>(lds + 8 * 32 * ELD * 4);  // [WN][BM] per-wave row partials
  float* rmean = red + WN * BM;                                    // [BM] tile mean, then the row mean
  float* rrstd = rmean + BM;                                       // [BM] row rstd
  const int c8 = (lane & 7) * 8;
  const bool col_ok = c8 < TN;  // TN = 48 (192-wide tiles): lanes 6, 7 of each row group idle
  const int n0 = bn + wn * TN + (col_ok ? c8 : 0);
  const EpiCol8 ec = epi_col_setup8(p, n0);
  const f32x4 lw0 = *reinterpret_cast<const f32x4*>(p.ln_w + n0), lw1 = *reinterpret_cast<const f32x4*>(p.ln_w + n0 + 4);
  const f32x4 lb0 = *reinterpret_cast<const f32x4*>(p.ln_b + n0), lb1 = *reinterpret_cast<const f32x4*>(p.ln_b + n0 + 4);
  f32x4 keep[NP][4][2];
  // 1. residual epilogue (the values stay in registers)
#pragma unroll
  for (int part = 0; part < NP; ++part) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i * 16 + g * 4 + r) * ELD + j * 16 + r16] = acc[part * 2 + i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int rloc = pass * 8 + (lane >> 3);
      const int m = bm + wm * TM + part * 32 + rloc;
      f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
      if (col_ok && m < p.M) {
        const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + rloc * ELD + c8);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + rloc * ELD + c8 + 4);
        const int64_t off = (int64_t)m * p.ldo + n0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v0[e] = lo[e] + ec.a.bv[e];
          v1[e] = hi[e] + ec.b.bv[e];
        }
        if (p.gamma) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v0[e] *= ec.a.gv[e];
            v1[e] *= ec.b.gv[e];
          }
        }
        v0 += *reinterpret_cast<const f32x4*>(p.resid1 + off);
        v1 += *reinterpret_cast<const f32x4*>(p.resid1 + off + 4);
      }
      keep[part][pass][0] = v0;  // stored to out_f32 after the band's arrival (step 3): the publish drain must not
      keep[part][pass][1] = v1;  // wait for the residual stream's stores
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // 2. tile row sums -> tile means
  const bool dskip = p.ln_skip & 16;  // (MAPA_LN_DIAG 16, timing only: no statistics, no exchange)
  float tsum = 0.f;
  if (!dskip) {
#pragma unroll
  for (int part = 0; part < NP; ++part)
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const f32x4 a = keep[part][pass][0], b = keep[part][pass][1];
      float s = ((a[0] + a[1]) + (a[2] + a[3])) + ((b[0] + b[1]) + (b[2] + b[3]));
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      if ((lane & 7) == 0) red[wn * BM + wm * TM + part * 32 + pass * 8 + (lane >> 3)] = s;
    }
  __syncthreads();
  if (tid < BM) {
#pragma unroll
    for (int w = 0; w < WN; ++w) tsum += red[w * BM + tid];
    rmean[tid] = tsum * (1.f / BN);
  }
  __syncthreads();
  // tile M2 about the tile mean
#pragma unroll
  for (int part = 0; part < NP; ++part)
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const float mu = rmean[wm * TM + part * 32 + pass * 8 + (lane >> 3)];
      float q = 0.f;
      if (col_ok) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float d = keep[part][pass][h][e] - mu;
            q += d * d;
          }
      }
      q += __shfl_xor(q, 1);
      q += __shfl_xor(q, 2);
      q += __shfl_xor(q, 4);
      if ((lane & 7) == 0) red[wn * BM + wm * TM + part * 32 + pass * 8 + (lane >> 3)] = q;
    }
  __syncthreads();
  }
  // 3. publish {epoch, sum, M2, ~epoch} per row as one 16-byte write-through granule: the data is its own flag (no
  // drain, no arrival counter); epoch = the band's generation word + 1, bumped by the band's last departing tile
  gi32* gen = (gi32*)(p.ln_ctr) + 2 * tm;
  gi32* depart = gen + 1;
  const unsigned epoch = dskip ? 1u : (unsigned)__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  // band tm's granules at a fixed stride of LN_MAX_NTN column tiles whatever this shape's ntn: a slot is only ever
  // written by band tm, with epochs from tm's own monotonic generation word, so no stale granule of another shape
  // (another ntn) can carry this launch's epoch
  const auto srs = __builtin_amdgcn_make_buffer_rsrc(p.ln_stats + (int64_t)tm * LN_MAX_NTN * BM * 4, 0, ntn * BM * 16,
                                                     0x00020000);
  if (tid < BM && !dskip && !((p.ln_skip & 1) && tm == 0 && tn == 0)) {  // (ln_skip: the test hook's missing tile)
    float m2 = 0.f;
#pragma unroll
    for (int w = 0; w < WN; ++w) m2 += red[w * BM + tid];
    const u32x4 gv = {epoch, __float_as_uint(tsum), __float_as_uint(m2), ~epoch};
    __builtin_amdgcn_raw_buffer_store_b128(gv, srs, (tn * BM + tid) * 16, 0, 16);  // sc1
  }
  // the new residual stream (epi_mode 2's out_f32), issued now so its stores drain while the band gathers
#pragma unroll
  for (int part = 0; part < NP; ++part)
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int m = bm + wm * TM + part * 32 + pass * 8 + (lane >> 3);
      if (col_ok && m < p.M && !(p.ln_skip & 8)) {
        const int64_t off = (int64_t)m * p.ldo + n0;
        *reinterpret_cast<f32x4*>(p.out_f32 + off) = keep[part][pass][0];
        *reinterpret_cast<f32x4*>(p.out_f32 + off + 4) = keep[part][pass][1];
      }
    }
  // 4. every row's ntn granules polled (write-through loads) until all carry this launch's epoch, then merged in
  // column order (Chan): the same value in every tile of the band
  if (tid < BM && dskip) {
    rmean[tid] = 0.f;
    rrstd[tid] = 1.f;
  } else if (tid < BM) {
    u32x4 gv[LN_MAX_NTN];
    unsigned spins = 0;
    for (;;) {
      if (p.ln_skip & 2) break;  // (MAPA_LN_DIAG timing only)
#pragma unroll
      for (int t = 0; t < LN_MAX_NTN; ++t)
        gv[t] = t < ntn ? __builtin_amdgcn_raw_buffer_load_b128(srs, (t * BM + tid) * 16, 0, 16) : u32x4{epoch, 0u, 0u, ~epoch};
      bool ok = true;
#pragma unroll
      for (int t = 0; t < LN_MAX_NTN; ++t) ok = ok && gv[t][0] == epoch && gv[t][3] == ~epoch;
      if (ok) break;
      __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");  // re-issue the granule loads every pass
      if (++spins > p.ln_spin) {  // a band tile never published: raise the fault word, do not hang the device
        if (p.fault)  // the calling thread's fault word (gemm_big.hip fault_word(), passed in)
          __hip_atomic_fetch_or(p.fault, (unsigned)MAPA_FAULT_LN_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAX_NTN; ++t)
      if (t < ntn) sum += __uint_as_float(gv[t][1]);
    const float mean = sum / (float)p.N;
    float m2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAX_NTN; ++t)
      if (t < ntn) {
        const float d = __uint_as_float(gv[t][1]) * (1.f / BN) - mean;
        m2 += __uint_as_float(gv[t][2]) + (float)BN * d * d;
      }
    rmean[tid] = mean;
    rrstd[tid] = rsqrtf(m2 / (float)p.N + p.ln_eps);
  }
  __syncthreads();
  if (tid == 0 && !dskip) {  // every tile of the band holds its granules: the last one out bumps the band's generation
    if (__hip_atomic_fetch_add(depart, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ntn - 1) {
      __hip_atomic_store(depart, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // 5. normalise this tile's columns
  bf16_t* lout = reinterpret_cast<bf16_t*>(p.ln_out);
#pragma unroll
  for (int part = 0; part < NP; ++part)
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int r = wm * TM + part * 32 + pass * 8 + (lane >> 3);
      const int m = bm + r;
      if (!col_ok || m >= p.M || (p.ln_skip & 4)) continue;
      const float mu = rmean[r], rs = rrstd[r];
      const f32x4 a = keep[part][pass][0], b = keep[part][pass][1];
      f32x4 y0, y1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y0[e] = (a[e] - mu) * rs * lw0[e] + lb0[e];
        y1[e] = (b[e] - mu) * rs * lw1[e] + lb1[e];
      }
      const uint4 u = {pack_bf16x2(y0[0], y0[1]), pack_bf16x2(y0[2], y0[3]), pack_bf16x2(y1[0], y1[1]),
                       pack_bf16x2(y1[2], y1[3])};
      *reinterpret_cast<uint4*>(lout + (int64_t)m * p.ln_ldo + n0) = u;
    }
}

template <int AMODE, int BN, int RB, int STAGES, int DIAG = 0, int PRIO = 0, int MINB = 1, int BM = BBM,
          bool F16 = false, bool LNF = false>
__global__ void __launch_bounds__(BTHREADS, MINB) gemm_big_kernel(GemmArgs p) {
  using C = Cfg<BN, RB, BM>;
  constexpr int MAIN = STAGES * C::STAGE;
  constexpr int EPI = C::EPI + (LNF ? (C::WN * BM + 2 * BM) * 4 : 0);  // + the LayerNorm row partials / statistics
  constexpr int LDS = MAIN > EPI ? MAIN : EPI;
  constexpr int NPT = C::NLA + C::NLB;  // LDS-DMA instructions per thread per K tile
  __shared__ __attribute__((aligned(1024))) char lds[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BM - 1) / BM;
  int tm, tn;
  if constexpr (LNF) {
    // this launch's bands [ln_band0, ln_band0 + ln_nbands); idle block of an XCD with one band fewer
    if (!mapa_idx::lnf_coords(blockIdx.x, p.ln_nbands, ntn, tm, tn)) return;
    tm += p.ln_band0;
  } else {
    mapa_idx::tile_coords_rt(blockIdx.x, p.tile_gm, ntm, ntn, tm, tn);
  }
  const int bm = tm * BM, bn = tn * BN;

  // ---- staging geometry: wave instruction i of this wave covers rows (i*8 + wave)*RPI .. +RPI-1
  const int lrow = lane / C::CPR, pos = lane % C::CPR;
  uint32_t a_src[C::NLA];  // stage_big's fast-path row offsets (bytes from A / W)
  int a_sc[C::NLA];
  int cv_pix[C::NLA], cv_yx[C::NLA];
  uint32_t w_src[C::NLB];
  int w_sc[C::NLB];
#pragma unroll
  for (int i = 0; i < C::NLA; ++i) {
    const int r = (i * 8 + wave) * C::RPI + lrow;
    a_sc[i] = pos ^ swz<RB>(r);
    const int m = min(bm + r, p.M - 1);
    if constexpr (AMODE == 0) {
      a_src[i] = (uint32_t)(((int64_t)m * p.lda + a_sc[i] * 8) * 2);
    } else {
      const int hw = p.cv_OH * p.cv_OW;
      const int img = m / hw, rem = m - img * hw;
      const int oy = rem / p.cv_OW, ox = rem - oy * p.cv_OW;
      conv_row_setup(p, img, oy, ox, cv_pix[i], cv_yx[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < C::NLB; ++i) {
    const int r = (i * 8 + wave) * C::RPI + lrow;
    w_sc[i] = pos ^ swz<RB>(r);
    const int n = min(bn + r, p.N - 1);
    w_src[i] = (uint32_t)(((int64_t)n * p.ldw + w_sc[i] * 8) * 2);
  }
  const int nk = (p.K + C::BK - 1) / C::BK;
  const bool k_exact = (p.K % C::BK) == 0;
  const bool fast = big_fast_staging<AMODE, C::BK>(p);
  const int lds_wave = wave * 1024;

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, r16 = lane & 15;
  // The implicit conv's staging state does not leave registers for every k-group's fragments of a 256x256 tile
  // (128 accumulators): there the fragments of one 32-deep k-group are read at a time (no scratch; the code-object
  // test checks every kernel).
  constexpr bool KG_AHEAD = !(AMODE == 1 && C::FM * C::FN >= 32 && C::KG > 1);
  auto compute = [&](int slot) __attribute__((always_inline)) {
    const char* As = lds + slot * C::STAGE;
    const char* Bs = As + C::A_BYTES;
    if constexpr (!KG_AHEAD) {
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg) {
        const int chunk = kg * 4 + g;
        bf16x8 a[C::FM], b[C::FN];
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          const int rb = wn * C::TN + j * 16 + r16;
          b[j] = *reinterpret_cast<const bf16x8*>(Bs + rb * RB + ((chunk ^ swz<RB>(rb)) << 4));
        }
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
          const int ra = wm * C::TM + i * 16 + r16;
          a[i] = *reinterpret_cast<const bf16x8*>(As + ra * RB + ((chunk ^ swz<RB>(ra)) << 4));
        }
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16x16x32<F16>(a[i], b[j], acc[i][j]);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
      }
      return;
    }
    bf16x8 a[C::KG][C::FM], b[C::KG][C::FN];
#pragma unroll
    for (int kg = 0; kg < C::KG; ++kg) {  // every k-group's fragment reads in flight before the first MFMA
      const int chunk = kg * 4 + g;
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int rb = wn * C::TN + j * 16 + r16;
        b[kg][j] = *reinterpret_cast<const bf16x8*>(Bs + rb * RB + ((chunk ^ swz<RB>(rb)) << 4));
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int ra = wm * C::TM + i * 16 + r16;
        a[kg][i] = *reinterpret_cast<const bf16x8*>(As + ra * RB + ((chunk ^ swz<RB>(ra)) << 4));
      }
    }
#pragma unroll
    for (int kg = 0; kg < C::KG; ++kg) {
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = mfma16x16x32<F16>(a[kg][i], b[kg][j], acc[i][j]);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  };

  if constexpr (STAGES == 2) {
    stage_big<AMODE, BN, RB, BM>(p, lds, 0, 0, lds_wave, k_exact, a_src, a_sc, cv_pix, cv_yx, w_src, w_sc, fast, bm, bn, wave, lane);
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();  // tile kt landed (vmcnt(0) before the barrier); every wave is done with tile kt-1
      if (kt + 1 < nk && DIAG != 1)
        stage_big<AMODE, BN, RB, BM>(p, lds, (kt + 1) & 1, kt + 1, lds_wave, k_exact, a_src, a_sc, cv_pix,
                                 cv_yx, w_src, w_sc, fast, bm, bn, wave, lane);
      if (DIAG != 2) compute(kt & 1);
    }
  } else {
    // ring of STAGES slots; tiles kt+1 .. kt+STAGES-2 stay in flight across the barrier of tile kt
#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
      if (s0 < nk)
        stage_big<AMODE, BN, RB, BM>(p, lds, s0, s0, lds_wave, k_exact, a_src, a_sc, cv_pix, cv_yx, w_src, w_sc, fast, bm, bn, wave, lane);
    int slot = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(STAGES - 2, nk - 1 - kt);  // tiles issued after kt that may still be in flight
      if (ahead >= STAGES - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * (STAGES - 2)) : "memory");
      else if (STAGES > 3 && ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * 2) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's DMA for tile kt landed; every wave done with tile kt-1
      __builtin_amdgcn_sched_barrier(0);
      if (kt + STAGES - 1 < nk && DIAG != 1) {
        const int ns = slot == 0 ? STAGES - 1 : slot - 1;  // (kt + STAGES - 1) % STAGES
        stage_big<AMODE, BN, RB, BM>(p, lds, ns, kt + STAGES - 1, lds_wave, k_exact, a_src, a_sc, cv_pix,
                                 cv_yx, w_src, w_sc, fast, bm, bn, wave, lane);
      }
      if (DIAG != 2) compute(slot);
      slot = slot + 1 == STAGES ? 0 : slot + 1;
    }
  }
  __syncthreads();  // all waves done with the last stage: LDS becomes the epilogue staging area
  if constexpr (DIAG == 3) {  // timing diagnostic: main loop only (the never-taken store keeps the MFMAs live)
    if (p.M < 0) big_epilogue<C::FM, C::FN, C::TM, C::TN>(p, acc, lds, bm, bn, wave, wm, wn, lane);
    return;
  }

  if constexpr (LNF)
    big_epilogue_ln<C::FM, C::FN, C::TM, C::TN, C::WN, BM>(p, acc, lds, tm, tn, ntn, wave, wm, wn, lane, tid);
  else
    big_epilogue<C::FM, C::FN, C::TM, C::TN>(p, acc, lds, bm, bn, wave, wm, wn, lane);
}

// ---- ping-pong schedule: two wave groups offset by one barrier ------------------------------------------------
// 256x256 tile, 32-deep K tiles (64-B LDS rows), a ring of NBUF K-tile buffers (32 KiB each).  Waves 0-3 (group 0,
// output rows 0-127) and 4-7 (group 1, rows 128-255) run the same program, group 1 one barrier behind, so on every
// SIMD one wave issues its 16-MFMA cluster while the other reads its next fragments from LDS and issues LDS-DMA:
//   per K tile t, per wave:  [stage A(t+D); read A0..3, B0..3; lgkm(0)] bar [16 MFMA] bar
//                            [stage B(t+D); vmcnt -> tile t+1 landed; read A4..7; lgkm(0)] bar [16 MFMA] bar
// RAW: every wave's vmcnt for tile t+1 precedes global barrier 4t+4 (group 1's one barrier later than group 0's),
// and the first reads of tile t+1 follow it.  WAR: tile t+D (D = NBUF-1) overwrites tile t-1's buffer, whose last
// reads (group 1, before global barrier 4t) were retired by lgkmcnt(0) before that barrier.
template <int AMODE, int NBUF>
__global__ void __launch_bounds__(BTHREADS, 1) gemm_pp_kernel(GemmArgs p) {
  using C = Cfg<256, 64>;
  constexpr int DIST = NBUF - 1;
  constexpr int MAIN = NBUF * C::STAGE;
  constexpr int LDS = MAIN > C::EPI ? MAIN : C::EPI;
  static_assert(C::NLA == 2 && C::NLB == 2 && C::FM == 8 && C::FN == 4 && C::KG == 1, "geometry");
  __shared__ __attribute__((aligned(1024))) char lds[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int ntn = (p.N + 255) / 256, ntm = (p.M + BBM - 1) / BBM;
  int tm, tn;
  tile_coords<4>(blockIdx.x, ntm, ntn, tm, tn);
  const int bm = tm * BBM, bn = tn * 256;

  const int lrow = lane / C::CPR, pos = lane % C::CPR;
  const char* a_src[C::NLA];
  int a_sc[C::NLA];
  int cv_pix[C::NLA], cv_yx[C::NLA];
  const char* w_src[C::NLB];
  int w_sc[C::NLB];
#pragma unroll
  for (int i = 0; i < C::NLA; ++i) {
    const int r = (i * 8 + wave) * C::RPI + lrow;
    a_sc[i] = pos ^ swz<64>(r);
    const int m = min(bm + r, p.M - 1);
    if constexpr (AMODE == 0) {
      a_src[i] = reinterpret_cast<const char*>(p.A) + ((int64_t)m * p.lda + a_sc[i] * 8) * 2;
    } else {
      const int hw = p.cv_OH * p.cv_OW;
      const int img = m / hw, rem = m - img * hw;
      const int oy = rem / p.cv_OW, ox = rem - oy * p.cv_OW;
      conv_row_setup(p, img, oy, ox, cv_pix[i], cv_yx[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < C::NLB; ++i) {
    const int r = (i * 8 + wave) * C::RPI + lrow;
    w_sc[i] = pos ^ swz<64>(r);
    const int n = min(bn + r, p.N - 1);
    w_src[i] = reinterpret_cast<const char*>(p.W) + ((int64_t)n * p.ldw + w_sc[i] * 8) * 2;
  }
  const int nk = (p.K + C::BK - 1) / C::BK;
  const bool k_exact = (p.K % C::BK) == 0;
  const int lds_wave = wave * 1024;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);

  auto stage_a = [&](int buf, int kt) __attribute__((always_inline)) {
    char* As = lds + buf * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::NLA; ++i) {
      const int kc = kt * C::BK + a_sc[i] * 8;
      const bool kin = k_exact || kc < p.K;
      const char* src;
      if constexpr (AMODE == 0) {
        src = kin ? a_src[i] + (int64_t)kt * C::BK * 2 - split_koff(p, kc, 2) : zero;
      } else {
        int tap, ci;
      conv_kmap(p, kc, tap, ci);
        const int ky = tap / 3, kx = tap - ky * 3;
        const bool ok = kin && conv_tap_in(p, cv_yx[i], ky, kx);
        src = ok ? reinterpret_cast<const char*>(p.A) + ((int64_t)(cv_pix[i] + ky * p.cv_IW + kx) * p.cv_Cp + ci) * 2
                 : zero;
      }
      __builtin_amdgcn_global_load_lds(src, As + lds_wave + i * 8192, 16, 0, 0);
    }
  };
  auto stage_b = [&](int buf, int kt) __attribute__((always_inline)) {
    char* Bs = lds + buf * C::STAGE + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < C::NLB; ++i) {
      const int kc = kt * C::BK + w_sc[i] * 8;
      const bool kin = k_exact || kc < p.K;
      __builtin_amdgcn_global_load_lds(kin ? w_src[i] + (int64_t)kt * C::BK * 2 : zero, Bs + lds_wave + i * 8192, 16,
                                       0, 0);
    }
  };

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  const int g = lane >> 4, r16 = lane & 15;
  // fragment byte offsets inside a K-tile buffer (16-B chunk g of the 32-deep row, swizzled)
  int a_off[C::FM], b_off[C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i) {
    const int ra = wm * C::TM + i * 16 + r16;
    a_off[i] = ra * 64 + ((g ^ swz<64>(ra)) << 4);
  }
#pragma unroll
  for (int j = 0; j < C::FN; ++j) {
    const int rb = wn * C::TN + j * 16 + r16;
    b_off[j] = C::A_BYTES + rb * 64 + ((g ^ swz<64>(rb)) << 4);
  }

  // prologue: K tiles 0 .. DIST-1 in flight; tile 0 landed everywhere before the first reads
#pragma unroll
  for (int s0 = 0; s0 < DIST; ++s0)
    if (s0 < nk) {
      stage_a(s0, s0);
      stage_b(s0, s0);
    }
  {
    const int later = min(DIST, nk) - 1;  // tiles after tile 0 in flight
    if (later >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (later == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

  int buf = 0, sbuf = DIST % NBUF;
  for (int kt = 0; kt < nk; ++kt) {
    const char* base = lds + buf * C::STAGE;
    const bool stage = kt + DIST < nk;
    // ---- phase A: rows 0-63 of the wave tile
    if (stage) stage_a(sbuf, kt + DIST);
    b8 bf[C::FN], af[4];
#pragma unroll
    for (int j = 0; j < C::FN; ++j) bf[j] = *reinterpret_cast<const b8*>(base + b_off[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const b8*>(base + a_off[i]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase B: rows 64-127; tile kt+1 must have landed (this wave's DMA) before the next barrier
    if (stage) stage_b(sbuf, kt + DIST);
    {
      const int later = min(DIST - 1, nk - 2 - kt);  // tiles after kt+1 whose DMA may stay in flight
      if (later >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (later == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const b8*>(base + a_off[4 + i]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    buf = buf + 1 == NBUF ? 0 : buf + 1;
    sbuf = sbuf + 1 == NBUF ? 0 : sbuf + 1;
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // rejoin: group 1's last MFMA cluster ends at this barrier
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue (as gemm_big_kernel): every LDS read retired before the barriers above
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * ELD;
  const int c4 = (lane & 15) * 4;
  const int n0 = bn + wn * C::TN + c4;
  const EpiCol ec = epi_col_setup(p, n0);
#pragma unroll
  for (int part = 0; part < C::FM / 2; ++part) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i * 16 + g * 4 + r) * ELD + j * 16 + r16] = acc[part * 2 + i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (n0 < p.N) {
#pragma unroll 2
      for (int pass = 0; pass < 8; ++pass) {
        const int rloc = pass * 4 + g;
        const int m = bm + wm * C::TM + part * 32 + rloc;
        if (m >= p.M) break;
        epi_store_row<bf16_t>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * ELD + c4));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---- stream-K: persistent grid, contiguous K-iteration ranges ---------------------------------------------
// The (tile, K-tile) iteration space [0, tiles * nk) is cut into G equal contiguous ranges, one per persistent
// workgroup (G = CUs x occupancy), so every CU does the same number of MFMA K-steps however badly the tile count
// divides the CU count (M = 10960 -> 43 row tiles; N = 768..1024 -> 6..8 column tiles: 258..344 tiles on 256 CUs).
// A tile whose iterations span several ranges is finished by its LAST-arriving contributor: each contributor stores
// its fp32 accumulators to a slab with write-through (sc1) stores and publishes (every wave vmcnt(0) -> barrier ->
// relaxed agent fetch_add on the tile's ticket; no release fence needed for sc1 payloads); the block drawing ticket
// nseg-1 reads every slab with sc1 loads (no acquire: no plain load of slab bytes anywhere), sums them in range
// order (bit-reproducible whatever the arrival order), resets the ticket and runs the fused epilogue.  No block ever waits on another, so the grid drains whatever the residency.
struct SkArgs : mapa_idx::SkPlan {  // dp_tiles / base / total / per / nk: the iteration plan (index_math.h)
  int* tickets;   // [tiles], zero at launch (zeroed once at workspace creation; the last arriver re-zeroes)
  float* slabs;   // [G][2][BBM * BN] fp32 accumulator images in fragment order
};

using mapa_idx::sk_slab;


template <int AMODE, int BN, int RB, int STAGES, int PRIO, int MINB, bool F16 = false>
__global__ void __launch_bounds__(BTHREADS, MINB) gemm_sk_kernel(GemmArgs p, SkArgs s) {
  using C = Cfg<BN, RB>;
  constexpr int MAIN = STAGES * C::STAGE;
  constexpr int BODY = MAIN > C::EPI ? MAIN : C::EPI;
  constexpr int LDS = BODY + 16;  // + the "last arriver" word (one LDS array: see the guide's 2nd-__shared__ trap)
  constexpr int NPT = C::NLA + C::NLB;
  constexpr int SLAB = BBM * BN;
  static_assert(STAGES >= 3, "ring pipeline");
  __shared__ __attribute__((aligned(1024))) char lds[LDS];
  int* last_word = reinterpret_cast<int*>(lds + BODY);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BBM - 1) / BBM;
  const int vb = xcd_remap(blockIdx.x, gridDim.x);  // consecutive ranges (shared tiles) on one XCD
  const bool k_exact = (p.K % C::BK) == 0;
  const bool fast = big_fast_staging<AMODE, C::BK>(p);
  const int lds_wave = wave * 1024;
  const int lrow = lane / C::CPR, pos = lane % C::CPR;
  const int g = lane >> 4, r16 = lane & 15;

  // data-parallel whole tiles first, then this block's stream-K iteration range (mapa_idx::sk_next)
  mapa_idx::SkCursor cur = mapa_idx::sk_begin(s, vb);
  for (;;) {
    int t, k0, k1;
    if (!mapa_idx::sk_next(s, gridDim.x, cur, t, k0, k1)) break;
    const int tb = t * s.nk;
    int tm, tn;
    group_coords<4>(t, ntm, ntn, tm, tn);
    const int bm = tm * BBM, bn = tn * BN;

    uint32_t a_src[C::NLA];  // stage_big's fast-path row offsets
    int a_sc[C::NLA];
    int cv_pix[C::NLA], cv_yx[C::NLA];
    uint32_t w_src[C::NLB];
    int w_sc[C::NLB];
#pragma unroll
    for (int i = 0; i < C::NLA; ++i) {
      const int r = (i * 8 + wave) * C::RPI + lrow;
      a_sc[i] = pos ^ swz<RB>(r);
      const int m = min(bm + r, p.M - 1);
      if constexpr (AMODE == 0) {
        a_src[i] = (uint32_t)(((int64_t)m * p.lda + a_sc[i] * 8) * 2);
      } else {
        const int hw = p.cv_OH * p.cv_OW;
        const int img = m / hw, rem = m - img * hw;
        const int oy = rem / p.cv_OW, ox = rem - oy * p.cv_OW;
        conv_row_setup(p, img, oy, ox, cv_pix[i], cv_yx[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < C::NLB; ++i) {
      const int r = (i * 8 + wave) * C::RPI + lrow;
      w_sc[i] = pos ^ swz<RB>(r);
      const int n = min(bn + r, p.N - 1);
      w_src[i] = (uint32_t)(((int64_t)n * p.ldw + w_sc[i] * 8) * 2);
    }

    f32x4 acc[C::FM][C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int slot) __attribute__((always_inline)) {
      const char* As = lds + slot * C::STAGE;
      const char* Bs = As + C::A_BYTES;
      bf16x8 a[C::KG][C::FM], b[C::KG][C::FN];  // raw 16-bit words: bf16, or fp16 with F16
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg) {
        const int chunk = kg * 4 + g;
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
          const int rb = wn * C::TN + j * 16 + r16;
          b[kg][j] = *reinterpret_cast<const bf16x8*>(Bs + rb * RB + ((chunk ^ swz<RB>(rb)) << 4));
        }
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
          const int ra = wm * C::TM + i * 16 + r16;
          a[kg][i] = *reinterpret_cast<const bf16x8*>(As + ra * RB + ((chunk ^ swz<RB>(ra)) << 4));
        }
      }
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            acc[i][j] = mfma16x16x32<F16>(a[kg][i], b[kg][j], acc[i][j]);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
      }
    };

    // ring of STAGES slots over K tiles k0 .. k1-1 (same pipeline as gemm_big_kernel)
    const int n = k1 - k0;
#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
      if (s0 < n)
        stage_big<AMODE, BN, RB>(p, lds, s0, k0 + s0, lds_wave, k_exact, a_src, a_sc, cv_pix, cv_yx, w_src,
                                 w_sc, fast, bm, bn, wave, lane);
    int slot = 0;
    for (int kk = 0; kk < n; ++kk) {
      const int ahead = min(STAGES - 2, n - 1 - kk);
      if (ahead >= STAGES - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * (STAGES - 2)) : "memory");
      else if (STAGES > 3 && ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * 2) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kk + STAGES - 1 < n) {
        const int ns = slot == 0 ? STAGES - 1 : slot - 1;
        stage_big<AMODE, BN, RB>(p, lds, ns, k0 + kk + STAGES - 1, lds_wave, k_exact, a_src, a_sc, cv_pix,
                                 cv_yx, w_src, w_sc, fast, bm, bn, wave, lane);
      }
      compute(slot);
      slot = slot + 1 == STAGES ? 0 : slot + 1;
    }
    __syncthreads();  // LDS free for the epilogue

    int lo, hi;
    mapa_idx::sk_contributors(s, t, lo, hi);
    if (lo != hi) {
      // split tile: publish this segment's partial sums.  Buffer stores/loads: the per-fragment offset is an
      // SGPR (soffset), the only VGPR is the lane's 16-B column -> no hoisted 64-bit addresses across the
      // persistent loop.
      const int voff = lane * 16;
      {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(s.slabs + sk_slab(vb, tb, s) * SLAB, 0, SLAB * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, voff,
                                                   ((wave * C::FM + i) * C::FN + j) * 1024, 16);  // sc1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
      __syncthreads();
      if (tid == 0) {
        const int ticket = __hip_atomic_fetch_add(&s.tickets[t], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = ticket == hi - lo;
        if (last) {
          __hip_atomic_store(&s.tickets[t], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *last_word = last;
      }
      __syncthreads();
      const int last = *last_word;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the slab loads below the ticket
      if (!last) continue;  // another contributor finishes this tile (LDS: the next segment re-stages after a
                            // barrier, and last_word is outside the staging area)
      // sum every contributor's slab (this block's included) in range order: bit-reproducible whatever the
      // arrival order.  Half a slab (8 x 16 B per lane) in flight at a time: the (dead) accumulators plus 32 VGPRs.
      for (int b = lo; b <= hi; ++b) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(s.slabs + sk_slab(b, tb, s) * SLAB, 0, SLAB * 4, 0x00020000);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 v[C::FM / 2][C::FN];
#pragma unroll
          for (int i = 0; i < C::FM / 2; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j)
              v[i][j] = __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                             rs, voff, ((wave * C::FM + h * (C::FM / 2) + i) * C::FN + j) * 1024, 16));
#pragma unroll
          for (int i = 0; i < C::FM / 2; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j) {
              f32x4& a = acc[h * (C::FM / 2) + i][j];
              a = b == lo ? v[i][j] : a + v[i][j];
            }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }

    // ---- fused epilogue (as gemm_big_kernel) ----
    float* ep = reinterpret_cast<float*>(lds) + wave * 32 * ELD;
    const int c4 = (lane & 15) * 4;
    const int n0 = bn + wn * C::TN + c4;
    const EpiCol ec = epi_col_setup(p, n0);
#pragma unroll
    for (int part = 0; part < C::FM / 2; ++part) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ep[(i * 16 + g * 4 + r) * ELD + j * 16 + r16] = acc[part * 2 + i][j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (n0 < p.N) {
#pragma unroll 2
        for (int pass = 0; pass < 8; ++pass) {
          const int rloc = pass * 4 + g;
          const int m = bm + wm * C::TM + part * 32 + rloc;
          if (m >= p.M) break;
          epi_store_row<bf16_t>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * ELD + c4));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();  // every wave done with the epilogue staging before the next segment's DMA
  }
}

}  // namespace
}  // namespace mapa_gemm_impl
