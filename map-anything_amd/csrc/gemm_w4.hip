// Four-wave 256-column bf16 MFMA GEMM / implicit-GEMM convolution for gfx950.
//
//   C[M,N] = A[M,K] * W[N,K]^T, bf16 operands, fp32 accumulate, the shared fused epilogue (gemm_internal.h).
//
// Why four waves: with eight waves of 128x64 (gemm_big.hip) every K step reads 192 KiB of fragments from LDS per CU
// on top of the 64 KiB the DMA writes — at 128 B/clk that is as long as the 2048 MFMA cycles of the step, so the
// LDS port, not the matrix cores, sets the pace.  Four waves of 128x128 (wave grid 2 x 2) read 128 KiB per step
// for the same flops (each fragment feeds 8 MFMAs instead of 4..8), at the price of 256 accumulator registers per
// lane: one wave per SIMD with the whole 512-entry register file (accumulators in AGPRs).
//  * 256 threads, 1 workgroup per CU, tile BM x 256 (BM = 256, or 192 when 256-row tiles would idle CUs).
//  * K tiles of 64 (128-B LDS rows), two stages (128 KiB at BM = 256), LDS-DMA (global_load_lds_dwordx4) with the
//    16-B chunk XOR swizzle (row & 7) on the source address -> conflict-free ds_read_b128 fragment reads.
//  * 16x16x32 MFMA tiles: wave tile (BM/2) x 128 = FM x 8 tiles; one barrier per K tile.
//  * Epilogue: each wave stages 32 x 64 fp32 through LDS per pass and stores 16-B row segments (epi_store_row).
#include "gemm_internal.h"

namespace mapa_gemm_impl {
namespace {

constexpr int W4_THREADS = 256, W4_BN = 256, W4_RB = 128, W4_BK = 64, W4_ELD = 68;

template <int BM>
struct W4 {
  static constexpr int WM = 2, WN = 2;
  static constexpr int TM = BM / WM, TN = W4_BN / WN;  // 128 (96) x 128
  static constexpr int FM = TM / 16, FN = TN / 16;     // 8 (6) x 8 MFMA tiles
  static constexpr int KG = W4_BK / 32;                // 32-deep k-groups per K tile
  static constexpr int RPI = 1024 / W4_RB;             // rows per 1-KiB wave instruction
  static constexpr int A_BYTES = BM * W4_RB, B_BYTES = W4_BN * W4_RB;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int NLA = BM / (4 * RPI), NLB = W4_BN / (4 * RPI);  // wave instructions per thread per tile
  static constexpr int EPI = 4 * 32 * W4_ELD * 4;
  static constexpr int LDS = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  static_assert(FM % 2 == 0 && BM % (4 * RPI) == 0, "geometry");
};

// LDS-DMA of K tile kt into stage buf: NLA 1-KiB wave instructions of A rows, NLB of W rows per wave (a device
// function, not a lambda in the kernel: as a lambda the host pass dropped the kernel stubs).
template <int AMODE, int BM>
__device__ __forceinline__ void w4_stage(const GemmArgs& p, char* lds, int buf, int kt, int lds_wave, bool k_exact,
                                         const char* const* a_src, const int* a_sc, const int* cv_base,
                                         const int* cv_iy, const int* cv_ix, const char* const* w_src,
                                         const int* w_sc) {
  using C = W4<BM>;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  char* As = lds + buf * C::STAGE;
  char* Bs = As + C::A_BYTES;
  const int64_t koff = (int64_t)kt * W4_BK * 2;
#pragma unroll
  for (int i = 0; i < C::NLA; ++i) {
    const int kc = kt * W4_BK + a_sc[i] * 8;
    const bool kin = k_exact || kc < p.K;
    const char* src;
    if constexpr (AMODE == 0) {
      src = kin ? a_src[i] + koff - split_koff(p, kc, 2) : zero;
    } else {
      int tap, ci;
      conv_kmap(p, kc, tap, ci);
      const int ky = tap / 3, kx = tap - ky * 3;
      const int iy = cv_iy[i] + ky, ix = cv_ix[i] + kx;
      const bool ok = kin && iy >= 0 && iy < p.cv_IH && ix >= 0 && ix < p.cv_IW;
      src = ok ? reinterpret_cast<const char*>(p.A) + ((int64_t)(cv_base[i] + iy * p.cv_IW + ix) * p.cv_Cp + ci) * 2
               : zero;
    }
    __builtin_amdgcn_global_load_lds(src, As + i * 4096 + lds_wave, 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < C::NLB; ++i) {
    const int kc = kt * W4_BK + w_sc[i] * 8;
    const bool kin = k_exact || kc < p.K;
    __builtin_amdgcn_global_load_lds(kin ? w_src[i] + koff : zero, Bs + i * 4096 + lds_wave, 16, 0, 0);
  }
}

template <int AMODE, int BM>
__global__ void __launch_bounds__(W4_THREADS, 1) gemm_w4_kernel(GemmArgs p) {
  using C = W4<BM>;
  __shared__ __attribute__((aligned(1024))) char lds[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int ntn = (p.N + W4_BN - 1) / W4_BN, ntm = (p.M + BM - 1) / BM;
  int tm, tn;
  tile_coords<4>(blockIdx.x, ntm, ntn, tm, tn);
  const int bm = tm * BM, bn = tn * W4_BN;

  // ---- staging geometry: wave instruction i of wave w covers tile rows (i*4 + w)*8 .. +7, lane = row*8 + chunk
  const int lrow = lane >> 3, pos = lane & 7;
  const char* a_src[C::NLA];
  int a_sc[C::NLA];
  int cv_base[C::NLA], cv_iy[C::NLA], cv_ix[C::NLA];
  const char* w_src[C::NLB];
  int w_sc[C::NLB];
#pragma unroll
  for (int i = 0; i < C::NLA; ++i) {
    const int r = (i * 4 + wave) * C::RPI + lrow;
    a_sc[i] = pos ^ (r & 7);
    const int m = min(bm + r, p.M - 1);
    if constexpr (AMODE == 0) {
      a_src[i] = reinterpret_cast<const char*>(p.A) + ((int64_t)m * p.lda + a_sc[i] * 8) * 2;
    } else {
      const int hw = p.cv_OH * p.cv_OW;
      const int img = m / hw, rem = m - img * hw;
      const int oy = rem / p.cv_OW, ox = rem - oy * p.cv_OW;
      cv_base[i] = img * p.cv_IH * p.cv_IW;
      cv_iy[i] = oy * p.cv_stride - 1;
      cv_ix[i] = ox * p.cv_stride - 1;
    }
  }
#pragma unroll
  for (int i = 0; i < C::NLB; ++i) {
    const int r = (i * 4 + wave) * C::RPI + lrow;
    w_sc[i] = pos ^ (r & 7);
    const int n = min(bn + r, p.N - 1);
    w_src[i] = reinterpret_cast<const char*>(p.W) + ((int64_t)n * p.ldw + w_sc[i] * 8) * 2;
  }
  const int nk = (p.K + W4_BK - 1) / W4_BK;
  const bool k_exact = (p.K % W4_BK) == 0;
  const int lds_wave = wave * 1024;
  auto stage = [&](int buf, int kt) __attribute__((always_inline)) {
    w4_stage<AMODE, BM>(p, lds, buf, kt, lds_wave, k_exact, a_src, a_sc, cv_base, cv_iy, cv_ix, w_src, w_sc);
  };

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  const int g = lane >> 4, r16 = lane & 15;
  auto compute = [&](int slot) __attribute__((always_inline)) {
    const char* As = lds + slot * C::STAGE;
    const char* Bs = As + C::A_BYTES;
#pragma unroll
    for (int kg = 0; kg < C::KG; ++kg) {
      const int chunk = kg * 4 + g;
      b8 a[C::FM], b[C::FN];
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const int rb = wn * C::TN + j * 16 + r16;
        b[j] = *reinterpret_cast<const b8*>(Bs + rb * W4_RB + ((chunk ^ (rb & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        const int ra = wm * C::TM + i * 16 + r16;
        a[i] = *reinterpret_cast<const b8*>(As + ra * W4_RB + ((chunk ^ (ra & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };

  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();  // tile kt landed (vmcnt(0) before the barrier); every wave is done with tile kt-1
    if (kt + 1 < nk) stage((kt + 1) & 1, kt + 1);
    compute(kt & 1);
  }
  __syncthreads();  // all waves done with the last stage: LDS becomes the epilogue staging area

  // ---- epilogue: per wave, 32 rows x 64 fp32 per pass through LDS, 16-B stores ------------------------------
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * W4_ELD;
  const int c4 = (lane & 15) * 4;
#pragma unroll
  for (int jh = 0; jh < 2; ++jh) {
    const int n0 = bn + wn * C::TN + jh * 64 + c4;
    const EpiCol ec = epi_col_setup(p, n0);
#pragma unroll
    for (int part = 0; part < C::FM / 2; ++part) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ep[(i * 16 + g * 4 + r) * W4_ELD + j * 16 + r16] = acc[part * 2 + i][jh * 4 + j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (n0 < p.N) {
#pragma unroll 2
        for (int pass = 0; pass < 8; ++pass) {
          const int rloc = pass * 4 + g;
          const int m = bm + wm * C::TM + part * 32 + rloc;
          if (m >= p.M) break;
          epi_store_row<bf16_t>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * W4_ELD + c4));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

}  // namespace

bool launch_gemm_w4(const GemmArgs& a, bool conv, int variant, hipStream_t stream) {
  if (variant < 0 || variant > 1) return false;
  const int BMv = variant == 0 ? 256 : 192;
  const int nblk = ((a.M + BMv - 1) / BMv) * ((a.N + W4_BN - 1) / W4_BN);
  void (*k)(GemmArgs);
  if (variant == 0) k = conv ? gemm_w4_kernel<1, 256> : gemm_w4_kernel<0, 256>;
  else k = conv ? gemm_w4_kernel<1, 192> : gemm_w4_kernel<0, 192>;
  hipLaunchKernelGGL(k, dim3(nblk), dim3(W4_THREADS), 0, stream, a);
  return true;
}

}  // namespace mapa_gemm_impl
