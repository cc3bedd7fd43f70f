// Four-wave bf16 MFMA GEMM for gfx950 with an explicitly ordered main loop (one wave per SIMD, 128x128 per wave).
//
//   C[M,N] = A[M,K] * W[N,K]^T, bf16 operands, fp32 accumulate, the shared fused epilogue (gemm_internal.h).
//
// The four-wave structure reads 2/3 of the LDS fragment bytes of the eight-wave kernels per MFMA, but with one wave
// per SIMD the wave has to hide its own LDS and DMA latency, and hipcc, left to itself, clusters the fragment reads
// and shuffles the 256 accumulators between VGPRs and AGPRs inside the loop.  Here:
//  * every MFMA is an inline-asm v_mfma_f32_16x16x32_bf16 with its accumulator constrained to AGPRs ("+a"): the
//    accumulators never leave the AGPR file;
//  * the body of K tile kt is written in issue order and fenced with sched_barrier: groups of 4 MFMAs (from the
//    fragments of tile kt, register set 0/1), each followed by one fragment read of tile kt+1 (the other set) for
//    the first 64 MFMAs' worth of reads, and by one LDS-DMA piece of tile kt+4 in the second half;
//  * 32-deep K tiles (64-B LDS rows, 16-B chunk swizzle on the source), a ring of 4 stages (128 KiB at BM = 256);
//    one barrier per tile, before it lgkmcnt(0) (tile kt+1's fragments are in) and vmcnt(2 tiles) (tile kt+2
//    landed; kt+3 and kt+4 stay in flight).  RAW/WAR as gemm_w4p: tile t is read in tile t-1's body after the
//    barrier that ended tile t-2 (whose vmcnt retired it); its slot is re-staged in tile t+1's body, after the
//    barrier ending tile t, which every wave reaches only after its lgkmcnt(0) for tile t's reads.
#include "gemm_internal.h"

namespace mapa_gemm_impl {
namespace {

constexpr int W4A_THREADS = 256, W4A_BN = 256, W4A_ELD = 68, W4A_S = 4;
typedef __bf16 w4ab8 __attribute__((ext_vector_type(8)));

template <int BM>
struct W4A {
  static constexpr int TM = BM / 2, TN = W4A_BN / 2;
  static constexpr int FM = TM / 16, FN = TN / 16;  // 8 (6) x 8
  static constexpr int A_BYTES = BM * 64, B_BYTES = W4A_BN * 64;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int NLA = A_BYTES / (W4A_THREADS * 16), NLB = B_BYTES / (W4A_THREADS * 16);
  static constexpr int NP = NLA + NLB;
  static constexpr int LDS = W4A_S * STAGE;
  static_assert(4 * 32 * W4A_ELD * 4 <= LDS && LDS <= 160 * 1024, "LDS");
};

__device__ __forceinline__ int w4a_swz(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }

template <int N>
__device__ __forceinline__ void w4a_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void w4a_mfma(f32x4& c, const w4ab8& a, const w4ab8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// one LDS-DMA piece i (0..NP-1) of K tile kt into slot `slot` (KEXACT: tiles past the last re-stage the last one)
// (a plain function with the tile constants as arguments, folded after inlining: as a template the host pass of
// hipcc rejects the call sites)
__device__ __forceinline__ void w4a_piece(const GemmArgs& p, char* lds, int slot, int kt, int nk, int lds_wave,
                                          const char* const* a_src, const char* const* w_src, int i, int NLA,
                                          int A_BYTES, int STAGE) {
  char* As = lds + slot * STAGE;
  const int k = min(kt, nk - 1);
  const int64_t koff = (int64_t)k * 64;
  if (i < NLA)
    __builtin_amdgcn_global_load_lds(a_src[i] + koff - split_koff(p, k * 32, 2), As + i * 4096 + lds_wave, 16, 0, 0);
  else
    __builtin_amdgcn_global_load_lds(w_src[i - NLA] + koff, As + A_BYTES + (i - NLA) * 4096 + lds_wave, 16, 0, 0);
}

template <int BM>
__device__ __forceinline__ void w4a_body(const GemmArgs& p, char* lds, int kt, int nk, int lds_wave,
                                         const char* const* a_src, const char* const* w_src, const int* a_off,
                                         const int* b_off, f32x4 (&acc)[W4A<BM>::FM][W4A<BM>::FN], const w4ab8* ac,
                                         const w4ab8* bc, w4ab8* an, w4ab8* bnx) {
  using C = W4A<BM>;
  constexpr int NM = C::FM * C::FN, NR = C::FM + C::FN;
  const char* rs = lds + ((kt + 1) & (W4A_S - 1)) * C::STAGE;
  const int sslot = kt & (W4A_S - 1);
  int m = 0;
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j, ++m) {
      w4a_mfma(acc[i][j], ac[i], bc[j]);
      // first half: a fragment read of tile kt+1 after every 2nd MFMA; second half: a DMA piece after every 4th
      int q = -1;
      if (m < NM / 2) {
        if (m % 2 == 1) q = m / 2;
      } else if (m % 4 == 3) {
        q = NR + (m - NM / 2) / 4;
      }
      if (q >= 0 && q < NR + C::NP) {
        __builtin_amdgcn_sched_barrier(0);
        if (q < C::FN) bnx[q] = *reinterpret_cast<const w4ab8*>(rs + b_off[q]);
        else if (q < NR) an[q - C::FN] = *reinterpret_cast<const w4ab8*>(rs + a_off[q - C::FN]);
        else w4a_piece(p, lds, sslot, kt + W4A_S, nk, lds_wave, a_src, w_src, q - NR, C::NLA, C::A_BYTES, C::STAGE);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  // slots the MFMA groups did not reach (BM = 192: 48 MFMAs)
  constexpr int REACHED = (NM / 2) / 2 < NR ? (NM / 2) / 2 : NR;
#pragma unroll
  for (int q = REACHED; q < NR; ++q) {
    if (q < C::FN) bnx[q] = *reinterpret_cast<const w4ab8*>(rs + b_off[q]);
    else an[q - C::FN] = *reinterpret_cast<const w4ab8*>(rs + a_off[q - C::FN]);
  }
  constexpr int PREACHED = (NM / 2) / 4 < C::NP ? (NM / 2) / 4 : C::NP;
#pragma unroll
  for (int q = PREACHED; q < C::NP; ++q) w4a_piece(p, lds, sslot, kt + W4A_S, nk, lds_wave, a_src, w_src, q, C::NLA, C::A_BYTES,
                                                   C::STAGE);
  w4a_vmcnt<2 * C::NP>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <int BM>
__global__ void __launch_bounds__(W4A_THREADS, 1) gemm_w4a_kernel(GemmArgs p) {
  using C = W4A<BM>;
  __shared__ __attribute__((aligned(1024))) char lds[C::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = (p.N + W4A_BN - 1) / W4A_BN, ntm = (p.M + BM - 1) / BM;
  int tm, tn;
  tile_coords<4>(blockIdx.x, ntm, ntn, tm, tn);
  const int bm = tm * BM, bn = tn * W4A_BN;

  const int lrow = lane >> 2, pos = lane & 3;
  const char* a_src[C::NLA];
  const char* w_src[C::NLB];
  const int sc = pos ^ w4a_swz(lrow);  // (i*4 + wave)*16 + lrow: the swizzle depends on lrow only
#pragma unroll
  for (int i = 0; i < C::NLA; ++i) {
    const int m = min(bm + (i * 4 + wave) * 16 + lrow, p.M - 1);
    a_src[i] = reinterpret_cast<const char*>(p.A) + ((int64_t)m * p.lda + sc * 8) * 2;
  }
#pragma unroll
  for (int i = 0; i < C::NLB; ++i) {
    const int n = min(bn + (i * 4 + wave) * 16 + lrow, p.N - 1);
    w_src[i] = reinterpret_cast<const char*>(p.W) + ((int64_t)n * p.ldw + sc * 8) * 2;
  }
  const int nk = p.K / 32;
  const int lds_wave = wave * 1024;

  const int g = lane >> 4, r16 = lane & 15;
  int a_off[C::FM], b_off[C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i) {
    const int ra = wm * C::TM + i * 16 + r16;
    a_off[i] = ra * 64 + ((g ^ w4a_swz(ra)) << 4);
  }
#pragma unroll
  for (int j = 0; j < C::FN; ++j) {
    const int rb = wn * C::TN + j * 16 + r16;
    b_off[j] = C::A_BYTES + rb * 64 + ((g ^ w4a_swz(rb)) << 4);
  }

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+a"(acc[i][j]));
    }
  w4ab8 a0[C::FM], b0[C::FN], a1[C::FM], b1[C::FN];

#pragma unroll
  for (int s0 = 0; s0 < W4A_S; ++s0)
#pragma unroll
    for (int i = 0; i < C::NP; ++i) w4a_piece(p, lds, s0, s0, nk, lds_wave, a_src, w_src, i, C::NLA, C::A_BYTES, C::STAGE);
  w4a_vmcnt<3 * C::NP>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < C::FN; ++j) b0[j] = *reinterpret_cast<const w4ab8*>(lds + b_off[j]);
#pragma unroll
  for (int i = 0; i < C::FM; ++i) a0[i] = *reinterpret_cast<const w4ab8*>(lds + a_off[i]);
  w4a_vmcnt<2 * C::NP>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    w4a_body<BM>(p, lds, kt, nk, lds_wave, a_src, w_src, a_off, b_off, acc, a0, b0, a1, b1);
    w4a_body<BM>(p, lds, kt + 1, nk, lds_wave, a_src, w_src, a_off, b_off, acc, a1, b1, a0, b0);
  }
  if (kt < nk) w4a_body<BM>(p, lds, kt, nk, lds_wave, a_src, w_src, a_off, b_off, acc, a0, b0, a1, b1);
  // the last MFMAs' results must be written back before the AGPRs are read (the compiler does not see asm latency)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * W4A_ELD;
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
            ep[(i * 16 + g * 4 + r) * W4A_ELD + j * 16 + r16] = acc[part * 2 + i][jh * 4 + j][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (n0 < p.N) {
#pragma unroll 2
        for (int pass = 0; pass < 8; ++pass) {
          const int rloc = pass * 4 + g;
          const int m = bm + wm * C::TM + part * 32 + rloc;
          if (m >= p.M) break;
          epi_store_row<bf16_t>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * W4A_ELD + c4));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

}  // namespace

// variant 0 = 256x256 tile, 1 = 192x256; dense A with K % 32 == 0 (split blocks too) only
bool launch_gemm_w4a(const GemmArgs& a, bool conv, int variant, hipStream_t stream) {
  if (conv || variant < 0 || variant > 1 || a.K % 32 != 0) return false;
  if (a.sp_half != 0x7fffffff && a.sp_half % 32 != 0) return false;
  const int BMv = variant == 0 ? 256 : 192;
  const int nblk = ((a.M + BMv - 1) / BMv) * ((a.N + W4A_BN - 1) / W4A_BN);
  if (variant == 0) hipLaunchKernelGGL(gemm_w4a_kernel<256>, dim3(nblk), dim3(W4A_THREADS), 0, stream, a);
  else hipLaunchKernelGGL(gemm_w4a_kernel<192>, dim3(nblk), dim3(W4A_THREADS), 0, stream, a);
  return true;
}

}  // namespace mapa_gemm_impl
