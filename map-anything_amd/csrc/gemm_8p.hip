// 256x256 bf16 MFMA GEMM / implicit-GEMM convolution for gfx950 with a phase-interleaved main loop.
//
//   C[M,N] = A[M,K] * W[N,K]^T, bf16 operands, fp32 accumulate, the shared fused epilogue (gemm_internal.h).
//
// Structure (the 8-phase schedule of the CDNA4 guide, re-derived for a deeper ring of half-tiles):
//  * 512 threads = 8 waves in two groups of four (waves 0-3, 4-7; one wave of each group per SIMD).  Wave (wr, wc)
//    owns output rows {wr*64 + [0,64)} u {128 + wr*64 + [0,64)} and columns {wc*32 + [0,32)} u {128 + wc*32 + [0,32)}
//    of the 256x256 tile: 2x2 quadrants of 64x32, quadrant (mh, nh) reading only A rows mh*128.. and W rows nh*128..
//  * A K tile (64 deep, 128-B LDS rows) is four half-tiles of 16 KiB: A0 (tile rows 0-127), W0, W1, A1 (staging
//    order = order of first use).  Half-tiles stream through a ring of S LDS slots, each DMA'd
//    (global_load_lds_dwordx4, 2 per thread) D = S - 2 half-tiles ahead: the measured lever is the DMA depth (the
//    L2 / Infinity-cache latency under load), so the default ring fills the CU's 160 KiB (S = 10, D = 8).
//  * One phase per quadrant, four per K tile: [fragment reads for the quadrant; DMA of half-tile ph+D; counted
//    vmcnt] barrier [16 MFMA 16x16x32] barrier.  Group 1 runs one barrier behind group 0, so on every SIMD one wave
//    issues MFMAs while the other reads fragments and issues DMA (ping-pong).  Quadrant order (0,0) (0,1) (1,1) (1,0);
//    every half-tile is read in exactly one phase.  BAL = 1: 8 / 4 / 8 / 4 fragment reads per phase (A0 in phase
//    0, W1 in 1, A1 in 2, the NEXT K tile's W0 in phase 3, W0 kept in registers for phases 0 and 3); BAL = 0:
//    12 / 4 / 8 / 0 (W0 read with A0 in phase 0).
//  * Hazards (phase ph = 4*kt + q; group 0 barriers 2ph, 2ph+1, group 1 one later): a DMA issued in phase s and
//    retired by the vmcnt of phase s+k is readable from phase s+k+1.  Each phase retires every half-tile
//    <= ph + 2 + BAL (the first reads of phase ph + 1), leaving KF = D - 2 - BAL half-tiles in flight (RAW).  A slot
//    is re-staged S half-tiles later, >= 2 phases after its last read, whose lgkmcnt retired it before the second
//    barrier of that phase (WAR; holds for D <= S - 2).
//  * Tile order as gemm_big.hip (XCD-contiguous ranges in 4-row groups); epilogue staged through LDS, 16-B stores.
#include "gemm_internal.h"

namespace mapa_gemm_impl {
namespace {

constexpr int P8_THREADS = 512, P8_HALF = 16384, P8_ELD = 68;
typedef __bf16 p8b8 __attribute__((ext_vector_type(8)));

template <int S_, int BAL_>
struct P8Cfg {
  static constexpr int S = S_, BAL = BAL_;
  static constexpr int U = S % 4 == 0 ? S / 4 * 2 : (S % 2 == 0 ? S : 2 * S);  // K tiles per unrolled block
  static_assert((4 * U) % S == 0 && U % 2 == 0, "unroll");
  static constexpr int D = S - 2;         // staging distance (half-tiles)
  static constexpr int KF = D - 2 - BAL;  // half-tiles left in flight by each phase's wait
  static_assert(KF >= 1 && KF <= 6 && D - 2 <= 6, "vmcnt table");
};

// Per-thread staging geometry.  Rows row0 + {0, 64} of half-tile hh are tile rows hh*128 + row0 + {0, 64}; rows past
// M / N read the zero page (edge tiles only).
struct P8Src {
  const char* a0;  // A row bm + row0 (dense A), source chunk applied
  const char* w0;  // W row bn + row0
  int am, wn;      // rows of A / W left from this thread's first row: M - (bm + row0), N - (bn + row0)
  int cv_base[2][2], cv_iy[2][2], cv_ix[2][2];
};

// DMA of half-tile J (0 = A0, 1 = W0, 2 = W1, 3 = A1) of K tile kt into LDS at dst (this wave's 1-KiB rows).
template <int AMODE, int J>
__device__ __forceinline__ void p8_stage(const GemmArgs& p, char* dst, int kt, bool k_exact, const P8Src& s,
                                         int w_sc) {
  constexpr bool IS_A = (J == 0 || J == 3);
  constexpr int HH = (J == 0 || J == 1) ? 0 : 1;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  const int64_t koff = (int64_t)kt * 128;
  const int kc = kt * 64 + w_sc * 8;
  const bool kin = k_exact || kc < p.K;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int RO = HH * 128 + i * 64;  // row offset of this wave instruction's rows
    const char* src;
    if constexpr (IS_A) {
      if constexpr (AMODE == 0) {
        src = (kin && RO < s.am) ? s.a0 + (int64_t)RO * p.lda * 2 + koff - split_koff(p, kc, 2) : zero;
      } else {
        int tap, ci;
      conv_kmap(p, kc, tap, ci);
        const int ky = tap / 3, kx = tap - ky * 3;
        const int iy = s.cv_iy[HH][i] + ky, ix = s.cv_ix[HH][i] + kx;
        const bool ok = kin && iy >= 0 && iy < p.cv_IH && ix >= 0 && ix < p.cv_IW;
        src = ok ? reinterpret_cast<const char*>(p.A) +
                       ((int64_t)(s.cv_base[HH][i] + iy * p.cv_IW + ix) * p.cv_Cp + ci) * 2
                 : zero;
      }
    } else {
      src = (kin && RO < s.wn) ? s.w0 + (int64_t)RO * p.ldw * 2 + koff : zero;
    }
    __builtin_amdgcn_global_load_lds(src, dst + i * 8192, 16, 0, 0);
  }
}

// Counted wait for this wave's DMA: at most rem (<= 6) half-tiles (2 instructions each) left in flight.
__device__ __forceinline__ void p8_vmwait(int rem) {
  if (rem >= 6) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (rem == 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if (rem == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (rem == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (rem == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (rem == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One phase: P = phase within a block of C::U K tiles (0 .. 4U-1), blk = index of the block.  4U is a multiple of
// S, so the ring slot of every half-tile the phase touches is a compile-time constant.
template <class C, int AMODE, int P, int DIAG>
__device__ __forceinline__ void p8_phase(const GemmArgs& p, char* lds, int blk, int H, int lds_wave, bool k_exact,
                                         const P8Src& s, int w_sc, int a_off0, int a_off1, int b_off0, int b_off1,
                                         f32x4 (&acc)[2][4][2][2], p8b8 (&af)[2][4], p8b8 (&bf)[2][2][2]) {
  constexpr int Q = P & 3;                        // quadrant
  constexpr int MH = (Q == 0 || Q == 1) ? 0 : 1;  // A half
  constexpr int NH = (Q == 1 || Q == 2) ? 1 : 0;  // W half
  // W fragments alternate between the two register sets when BAL: the K tile of parity E keeps its W0 in bf[E] and
  // its W1 in bf[1-E] (W1 is dead after phase 2, so phase 3 refills that set with the next tile's W0)
  constexpr int E = C::BAL ? ((P >> 2) & 1) : 0;
  const int ph = 4 * C::U * blk + P;
  constexpr int H0 = P - Q;  // half-tile A0 of this K tile (relative to the block; slots mod S)
  // ---- fragment reads
  if constexpr ((DIAG & 2) != 0) {  // timing diagnostic: no fragment reads (MFMA on the registers as they are)
#pragma unroll
    for (int kg = 0; kg < 2; ++kg) {
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(af[kg][i]));
#pragma unroll
      for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(bf[NH == 0 ? E : 1 - E][kg][j]));
    }
  } else {
    if constexpr (Q == 0 || Q == 2) {
      const char* hb = lds + ((H0 + (Q == 0 ? 0 : 3)) % C::S) * P8_HALF;
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int i = 0; i < 4; ++i) af[kg][i] = *reinterpret_cast<const p8b8*>(hb + i * 2048 + (kg ? a_off1 : a_off0));
    }
    if constexpr (Q == 0 && !C::BAL) {
      const char* hb = lds + ((H0 + 1) % C::S) * P8_HALF;
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[0][kg][j] = *reinterpret_cast<const p8b8*>(hb + j * 2048 + (kg ? b_off1 : b_off0));
    }
    if constexpr (Q == 1) {
      const char* hb = lds + ((H0 + 2) % C::S) * P8_HALF;
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[1 - E][kg][j] = *reinterpret_cast<const p8b8*>(hb + j * 2048 + (kg ? b_off1 : b_off0));
    }
    if constexpr (Q == 3 && C::BAL) {
      if (ph + 1 < H) {  // W0 of K tile t + 1 (half-tile A0 + 5)
        const char* hb = lds + ((H0 + 5) % C::S) * P8_HALF;
#pragma unroll
        for (int kg = 0; kg < 2; ++kg)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bf[1 - E][kg][j] = *reinterpret_cast<const p8b8*>(hb + j * 2048 + (kg ? b_off1 : b_off0));
      }
    }
  }
  // ---- DMA of half-tile ph + D
  {
    const int h = ph + C::D;
    constexpr int JS = (P + C::D) & 3;
    constexpr bool SKIP = (DIAG & 1) != 0 || ((DIAG & 4) != 0 && (JS == 0 || JS == 3));  // diagnostics
    if (!SKIP && h < H)
      p8_stage<AMODE, JS>(p, lds + ((P + C::D) % C::S) * P8_HALF + lds_wave, h >> 2, k_exact, s, w_sc);
  }
  p8_vmwait(min(C::KF, H - 3 - C::BAL - ph));  // every half-tile <= ph + 2 + BAL landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[MH][i][NH][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kg][i], bf[NH == 0 ? E : 1 - E][kg][j],
                                                                    acc[MH][i][NH][j], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <class C, int AMODE, int DIAG = 0>
__global__ void __launch_bounds__(P8_THREADS, 1) gemm_8p_kernel(GemmArgs p) {
  constexpr int LDS = C::S * P8_HALF;  // the epilogue staging (8 x 32 x 68 fp32) reuses it
  static_assert(8 * 32 * P8_ELD * 4 <= LDS && LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char lds[LDS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int ntn = (p.N + 255) / 256, ntm = (p.M + 255) / 256;
  int tm, tn;
  tile_coords<4>(blockIdx.x, ntm, ntn, tm, tn);
  const int bm = tm * 256, bn = tn * 256;

  // ---- staging geometry: wave instruction i of this wave covers half-tile rows (i*8 + wave)*8 + [0, 8)
  const int lrow = lane >> 3, pos = lane & 7;
  P8Src s;
  const int row0 = wave * 8 + lrow;  // rows row0 + {0, 64, 128, 192} of the tile; row0 & 7 == lrow
  const int w_sc = pos ^ lrow;        // swizzled source chunk (LDS chunk pos holds chunk pos ^ (row & 7))
  s.am = p.M - (bm + row0);
  s.wn = p.N - (bn + row0);
  s.a0 = reinterpret_cast<const char*>(p.A) + ((int64_t)(bm + row0) * p.lda + w_sc * 8) * 2;
  s.w0 = reinterpret_cast<const char*>(p.W) + ((int64_t)(bn + row0) * p.ldw + w_sc * 8) * 2;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if constexpr (AMODE == 1) {
        const int m = min(bm + hh * 128 + i * 64 + row0, p.M - 1);
        const int hw = p.cv_OH * p.cv_OW;
        const int img = m / hw, rem = m - img * hw;
        const int oy = rem / p.cv_OW, ox = rem - oy * p.cv_OW;
        s.cv_base[hh][i] = img * p.cv_IH * p.cv_IW;
        s.cv_iy[hh][i] = oy * p.cv_stride - 1;
        s.cv_ix[hh][i] = ox * p.cv_stride - 1;
      } else {
        s.cv_base[hh][i] = s.cv_iy[hh][i] = s.cv_ix[hh][i] = 0;
      }
    }
  const int nk = (p.K + 63) / 64;
  const int H = 4 * nk;  // half-tiles
  const bool k_exact = (p.K % 64) == 0;
  const int lds_wave = wave * 1024;

  // ---- fragment read offsets inside a half-tile (16-B chunk kg*4 + g of the row, swizzled by row & 7 = r16 & 7)
  const int g = lane >> 4, r16 = lane & 15;
  const int a_row = (wr * 64 + r16) * 128, b_row = (wc * 32 + r16) * 128;
  const int c0 = ((0 * 4 + g) ^ (r16 & 7)) << 4, c1 = ((1 * 4 + g) ^ (r16 & 7)) << 4;
  const int a_off0 = a_row + c0, a_off1 = a_row + c1, b_off0 = b_row + c0, b_off1 = b_row + c1;

  f32x4 acc[2][4][2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][i][b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  p8b8 af[2][4], bf[2][2][2];

  // ---- prologue: half-tiles 0 .. D-1 in flight; 0 and 1 (the first reads) landed everywhere
#pragma unroll
  for (int h = 0; h < C::D; ++h) {
    if (h < H) {
      char* dst = lds + h * P8_HALF + lds_wave;
      switch (h & 3) {
        case 0: p8_stage<AMODE, 0>(p, dst, h >> 2, k_exact, s, w_sc); break;
        case 1: p8_stage<AMODE, 1>(p, dst, h >> 2, k_exact, s, w_sc); break;
        case 2: p8_stage<AMODE, 2>(p, dst, h >> 2, k_exact, s, w_sc); break;
        default: p8_stage<AMODE, 3>(p, dst, h >> 2, k_exact, s, w_sc); break;
      }
    }
  }
  p8_vmwait(min(C::D - 2, H - 2));  // every half-tile <= 1 landed
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  if constexpr (C::BAL && (DIAG & 2) == 0) {  // W0 of K tile 0 (later tiles' W0 is read in phase 3 of the tile before)
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bf[0][kg][j] = *reinterpret_cast<const p8b8*>(lds + 1 * P8_HALF + j * 2048 + (kg ? b_off1 : b_off0));
  }
  if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind
  __builtin_amdgcn_sched_barrier(0);

#define P8_ARGS p, lds, blk, H, lds_wave, k_exact, s, w_sc, a_off0, a_off1, b_off0, b_off1, acc, af, bf
#define P8_TILE(u)                                     \
  if (C::U * blk + (u) < nk) {                         \
    p8_phase<C, AMODE, 4 * (u) + 0, DIAG>(P8_ARGS);    \
    p8_phase<C, AMODE, 4 * (u) + 1, DIAG>(P8_ARGS);    \
    p8_phase<C, AMODE, 4 * (u) + 2, DIAG>(P8_ARGS);    \
    p8_phase<C, AMODE, 4 * (u) + 3, DIAG>(P8_ARGS);    \
  }
  static_assert(C::U <= 10, "P8_TILE list");
  for (int blk = 0; C::U * blk < nk; ++blk) {
    P8_TILE(0) P8_TILE(1)
    if constexpr (C::U > 2) { P8_TILE(2) P8_TILE(3) }
    if constexpr (C::U > 4) { P8_TILE(4) P8_TILE(5) }
    if constexpr (C::U > 6) { P8_TILE(6) P8_TILE(7) }
    if constexpr (C::U > 8) { P8_TILE(8) P8_TILE(9) }
  }
#undef P8_TILE
#undef P8_ARGS
  if (wr == 0) __builtin_amdgcn_s_barrier();  // rejoin: group 1's last MFMA cluster ends at this barrier
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();  // every fragment read retired (lgkmcnt before each MFMA cluster), every DMA landed (vmcnt(0))

  // ---- epilogue: per pass 32 rows x 64 columns (the wave's two 32-column blocks side by side) through LDS
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * P8_ELD;
  const int c4 = (lane & 15) * 4;
  const int n0 = bn + (c4 < 32 ? wc * 32 + c4 : 128 + wc * 32 + c4 - 32);
  const EpiCol ec = epi_col_setup(p, n0);
#pragma unroll
  for (int part = 0; part < 4; ++part) {
    const int mh = part >> 1, i0 = (part & 1) * 2;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            ep[(ii * 16 + g * 4 + r) * P8_ELD + nh * 32 + j * 16 + r16] = acc[mh][i0 + ii][nh][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (n0 < p.N) {
#pragma unroll 2
      for (int pass = 0; pass < 8; ++pass) {
        const int rloc = pass * 4 + g;
        const int m = bm + mh * 128 + wr * 64 + (part & 1) * 32 + rloc;
        if (m >= p.M) break;
        epi_store_row<bf16_t>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * P8_ELD + c4));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

}  // namespace

// cfg: 0 = 10-slot ring (160 KiB) with balanced reads, 1 = 10 slots / W0 read with A0, 2 = 8 slots (128 KiB) /
// balanced, 3 = 8 slots / W0 with A0; 4 = timing diagnostic of cfg 0 without the main-loop DMA, 5 = of cfg 1
// without the main-loop A DMA (both wrong results).
bool launch_gemm_8p(const GemmArgs& a, bool conv, int cfg, hipStream_t stream) {
  const int nblk = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  void (*k)(GemmArgs) = nullptr;
  switch (cfg) {
    case 0: k = conv ? gemm_8p_kernel<P8Cfg<10, 1>, 1> : gemm_8p_kernel<P8Cfg<10, 1>, 0>; break;
    case 1: k = conv ? gemm_8p_kernel<P8Cfg<10, 0>, 1> : gemm_8p_kernel<P8Cfg<10, 0>, 0>; break;
    case 2: k = conv ? gemm_8p_kernel<P8Cfg<8, 1>, 1> : gemm_8p_kernel<P8Cfg<8, 1>, 0>; break;
    case 3: k = conv ? gemm_8p_kernel<P8Cfg<8, 0>, 1> : gemm_8p_kernel<P8Cfg<8, 0>, 0>; break;
    case 4:
      if (conv) return false;
      k = gemm_8p_kernel<P8Cfg<10, 1>, 0, 1>;
      break;
    case 5:  // timing diagnostic of cfg 1 without the main-loop A DMA (wrong results)
      k = conv ? gemm_8p_kernel<P8Cfg<10, 0>, 1, 4> : gemm_8p_kernel<P8Cfg<10, 0>, 0, 4>;
      break;
    default: return false;
  }
  hipLaunchKernelGGL(k, dim3(nblk), dim3(P8_THREADS), 0, stream, a);
  return true;
}

}  // namespace mapa_gemm_impl
