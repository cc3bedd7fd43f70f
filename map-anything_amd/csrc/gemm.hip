// MFMA GEMM / implicit-GEMM convolution for gfx950.
//
//   C[M,N] = A[M,K] * W[N,K]^T   (both operands K-contiguous: nn.Linear / NHWC-conv weight layout)
//
// Replaces every nn.Linear / nn.Conv2d / nn.ConvTranspose2d call of the hot path:
// DINOv2 patch-embed + qkv/proj/fc1/fc2 (vision_transformer.py, layers/block.py), AAT proj_embed/qkv/proj/
// fc1/fc2 (transformer_blocks.py:65-212), the DPT 1x1/3x3/transposed convs (dpt.py:94-311, dpt_block.py:114-255),
// the pose-head 1x1 convs (pose_head.py:18-48) and the dense-rep encoder convs (dense_rep_encoder.py).
//
// Design (MI355X-first):
//  * 256 threads = 4 waves (2x2), block tile 128x128, wave tile 64x64 = 4x4 MFMA 16x16 tiles.
//  * Operands staged HBM -> LDS with global_load_lds (16 B per lane, LDS image lane-linear); the 16-B chunk
//    XOR swizzle (chunk ^ row&7) is applied on the per-lane SOURCE address so that the ds_read_b128 fragment
//    reads are bank-conflict free.  Two LDS stages (double buffer), one barrier per K tile.  The wave index is
//    made provably uniform (readfirstlane) so the LDS-DMA destination (M0) never needs a waterfall loop, and
//    every per-lane source address is precomputed once: the K loop adds a byte offset and issues the DMA.
//  * Rows past M / N are clamped to the last row (their results are never stored); K-tail chunks and conv
//    halo taps read a 16-byte zero page.
//  * Two arithmetic variants behind one loader/epilogue: bf16 operands with v_mfma_f32_16x16x32_bf16
//    (fast path), and fp32 operands with v_mfma_f32_16x16x4_f32 (exact-fp32 "precise" parity mode).
//    Each LDS row is 128 B in both (64 bf16 or 32 fp32 of K), so the staging code is shared.
//  * A operand modes (template): dense rows, or implicit 3x3 convolution (pad 1, stride 1/2) over NHWC.
//  * Epilogue staged through LDS so every lane stores 16 contiguous output bytes: out = resid1 + resid2 +
//    gamma * act(acc + bias); fp32 and/or low-precision and/or ReLU'd low-precision outputs; row-major or
//    pixel-shuffle (ConvTranspose k=s) addressing.
//  * XCD-aware tile order (bijective remap: consecutive tiles share an XCD's L2).
#include <stdlib.h>

#include "gemm_internal.h"

namespace mapa_gemm_impl {

constexpr int BM = 128, BN = 128, NTHREADS = 256;
constexpr int EPI_LD = 68;                           // fp32 row stride of the epilogue staging tile
constexpr int EPI_LDS = 4 * 32 * EPI_LD * 4;         // 4 waves x 32 rows (the wave tile in two halves)

// LDS image of one K tile: BM rows of RB bytes (RB = 128: 64 bf16 / 32 fp32 of K; RB = 64: half that).
// 16-B chunk position = chunk ^ swz(row) (applied on the LDS-DMA source address, read with the same XOR):
// conflict-free ds_read_b128 for the 16x16 fragment pattern at both row sizes.
template <int RB>
__device__ __forceinline__ int swz(int row) {
  if constexpr (RB == 128) return row & 7;
  else return (0x1320 >> (((row >> 2) & 3) * 4)) & 3;  // [0, 2, 3, 1][(row >> 2) & 3]
}

struct TraitsBF16 {
  using T = bf16_t;
  static constexpr int E = 8;    // elements per 16-B chunk
  static constexpr bool F16 = false;
};
struct TraitsF16 {  // fp16 operands (the fp16 autocast recipe): same 16-bit storage and tiles, f16 MFMA
  using T = bf16_t;
  static constexpr int E = 8;
  static constexpr bool F16 = true;
};
struct TraitsF32 {
  using T = float;
  static constexpr int E = 4;
  static constexpr bool F16 = false;
};

template <typename Tr, int RB>
__device__ __forceinline__ void mfma_kgroup(const char* As, const char* Bs, int wm, int wn, int lane, int kg,
                                            f32x4 (&acc)[4][4]) {
  constexpr int ROW_BYTES = RB;
  const int g = lane >> 4, r16 = lane & 15;
  const int chunk = kg * 4 + g;
  if constexpr (sizeof(typename Tr::T) == 2) {
    bf16x8 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ra = wm * 64 + i * 16 + r16;
      a[i] = *reinterpret_cast<const bf16x8*>(As + ra * ROW_BYTES + ((chunk ^ swz<RB>(ra)) << 4));
      const int rb = wn * 64 + i * 16 + r16;
      b[i] = *reinterpret_cast<const bf16x8*>(Bs + rb * ROW_BYTES + ((chunk ^ swz<RB>(rb)) << 4));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32<Tr::F16>(a[i], b[j], acc[i][j]);
  } else {
    f32x4 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ra = wm * 64 + i * 16 + r16;
      a[i] = *reinterpret_cast<const f32x4*>(As + ra * ROW_BYTES + ((chunk ^ swz<RB>(ra)) << 4));
      const int rb = wn * 64 + i * 16 + r16;
      b[i] = *reinterpret_cast<const f32x4*>(Bs + rb * ROW_BYTES + ((chunk ^ swz<RB>(rb)) << 4));
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  }
}


// LDS-DMA of K tile kt into ring slot buf: NLD 16-B chunks of A and of W per thread (lane-linear LDS image).
template <typename Tr, int AMODE, int RB>
__device__ __forceinline__ void stage_tile(const GemmArgs& p, char* lds, int buf, int kt, int lds_base, bool k_exact,
                                           const char* const* a_src, const char* const* w_src, const int* sc,
                                           const int* cv_pix, const int* cv_yx) {
  using T = typename Tr::T;
  constexpr int E = Tr::E;
  constexpr int BK = (RB / 16) * E;
  constexpr int NLD = BM / (4 * (1024 / RB));
  constexpr int TILE_BYTES = BM * RB;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  char* As = lds + buf * 2 * TILE_BYTES;
  char* Bs = As + TILE_BYTES;
  const int64_t koff = (int64_t)kt * BK * sizeof(T);
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const int off = lds_base + i * 4 * 1024;
    const int kc = kt * BK + sc[i] * E;
    const bool kin = k_exact || kc < p.K;
    const char* src;
    if constexpr (AMODE == 0) {
      src = kin ? a_src[i] + koff - split_koff(p, kc, (int)sizeof(T)) : zero;
    } else {
      int tap, ci;
      conv_kmap(p, kc, tap, ci);
      const int ky = tap / 3, kx = tap - ky * 3;
      const bool ok = kin && conv_tap_in(p, cv_yx[i], ky, kx);
      src = ok ? reinterpret_cast<const char*>(p.A) +
                     ((int64_t)(cv_pix[i] + ky * p.cv_IW + kx) * p.cv_Cp + ci) * sizeof(T)
               : zero;
    }
    __builtin_amdgcn_global_load_lds(src, As + off, 16, 0, 0);
    __builtin_amdgcn_global_load_lds(kin ? w_src[i] + koff : zero, Bs + off, 16, 0, 0);
  }
}

// RB: LDS row bytes of a K tile (128 or 64); STAGES: LDS ring depth.  With STAGES > 2 the LDS-DMA for tile
// t+STAGES-1 stays in flight across the barrier of tile t (counted vmcnt + raw s_barrier, no vmcnt(0) drain).
template <typename Tr, int AMODE, int RB, int STAGES>
__global__ void __launch_bounds__(NTHREADS) gemm_kernel(GemmArgs p) {
  using T = typename Tr::T;
  constexpr int E = Tr::E;
  constexpr int CPR = RB / 16;                     // 16-B chunks per LDS row
  constexpr int BK = CPR * E;                      // K elements per tile
  constexpr int RPI = 1024 / RB;                   // rows per 1-KiB wave instruction
  constexpr int NLD = BM / (4 * RPI);              // load instructions per operand per thread
  constexpr int TILE_BYTES = BM * RB;
  constexpr int MAIN_LDS = STAGES * 2 * TILE_BYTES;
  constexpr int LDS_BYTES = MAIN_LDS > EPI_LDS ? MAIN_LDS : EPI_LDS;
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform: no M0 waterfall
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BM - 1) / BM;
  int tm, tn;
  tile_coords<8>(blockIdx.x, ntm, ntn, tm, tn);
  const int bm = tm * BM, bn = tn * BN;

  // ---- per-thread staging geometry: NLD rows (one per load instruction), one fixed source chunk ---------
  const int lrow = lane / CPR, pos = lane % CPR;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  const char* a_src[NLD];
  const char* w_src[NLD];
  int sc[NLD];
  int cv_pix[NLD], cv_yx[NLD];
#pragma unroll
  for (int i = 0; i < NLD; ++i) {
    const int r = (i * 4 + wave) * RPI + lrow;
    sc[i] = pos ^ swz<RB>(r);  // pre-swizzled source chunk
    const int m = min(bm + r, p.M - 1), n = min(bn + r, p.N - 1);
    w_src[i] = reinterpret_cast<const char*>(p.W) + ((int64_t)n * p.ldw + sc[i] * E) * sizeof(T);
    if constexpr (AMODE == 0) {
      a_src[i] = reinterpret_cast<const char*>(p.A) + ((int64_t)m * p.lda + sc[i] * E) * sizeof(T);
    } else {
      const int hw = p.cv_OH * p.cv_OW;
      const int img = m / hw, rem = m - img * hw;
      const int oy = rem / p.cv_OW, ox = rem - oy * p.cv_OW;
      conv_row_setup(p, img, oy, ox, cv_pix[i], cv_yx[i]);
    }
  }
  const int nk = (p.K + BK - 1) / BK;
  const bool k_exact = (p.K % BK) == 0;
  const int lds_base = wave * 1024;


  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (STAGES == 2) {
    stage_tile<Tr, AMODE, RB>(p, lds, 0, 0, lds_base, k_exact, a_src, w_src, sc, cv_pix, cv_yx);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) stage_tile<Tr, AMODE, RB>(p, lds, cur ^ 1, kt + 1, lds_base, k_exact, a_src, w_src, sc, cv_pix, cv_yx);
      const char* As = lds + cur * 2 * TILE_BYTES;
      const char* Bs = As + TILE_BYTES;
#pragma unroll
      for (int kg = 0; kg < CPR / 4; ++kg) mfma_kgroup<Tr, RB>(As, Bs, wm, wn, lane, kg, acc);
      __syncthreads();
    }
  } else {
    // prologue: tiles 0 .. STAGES-2 in flight
#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
      if (s0 < nk) stage_tile<Tr, AMODE, RB>(p, lds, s0, s0, lds_base, k_exact, a_src, w_src, sc, cv_pix, cv_yx);
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt landed (this thread's DMAs): later tiles may stay in flight
      if (kt + STAGES - 2 < nk) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NLD * (STAGES - 2)) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's DMA for tile kt landed; every wave done with tile kt-1
      __builtin_amdgcn_sched_barrier(0);
      if (kt + STAGES - 1 < nk) stage_tile<Tr, AMODE, RB>(p, lds, (kt + STAGES - 1) % STAGES, kt + STAGES - 1, lds_base, k_exact, a_src, w_src, sc, cv_pix, cv_yx);
      const char* As = lds + (kt % STAGES) * 2 * TILE_BYTES;
      const char* Bs = As + TILE_BYTES;
#pragma unroll
      for (int kg = 0; kg < CPR / 4; ++kg) mfma_kgroup<Tr, RB>(As, Bs, wm, wn, lane, kg, acc);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: accumulators -> LDS (per-wave 32 x 64 fp32 half tile) -> 16-B row segments ------------
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * EPI_LD;
  const int c8 = (lane & 7) * 8;  // 8 columns per lane (16-B bf16 stores, epi_store_row8)
  const int n0 = bn + wn * 64 + c8;
  const EpiCol8 ec = epi_col_setup8(p, n0);
  const int g = lane >> 4, c16 = lane & 15;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i * 16 + g * 4 + r) * EPI_LD + j * 16 + c16] = acc[half * 2 + i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (n0 < p.N) {
#pragma unroll 2
      for (int pass = 0; pass < 4; ++pass) {
        const int rloc = pass * 8 + (lane >> 3);
        const int m = bm + wm * 64 + half * 32 + rloc;
        if (m >= p.M) break;
        epi_store_row8<T>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * EPI_LD + c8),
                          *reinterpret_cast<const f32x4*>(ep + rloc * EPI_LD + c8 + 4));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// variant = RB * 10 + STAGES (runtime-selectable for tuning: MAPA_GEMM_VARIANT)
template <typename Tr, int AMODE>
void launch_variant(int variant, int nblk, hipStream_t stream, const GemmArgs& a) {
  void (*k)(GemmArgs);
  switch (variant) {
    case 643: k = gemm_kernel<Tr, AMODE, 64, 3>; break;
    case 644: k = gemm_kernel<Tr, AMODE, 64, 4>; break;
    case 1283: k = gemm_kernel<Tr, AMODE, 128, 3>; break;
    default: k = gemm_kernel<Tr, AMODE, 128, 2>; break;
  }
  hipLaunchKernelGGL(k, dim3(nblk), dim3(NTHREADS), 0, stream, a);
}

// Kernel choice per shape, from tools/kbench.py sweeps of the path's shapes on MI355X (TF/s in DESIGN.md):
//   2568 = 256x256 tile, 1 workgroup/CU, s_setprio around the MFMA bursts (long K, wide convs)
//   2570/2571 = 256x128 tile, 2 workgroups/CU (one tile's epilogue overlaps the other's main loop)
//   2574 = 192x256 tile, 1 workgroup/CU (tile quantization: more tiles in the one wave)
//   2587 = 192x192 tile, 1 workgroup/CU (N = 768: a fuller single wave)
//   1282 / 643 = 128x128 tiles (fp32 parity mode; problems too small to fill the chip with 256-row tiles)
int pick_variant(int dtype, bool conv, int M, int N, int K) {
  if (dtype == MAPA_F32) return (conv || K < 1024) ? 643 : 1282;
  const int64_t big_tiles = (int64_t)((M + 255) / 256) * ((N + 127) / 128);
  if (big_tiles < 256) return (conv || K < 1024) ? 643 : 1282;
  // 192x256 tiles when they fit one wave on the CUs and 256-row tiles leave a quarter of them idle: the path's
  // N <= 1024 linears at 8 views (M = 10960: 58 vs 43 row tiles) and the 74x74 DPT convs
  const int64_t t192 = (int64_t)((M + 191) / 192) * ((N + 255) / 256);
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  // 192x192 when it still fits one wave and N is a multiple of 192 (N = 768 at 8 views: 232 tiles instead of 174
  // of 192x256; kbench aat.proj 29.3 -> 27.3 us, aat.fc2 68.8 -> 62.1)
  const int64_t t192sq = (int64_t)((M + 191) / 192) * ((N + 191) / 192);
  if (!conv && N % 192 == 0 && t192sq <= 256 && t192sq > t192) return 2587;
  if (t192 <= 256 && t256 <= 192 && N >= 256) return 2574;
  if (conv) return N >= 256 ? 2568 : 2571;
  // 256x128 tiles at 2 / CU leaving a nearly empty last round (enc.qkv at 8 views: 1032 tiles on 512 slots) with
  // K >= 1024: 192x256 tiles at 1 / CU (696 tiles, 2.7 rounds) measured 97.2 -> 93.0 us (K = 768: equal)
  if (K >= 1024 && K < 4096 && big_tiles > 512 && big_tiles % 512 != 0 && (big_tiles % 512) * 8 < 512) return 2574;
  if (K >= 4096) return 2568;
  if (N >= 3072 && K <= 1024) return 2570;
  return 2571;
}

// LDS halo-window conv (conv_halo.hip) for stride-1 bf16 convs in the 32-channel-slice K order, when its 16x16-pixel
// blocks fill the CUs (the 148^2 .. 518^2 DPT head convs); the small-image convs keep the implicit GEMM / stream-K.
// Measured (kbench, 8 views): the 128-wide tile at 2 workgroups / CU beats the 256-wide one on every head conv
// (reg2@518 1794 vs 2567 us, rn1@148 652 vs 781) and the implicit GEMM from 148^2 up (2207 / 734 us); at 74^2 and
// below (<= 400 tiles) the implicit GEMM / stream-K stay ahead.  N = 256 (the 148^2 DPT convs) runs 8x16-pixel
// blocks with 256-wide tiles, 2 / CU (rn1@148 643 -> 613 us, l1rn@148 284 -> 260: fewer idle rows at 148, 2.97
// instead of 3.1 rounds); N = 128 keeps 16x16 blocks.
static int g_halo = 1;     // mapa_gemm_tune(MAPA_TUNE_CONV_HALO, .)
static int g_tail_sk = 0;  // mapa_gemm_tune(MAPA_TUNE_TAIL_STREAMK, .)
static bool pick_halo(int M, int N, int OH, int OW, int kb) {
  if (kb != 32 || !g_halo || N % 128 != 0) return false;
  const int64_t blocks = (int64_t)(M / (OH * OW)) * ((OH + 15) / 16) * ((OW + 15) / 16);
  // >= 400 tiles of 128 columns: from the 74^2 DPT convs up (8 views: 400 tiles; kbench after the round-3 window
  // swizzle: rn2@74 167.6 -> 149.9 us, l2rn@74 140.7 -> 121.1 vs the implicit GEMM)
  return blocks * (N / 128) >= 400;
}

// 8-row blocks with 256-wide tiles only where they cover fewer idle rows than 16-row blocks (148^2: 152 vs 160
// rows; 74^2: 80 either way, and there the 128-wide 16x16 tile is faster: rn2@74 149.9 vs 156.4 us)
static bool halo_rows8(const GemmArgs& a) {
  return a.N % 256 == 0 && (g_halo == 1 || g_halo == 3) && ((a.cv_OH + 7) / 8) * 8 < ((a.cv_OH + 15) / 16) * 16;
}

// Flat-raster halo conv with split K (conv_halo.hip FLAT) for the stride-1 convs too small for 16x16 blocks (the
// 19^2 / 37^2 DPT convs: 26-144 tiles of 16x16 blocks, 41-65 % of their pixels idle), which the stream-K implicit
// GEMM ran before.  Returns the K part count, 0 = not this kernel.
static int g_halo_split = 0;  // mapa_gemm_tune(MAPA_TUNE_HALO_SPLIT, .): 0 = automatic part count
static int g_tile_gm = 4;     // mapa_gemm_tune(MAPA_TUNE_TILE_GROUP, .): tile rows per group of gemm_big_kernel
static int g_ln_fuse = -1;    // mapa_gemm_tune(MAPA_TUNE_LN_FUSE, .) / env MAPA_LN_FUSE (A/B switch); -1: env not read

// The residual linears whose automatic tile choice is the 192-row data-parallel kernel (the path's proj / fc2 at
// 8 views) fuse a requested output LayerNorm (launch_gemm_big_ln); everything else runs it as its own launch.
// g_ln_fuse 2 (default): every qualifying bf16 residual linear on the fused kernel whatever its automatic tile choice
// (the batched-scene shapes too: more bands than the device holds at once run as several launches of co-resident
// bands, launch_gemm_big_ln; B = 2 x 8 views 254.4 / 256.9 vs 251.4 / 250.8 views/s in mode 1, the B = 1 launches
// identical); 1 = only where the automatic choice is the 192-row kernel; 0 = GEMM, then mapa_layernorm.
static int pick_ln_fused(const mapa_gemm_desc* d, int variant, int sk) {
  if (g_ln_fuse < 0) g_ln_fuse = getenv("MAPA_LN_FUSE") ? atoi(getenv("MAPA_LN_FUSE")) : 2;
  if (!d->ln_out || !g_ln_fuse || d->dtype != MAPA_BF16 || d->a_mode != MAPA_A_DENSE || d->a_split || sk) return 0;
  if (g_ln_fuse == 2) return d->N % 256 == 0 ? 14 : d->N % 192 == 0 ? 15 : 0;
  if (g_ln_fuse == 3) return d->N % 256 == 0 ? 14 : 0;  // A/B: the 192x256 form only (whole model: = mode 2)
  return variant == 2574 ? 14 : variant == 2587 ? 15 : 0;
}
static int pick_flat(const GemmArgs& a) {
  if (g_halo != 1 || pick_halo(a.M, a.N, a.cv_OH, a.cv_OW, a.cv_kb)) return 0;
  return conv_halo_flat_split(a, gemm_streamk_slots(0), g_halo_split);
}

// Persistent register-epilogue kernel (gemm_pers.hip) for the dense transformer linears: mapa_gemm_tune(MAPA_TUNE_PERS,
// .) / env MAPA_GEMM_PERS: 0 = off, 1 = on with the automatic tile shape, 2 + s = tile shape s; -1: env not read.
static int g_pers = -1;
static int pers_mode() {
  if (g_pers < 0) g_pers = getenv("MAPA_GEMM_PERS") ? atoi(getenv("MAPA_GEMM_PERS")) : 1;
  return g_pers;
}

// The LayerNorm-fused residual linears on the persistent kernel (launch_gemm_pers_ln) instead of gemm_big's LNF tiles:
// mapa_gemm_tune(MAPA_TUNE_PERS_LN, .) / env MAPA_GEMM_PERS_LN, 1 = always, 2 = where K <= 1024, 0 = never (default:
// in isolation the persistent form was faster on the proj linears — enc.proj 45.5 vs 48.2 us, aat.proj 36.9 vs 37.8 —
// and slower at K = 3072 / 4096, aat.fc2 76.7 vs 73.4, but inside the model mode 2 measured 321.8 vs 323.5 views/s,
// profiles/r6/ln_forms_ab.txt); -1: env not read.
static int g_pers_ln = -1;
static int pers_ln_mode() {
  if (g_pers_ln < 0) g_pers_ln = getenv("MAPA_GEMM_PERS_LN") ? atoi(getenv("MAPA_GEMM_PERS_LN")) : 0;
  return g_pers_ln;
}
static bool pers_ln_takes(int K) { return pers_ln_mode() == 1 || (pers_ln_mode() == 2 && K <= 1024); }

static int g_forced = -1;  // -1: not read yet; 0: automatic; else a kernel variant code (tuning / tests)

static int forced_variant() {
  if (g_forced < 0) {
    const char* ev = getenv("MAPA_GEMM_VARIANT");
    g_forced = ev ? atoi(ev) : 0;
  }
  return g_forced;
}

// Stream-K variants (2580 + v) are chosen only when the caller passes a workspace; 0 = none.  None is picked
// automatically: on the path shapes the data-parallel kernels measured faster (2580/2581), or equal within noise at
// the bench level (2582, tail-only stream-K: every full wave of 256x128 tiles data-parallel, only the last partial
// wave split; enc.qkv 108 -> 97 us and aat.fc1 77 -> 75 us in isolation, 266 vs 266 views/s in the bench).
// Automatic stream-K: problems with fewer 256x128 tiles than CUs and a long K (the fp32-exact split-precision DPT
// convs at 19x19 and 37x37: K = 27*C = 6912..20736, M = views*361 or views*1369) leave most of the chip idle in
// the data-parallel schedule; splitting K over the persistent grid measured 1.5-3.2x faster (kbench, 8 views:
// layer4_rn 392 -> 122 us, input_process.3 conv 394 -> 177, layer3_rn 194 -> 102, refinenet3/4 convs 142 -> 100).
// The stride-1 ones among them now run the flat-raster halo conv (pick_flat, checked first in mapa_gemm); the
// stride-2 input_process.3 conv stays here.
int pick_streamk(int dtype, bool conv, int M, int N, int K) {
  const int f = forced_variant();
  if (f) return f >= 2580 && f <= 2582 ? f : 0;
  if (dtype != MAPA_BF16 && dtype != MAPA_F16) return 0;
  const int64_t big_tiles = (int64_t)((M + 255) / 256) * ((N + 127) / 128);
  // 256x256 stream-K tiles from N = 512 up at a few thousand rows (the stride-2 768-channel DPT conv at 37 -> 19,
  // M = views * 361: 244 -> 152 us); the 224^2 geometric encoders (M = views * 256) keep 256x128
  // (convs always take the 256x256 form: the 256x128 conv instantiation at 2 workgroups / CU does not fit its
  // 128-VGPR budget without scratch)
  if (big_tiles < 256 && K >= 4096) return conv || (N >= 512 && M >= 2048) ? 2581 : 2580;
  // tail-only stream-K where the 256x128 data-parallel schedule leaves a nearly empty last wave (enc.qkv / aat.fc1
  // at 8 views: 1032 tiles on 512 slots -> a third wave of 8 tiles)
  if (g_tail_sk && !conv) {
    const int slots = gemm_streamk_slots(2);
    const int64_t rem = big_tiles % slots;
    if (big_tiles > slots && rem > 0 && rem * 8 < slots) return 2582;
  }
  return 0;
}

}  // namespace mapa_gemm_impl
using namespace mapa_gemm_impl;

static int gemm_args(const mapa_gemm_desc* d, GemmArgs& a) {
  MAPA_CHECK_ARG(d != nullptr, "mapa_gemm: null descriptor");
  MAPA_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0, "mapa_gemm: bad shape M=%d N=%d K=%d", d->M, d->N, d->K);
  MAPA_CHECK_ARG(d->dtype == MAPA_BF16 || d->dtype == MAPA_F32 || d->dtype == MAPA_F16,
                 "mapa_gemm: dtype must be bf16, f16 or f32");
  // fp16: the transformer linears of the fp16 autocast recipe, and the TF32-equivalent heads (MAPA_F16X2 operands:
  // split rows [hi | lo] read as a plain 2C-wide f16 operand against weights [w | w]; out_s3 then writes f16 splits)
  MAPA_CHECK_ARG(d->dtype != MAPA_F16 || !d->a_split, "mapa_gemm: a_split is the bf16 split (MAPA_BF16X3) only");
  const int E = d->dtype == MAPA_F32 ? 4 : 8;
  MAPA_CHECK_ARG(d->K % E == 0, "mapa_gemm: K=%d must be a multiple of %d", d->K, E);
  MAPA_CHECK_ARG(d->A && d->W, "mapa_gemm: null operand");
  MAPA_CHECK_ARG(d->dtype != MAPA_F32 || (!d->out_s3 && !d->out_s3_relu),
                 "mapa_gemm: split outputs need dtype bf16 (MAPA_BF16X3 rows) or f16 (MAPA_F16X2 rows)");
  a.lp_f16 = d->dtype == MAPA_F16 ? 1 : 0;
  MAPA_CHECK_ARG(d->act >= MAPA_ACT_NONE && d->act <= MAPA_ACT_GELU_POST, "mapa_gemm: bad act %d", d->act);
  MAPA_CHECK_ARG(d->act != MAPA_ACT_GELU_POST || !d->gamma, "mapa_gemm: GELU_POST takes no gamma");
  if (d->a_mode == MAPA_A_CONV3X3) {
    MAPA_CHECK_ARG(d->conv_C % E == 0 && d->K == 9 * d->conv_C, "mapa_gemm: conv K=%d must be 9*C (C=%d, C%%%d==0)",
                   d->K, d->conv_C, E);
    MAPA_CHECK_ARG(d->conv_stride == 1 || d->conv_stride == 2, "mapa_gemm: conv stride must be 1 or 2");
    const int oh = (d->conv_IH + 2 - 3) / d->conv_stride + 1, ow = (d->conv_IW + 2 - 3) / d->conv_stride + 1;
    MAPA_CHECK_ARG(oh == d->conv_OH && ow == d->conv_OW, "mapa_gemm: conv out %dx%d != expected %dx%d",
                   d->conv_OH, d->conv_OW, oh, ow);
    MAPA_CHECK_ARG((int64_t)d->conv_OH * d->conv_OW > 0 && d->M % (d->conv_OH * d->conv_OW) == 0,
                   "mapa_gemm: conv M must be images * OH * OW");
    MAPA_CHECK_ARG(d->conv_kblock == 0 || (d->conv_kblock > 0 && d->conv_kblock % 8 == 0 && d->conv_C % d->conv_kblock == 0),
                   "mapa_gemm: conv_kblock=%d must be 0 or a multiple of 8 dividing conv_C=%d", d->conv_kblock,
                   d->conv_C);
  } else {
    MAPA_CHECK_ARG(d->a_mode == MAPA_A_DENSE, "mapa_gemm: bad a_mode");
    MAPA_CHECK_ARG((d->a_split || d->lda >= d->K) && d->lda % E == 0, "mapa_gemm: lda must be >= K and keep 16-B rows");
  }
  MAPA_CHECK_ARG(d->ldw >= d->K && d->ldw % E == 0, "mapa_gemm: ldw must be >= K and keep 16-B rows");
  if (d->a_split) {
    const int lw = d->a_mode == MAPA_A_CONV3X3 ? d->conv_C : d->K;  // logical [hi | hi | lo] width
    MAPA_CHECK_ARG(d->dtype == MAPA_BF16 && lw % 3 == 0 && (lw / 3) % 8 == 0,
                   "mapa_gemm: a_split needs bf16 and a logical width 3*C with C %% 8 == 0 (got %d)", lw);
    MAPA_CHECK_ARG(d->a_mode == MAPA_A_CONV3X3 || d->lda >= 2 * (d->K / 3),
                   "mapa_gemm: a_split lda must be >= the stored width 2K/3");
  }
  if (d->out_mode == MAPA_OUT_PIXSHUF) {
    MAPA_CHECK_ARG(d->ps_s > 0 && d->ps_cout > 0 && d->N == d->ps_s * d->ps_s * d->ps_cout &&
                       d->M % (d->ps_h * d->ps_w) == 0 && d->ps_cout % 4 == 0,
                   "mapa_gemm: bad pixel-shuffle geometry");
  } else {
    MAPA_CHECK_ARG(d->ldo >= d->N, "mapa_gemm: ldo < N");
  }
  a.A = d->A; a.lda = d->lda; a.W = d->W; a.ldw = d->ldw;
  a.M = d->M; a.N = d->N; a.K = d->K;
  a.cv_C = d->conv_C; a.cv_IH = d->conv_IH; a.cv_IW = d->conv_IW; a.cv_OH = d->conv_OH; a.cv_OW = d->conv_OW;
  a.cv_stride = d->conv_stride;
  a.sp_half = 0x7fffffff;
  a.cv_Cp = d->conv_C;
  a.cv_kb = d->a_mode == MAPA_A_CONV3X3 ? d->conv_kblock : 0;
  if (d->a_split) {
    a.sp_half = (d->a_mode == MAPA_A_CONV3X3 ? d->conv_C : d->K) / 3;
    if (d->a_mode == MAPA_A_CONV3X3) a.cv_Cp = 2 * a.sp_half;
  }
  a.bias = d->bias; a.bias_mod = d->bias_mod > 0 ? d->bias_mod : d->N;
  a.gamma = d->gamma; a.act = d->act;
  a.resid1 = d->resid1; a.resid2 = d->resid2;
  a.out_f32 = d->out_f32; a.out_lp = d->out_lp; a.out_lp_relu = d->out_lp_relu; a.ldo = d->ldo;
  a.out_s3 = d->out_s3; a.out_s3_relu = d->out_s3_relu;
  a.out_mode = d->out_mode; a.ps_s = d->ps_s; a.ps_h = d->ps_h; a.ps_w = d->ps_w; a.ps_cout = d->ps_cout;
  a.vec_ok = (d->N % 4 == 0) && (d->out_mode == MAPA_OUT_PIXSHUF || d->ldo % 4 == 0);
  a.tile_gm = g_tile_gm;
  a.fault = fault_word();
  if (d->ln_out) {
    MAPA_CHECK_ARG(d->ln_w && d->ln_b && d->out_f32 && d->out_mode == MAPA_OUT_ROWMAJOR,
                   "mapa_gemm: ln_out needs ln_w, ln_b and a row-major out_f32");
    MAPA_CHECK_ARG(d->N == 256 || d->N == 512 || d->N == 768 || d->N == 1024, "mapa_gemm: LayerNorm width N=%d", d->N);
    MAPA_CHECK_ARG(d->ln_ldo >= d->N && d->ln_ldo % 4 == 0 && d->ldo % 4 == 0,
                   "mapa_gemm: ln_ldo must be >= N and ln_ldo, ldo multiples of 4");
  }
  a.ln_w = d->ln_w; a.ln_b = d->ln_b; a.ln_eps = d->ln_eps; a.ln_out = d->ln_out; a.ln_ldo = d->ln_ldo;
  a.ln_ctr = nullptr; a.ln_stats = nullptr;
  a.stagger = 0;
  MAPA_CHECK_ARG(a.vec_ok || d->out_mode == MAPA_OUT_ROWMAJOR, "mapa_gemm: pixel shuffle needs N %% 4 == 0");
  return 0;
}

extern "C" int mapa_gemm(const mapa_gemm_desc* d, hipStream_t stream) {
  GemmArgs a;
  if (int rc = gemm_args(d, a)) return rc;
  MAPA_CHECK_ARG(d->out_f32 || d->out_lp || d->out_lp_relu || d->out_s3 || d->out_s3_relu, "mapa_gemm: no output");
  const int nblk = ((d->M + BM - 1) / BM) * ((d->N + BN - 1) / BN);
  const bool conv = d->a_mode == MAPA_A_CONV3X3;
  // Tile-pipeline variant (RB*10 + STAGES).  Measured on MI355X (tools/kbench.py): 64-B rows x 3 stages (occupancy
  // 3) wins for the implicit convs and K < 1024; 128-B rows x 2 stages for the K >= 1024 linears.
  const int forced = forced_variant();
  const int variant = forced ? forced : pick_variant(d->dtype, conv, d->M, d->N, d->K);
  const bool lp16 = d->dtype == MAPA_BF16 || d->dtype == MAPA_F16;
  const int sk = lp16 ? pick_streamk(d->dtype, conv, d->M, d->N, d->K) : 0;
  const bool halo = conv && lp16 &&
                    (forced ? (forced >= 2584 && forced <= 2586) || forced == 2588
                            : pick_halo(a.M, a.N, a.cv_OH, a.cv_OW, a.cv_kb));
  const int flat = !conv || !lp16 ? 0
                   : forced ? (forced == 2589 ? conv_halo_flat_split(a, gemm_streamk_slots(0), g_halo_split) : 0)
                            : pick_flat(a);
  const int lnf = pick_ln_fused(d, variant, sk);
  if (lnf && pers_ln_takes(d->K) && !forced &&
      launch_gemm_pers_ln(a, d->workspace, d->workspace_bytes, gemm_streamk_slots(1), stream)) {
    MAPA_CHECK_LAUNCH("mapa_gemm (LayerNorm fused, persistent)");
    return 0;
  }
  if (lnf && launch_gemm_big_ln(a, lnf, d->workspace, d->workspace_bytes, stream)) {
    MAPA_CHECK_LAUNCH("mapa_gemm (LayerNorm fused)");
    return 0;  // launched (residual linear + the LayerNorm of its output rows)
  }
  const bool pers_forced = forced >= 2600 && forced <= 2608;
  const bool pers_auto = !forced && pers_mode() && !sk && ((variant >= 2560 && variant <= 2574) || variant == 2587);
  if (flat && launch_conv_halo_flat(a, flat, d->workspace, d->workspace_bytes, GEMM_TICKET_BYTES, stream)) {
    // launched (flat-raster halo conv, split K)
  } else if (!conv && lp16 && !d->ln_out && (pers_forced || pers_auto) &&
             launch_gemm_pers(a, pers_forced ? forced - 2600 : pers_mode() >= 2 ? pers_mode() - 2 : -1,
                              gemm_streamk_slots(1), stream)) {
    // launched (persistent register-epilogue kernel)
  } else if (sk && launch_gemm_streamk(a, conv, sk - 2580, d->workspace, d->workspace_bytes, stream)) {
    // launched (persistent stream-K grid)
  } else if (halo && (forced ? launch_conv_halo(a, forced == 2585 || forced == 2588 ? 256 : 128, stream,
                                                forced == 2588 ? 8 : 16)
                              : launch_conv_halo(a, halo_rows8(a) ? 256 : 128, stream, halo_rows8(a) ? 8 : 16))) {
    // launched (LDS halo-window conv)
  } else if (d->dtype != MAPA_F32 && ((variant >= 2560 && variant <= 2574) || variant == 2587 ||
                                      (variant >= 2591 && variant <= 2596)) &&
             launch_gemm_big(a, conv, variant == 2587 ? 15 : variant >= 2591 ? variant - 2575 : variant - 2560,
                             stream)) {
    // launched (bf16, or f16 for the tile kernels that carry an fp16 instantiation)
  } else if (d->dtype == MAPA_F16) {
    if (conv) launch_variant<TraitsF16, 1>(variant >= 2560 ? 643 : variant, nblk, stream, a);
    else launch_variant<TraitsF16, 0>(variant >= 2560 ? 1282 : variant, nblk, stream, a);
  } else if (d->dtype == MAPA_BF16) {
    if (conv) launch_variant<TraitsBF16, 1>(variant, nblk, stream, a);
    else launch_variant<TraitsBF16, 0>(variant, nblk, stream, a);
  } else {
    if (conv) launch_variant<TraitsF32, 1>(variant, nblk, stream, a);
    else launch_variant<TraitsF32, 0>(variant, nblk, stream, a);
  }
  MAPA_CHECK_LAUNCH("mapa_gemm");
  if (d->ln_out)  // the requested LayerNorm as its own launch (same stream, after the GEMM)
    return mapa_layernorm(d->out_f32, d->ldo, d->M, d->N, d->ln_w, d->ln_b, d->ln_eps, nullptr, d->ln_out,
                          d->dtype, d->ln_ldo, 0, 0, 0, stream);
  return 0;
}

extern "C" int mapa_regressor_head_out(const mapa_gemm_desc* d, const float* w6, const float* b6,
                                       const float* pose_out, const float* scale, int views_per_scale,
                                       float* pts3d, float* pts3d_cam,
                                       float* rays, float* depth, float* conf, float* logits, uint8_t* mask,
                                       hipStream_t stream) {
  GemmArgs a;
  if (int rc = gemm_args(d, a)) return rc;
  MAPA_CHECK_ARG(w6 && b6 && pose_out && scale && pts3d && pts3d_cam && rays && depth && conf && logits && mask,
                 "mapa_regressor_head_out: null output or parameter");
  MAPA_CHECK_ARG(views_per_scale > 0, "mapa_regressor_head_out: views_per_scale %d must be > 0", views_per_scale);
  MAPA_CHECK_ARG((d->dtype == MAPA_BF16 || d->dtype == MAPA_F16) && d->a_mode == MAPA_A_CONV3X3 && !d->out_f32 &&
                     !d->out_lp &&
                     !d->out_lp_relu && !d->out_s3 && !d->out_s3_relu && !d->resid1 && !d->resid2 && !d->gamma,
                 "mapa_regressor_head_out: needs a bf16 / f16 3x3 conv descriptor without other outputs");
  MAPA_CHECK_ARG(launch_conv_halo_headout(a, w6, b6, pose_out, scale, views_per_scale, pts3d, pts3d_cam, rays, depth, conf, logits,
                                          mask, stream),
                 "mapa_regressor_head_out: conv must be stride 1, conv_kblock 32, N 128, ReLU with bias");
  MAPA_CHECK_LAUNCH("mapa_regressor_head_out");
  return 0;
}

extern "C" int mapa_gemm_tune(int key, int value) {
  MAPA_CHECK_ARG(key == MAPA_TUNE_CONV_HALO || key == MAPA_TUNE_TAIL_STREAMK || key == MAPA_TUNE_HALO_SPLIT ||
                     key == MAPA_TUNE_TILE_GROUP || key == MAPA_TUNE_LN_FUSE || key == MAPA_TUNE_LN_SPIN ||
                     key == MAPA_TUNE_LN_TEST_SKIP || key == MAPA_TUNE_DIAG_GRID || key == MAPA_TUNE_PERS ||
                     key == MAPA_TUNE_PERS_LN || key == MAPA_TUNE_PERS_STAGGER,
                 "mapa_gemm_tune: unknown key %d", key);
  MAPA_CHECK_ARG((key != MAPA_TUNE_LN_SPIN && key != MAPA_TUNE_LN_TEST_SKIP) || value >= 0,
                 "mapa_gemm_tune: negative value %d", value);
  if (key == MAPA_TUNE_LN_SPIN) {
    ln_set_spin((unsigned)value);
    return 0;
  }
  if (key == MAPA_TUNE_LN_TEST_SKIP) {
    ln_arm_test_skip(value);
    return 0;
  }
  if (key == MAPA_TUNE_PERS_STAGGER) {
    MAPA_CHECK_ARG(value >= -1 && value <= 100000, "mapa_gemm_tune: stagger %d", value);
    pers_set_stagger(value);
    return 0;
  }
  if (key == MAPA_TUNE_PERS_LN) {
    g_pers_ln = value == 2 ? 2 : value ? 1 : 0;
    return 0;
  }
  if (key == MAPA_TUNE_PERS) {
    MAPA_CHECK_ARG(value >= 0 && value <= 8, "mapa_gemm_tune: persistent mode %d", value);
    g_pers = value;
    return 0;
  }
  if (key == MAPA_TUNE_DIAG_GRID) {
    MAPA_CHECK_ARG(value >= 0, "mapa_gemm_tune: grid %d", value);
    diag_set_grid(value);
    return 0;
  }
  MAPA_CHECK_ARG(key != MAPA_TUNE_HALO_SPLIT || (value >= 0 && value <= 64), "mapa_gemm_tune: split %d", value);
  MAPA_CHECK_ARG(key != MAPA_TUNE_TILE_GROUP || (value >= 0 && value <= 1024), "mapa_gemm_tune: group %d", value);
  if (key == MAPA_TUNE_CONV_HALO) g_halo = value == 2 || value == 3 ? value : value ? 1 : 0;
  else if (key == MAPA_TUNE_HALO_SPLIT) g_halo_split = value;
  else if (key == MAPA_TUNE_TILE_GROUP) g_tile_gm = value ? value : 4;
  else if (key == MAPA_TUNE_LN_FUSE) g_ln_fuse = value >= 2 && value <= 3 ? value : value ? 1 : 0;
  else g_tail_sk = value ? 1 : 0;
  return 0;
}

extern "C" int mapa_gemm_set_variant(int variant) {
  MAPA_CHECK_ARG(variant == 0 || variant == 643 || variant == 644 || variant == 1282 || variant == 1283 ||
                     (variant >= 2560 && variant <= 2574) || (variant >= 2580 && variant <= 2582) ||
                     (variant >= 2584 && variant <= 2589) || (variant >= 2591 && variant <= 2596) ||
                     (variant >= 2600 && variant <= 2608),
                 "mapa_gemm_set_variant: unknown variant %d", variant);
  g_forced = variant;
  return 0;
}

extern "C" int64_t mapa_gemm_workspace_bytes(const mapa_gemm_desc* d) {
  if (!d || (d->dtype != MAPA_BF16 && d->dtype != MAPA_F16) || d->M <= 0 || d->N <= 0 || d->K <= 0) return 0;
  if (d->ln_out && !forced_variant()) {
    const bool conv = d->a_mode == MAPA_A_CONV3X3;
    const int lnf = pick_ln_fused(d, pick_variant(d->dtype, conv, d->M, d->N, d->K),
                                  pick_streamk(d->dtype, conv, d->M, d->N, d->K));
    const int64_t b = lnf ? ln_stats_bytes(d->M, d->N, lnf) : -1;
    if (b >= 0) return GEMM_TICKET_BYTES + b;
  }
  if (d->a_mode == MAPA_A_CONV3X3) {
    GemmArgs a;
    if (gemm_args(d, a) != 0) return 0;  // a bad descriptor is reported by mapa_gemm itself
    const int forced = forced_variant();
    const int flat = forced ? (forced == 2589 ? conv_halo_flat_split(a, gemm_streamk_slots(0), g_halo_split) : 0)
                            : pick_flat(a);
    if (flat) {
      const int64_t b = conv_halo_flat_workspace_bytes(a, flat, GEMM_TICKET_BYTES);
      if (b >= 0) return b;
    }
  }
  const int sk = pick_streamk(d->dtype, d->a_mode == MAPA_A_CONV3X3, d->M, d->N, d->K);
  return sk ? streamk_workspace_bytes(d->M, d->N, sk - 2580) : 0;
}
