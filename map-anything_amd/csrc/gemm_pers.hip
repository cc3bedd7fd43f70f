// Persistent bf16 / fp16 GEMM for the transformer linears (gfx950):
//
//   C[M,N] = A[M,K] * W[N,K]^T with the two transformer-block epilogues (gemm_internal.h epi_mode):
//     mode 1: act(acc + bias) -> 16-bit out_lp      (DINOv2 / AAT qkv, fc1 + GELU)
//     mode 2: out_f32 = resid1 + gamma * (acc + bias), in place   (attn proj, fc2 residual updates)
//   dinov2 layers/block.py:93-118, uniception transformer_blocks.py:65-212.
//
// Why a second data-parallel kernel beside gemm_big (profiles/r6/gemm_breakdown.json, MI355X): on the path shapes the
// 256-row kernels spend 23-32 % of their time in the epilogue (LDS round trip of the fp32 accumulators, wave barriers,
// then the stores, with nothing overlapping them) and 16-32 % in a partly empty last wave of tiles.  Here:
//  * the MFMA operands are swapped (W fragment first), so each lane's accumulator holds 4 consecutive COLUMNS of one
//    output row: the epilogue goes straight from registers to 8-byte (16-bit outputs) / 16-byte (fp32) global stores,
//    no LDS, no barriers;
//  * the grid is persistent (resident workgroups only): as soon as a tile's last K step has been read from LDS, the
//    LDS-DMA prologue of the workgroup's NEXT tile is issued, and the epilogue's VALU work and stores of the finished
//    tile run while that DMA is in flight;
//  * the tile shape is chosen per problem from the round count (launch_gemm_pers), so a near-empty last round
//    (e.g. 1032 tiles on 512 slots) is traded for a fuller one.
// Main loop as gemm_big's: LDS-DMA (global_load_lds_dwordx4) into a ring of K tiles with the 16-B chunk XOR swizzle
// on the source address, conflict-free ds_read_b128 fragments, counted vmcnt + raw s_barrier, 16x16x32 MFMA.
#include <stdlib.h>

#include <algorithm>

#include "gemm_internal.h"

namespace mapa_gemm_impl {
namespace {

constexpr int PTHREADS = 512;
constexpr int LN_MAX_NTN_P = 8;  // column tiles per band the LayerNorm merge holds (= gemm_big's LN_MAX_NTN: one
                                 // workspace layout for both LayerNorm-fused kernels)
typedef unsigned int u32x4p __attribute__((ext_vector_type(4)));

template <int BM, int BN, int RB, int WM, int NW = 8>
struct PCfg {
  static constexpr int WN = NW / WM;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int CPR = RB / 16;  // 16-B chunks per LDS row
  static constexpr int BK = CPR * 8;   // K per tile
  static constexpr int KG = CPR / 4;   // 32-deep MFMA k-groups per tile
  static constexpr int RPI = 1024 / RB;
  static constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB, STAGE = A_BYTES + B_BYTES;
  static constexpr int NLA = BM / (NW * RPI), NLB = BN / (NW * RPI);
  static_assert(BM % (NW * RPI) == 0 && BN % (NW * RPI) == 0, "whole 1-KiB wave instructions per operand");
  static_assert(TM % 16 == 0 && TN % 16 == 0, "16x16 MFMA tiles");
};

template <int RB>
__device__ __forceinline__ int pswz(int row) {
  if constexpr (RB == 128) return row & 7;
  else return (0x1320 >> (((row >> 2) & 3) * 4)) & 3;  // [0, 2, 3, 1][(row >> 2) & 3]
}

// Per-tile staging state: the per-lane source rows (clamped past M / N; their results are never stored).  TAG makes
// every kernel instantiation use a Src type of its own: with two kernels sharing one Src instantiation, hipcc (ROCm
// 7.2) emitted the host-side launch stubs of the first kernel only (the others' stayed undefined at link time).
template <int BM, int BN, int RB, int WM, int TAG, int NW = 8>
struct Src {
  using C = PCfg<BM, BN, RB, WM, NW>;
  // per-lane byte offsets of this lane's source rows from A / W (rows clamped to M-1 / N-1); the K offset of a tile
  // rides in the buffer load's soffset, so no 64-bit per-lane pointer lives across the K loop (fast path: K a
  // multiple of BK and both operands under 2 GiB — the path's linears; otherwise the zero-page form below)
  uint32_t ao[C::NLA], wo[C::NLB];
  __device__ __forceinline__ void setup(const GemmArgs& p, int bm, int bn, int wave, int lane) {
    const int lrow = lane / C::CPR, pos = lane % C::CPR;
#pragma unroll
    for (int i = 0; i < C::NLA; ++i) {
      const int r = (i * NW + wave) * C::RPI + lrow;
      const int m = min(bm + r, p.M - 1);
      ao[i] = (uint32_t)(((int64_t)m * p.lda + (pos ^ pswz<RB>(r)) * 8) * 2);
    }
#pragma unroll
    for (int i = 0; i < C::NLB; ++i) {
      const int r = (i * NW + wave) * C::RPI + lrow;
      const int n = min(bn + r, p.N - 1);
      wo[i] = (uint32_t)(((int64_t)n * p.ldw + (pos ^ pswz<RB>(r)) * 8) * 2);
    }
  }
  // LDS-DMA of K tile kt into ring slot `slot`
  __device__ __forceinline__ void stage(const GemmArgs& p, char* lds, int slot, int kt, int lds_wave, bool fast,
                                        int wave, int lane) const {
    char* As = lds + slot * C::STAGE;
    char* Bs = As + C::A_BYTES;
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    if (fast) {
      const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, 0x7fffffff, 0x00020000);
      const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)p.W, 0, 0x7fffffff, 0x00020000);
      const int koff = kt * C::BK * 2;
#pragma unroll
      for (int i = 0; i < C::NLA; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(As + lds_wave + i * NW * 1024), 16, (int)ao[i], koff,
                                                 0, 0);
#pragma unroll
      for (int i = 0; i < C::NLB; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(Bs + lds_wave + i * NW * 1024), 16, (int)wo[i], koff,
                                                 0, 0);
      return;
    }
    // K-tail form: the same offsets as plain pointers, the chunks past K from the zero page (the empty asm hides the
    // offsets' loop invariance, so no 64-bit pointer per piece is hoisted into registers across the K loop)
    const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
    const int lrow = lane / C::CPR, pos = lane % C::CPR;
    const int64_t koff = (int64_t)kt * C::BK * 2;
#pragma unroll
    for (int i = 0; i < C::NLA; ++i) {
      const int r = (i * NW + wave) * C::RPI + lrow;
      const bool kin = kt * C::BK + (pos ^ pswz<RB>(r)) * 8 < p.K;
      uint32_t off = ao[i];
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_global_load_lds(kin ? reinterpret_cast<const char*>(p.A) + off + koff : zero,
                                       As + lds_wave + i * NW * 1024, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < C::NLB; ++i) {
      const int r = (i * NW + wave) * C::RPI + lrow;
      const bool kin = kt * C::BK + (pos ^ pswz<RB>(r)) * 8 < p.K;
      uint32_t off = wo[i];
      asm volatile("" : "+v"(off));
      __builtin_amdgcn_global_load_lds(kin ? reinterpret_cast<const char*>(p.W) + off + koff : zero,
                                       Bs + lds_wave + i * NW * 1024, 16, 0, 0);
    }
  }
};

// The buffer-offset staging form applies: whole K tiles (both operands are under 2 GiB: launch_gemm_pers checks)
template <int BK>
__device__ __forceinline__ bool pers_fast_staging(const GemmArgs& p) {
  return p.K % BK == 0;
}

// 32-bit byte offsets reach every staged element (ao / wo + the K offset of the last tile)
static bool pers_operands_fit(const GemmArgs& a) {
  return (int64_t)a.M * a.lda * 2 + (int64_t)a.K * 2 + 256 < 0x7fffffff &&
         (int64_t)a.N * a.ldw * 2 + (int64_t)a.K * 2 + 256 < 0x7fffffff;
}

// Epilogue of one tile straight from the (swapped-operand) accumulators: lane (r16 = lane & 15, g = lane >> 4) holds
// output row bm + wm*TM + i*16 + r16, columns bn + wn*TN + j*16 + g*4 + {0..3} in acc[i][j].
// act(acc + bias) of one 4-column group -> two packed 16-bit words (the fault check for binary16 outputs)
template <bool F16>
__device__ __forceinline__ uint2 pers_act_pack(const GemmArgs& p, f32x4 v) {
  if (p.act == MAPA_ACT_GELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = F16 ? gelu_erf(v[e]) : gelu_bf16out(v[e]);
  }
  if constexpr (F16) {
    f16_check4(p.fault, v);
    return uint2{pack_f16x2(v[0], v[1]), pack_f16x2(v[2], v[3])};
  } else {
    return uint2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
  }
}

// The act -> 16-bit epilogue with 16-byte stores (N % 16 == 0, 16-B aligned rows): of the two 16-column blocks j0, j1
// of a row, lanes g = 0 / 2 store columns 0-7 / 8-15 of j0 and lanes g = 1 / 3 those of j1, the missing half of each
// 8-column group swapped with the partner lane (lane ^ 16) — half the store instructions of the 8-byte form, whose
// issue (not HBM) set the epilogue's time (MI355X_MICROARCH.md: dwordx2 tails are store-issue-bound).
template <bool F16, int FM, int FN, int TM, int TN>
__device__ __forceinline__ void pers_epilogue_wide(const GemmArgs& p, const f32x4 (&acc)[FM][FN], int bm, int bn,
                                                   int wm, int wn, int lane) {
  static_assert(FN % 2 == 0, "16-column block pairs");
  const int r16 = lane & 15, g = lane >> 4;
  const bool odd = g & 1;
  const int row0 = bm + wm * TM + r16;
#pragma unroll
  for (int q = 0; q < FN / 2; ++q) {
    const int c0 = bn + wn * TN + q * 32;  // first column of block j0 = 2q (j1 = 2q + 1 starts at c0 + 16)
    const int n_a = c0 + g * 4, n_b = c0 + 16 + g * 4;
    const bool in_a = c0 < p.N, in_b = c0 + 16 < p.N;  // N % 16 == 0: whole blocks
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    const f32x4 ba = p.bias && in_a ? *reinterpret_cast<const f32x4*>(p.bias + n_a) : zero;
    const f32x4 bb = p.bias && in_b ? *reinterpret_cast<const f32x4*>(p.bias + n_b) : zero;
    const int col = (odd ? c0 + 16 : c0) + (g >> 1) * 8;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const uint2 ua = pers_act_pack<F16>(p, acc[i][2 * q] + ba);
      const uint2 ub = pers_act_pack<F16>(p, acc[i][2 * q + 1] + bb);
      const uint2 snd = odd ? ua : ub;
      uint2 rcv;
      rcv.x = __shfl_xor(snd.x, 16);
      rcv.y = __shfl_xor(snd.y, 16);
      const int m = row0 + i * 16;
      if (m < p.M && (odd ? in_b : in_a)) {
        const uint4 w = odd ? uint4{rcv.x, rcv.y, ub.x, ub.y} : uint4{ua.x, ua.y, rcv.x, rcv.y};
        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p.out_lp) + (int64_t)m * p.ldo + col) = w;
      }
    }
  }
}

template <int MODE, bool F16, int FM, int FN, int TM, int TN>
__device__ __forceinline__ void pers_epilogue(const GemmArgs& p, const f32x4 (&acc)[FM][FN], int bm, int bn, int wm,
                                              int wn, int lane) {
  if constexpr (MODE == 1 && FN % 2 == 0) {
    if (p.N % 16 == 0 && p.ldo % 8 == 0 && (reinterpret_cast<uintptr_t>(p.out_lp) & 15) == 0) {
      pers_epilogue_wide<F16, FM, FN, TM, TN>(p, acc, bm, bn, wm, wn, lane);
      return;
    }
  }
  const int r16 = lane & 15, g = lane >> 4;
  const int row0 = bm + wm * TM + r16;
  const int col0 = bn + wn * TN + g * 4;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n0 = col0 + j * 16;
    if (n0 >= p.N) continue;  // N % 4 == 0: a lane's 4 columns are all in range or all out
    const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n0) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 gv = {1.f, 1.f, 1.f, 1.f};
    if (MODE == 2 && p.gamma) gv = *reinterpret_cast<const f32x4*>(p.gamma + n0);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = row0 + i * 16;
      if (m >= p.M) continue;
      f32x4 v = acc[i][j] + bv;
      const int64_t off = (int64_t)m * p.ldo + n0;
      if constexpr (MODE == 1) {
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.out_lp) + off) = pers_act_pack<F16>(p, v);
      } else {  // the arithmetic of epi_store_row8_mode<2> (gamma multiply and residual add rounded separately)
        if (p.gamma) v *= gv;
        v += *reinterpret_cast<const f32x4*>(p.resid1 + off);
        *reinterpret_cast<f32x4*>(p.out_f32 + off) = v;
      }
    }
  }
}

// PRIO: s_setprio 1 around each tile's MFMA burst.  DIAG (timing diagnostic, wrong results): 1 = no epilogue.
template <int MODE, int BM, int BN, int RB, int WM, int STAGES, int MINB, bool F16, int PRIO = 0, int DIAG = 0,
          int NW = 8>
__global__ void __launch_bounds__(NW * 64, MINB) gemm_pers_kernel(GemmArgs p) {
  using C = PCfg<BM, BN, RB, WM, NW>;
  constexpr int NPT = C::NLA + C::NLB;
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * C::STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int ntm = (p.M + BM - 1) / BM, ntn = (p.N + BN - 1) / BN;
  const int tiles = ntm * ntn, G = gridDim.x;
  const int nk = (p.K + C::BK - 1) / C::BK;
  const bool fast = pers_fast_staging<C::BK>(p);
  const int lds_wave = wave * 1024;
  const int g = lane >> 4, r16 = lane & 15;

  // fragment byte offsets inside a ring slot (k-group kg adds kg * 64 B before the swizzle)
  int a_off[C::KG][C::FM], b_off[C::KG][C::FN];
#pragma unroll
  for (int kg = 0; kg < C::KG; ++kg) {
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const int ra = wm * C::TM + i * 16 + r16;
      a_off[kg][i] = ra * RB + (((kg * 4 + g) ^ pswz<RB>(ra)) << 4);
    }
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      const int rb = wn * C::TN + j * 16 + r16;
      b_off[kg][j] = C::A_BYTES + rb * RB + (((kg * 4 + g) ^ pswz<RB>(rb)) << 4);
    }
  }

  int r = 0, tm, tn;
  if (!mapa_idx::pers_tile(blockIdx.x, G, r, tiles, p.tile_gm, ntm, ntn, tm, tn)) return;
  Src<BM, BN, RB, WM, MODE * 2 + (F16 ? 1 : 0) + 4 * PRIO + 8 * DIAG + 32 * NW, NW> src;
  src.setup(p, tm * BM, tn * BN, wave, lane);
#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < nk) src.stage(p, lds, s0, s0, lds_wave, fast, wave, lane);
  // Stagger: the workgroups with one tile fewer (no tile in the last, partial round) start p.stagger ticks late, so
  // their tile boundaries fall mid-tile of the others' and the chip's epilogue store bursts no longer coincide; they
  // still finish before the full-length workgroups as long as the delay is under one tile time.
  if (p.stagger > 0) {
    const int rem = tiles % G;
    if (rem && (int)blockIdx.x >= rem) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)p.stagger) __builtin_amdgcn_s_sleep(8);
    }
  }

  f32x4 acc[C::FM][C::FN];
  for (;;) {
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // ---- main loop over the ring: tiles kt+1 .. kt+STAGES-2 stay in flight across the barrier of tile kt.  The
    // waits count only this tile's DMA (issued in order before anything else of this tile), and every vector-memory
    // op issued earlier (the previous tile's epilogue stores) is older still: a wait for the DMA also covers them.
    int slot = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(STAGES - 2, nk - 1 - kt);
      if (ahead >= STAGES - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * (STAGES - 2)) : "memory");
      else if (STAGES > 3 && ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * 2) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's DMA for tile kt landed; every wave done with tile kt-1
      __builtin_amdgcn_sched_barrier(0);
      if (kt + STAGES - 1 < nk) src.stage(p, lds, slot == 0 ? STAGES - 1 : slot - 1, kt + STAGES - 1, lds_wave, fast, wave, lane);
      const char* base = lds + slot * C::STAGE;
      bf16x8 af[C::KG][C::FM], bfr[C::KG][C::FN];
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg) {
#pragma unroll
        for (int j = 0; j < C::FN; ++j) bfr[kg][j] = *reinterpret_cast<const bf16x8*>(base + b_off[kg][j]);
#pragma unroll
        for (int i = 0; i < C::FM; ++i) af[kg][i] = *reinterpret_cast<const bf16x8*>(base + a_off[kg][i]);
      }
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16x16x32<F16>(bfr[kg][j], af[kg][i], acc[i][j]);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
      }
      slot = slot + 1 == STAGES ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's last fragment reads retired: the ring is free
    __builtin_amdgcn_sched_barrier(0);
    // ---- the next tile's prologue DMA, then this tile's epilogue under it
    const int bm = tm * BM, bn = tn * BN;
    ++r;
    const bool more = mapa_idx::pers_tile(blockIdx.x, G, r, tiles, p.tile_gm, ntm, ntn, tm, tn);
    if (more) {
      src.setup(p, tm * BM, tn * BN, wave, lane);
#pragma unroll
      for (int s0 = 0; s0 < STAGES - 1; ++s0)
        if (s0 < nk) src.stage(p, lds, s0, s0, lds_wave, fast, wave, lane);
    }
    if (DIAG != 1 || p.M < 0) pers_epilogue<MODE, F16, C::FM, C::FN, C::TM, C::TN>(p, acc, bm, bn, wm, wn, lane);
    if (!more) break;
  }
}

// ---- LayerNorm-fused residual epilogue (the in-place residual pattern + nn.LayerNorm of the output rows; dinov2
// layers/block.py:93-118 norm1 / norm2, transformer_blocks.py:452-469), from registers.  A row's N columns are the
// ntn column tiles of its BM-row band; the band's tiles exchange {sum, M2} per row through 16-byte write-through
// granules {epoch, sum, M2, ~epoch} in the workspace (the protocol of gemm_big_kernels.h big_epilogue_ln, same slots,
// same generation / departure words), so every tile normalises its own columns with the row's full statistics:
//  1. v = resid1 + gamma * (acc + bias) in place in the accumulators (epi_store_row8_mode<2>'s rounding);
//  2. per row: the sum over the tile's columns (the 4 lanes sharing a row by two butterflies, the WN column waves in
//     LDS in wave order), the tile mean, then M2 about it the same way (two-pass inside the tile);
//  3. the granule of every row published (write-through store: the data is its own flag); the residual rows stored;
//  4. the band's granules polled (bounded: MAPA_FAULT_LN_BARRIER on expiry) and merged in column order (Chan);
//  5. the band's last departing tile bumps the band's generation word; each tile writes (v - mean) * rstd * w + b as
//     bf16 for its own columns.
// LDS: the first (2 * WN + 2) * BM floats of the ring (free: the next tile's prologue is issued after this).
template <int FM, int FN, int TM, int TN, int WN, int BM, int BN>
__device__ __forceinline__ void pers_epilogue_ln(const GemmArgs& p, f32x4 (&acc)[FM][FN], char* lds, int tm, int tn,
                                                 int ntn, int wm, int wn, int lane, int tid) {
  const int r16 = lane & 15, g = lane >> 4;
  const int bm = tm * BM, bn = tn * BN;
  float* red = reinterpret_cast<float*>(lds);  // [WN][BM] row sums of each column wave
  float* red2 = red + WN * BM;                   // [WN][BM] row M2 about the tile mean
  float* rmean = red2 + WN * BM;                 // [BM] the row's mean over N
  float* rrstd = rmean + BM;                     // [BM] the row's rstd
  const int col0 = bn + wn * TN + g * 4;
  // 1. the new residual, in the accumulators (rows past M: zeros, never stored)
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n0 = col0 + j * 16;
    const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n0) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 gv = p.gamma ? *reinterpret_cast<const f32x4*>(p.gamma + n0) : f32x4{1.f, 1.f, 1.f, 1.f};
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = bm + wm * TM + i * 16 + r16;
      f32x4 v = acc[i][j] + bv;
      if (p.gamma) v *= gv;
      if (m < p.M) v += *reinterpret_cast<const f32x4*>(p.resid1 + (int64_t)m * p.ldo + n0);
      else v = f32x4{0.f, 0.f, 0.f, 0.f};
      acc[i][j] = v;
    }
  }
  // 2. tile row sums -> tile means -> M2 about them
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) sum += (acc[i][j][0] + acc[i][j][1]) + (acc[i][j][2] + acc[i][j][3]);
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    if (g == 0) red[wn * BM + wm * TM + i * 16 + r16] = sum;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int rl = wm * TM + i * 16 + r16;
    float ts = 0.f;
#pragma unroll
    for (int w = 0; w < WN; ++w) ts += red[w * BM + rl];
    const float mu = ts * (1.f / BN);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = acc[i][j][e] - mu;
        q += d * d;
      }
    q += __shfl_xor(q, 16);
    q += __shfl_xor(q, 32);
    if (g == 0) red2[wn * BM + rl] = q;
  }
  __syncthreads();
  // 3. publish {epoch, sum, M2, ~epoch} per row (write-through: the data is its own flag); the residual rows
  typedef __attribute__((address_space(1))) int gi32;
  gi32* gen = (gi32*)(p.ln_ctr) + 2 * tm;
  gi32* depart = gen + 1;
  const unsigned epoch = (unsigned)__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const auto srs = __builtin_amdgcn_make_buffer_rsrc(p.ln_stats + (int64_t)tm * LN_MAX_NTN_P * BM * 4, 0,
                                                     ntn * BM * 16, 0x00020000);
  float tsum = 0.f;
  if (tid < BM) {
#pragma unroll
    for (int w = 0; w < WN; ++w) tsum += red[w * BM + tid];
    if (!((p.ln_skip & 1) && tm == 0 && tn == 0)) {  // (ln_skip: the test hook's missing tile)
      float m2 = 0.f;
#pragma unroll
      for (int w = 0; w < WN; ++w) m2 += red2[w * BM + tid];
      const u32x4p gv = {epoch, __float_as_uint(tsum), __float_as_uint(m2), ~epoch};
      __builtin_amdgcn_raw_buffer_store_b128(gv, srs, (tn * BM + tid) * 16, 0, 16);  // sc1
    }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = bm + wm * TM + i * 16 + r16;
      if (m < p.M && !(p.ln_skip & 8)) *reinterpret_cast<f32x4*>(p.out_f32 + (int64_t)m * p.ldo + col0 + j * 16) = acc[i][j];
    }
  // 4. the band's granules, merged in column order
  if (tid < BM) {
    u32x4p gv[LN_MAX_NTN_P];
    unsigned spins = 0;
    for (;;) {
      if (p.ln_skip & 2) break;  // (MAPA_LN_DIAG timing only)
#pragma unroll
      for (int t = 0; t < LN_MAX_NTN_P; ++t)
        gv[t] = t < ntn ? __builtin_amdgcn_raw_buffer_load_b128(srs, (t * BM + tid) * 16, 0, 16)
                        : u32x4p{epoch, 0u, 0u, ~epoch};
      bool ok = true;
#pragma unroll
      for (int t = 0; t < LN_MAX_NTN_P; ++t) ok = ok && gv[t][0] == epoch && gv[t][3] == ~epoch;
      if (ok) break;
      __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
      if (++spins > p.ln_spin) {  // a band tile never published: raise the fault word, do not hang the device
        if (p.fault)
          __hip_atomic_fetch_or(p.fault, (unsigned)MAPA_FAULT_LN_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAX_NTN_P; ++t)
      if (t < ntn) sum += __uint_as_float(gv[t][1]);
    const float mean = sum / (float)p.N;
    float m2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAX_NTN_P; ++t)
      if (t < ntn) {
        const float d = __uint_as_float(gv[t][1]) * (1.f / BN) - mean;
        m2 += __uint_as_float(gv[t][2]) + (float)BN * d * d;
      }
    rmean[tid] = mean;
    rrstd[tid] = rsqrtf(m2 / (float)p.N + p.ln_eps);
  }
  __syncthreads();
  if (tid == 0) {  // every tile of the band holds its granules: the last one out bumps the band's generation
    if (__hip_atomic_fetch_add(depart, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ntn - 1) {
      __hip_atomic_store(depart, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // 5. normalise this tile's columns: 16-byte bf16 stores, the two 16-column blocks of a pair split between lane
  // partners (lane ^ 16) as in pers_epilogue_wide
  static_assert(FN % 2 == 0, "16-column block pairs");
  bf16_t* lout = reinterpret_cast<bf16_t*>(p.ln_out);
  const bool odd = g & 1;
#pragma unroll
  for (int q = 0; q < FN / 2; ++q) {
    const int na = col0 + 2 * q * 16, nb = na + 16;
    const f32x4 lwa = *reinterpret_cast<const f32x4*>(p.ln_w + na), lba = *reinterpret_cast<const f32x4*>(p.ln_b + na);
    const f32x4 lwb = *reinterpret_cast<const f32x4*>(p.ln_w + nb), lbb = *reinterpret_cast<const f32x4*>(p.ln_b + nb);
    const int col = bn + wn * TN + q * 32 + (odd ? 16 : 0) + (g >> 1) * 8;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rl = wm * TM + i * 16 + r16;
      const float mu = rmean[rl], rs = rrstd[rl];
      f32x4 ya, yb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ya[e] = (acc[i][2 * q][e] - mu) * rs * lwa[e] + lba[e];
        yb[e] = (acc[i][2 * q + 1][e] - mu) * rs * lwb[e] + lbb[e];
      }
      const uint2 ua = {pack_bf16x2(ya[0], ya[1]), pack_bf16x2(ya[2], ya[3])};
      const uint2 ub = {pack_bf16x2(yb[0], yb[1]), pack_bf16x2(yb[2], yb[3])};
      const uint2 snd = odd ? ua : ub;
      uint2 rcv;
      rcv.x = __shfl_xor(snd.x, 16);
      rcv.y = __shfl_xor(snd.y, 16);
      if (bm + rl < p.M && !(p.ln_skip & 4))
        *reinterpret_cast<uint4*>(lout + (int64_t)(bm + rl) * p.ln_ldo + col) =
            odd ? uint4{rcv.x, rcv.y, ub.x, ub.y} : uint4{ua.x, ua.y, rcv.x, rcv.y};
    }
  }
}

// The residual linear + LayerNorm over persistent band rounds: grid G = whole bands that fit the co-resident
// workgroups (launch_gemm_pers_ln), tile t of round r = r * G + xcd_remap(b, n_r), band-major (t / ntn = band): every
// round holds whole bands, all of them resident, so a band's barrier never waits for a tile that cannot run.
template <int BM, int BN, int RB, int WM, int STAGES, int MINB>
__global__ void __launch_bounds__(PTHREADS, MINB) gemm_pers_ln_kernel(GemmArgs p) {
  using C = PCfg<BM, BN, RB, WM>;
  constexpr int NPT = C::NLA + C::NLB;
  static_assert(STAGES * C::STAGE >= (2 * C::WN + 2) * BM * 4, "LN scratch fits the ring");
  __shared__ __attribute__((aligned(1024))) char lds[STAGES * C::STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int ntm = (p.M + BM - 1) / BM, ntn = p.N / BN;
  const int tiles = ntm * ntn, G = gridDim.x;
  const int nk = (p.K + C::BK - 1) / C::BK;
  const bool fast = pers_fast_staging<C::BK>(p);
  const int lds_wave = wave * 1024;
  const int g = lane >> 4, r16 = lane & 15;
  int a_off[C::KG][C::FM], b_off[C::KG][C::FN];
#pragma unroll
  for (int kg = 0; kg < C::KG; ++kg) {
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const int ra = wm * C::TM + i * 16 + r16;
      a_off[kg][i] = ra * RB + (((kg * 4 + g) ^ pswz<RB>(ra)) << 4);
    }
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      const int rb = wn * C::TN + j * 16 + r16;
      b_off[kg][j] = C::A_BYTES + rb * RB + (((kg * 4 + g) ^ pswz<RB>(rb)) << 4);
    }
  }
  Src<BM, BN, RB, WM, 100> src;
  f32x4 acc[C::FM][C::FN];
  for (int base = 0; base < tiles; base += G) {
    const int n = min(G, tiles - base);
    if ((int)blockIdx.x >= n) break;
    const int t = base + mapa_idx::xcd_remap(blockIdx.x, n);
    const int tm = t / ntn, tn = t - tm * ntn;
    src.setup(p, tm * BM, tn * BN, wave, lane);
#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
      if (s0 < nk) src.stage(p, lds, s0, s0, lds_wave, fast, wave, lane);
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int slot = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(STAGES - 2, nk - 1 - kt);
      if (ahead >= STAGES - 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * (STAGES - 2)) : "memory");
      else if (STAGES > 3 && ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT * 2) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + STAGES - 1 < nk) src.stage(p, lds, slot == 0 ? STAGES - 1 : slot - 1, kt + STAGES - 1, lds_wave, fast, wave, lane);
      const char* sb = lds + slot * C::STAGE;
      bf16x8 af[C::KG][C::FM], bfr[C::KG][C::FN];
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg) {
#pragma unroll
        for (int j = 0; j < C::FN; ++j) bfr[kg][j] = *reinterpret_cast<const bf16x8*>(sb + b_off[kg][j]);
#pragma unroll
        for (int i = 0; i < C::FM; ++i) af[kg][i] = *reinterpret_cast<const bf16x8*>(sb + a_off[kg][i]);
      }
#pragma unroll
      for (int kg = 0; kg < C::KG; ++kg)
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16x16x32<false>(bfr[kg][j], af[kg][i], acc[i][j]);
      slot = slot + 1 == STAGES ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // the ring is free: the LayerNorm scratch
    pers_epilogue_ln<C::FM, C::FN, C::TM, C::TN, C::WN, BM, BN>(p, acc, lds, tm, tn, ntn, wm, wn, lane, tid);
    __syncthreads();  // scratch reads done before the next tile's prologue DMA
  }
}

}  // namespace

// Shapes: 0 = 256x128 (64-B rows, 3 stages, 2 workgroups / CU), 1 = 192x256 (128-B rows, 2 stages, 1 / CU),
// 2 = 256x256 (128-B rows, 2 stages, 1 / CU), 3 = 192x128 (128-B rows, 2 stages, 2 / CU); 4 = 3 with s_setprio
// around the MFMA bursts; 5 / 6 = 3 / 0 without the epilogue (timing diagnostics, wrong results).
static void pers_shape(int s, int& bm, int& bn, int& per_cu, int& nw) {
  static const int BMs[9] = {256, 192, 256, 192, 192, 192, 256, 192, 256},
                   BNs[9] = {128, 256, 256, 128, 128, 128, 128, 128, 128}, PCs[9] = {2, 1, 1, 2, 2, 2, 2, 2, 2},
                   NWs[9] = {8, 8, 8, 8, 8, 8, 8, 4, 4};
  bm = BMs[s];
  bn = BNs[s];
  per_cu = PCs[s];
  nw = NWs[s];
}

// Start delay of the workgroups with one tile fewer (gemm_pers_kernel): mapa_gemm_tune(MAPA_TUNE_PERS_STAGGER, .) /
// env MAPA_GEMM_STAGGER = 100-MHz ticks, 0 = off (default), -1 = automatic (pers_auto_stagger); -2: env not read yet.
// Off by default: the bench-level gain did not hold across boxes (+0.5 % on one, -0.2 / -0.5 % at 35 / 40 % on
// another, profiles/r6/stagger_bench_ab.txt) — a fixed delay in ticks cannot track the box's clock.
static int g_pers_stagger = -2;

// Automatic stagger: half a tile's time (2 BM BN K flop at ~1.65 TFLOP/s per resident workgroup, the path rate) where
// the short workgroups are a minority (< 40 % of the grid): then they still finish first, and the chip's epilogue
// bursts split into two half-size ones that fall mid-tile of the other group.  Measured (tools/stagger_ab.py,
// profiles/r6/stagger_ab.json, 192x128 tiles): enc.qkv 81.3 -> 78.2 us at 1500 ticks, enc.fc1 111.6 -> 109.5;
// aat.fc1 neutral; where most workgroups are short (aat.qkv: 492 of 512) any delay only adds to the kernel
// (49.1 -> 52.1 us at 500 ticks), so none is applied there.  Bitwise-neutral: the same tiles, the same K order.
static int pers_auto_stagger(int64_t tiles, int G, int bm, int bn, int K) {
  const int64_t rem = tiles % G;
  static int pct = -1;  // MAPA_GEMM_STAGGER_PCT: the short-workgroup share below which the stagger applies (A/B)
  if (pct < 0) pct = getenv("MAPA_GEMM_STAGGER_PCT") ? atoi(getenv("MAPA_GEMM_STAGGER_PCT")) : 40;
  if (rem == 0 || tiles < G || (G - rem) * 100 >= pct * (int64_t)G) return 0;
  const double tile_us = 2.0 * bm * bn * (double)K / 1.65e6;
  return (int)(0.5 * tile_us * 100.0);  // 100 ticks per microsecond
}

int pers_pick_shape(int M, int N, int K, int cus) {
  // 192x128 tiles at 2 workgroups per CU measured fastest on every path shape with the act -> 16-bit epilogue
  // (tools/pers_ab.py, profiles/r6/pers_ab_v1.json: enc.qkv 84.1 us vs 92.9 / 93.7 / 111.7 for the other shapes,
  // enc.fc1 114.4 vs 121.3-132.1, aat.qkv 53.3 vs 63.4-76.6, aat.fc1 71.0 vs 83.3-100.8): the 64-deep K tiles halve
  // the barriers of the 256x128 ring and the extra row tiles fill the last round
  (void)M;
  (void)N;
  (void)K;
  (void)cus;
  return 3;
}

static GemmKernel pers_kernel_diag(int s) {  // bf16, act -> 16-bit epilogue only
  switch (s) {
    case 4: return gemm_pers_kernel<1, 192, 128, 128, 4, 2, 2, false, 1>;
    case 5: return gemm_pers_kernel<1, 192, 128, 128, 4, 2, 2, false, 0, 1>;
    case 6: return gemm_pers_kernel<1, 256, 128, 64, 4, 3, 2, false, 0, 1>;
    // 4-wave workgroups (2 waves / SIMD at 2 per CU, 256 VGPRs): 192x128 as 2x2 waves of 96x64; 256x128 in 32-deep K
    // tiles, 3 stages, 2x2 waves of 128x64
    case 7: return gemm_pers_kernel<1, 192, 128, 128, 2, 2, 2, false, 0, 0, 4>;
    case 8: return gemm_pers_kernel<1, 256, 128, 64, 2, 3, 2, false, 0, 0, 4>;
    default: return nullptr;
  }
}

static GemmKernel pers_kernel(int mode, bool f16, int s) {
  if (s >= 4) return mode == 1 && !f16 ? pers_kernel_diag(s) : nullptr;
  switch ((mode == 1 ? 0 : 8) + (f16 ? 4 : 0) + s) {
    case 0: return gemm_pers_kernel<1, 256, 128, 64, 4, 3, 2, false>;
    case 1: return gemm_pers_kernel<1, 192, 256, 128, 2, 2, 1, false>;
    case 2: return gemm_pers_kernel<1, 256, 256, 128, 2, 2, 1, false>;
    case 3: return gemm_pers_kernel<1, 192, 128, 128, 4, 2, 2, false>;
    case 4: return gemm_pers_kernel<1, 256, 128, 64, 4, 3, 2, true>;
    case 5: return gemm_pers_kernel<1, 192, 256, 128, 2, 2, 1, true>;
    case 6: return gemm_pers_kernel<1, 256, 256, 128, 2, 2, 1, true>;
    case 7: return gemm_pers_kernel<1, 192, 128, 128, 4, 2, 2, true>;
    case 8: return gemm_pers_kernel<2, 256, 128, 64, 4, 3, 2, false>;
    case 9: return gemm_pers_kernel<2, 192, 256, 128, 2, 2, 1, false>;
    case 10: return gemm_pers_kernel<2, 256, 256, 128, 2, 2, 1, false>;
    case 11: return gemm_pers_kernel<2, 192, 128, 128, 4, 2, 2, false>;
    case 12: return gemm_pers_kernel<2, 256, 128, 64, 4, 3, 2, true>;
    case 13: return gemm_pers_kernel<2, 192, 256, 128, 2, 2, 1, true>;
    case 14: return gemm_pers_kernel<2, 256, 256, 128, 2, 2, 1, true>;
    case 15: return gemm_pers_kernel<2, 192, 128, 128, 4, 2, 2, true>;
    default: return nullptr;
  }
}

bool launch_gemm_pers(const GemmArgs& a, int shape, int cus, hipStream_t stream) {
  // dense A, one of the two transformer epilogue patterns, 16-B aligned rows
  const int mode = epi_mode(a);
  if (!mode || a.sp_half != 0x7fffffff || a.N % 4 || a.ldo % 4 || a.lda % 8 || a.ldw % 8 || !pers_operands_fit(a))
    return false;
  if (mode == 1 && a.act != MAPA_ACT_NONE && a.act != MAPA_ACT_GELU) return false;
  if (shape < 0) {
    if (mode != 1) return false;  // the residual pattern: the tile kernels measured as fast or faster (pers_ab)
    shape = pers_pick_shape(a.M, a.N, a.K, cus);
  }
  if (shape > 8) return false;
  int bm, bn, pc, nw;
  pers_shape(shape, bm, bn, pc, nw);
  const int64_t tiles = (int64_t)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  const int G = (int)std::min<int64_t>(tiles, (int64_t)cus * pc);
  const GemmKernel k = pers_kernel(mode, a.lp_f16 != 0, shape);
  if (!k) return false;
  GemmArgs b = a;
  if (g_pers_stagger == -2) g_pers_stagger = getenv("MAPA_GEMM_STAGGER") ? atoi(getenv("MAPA_GEMM_STAGGER")) : 0;
  b.stagger = g_pers_stagger >= 0 ? g_pers_stagger : pers_auto_stagger(tiles, G, bm, bn, a.K);
  hipLaunchKernelGGL(k, dim3(G), dim3(nw * 64), 0, stream, b);
  return true;
}

void pers_set_stagger(int ticks) { g_pers_stagger = ticks >= 0 ? ticks : -1; }

// The LayerNorm-fused residual linear on 192x128 tiles, 2 workgroups per CU (gemm_pers_ln_kernel): N = 768 or 1024
// (6 / 8 column tiles per band), bf16, the in-place residual pattern.  Workspace as launch_gemm_big_ln (the GEMM
// ticket head's top LN_TICKET_WORDS words + ln_stats_bytes of granule slots, 192-row bands).
bool launch_gemm_pers_ln(const GemmArgs& a, void* ws, int64_t ws_bytes, int cus, hipStream_t stream) {
  constexpr int BM = 192, BN = 128;
  if (a.N % BN || a.N / BN > LN_MAX_NTN_P || a.lp_f16 || !a.ln_out || !a.ln_w || !a.ln_b || a.ln_ldo % 8 ||
      (reinterpret_cast<uintptr_t>(a.ln_out) & 15))
    return false;
  if (a.out_mode != 0 || !a.out_f32 || !a.resid1 || a.resid2 || a.out_lp || a.out_lp_relu || a.out_s3 ||
      a.out_s3_relu || a.act != MAPA_ACT_NONE || a.ldo % 4 || a.lda % 8 || a.ldw % 8 || a.sp_half != 0x7fffffff ||
      !pers_operands_fit(a))
    return false;
  const int ntm = (a.M + BM - 1) / BM, ntn = a.N / BN;
  if (2 * ntm >= LN_TICKET_WORDS || !ws || ws_bytes < GEMM_TICKET_BYTES + (int64_t)ntm * LN_MAX_NTN_P * BM * 16)
    return false;
  const GemmKernel k = gemm_pers_ln_kernel<BM, BN, 128, 4, 2, 2>;
  static int per_cu_of[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int& per_cu = per_cu_of[dev];
  if (!per_cu) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, PTHREADS, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
  }
  const int slots = per_cu * cus;
  const int G = std::min(ntm, slots / ntn) * ntn;  // whole bands, all co-resident
  if (G <= 0) return false;
  GemmArgs b = a;
  b.ln_ctr = reinterpret_cast<int*>(ws) + (GEMM_TICKET_BYTES / 4 - LN_TICKET_WORDS);
  b.ln_stats = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) + GEMM_TICKET_BYTES);
  b.ln_skip = ln_take_test_skip() | ln_diag_bits();
  b.ln_spin = ln_spin_value();
  hipLaunchKernelGGL(k, dim3(G), dim3(PTHREADS), 0, stream, b);
  return true;
}

}  // namespace mapa_gemm_impl
