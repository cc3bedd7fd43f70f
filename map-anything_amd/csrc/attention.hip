// Flash-attention forward for gfx950, head_dim 64, non-causal, softmax scale 1/8.
//
// Replaces F.scaled_dot_product_attention of the DINOv2 SDPA wrapper (uniception/models/encoders/dinov2.py:136,
// q,k,v (V*B, 16, 1370, 64)) and of the AAT SelfAttentionBlock (uniception/models/utils/transformer_blocks.py:
// 198-201): global layers over all V*1369+1 tokens, frame layers per view over 1369 tokens.
//
// Structure (one workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32 query rows):
//  * Q stays in registers for the whole K/V sweep; K/V tiles of 64 keys are staged HBM -> LDS with
//    global_load_lds into a two-slot ring (one barrier per tile).
//  * Swapped QK^T: S^T = K * Q^T with v_mfma_f32_32x32x16_bf16, so a lane owns one query row (lane & 31) and
//    32 of its key scores in registers: the row max / row sum are in-lane plus one cross-half exchange.
//  * The S^T accumulator is re-used directly as the B operand of O^T = V^T * P^T (accumulator-as-operand,
//    no LDS round trip for P); V^T fragments come from ds_read_b64_tr_b16 transposed LDS reads.
//  * Online softmax in the log2 domain (v_exp_f32), fp32 running max / sum, O^T in 32 fp32 accumulators.
//  * K LDS rows are XOR-swizzled by (row>>1)&7 and V rows by ((row>>1)&1)<<2 (applied on the LDS-DMA source
//    address), which makes both the b128 K reads and the transposed V reads bank-conflict free.
//  * Precise variant (dtype f32): identical dataflow on v_mfma_f32_32x32x2_f32 (exact fp32 products).
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "mapa_common.h"
#include "index_math.h"

namespace {

constexpr int NT = 256;        // 4 waves
constexpr int QBLK = 128;      // query rows per workgroup
constexpr int KT = 64;         // keys per K/V tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

struct AttnArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  int64_t qb, qr, kb, kr, vb, vr, ob, orr;
  int batch, heads, seq_q, seq_kv;
  float qscale;  // softmax scale on q.k (natural units; the bf16 kernel multiplies by log2(e) as well)
  int nseg;
  int seg_start[MAPA_MAX_KV_SEGMENTS];
  int seg_len[MAPA_MAX_KV_SEGMENTS];
};

// logical key -> physical K/V row (identity unless the keys are split into segments).  The segment loop is
// wave-uniform (scalar loads of the descriptor; no divergent indexing, no vector load + vmcnt wait that would
// drain the in-flight LDS-DMA).
__device__ __forceinline__ int kv_row(const AttnArgs& p, int key) {
  if (p.nseg == 0) return key;
  int off = p.seg_start[0], cum = p.seg_len[0];
#pragma unroll 1
  for (int s = 1; s < p.nseg; ++s) {
    if (key >= cum) off = p.seg_start[s] - cum;
    cum += p.seg_len[s];
  }
  return key + off;
}

using mapa_idx::xcd_remap;

typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ s4v tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(p));
}

// ------------------------------------------------------------------------------------------------ bf16
// Row sums are plain f32 adds: attention.o is built with -fno-slp-vectorize so -O3 does not pack them into
// v_pk_add_f32, which costs ~12 extra cycles per instruction beside MFMAs (MI355X_MICROARCH.md, per-instruction
// cycle constants).  (An inline-asm v_add would dodge the packing too, but hipcc pads no hazards into asm: the
// v_exp_f32 -> VALU and MFMA -> VALU wait states would be missing.)
__device__ __forceinline__ float add_s(float a, float b) { return a + b; }

// Softmax bookkeeping relative to a per-row REFERENCE max m_ref (log2 domain) instead of the exact running max:
//  * the QK^T accumulator is initialised with -m_ref, so the MFMA itself produces s - m_ref (no per-score subtract);
//  * P = exp2(s - m_ref) is used as long as every row sum of the tile stays <= 2^8 (then every P <= 256: no
//    overflow, and bf16 P keeps its relative precision at any magnitude);
//  * otherwise (rare, wave-uniform branch) the rows are rebased onto their true running max: O and l scaled by
//    exp2(-d), P recomputed.  The first tile always takes the exact path (m_ref := its row max).
// Exact softmax either way: O / l is invariant to the reference (the LSE output adds m_ref back).
constexpr float REBASE_SUM = 256.f;

// Work split.  A task = (batch, head, 128-row query block).  The grid holds n_dp whole tasks (data-parallel, the
// full waves of the device's resident workgroup slots) followed by the remaining tasks each cut into `chunks`
// contiguous K/V tile ranges so that the last, partial wave is spread over all slots instead of leaving most of
// the chip idle for a whole task time (e.g. 1032 global-layer tasks on 512 slots: 2 waves + 8 tasks -> the 8 tasks
// run as 8 x 43 chunks).  Chunks leave normalised fp32 rows + LSE in the workspace (slot = tail workgroup index)
// and attn_split_merge combines them.  The tail workgroups have the highest ids, so they are dispatched last.
struct SplitArgs {
  float* part_o;    // [slots][128][64] fp32
  float* part_lse;  // [slots][128]     natural-log LSE
  int n_dp;         // whole tasks (grid ids [0, n_dp))
  int chunks;       // K/V chunks per remaining task (grid ids n_dp + j: task n_dp + j / chunks, chunk j % chunks)
};

// F16: fp16 operands (the fp16 autocast recipe): same structure, f16 MFMAs, P rounded to fp16
template <int NW, bool SEG, bool F16 = false>
__global__ void __launch_bounds__(NW * 64, 2) attn_fwd_bf16(AttnArgs p, SplitArgs sp) {
  constexpr int TILE = KT * 128;  // 64 rows x 128 B
  constexpr int QBLK_WG = NW * 32;
  constexpr int NP = 16 / NW;     // 1-KiB LDS-DMA pieces per wave per K/V tile (first half K, second half V)
  static_assert(NW == 4 || NW == 8, "pieces are dealt K-first over 4 or 8 waves");
  __shared__ __attribute__((aligned(1024))) char lds[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane >> 5, l32 = lane & 31;
  const int nqt = (p.seq_q + QBLK_WG - 1) / QBLK_WG;
  const int nkt = (p.seq_kv + KT - 1) / KT;
  const bool has_tail = (p.seq_kv % KT) != 0;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  int task, k0, k1, slot;
  mapa_idx::attn_block_work(blockIdx.x, sp.n_dp, sp.chunks, nkt, task, k0, k1, slot);

  // Staging: piece = i*NW + wave is 8 rows x 128 B of K (piece < 8) or V; this lane's 16 B sit at tile row
  // srow[i] (XOR-swizzled 16-B column on the source so the LDS image stays lane-linear).  The byte offset inside
  // a tile is loop-invariant; a full tile adds one wave-uniform base per tile.
  // (the row and column are recomputed from the lane where the slow path needs them: keeping them as arrays
  // costs the segmented kernel its last free registers)
  auto srow = [&](int i) __attribute__((always_inline)) { return ((i * NW + wave) & 7) * 8 + (lane >> 3); };
  auto scol = [&](int i) __attribute__((always_inline)) {
    const int row = srow(i), pos = lane & 7;
    return (i >= NP / 2 ? (pos ^ (((row >> 1) & 1) << 2)) : (pos ^ ((row >> 1) & 7))) * 16;
  };
  uint32_t soff[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) soff[i] = (uint32_t)(srow(i) * (i >= NP / 2 ? p.vr : p.kr) * 2 + scol(i));
  // physical row of logical key `key0` when the whole tile [key0, key0+64) sits in one K/V segment, else -1
  auto seg_base = [&](int key0) -> int {
    if (!SEG) return key0;
    const int key1 = min(key0 + KT, p.seq_kv) - 1;
    int cum = 0;
#pragma unroll 1
    for (int s = 0; s < p.nseg; ++s) {
      const int len = p.seg_len[s];
      if (key0 >= cum && key0 < cum + len) return key1 < cum + len ? p.seg_start[s] + (key0 - cum) : -1;
      cum += len;
    }
    return -1;
  };

  {
    const int qt = task % nqt, hb = task / nqt, h = hb % p.heads, b = hb / p.heads;
    const bf16_t* qbase = reinterpret_cast<const bf16_t*>(p.q) + b * p.qb + h * 64;
    const char* kbase = reinterpret_cast<const char*>(reinterpret_cast<const bf16_t*>(p.k) + b * p.kb + h * 64);
    const char* vbase = reinterpret_cast<const char*>(reinterpret_cast<const bf16_t*>(p.v) + b * p.vb + h * 64);
    const int qrow = qt * QBLK_WG + wave * 32 + l32;

    auto stage = [&](int slot, int kt) {
      char* dst = lds + slot * 2 * TILE;
      const int key0 = kt * KT;
      const int r0 = seg_base(key0);
      const bool tail = key0 + KT > p.seq_kv;
      if (r0 >= 0 && !tail) {  // wave-uniform fast path: per-tile buffer descriptors + loop-invariant lane offsets
        const __amdgpu_buffer_rsrc_t rk =
            __builtin_amdgcn_make_buffer_rsrc((void*)(kbase + (int64_t)r0 * p.kr * 2), 0, 0x7fffffff, 0x00020000);
        const __amdgpu_buffer_rsrc_t rv =
            __builtin_amdgcn_make_buffer_rsrc((void*)(vbase + (int64_t)r0 * p.vr * 2), 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int i = 0; i < NP; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= NP / 2 ? rv : rk, (lds_ptr_t)(dst + (i * NW + wave) * 1024),
                                                   16, (int)soff[i], 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const bool isv = i >= NP / 2;
          const int key = key0 + srow(i);
          const int pr = SEG ? kv_row(p, key) : key;
          const int c_off = scol(i);
          const char* src = key < p.seq_kv
                                ? (isv ? vbase : kbase) + (int64_t)pr * (isv ? p.vr : p.kr) * 2 + c_off
                                : zero;
          __builtin_amdgcn_global_load_lds(src, dst + (i * NW + wave) * 1024, 16, 0, 0);
        }
      }
    };
    stage(0, k0);  // the first tile's DMA flies while Q is read

    // Q^T fragments (B operand): lane holds Q[q][kk*16 + 8*hl + j], pre-scaled by 1/8 * log2(e) so the
    // scores come out of the MFMA already in the log2 domain (one bf16 rounding of the scaled Q).
    bf16x8 qf[4];  // raw 16-bit operand words (bf16, or fp16 with F16)
    {
      const int qrow_c = qrow < p.seq_q ? qrow : p.seq_q - 1;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const s8v raw = *reinterpret_cast<const s8v*>(qbase + (int64_t)qrow_c * p.qr + kk * 16 + 8 * hl);
        if constexpr (F16) {
          f16x8_t sc;
#pragma unroll
          for (int j = 0; j < 8; ++j) sc[j] = (_Float16)(f16_to_f32((uint16_t)raw[j]) * (p.qscale * LOG2E));
          qf[kk] = __builtin_bit_cast(bf16x8, sc);
        } else {
          b8 sc;
#pragma unroll
          for (int j = 0; j < 8; ++j) sc[j] = (__bf16)(bf16_to_f32((bf16_t)raw[j]) * (p.qscale * LOG2E));
          qf[kk] = __builtin_bit_cast(bf16x8, sc);
        }
      }
    }

    f32x16 o[2];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
    float m_ref = 0.f, l_run = 0.f;
    // C operand of the first QK^T MFMA of every full tile: -m_ref in every element, kept in its own registers and
    // rewritten only when m_ref moves (no per-tile splat)
    f32x16 csplat;
#pragma unroll
    for (int r = 0; r < 16; ++r) csplat[r] = 0.f;
    auto set_ref = [&](float m) __attribute__((always_inline)) {
      m_ref = m;
#pragma unroll
      for (int r = 0; r < 16; ++r) csplat[r] = -m;
    };

    // One K/V tile: S^T = K Q^T, softmax, O^T += V^T P^T.  FIRST (a segment's first tile) sets m_ref; TAIL (the
    // last, partial tile of the key range) masks keys past seq_kv; SLOT = the LDS ring slot as a compile-time
    // constant (tiles alternate slots; the loops below unroll by two) so LDS addresses fold into immediates.
    auto tile = [&](int kt, auto first_tag, auto tail_tag, auto slot_tag) __attribute__((always_inline)) {
      constexpr bool FIRST = decltype(first_tag)::value;
      constexpr bool TAIL = decltype(tail_tag)::value;
      constexpr int cur = decltype(slot_tag)::value;
      const char* Ks = lds + cur * 2 * TILE;
      const char* Vs = Ks + TILE;
      // every LDS read of this tile is issued before the next tile's DMA, so the compiler's conservative
      // vmcnt(0) (an LDS-DMA may alias any LDS read) never lands inside the tile
      bf16x8 kf[2][4];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int row = kb * 32 + l32;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int chunk = kk * 2 + hl;
          kf[kb][kk] = *reinterpret_cast<const bf16x8*>(Ks + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
        }
      }
      // S^T - m_ref = K Q^T + C, C = -m_ref (masked keys of the tail tile: -inf)
      f32x16 st[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if constexpr (TAIL) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kt * KT + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
            st[kb][r] = key < p.seq_kv ? csplat[r] : -INFINITY;
          }
          st[kb] = mfma32x32x16<F16>(kf[kb][0], qf[0], st[kb]);
        } else {
          st[kb] = mfma32x32x16<F16>(kf[kb][0], qf[0], csplat);
        }
#pragma unroll
        for (int kk = 1; kk < 4; ++kk)
          st[kb] = mfma32x32x16<F16>(kf[kb][kk], qf[kk], st[kb]);
      }
      // V^T fragments (transposed LDS reads), then the next tile's DMA
      bf16x8 vf[2][2][2];
      {
        const int i4 = lane & 15, q4 = i4 >> 2, p4 = i4 & 3, grp = (lane >> 4) & 1;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int cc = dt * 32 + 16 * grp + 4 * p4;
          const int chunk = cc >> 3, within = (cc & 7) * 2;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              const int R0 = kb * 32 + 16 * s + 4 * hl + q4;
              const int R1 = R0 + 8;
              const s4v lo = tr_read(Vs + R0 * 128 + ((chunk ^ (((R0 >> 1) & 1) << 2)) << 4) + within);
              const s4v hi = tr_read(Vs + R1 * 128 + ((chunk ^ (((R1 >> 1) & 1) << 2)) << 4) + within);
              const s8v vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
              vf[dt][kb][s] = vv;
            }
        }
      }
      if (kt + 1 < k1) stage(cur ^ 1, kt + 1);

      // P = exp2(S - m_ref) -> bf16 fragments, row partial sums (this lane's 32 keys)
      bf16x8 pf[2][2];
      float ls;
      auto exp_pack = [&](float shift) __attribute__((always_inline)) {
        // four partial sums, seeded with the first four values (0 + e is not foldable: it would cost 4 adds)
        float a[4];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            if constexpr (F16) {
              f16x8_t t;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float e = __builtin_amdgcn_exp2f(st[kb][8 * s + j] - shift);
                a[j & 3] = (kb == 0 && s == 0 && j < 4) ? e : add_s(a[j & 3], e);
                t[j] = (_Float16)e;
              }
              pf[kb][s] = __builtin_bit_cast(bf16x8, t);
            } else {
              b8 t;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float e = __builtin_amdgcn_exp2f(st[kb][8 * s + j] - shift);
                a[j & 3] = (kb == 0 && s == 0 && j < 4) ? e : add_s(a[j & 3], e);
                t[j] = (__bf16)e;
              }
              pf[kb][s] = __builtin_bit_cast(bf16x8, t);
            }
          }
        ls = add_s(add_s(a[0], a[1]), add_s(a[2], a[3]));
      };
      auto row_max = [&]() __attribute__((always_inline)) {
        float mx = st[0][0];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[kb][r]);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        return fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      };
      if constexpr (FIRST) {
        const float d = row_max();  // finite: a segment's first tile always holds a valid key
        set_ref(d);
        exp_pack(d);
      } else {
        const float cur_ref = 0.f;  // (x - 0 folds: the MFMA produced s - m_ref)
        exp_pack(cur_ref);
        if (__builtin_expect(__any(!(ls <= REBASE_SUM)), 0)) {  // rebase (NaN-safe compare: inf sums rebase)
          const float d = fmaxf(row_max() - cur_ref, 0.f);
          set_ref(m_ref + d);
          const float alpha = __builtin_amdgcn_exp2f(-d);
          l_run *= alpha;
#pragma unroll
          for (int dt = 0; dt < 2; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
          exp_pack(cur_ref + d);
        }
      }
      l_run = add_s(l_run, ls);
      // O^T += V^T P^T : B = P^T straight from the S^T accumulator, A = V^T
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            o[dt] = mfma32x32x16<F16>(vf[dt][kb][s], pf[kb][s], o[dt]);
      __syncthreads();
    };

    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    __syncthreads();
    const bool tail_last = has_tail && k1 == nkt;
    const int kf_end = tail_last ? k1 - 1 : k1;  // full tiles of this segment: [k0, kf_end)
    if (kf_end == k0) {
      tile(k0, T_(), T_(), S0());  // a one-tile segment on the partial last tile
    } else {
      tile(k0, T_(), F_(), S0());
      int kt = k0 + 1;
#pragma unroll 1
      for (; kt + 1 < kf_end; kt += 2) {
        tile(kt, F_(), F_(), S1());
        tile(kt + 1, F_(), F_(), S0());
      }
      if (kt < kf_end) {
        tile(kt, F_(), F_(), S1());
        ++kt;
      }
      if (tail_last) {
        if ((kt - k0) & 1) tile(kt, F_(), T_(), S1());
        else tile(kt, F_(), T_(), S0());
      }
    }

    const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
    const float inv = 1.f / l_tot;
    if (k0 == 0 && k1 == nkt) {  // whole task in this workgroup: final output
      if (qrow < p.seq_q) {
        bf16_t* obase = reinterpret_cast<bf16_t*>(p.o) + b * p.ob + (int64_t)qrow * p.orr + h * 64;
        // lanes l and l+32 hold the two 4-column halves of each 8-column chunk of the same row: one permlane32_swap
        // per packed word hands lane l the chunk's second half of an even chunk pair and lane l+32 the first half of
        // the odd one, so every lane stores whole 16-B row segments (4 stores instead of 8 of 8 B)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int gp = 0; gp < 2; ++gp) {
            uint32_t y[2], x[2];  // y: chunk 2gp (columns +4*hl), x: chunk 2gp+1
#pragma unroll
            for (int w = 0; w < 2; ++w) {
              y[w] = pack_lp2(F16, o[dt][8 * gp + 2 * w] * inv, o[dt][8 * gp + 2 * w + 1] * inv);
              x[w] = pack_lp2(F16, o[dt][8 * gp + 4 + 2 * w] * inv, o[dt][8 * gp + 4 + 2 * w + 1] * inv);
              const auto sw = __builtin_amdgcn_permlane32_swap(y[w], x[w], false, false);
              y[w] = sw[0];
              x[w] = sw[1];
            }
            // lane hl = 0: columns 16gp .. +7 = (y, x); hl = 1: columns 16gp + 8 .. +15 = (y, x)
            const int d = dt * 32 + 16 * gp + 8 * hl;
            *reinterpret_cast<uint4*>(obase + d) = make_uint4(y[0], y[1], x[0], x[1]);
          }
        if (p.lse && hl == 0)
          p.lse[((int64_t)b * p.heads + h) * p.seq_q + qrow] = (m_ref + __log2f(l_tot)) * LN2;
      }
    } else {  // partial over tiles [k0, k1): normalised fp32 rows + LSE into this workgroup's slot
      const int r = wave * 32 + l32;
      float* po = sp.part_o + ((int64_t)slot * QBLK_WG + r) * 64;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int d = dt * 32 + 8 * gq + 4 * hl;
          const f32x4 v = {o[dt][4 * gq] * inv, o[dt][4 * gq + 1] * inv, o[dt][4 * gq + 2] * inv,
                           o[dt][4 * gq + 3] * inv};
          *reinterpret_cast<f32x4*>(po + d) = v;
        }
      if (hl == 0) sp.part_lse[(int64_t)slot * QBLK_WG + r] = (m_ref + __log2f(l_tot)) * LN2;
    }
  }
}

// Combines the K/V-chunk partials of the split tasks: MERGE_G adjacent lanes per (row, 4 columns) of a split task,
// each over every MERGE_G-th chunk, combined by a fixed butterfly (deterministic): ~43 chunks per row were a
// latency-bound serial walk in one thread (14.5 us per 8-view global layer).
constexpr int MERGE_G = 8;
template <int NW, bool F16 = false>
__global__ void __launch_bounds__(256) attn_split_merge(AttnArgs p, SplitArgs sp, int nsplit_rows) {
  constexpr int QBLK_WG = NW * 32;
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int g = e & (MERGE_G - 1), rc = e / MERGE_G;
  // every lane of a group stays for the shuffles; only the writes are predicated
  const bool live = rc < nsplit_rows * 16;
  const int c4 = rc & 15, rr = live ? rc >> 4 : 0;
  const int tt = rr / QBLK_WG, r = rr % QBLK_WG;  // split-task index, row in the block
  const int t = sp.n_dp + tt;
  const int nqt = (p.seq_q + QBLK_WG - 1) / QBLK_WG;
  const int qt = t % nqt, hb = t / nqt, h = hb % p.heads, b = hb / p.heads;
  const int qrow = qt * QBLK_WG + r;
  const int s0 = tt * sp.chunks;
  float mx = -INFINITY;
#pragma unroll 4
  for (int c = g; c < sp.chunks; c += MERGE_G) mx = fmaxf(mx, sp.part_lse[(int64_t)(s0 + c) * QBLK_WG + r]);
#pragma unroll
  for (int o = 1; o < MERGE_G; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float wsum = 0.f;
#pragma unroll 4
  for (int c = g; c < sp.chunks; c += MERGE_G) {
    const float w = __expf(sp.part_lse[(int64_t)(s0 + c) * QBLK_WG + r] - mx);
    wsum += w;
    acc += w * *reinterpret_cast<const f32x4*>(sp.part_o + ((int64_t)(s0 + c) * QBLK_WG + r) * 64 + c4 * 4);
  }
#pragma unroll
  for (int o = 1; o < MERGE_G; o <<= 1) {
    wsum += __shfl_xor(wsum, o, 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += __shfl_xor(acc[k], o, 64);
  }
  if (!live || g != 0 || qrow >= p.seq_q) return;
  const float inv = 1.f / wsum;
  uint2 pk;
  pk.x = pack_lp2(F16, acc[0] * inv, acc[1] * inv);
  pk.y = pack_lp2(F16, acc[2] * inv, acc[3] * inv);
  *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.o) + b * p.ob + (int64_t)qrow * p.orr + h * 64 + c4 * 4) = pk;
  if (p.lse && c4 == 0) p.lse[((int64_t)b * p.heads + h) * p.seq_q + qrow] = mx + __logf(wsum);
}

// ------------------------------------------------------------------------------------------------ f32
__global__ void __launch_bounds__(NT, 1) attn_fwd_f32(AttnArgs p) {
  constexpr int TILE = KT * 256;  // 64 rows x 256 B
  __shared__ __attribute__((aligned(1024))) char lds[2 * 2 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hl = lane >> 5, l32 = lane & 31;
  const int nqt = (p.seq_q + QBLK - 1) / QBLK;
  const int nblk = nqt * p.heads * p.batch;
  const int bid = xcd_remap(blockIdx.x, nblk);
  const int qt = bid % nqt, hb = bid / nqt, h = hb % p.heads, b = hb / p.heads;

  const float* qbase = reinterpret_cast<const float*>(p.q) + b * p.qb + h * 64;
  const float* kbase = reinterpret_cast<const float*>(p.k) + b * p.kb + h * 64;
  const float* vbase = reinterpret_cast<const float*>(p.v) + b * p.vb + h * 64;
  const int qrow = qt * QBLK + wave * 32 + l32;
  const int qrow_c = qrow < p.seq_q ? qrow : p.seq_q - 1;

  // lane half hl owns hd chunks 2c+hl (c = 0..7); step s of chunk-pair c uses hd 8c + 4hl + s
  f32x4 qf[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    qf[c] = *reinterpret_cast<const f32x4*>(qbase + (int64_t)qrow_c * p.qr + (2 * c + hl) * 4);
    qf[c] *= p.qscale;
  }
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  const int nkt = (p.seq_kv + KT - 1) / KT;

  auto stage = [&](int slot, int kt) {
    char* Ks = lds + slot * 2 * TILE;
    char* Vs = Ks + TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (i * 4 + wave) * 4 + (lane >> 4), pos = lane & 15;
      const int key = kt * KT + row;
      const int kc = pos ^ (row & 15);
      const int pr = kv_row(p, key);
      const char* ks = key < p.seq_kv ? reinterpret_cast<const char*>(kbase + (int64_t)pr * p.kr + kc * 4) : zero;
      const char* vs = key < p.seq_kv ? reinterpret_cast<const char*>(vbase + (int64_t)pr * p.vr + pos * 4) : zero;
      const int base = (i * 4 + wave) * 64 * 16;
      __builtin_amdgcn_global_load_lds(ks, Ks + base, 16, 0, 0);
      __builtin_amdgcn_global_load_lds(vs, Vs + base, 16, 0, 0);
    }
  };

  f32x16 o[2];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) stage(cur ^ 1, kt + 1);
    const char* Ks = lds + cur * 2 * TILE;
    const float* Vs = reinterpret_cast<const float*>(Ks + TILE);

    f32x16 st[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) st[kb][r] = 0.f;
      const int row = kb * 32 + l32;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int chunk = 2 * c + hl;
        const f32x4 kf = *reinterpret_cast<const f32x4*>(Ks + row * 256 + ((chunk ^ (row & 15)) << 4));
#pragma unroll
        for (int s = 0; s < 4; ++s) st[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[s], qf[c][s], st[kb], 0, 0, 0);
      }
    }
    const bool tail = (kt + 1) * KT > p.seq_kv;
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float s = st[kb][r] * LOG2E;
        if (tail) {
          const int key = kt * KT + kb * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
          if (key >= p.seq_kv) s = -INFINITY;
        }
        st[kb][r] = s;
        mx = fmaxf(mx, s);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float ls = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = exp2f(st[kb][r] - m_new);
        st[kb][r] = e;
        ls += e;
      }
    l_run = l_run * alpha + ls;
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[d][r] *= alpha;
    // O^T += V^T P^T, k-step s of key block kb uses key (s&3) + 8(s>>2) + 4hl: register s of the S^T tile.
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int key = kb * 32 + (s & 3) + 8 * (s >> 2) + 4 * hl;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[key * 64 + dt * 32 + l32], st[kb][s], o[dt], 0, 0, 0);
      }
    __syncthreads();
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  if (qrow < p.seq_q) {
    const float inv = 1.f / l_tot;
    float* obase = reinterpret_cast<float*>(p.o) + b * p.ob + (int64_t)qrow * p.orr + h * 64;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hl;
        f32x4 v = {o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv};
        *reinterpret_cast<f32x4*>(obase + d) = v;
      }
    if (p.lse && hl == 0) p.lse[((int64_t)b * p.heads + h) * p.seq_q + qrow] = (m_run + log2f(l_tot)) * LN2;
  }
}

// Merge of two attention partials over disjoint key sets (flash-decoding style):
//   w_a = exp(lse_a - m), w_b = exp(lse_b - m), m = max(lse_a, lse_b);  o = (w_a o_a + w_b o_b) / (w_a + w_b)
// o rows [rows][heads*64] (row stride ld), lse [heads][rows] (natural log, as attn_fwd writes it).
template <typename T, bool F16 = false>
__global__ void attn_merge_kernel(const T* __restrict__ oa, const float* __restrict__ la, const T* __restrict__ ob,
                                  const float* __restrict__ lb, T* __restrict__ out, float* __restrict__ lse_out,
                                  int rows, int heads, int64_t ld) {
  const int64_t total = (int64_t)rows * heads * 16;  // 4 values per thread
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int d4 = (int)(e % 16) * 4;
    const int64_t rh = e / 16;
    const int h = (int)(rh % heads);
    const int r = (int)(rh / heads);
    const float a = la[(int64_t)h * rows + r], b = lb[(int64_t)h * rows + r];
    const float m = fmaxf(a, b);
    const float wa = __expf(a - m), wb = __expf(b - m);
    const float inv = 1.f / (wa + wb);
    const int64_t o = (int64_t)r * ld + h * 64 + d4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float va, vb;
      if constexpr (sizeof(T) == 2) {
        va = lp_to_f32(F16, oa[o + j]);
        vb = lp_to_f32(F16, ob[o + j]);
      } else {
        va = oa[o + j];
        vb = ob[o + j];
      }
      const float v = (wa * va + wb * vb) * inv;
      if constexpr (sizeof(T) == 2) out[o + j] = f32_to_lp(F16, v);
      else out[o + j] = v;
    }
    if (lse_out && d4 == 0) lse_out[(int64_t)h * rows + r] = m + __logf(wa + wb);
  }
}

}  // namespace

extern "C" int mapa_attn_merge(const void* o_a, const float* lse_a, const void* o_b, const float* lse_b, void* o_out,
                               float* lse_out, int dtype, int rows, int heads, int64_t ld, hipStream_t stream) {
  MAPA_CHECK_ARG(o_a && lse_a && o_b && lse_b && o_out && rows > 0 && heads > 0 && ld >= (int64_t)heads * 64,
                 "mapa_attn_merge: bad args");
  const int64_t total = (int64_t)rows * heads * 16;
  int64_t g = (total + 255) / 256;
  if (g > 65536) g = 65536;
  if (dtype == MAPA_BF16)
    hipLaunchKernelGGL(attn_merge_kernel<bf16_t>, dim3((unsigned)g), dim3(256), 0, stream, (const bf16_t*)o_a, lse_a,
                       (const bf16_t*)o_b, lse_b, (bf16_t*)o_out, lse_out, rows, heads, ld);
  else if (dtype == MAPA_F16)
    hipLaunchKernelGGL((attn_merge_kernel<bf16_t, true>), dim3((unsigned)g), dim3(256), 0, stream, (const bf16_t*)o_a,
                       lse_a, (const bf16_t*)o_b, lse_b, (bf16_t*)o_out, lse_out, rows, heads, ld);
  else
    hipLaunchKernelGGL(attn_merge_kernel<float>, dim3((unsigned)g), dim3(256), 0, stream, (const float*)o_a, lse_a,
                       (const float*)o_b, lse_b, (float*)o_out, lse_out, rows, heads, ld);
  MAPA_CHECK_LAUNCH("mapa_attn_merge");
  return 0;
}

namespace {
constexpr int SK_NW = 4;  // waves per workgroup (4 x 32 query rows); 6/8-wave workgroups measured slower
constexpr int SK_QBLK = SK_NW * 32;

// Workgroups of attn_fwd_bf16 resident per CU: the 512-entry VGPR file over the kernel's allocation (one wave of
// the 4-wave workgroup per SIMD), capped by LDS; MAPA_ATTN_WG_PER_CU overrides.  Cached per device.
int sk_slots() {
  static int cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cache[dev]) return cache[dev];
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  hipFuncAttributes fa;
  int per_cu = 2;
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&attn_fwd_bf16<SK_NW, false>)) == hipSuccess &&
      fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    per_cu = 512 / alloc;
    const int lds_cap = (160 * 1024) / (int)(fa.sharedSizeBytes > 0 ? fa.sharedSizeBytes : 32768);
    if (lds_cap < per_cu) per_cu = lds_cap;
    if (per_cu < 1) per_cu = 1;
  }
  if (const char* e = getenv("MAPA_ATTN_WG_PER_CU")) per_cu = atoi(e) > 0 ? atoi(e) : per_cu;
  return cache[dev] = cus * per_cu;
}

int64_t sk_workspace_bytes(int slots) { return (int64_t)slots * SK_QBLK * (64 + 1) * sizeof(float); }
}  // namespace

extern "C" int64_t mapa_attention_workspace_bytes(const mapa_attn_desc* d) {
  if (!d || d->dtype != MAPA_BF16) return 0;
  return sk_workspace_bytes(sk_slots());
}

extern "C" int mapa_attention(const mapa_attn_desc* d, hipStream_t stream) {
  MAPA_CHECK_ARG(d != nullptr, "mapa_attention: null descriptor");
  MAPA_CHECK_ARG(d->batch > 0 && d->heads > 0 && d->seq_q > 0 && d->seq_kv > 0,
                 "mapa_attention: bad shape b=%d h=%d q=%d kv=%d", d->batch, d->heads, d->seq_q, d->seq_kv);
  MAPA_CHECK_ARG(d->q && d->k && d->v && d->o, "mapa_attention: null pointer");
  MAPA_CHECK_ARG(d->dtype == MAPA_BF16 || d->dtype == MAPA_F16 || d->dtype == MAPA_F32, "mapa_attention: bad dtype");
  const int align = d->dtype == MAPA_F32 ? 4 : 8;
  MAPA_CHECK_ARG(d->q_rstride % align == 0 && d->k_rstride % align == 0 && d->v_rstride % align == 0 &&
                     d->o_rstride % align == 0 && d->o_bstride % align == 0 &&
                     (reinterpret_cast<uintptr_t>(d->o) & 15) == 0,
                 "mapa_attention: output base and row / batch strides must keep 16-B alignment (16-B row stores)");
  AttnArgs a;
  a.q = d->q; a.k = d->k; a.v = d->v; a.o = d->o; a.lse = d->lse;
  a.qb = d->q_bstride; a.qr = d->q_rstride; a.kb = d->k_bstride; a.kr = d->k_rstride;
  a.vb = d->v_bstride; a.vr = d->v_rstride; a.ob = d->o_bstride; a.orr = d->o_rstride;
  a.batch = d->batch; a.heads = d->heads; a.seq_q = d->seq_q; a.seq_kv = d->seq_kv;
  MAPA_CHECK_ARG(d->scale >= 0.f && d->scale < 1e30f, "mapa_attention: bad scale %g", (double)d->scale);
  a.qscale = d->scale > 0.f ? d->scale : 0.125f;
  MAPA_CHECK_ARG(d->kv_nseg >= 0 && d->kv_nseg <= MAPA_MAX_KV_SEGMENTS, "mapa_attention: kv_nseg out of range");
  a.nseg = d->kv_nseg;
  int64_t tot = 0;
  for (int s = 0; s < d->kv_nseg; ++s) {
    a.seg_start[s] = d->kv_seg_start[s];
    a.seg_len[s] = d->kv_seg_len[s];
    MAPA_CHECK_ARG(d->kv_seg_len[s] >= 0 && d->kv_seg_start[s] >= 0, "mapa_attention: bad kv segment");
    tot += d->kv_seg_len[s];
  }
  MAPA_CHECK_ARG(d->kv_nseg == 0 || tot == d->seq_kv, "mapa_attention: kv segments sum %lld != seq_kv %d",
                 (long long)tot, d->seq_kv);
  if (d->dtype != MAPA_F32) {  // bf16 or fp16 operands: the MFMA flash kernel
    const bool f16 = d->dtype == MAPA_F16;
    const int ntask = ((d->seq_q + SK_QBLK - 1) / SK_QBLK) * d->heads * d->batch;
    const int nkt = (d->seq_kv + KT - 1) / KT;
    SplitArgs sp;
    sp.part_o = nullptr;
    sp.part_lse = nullptr;
    sp.n_dp = ntask;
    sp.chunks = 1;
    // the remainder after the full waves of resident slots is cut into K/V chunks of >= 4 tiles (or not at all
    // without a workspace)
    const int slots = sk_slots();
    int n_dp, chunks;
    mapa_idx::attn_split_plan(ntask, nkt, slots, n_dp, chunks);
    if (chunks > 1 && d->workspace && d->workspace_bytes >= sk_workspace_bytes(slots) &&
        getenv("MAPA_ATTN_NO_SPLIT") == nullptr) {
      sp.n_dp = n_dp;
      sp.chunks = chunks;
      sp.part_o = reinterpret_cast<float*>(d->workspace);
      sp.part_lse = sp.part_o + (int64_t)slots * SK_QBLK * 64;
    }
    const int grid = sp.n_dp + (ntask - sp.n_dp) * sp.chunks;
    if (f16) {
      if (a.nseg > 0)
        hipLaunchKernelGGL((attn_fwd_bf16<SK_NW, true, true>), dim3(grid), dim3(SK_NW * 64), 0, stream, a, sp);
      else
        hipLaunchKernelGGL((attn_fwd_bf16<SK_NW, false, true>), dim3(grid), dim3(SK_NW * 64), 0, stream, a, sp);
    } else if (a.nseg > 0) {
      hipLaunchKernelGGL((attn_fwd_bf16<SK_NW, true>), dim3(grid), dim3(SK_NW * 64), 0, stream, a, sp);
    } else {
      hipLaunchKernelGGL((attn_fwd_bf16<SK_NW, false>), dim3(grid), dim3(SK_NW * 64), 0, stream, a, sp);
    }
    MAPA_CHECK_LAUNCH("mapa_attention");
    if (sp.n_dp < ntask) {
      const int rows = (ntask - sp.n_dp) * SK_QBLK;
      if (f16)
        hipLaunchKernelGGL((attn_split_merge<SK_NW, true>), dim3((rows * 16 * MERGE_G + 255) / 256), dim3(256), 0,
                           stream, a, sp, rows);
      else
        hipLaunchKernelGGL((attn_split_merge<SK_NW>), dim3((rows * 16 * MERGE_G + 255) / 256), dim3(256), 0, stream,
                           a, sp, rows);
      MAPA_CHECK_LAUNCH("mapa_attention (split merge)");
    }
    return 0;
  }
  const int nblk = ((d->seq_q + QBLK - 1) / QBLK) * d->heads * d->batch;
  hipLaunchKernelGGL(attn_fwd_f32, dim3(nblk), dim3(NT), 0, stream, a);
  MAPA_CHECK_LAUNCH("mapa_attention");
  return 0;
}
