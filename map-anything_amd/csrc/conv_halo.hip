// 3x3 stride-1 convolution (pad 1) as an MFMA GEMM whose A operand is read from an LDS halo window, for gfx950.
//
//   out[img][oy][ox][n] = sum_{ky,kx,c} X[img][oy+ky-1][ox+kx-1][c] * W[n][c/32][ky*3+kx][c%32]   (+ fused epilogue)
//
// Why: the implicit-GEMM conv (gemm_big.hip, A mode 1) stages every input pixel once per tap — 9 copies of the
// 256-pixel tile's neighbourhood per 32-channel slice through L2 -> LDS.  Timing without that A staging measured
// 1.5-1.6x faster on the DPT head convs (rn1/l1rn at 148^2), so here the tile's 18x18 input window of a 32-channel
// slice is DMA'd ONCE (20.7 KiB) and the 9 taps read their A fragments from it at shifted addresses: 7x less
// operand staging for A.  Weights use the channel-block-major K order of mapa_gemm_desc.conv_kblock = 32, so K tile
// kt is (slice kt / 9, tap kt % 9) and the W tile of kt is 32 contiguous columns.
//  * Output tile: a 16x16 pixel block (M = 256 rows, pixel (py, px) = row py*16 + px) x BN output channels.
//    BN = 256: 8 waves as 2 (M) x 4 (N), wave tile 128x64 (1 workgroup / CU); BN = 128: 4 x 2, wave tile 64x64,
//    <= 128 VGPRs (2 workgroups / CU: one tile's epilogue overlaps the other's main loop).
//  * A fragment (16x16x32 MFMA) for block row py and tap (ky, kx): lane (px, g) reads 16 B = channels 8g..8g+7 of
//    window pixel wp = (py+ky)*18 + px+kx.  Window image: pixel-major, 64 B per pixel, 16-B chunk g stored at
//    position win_pos(g, wp): conflict-free in ds_read_b128's lane groups for every tap shift (see win_pos; the
//    earlier g ^ ((wp >> 2) & 3) was 2-way in those groups: 29 % of the LDS cycles were conflict cycles).
//  * W tiles (BN x 64 B, 16-B chunks XOR-swizzled as gemm_big's 64-B rows) stream through a ring of S slots,
//    each DMA'd S-1 K tiles ahead; the window of slice c+1 rides in the DMA group of K tile 9(c+1) (two window
//    buffers).  Counted vmcnt over the groups still in flight + raw s_barrier (no drain in the loop).
//  * The 9 taps of a slice are unrolled: vmcnt depths, tap shifts and window staging are compile-time, and every A
//    fragment read is one of 8 per-slice base addresses + an immediate (no per-read VALU, few SALU per step).
#include <type_traits>

#include "gemm_internal.h"

namespace mapa_gemm_impl {
namespace {

constexpr int HT = 512;           // threads
constexpr int BW = 16;            // output block width (pixels): one MFMA row fragment = one block row
constexpr int WE = BW + 2;        // window width
constexpr int H_ELD = 68;

// BN output channels x a BH x 16 pixel block.  BH = 16: (BN 256) 8 waves 2 x 4 of 128x64, 1 workgroup / CU, or
// (BN 128) 4 x 2 of 64x64, 2 / CU.  BH = 8 with BN 256: 2 x 4 waves of 64x64, 2 / CU — for 148^2 maps, where 16-row
// blocks leave 17 % of the pixels idle (160 vs 148 rows) and 1600 tiles fill 3.1 rounds of 512 slots, 8-row blocks
// cover 152 rows in 1520 tiles (2.97 rounds) and stage each window once for all 256 output channels.
template <int BN, int BH = 16>
struct HCfg {
  static constexpr int WM = (BN == 256) ? 2 : 4, WN = 8 / WM;
  static constexpr int TM = BH * BW / WM, TN = BN / WN;  // 128x64, 64x64 or 64x64
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int S = BH == 8 ? 3 : BN == 256 ? 6 : 4;  // W ring slots
  static constexpr int WT = BN * 64;                          // W tile bytes (32 bf16 per row)
  static constexpr int NWG = WT / (HT * 16);                  // W DMA instructions per thread per K tile (2 or 1)
  static constexpr int WH = BH + 2;                           // window rows
  static constexpr int WPIECES = WH * WE * 4;                 // 16-B pieces per window (64 B per pixel)
  static constexpr int WROUNDS = (WPIECES + HT - 1) / HT;     // DMA instructions per thread per window (3 or 2)
  static constexpr int WBYTES = WROUNDS * HT * 16;            // window buffer (tail pieces land in padding)
  static constexpr int LDS = S * WT + 2 * WBYTES;             // 144, 80 or 80 KiB
  static constexpr int MINB = (BN == 256 && BH == 16) ? 1 : 2;
  static_assert(TN == 64 && FM % 2 == 0 && FM * WM == BH, "epilogue: 64-column wave tiles, 32-row passes");
  static_assert(8 * 32 * H_ELD * 4 <= LDS, "epilogue staging");
};

// Fused regressor tail (HO = true, BN = 128): instead of the ReLU'd 128-channel hidden map, the epilogue computes the
// 1x1 conv 128 -> 6 of every pixel and the dense-head adaptors / output assembly (dense_head_pixel).
struct HeadOut {
  const float* w6;    // [6][128]
  const float* b6;    // [6]
  const float* pose;  // [views][19] pose_out rows of this launch's views
  const float* scale; // metric scale: scale[img / vps] for the launch's image img
  int vps;            // consecutive images sharing one scale value (>= the launch's images: one scene)
  float *pts3d, *pts3d_cam, *rays, *depth, *conf, *logits;
  uint8_t* mask;
};

// Flat-raster blocks (FLAT = true; maps up to 62 pixels wide: the 19^2 / 37^2 DPT convs, where 16x16 blocks leave
// 41-65 % of the pixels idle and give only 26-144 tiles): a block is 256 consecutive positions of the images' padded
// raster (mapa_idx::flat_pixel: rows of OW + 1, OH + 1 rows per image, 94-95 % of the positions real pixels); the 9
// taps read the 1-D window of 256 + 2(OW+1) + 2 positions at shifts dy(OW+1) + dx.  Too few tiles for the CUs, so
// the 32-channel slices are split over nsplit workgroups per tile: each stores its fp32 partial sums to a slab with
// write-through (sc1) stores and draws a ticket (agent-scope relaxed add, as gemm_big.hip's stream-K); the last
// arriver reads every slab with sc1 loads, sums them in part order (bit-reproducible whatever the arrival order),
// re-zeroes the ticket and runs the epilogue.  No workgroup waits on another.
struct HSplit {
  int nsplit;    // K parts per tile (1: no slabs, no tickets)
  int nblk;      // flat blocks
  int* tickets;  // [tiles], zero between launches
  float* slabs;  // [tiles * nsplit][256 * BN] fp32 accumulator images in fragment order
};
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int FLAT_MAX_WP = 63;  // window of 256 + 2 * Wp + 2 <= 384 positions (the 3-round window buffer)

__device__ __forceinline__ int swz64(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }

template <int N>
__device__ __forceinline__ void vm_wait_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(n) for a runtime n in [0, 15]
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    case 0: vm_wait_le<0>(); break;
    case 1: vm_wait_le<1>(); break;
    case 2: vm_wait_le<2>(); break;
    case 3: vm_wait_le<3>(); break;
    case 4: vm_wait_le<4>(); break;
    case 5: vm_wait_le<5>(); break;
    case 6: vm_wait_le<6>(); break;
    case 7: vm_wait_le<7>(); break;
    case 8: vm_wait_le<8>(); break;
    case 9: vm_wait_le<9>(); break;
    case 10: vm_wait_le<10>(); break;
    case 11: vm_wait_le<11>(); break;
    case 12: vm_wait_le<12>(); break;
    case 13: vm_wait_le<13>(); break;
    case 14: vm_wait_le<14>(); break;
    default: vm_wait_le<15>(); break;
  }
}

// Window image chunk position of channel chunk g (channels 8g..8g+7) of window pixel wp: pos = bswap2(g) ^ bit 2 of
// wp.  ds_read_b128 serves a wave in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and the same +32),
// and an A fragment's lanes read 16 consecutive window pixels from an arbitrary start (the tap shift): in every
// group each pixel residue mod 4 (= its 64-B bank quarter) is read by 4 lanes at pixels P, P+4, P+8, P+12 with
// chunks {0,1,1,0} or {1,0,0,1} (+2 for the upper half-wave), and this map sends those to 4 distinct 16-B slots for
// every P — conflict-free (the plain g ^ ((wp >> 2) & 3) of 16 contiguous lanes is 2-way in these groups).
__device__ __forceinline__ int win_pos(int g, int wp) { return (((g & 1) << 1) | (g >> 1)) ^ ((wp >> 2) & 1); }
// its inverse: the chunk stored at position pos
__device__ __forceinline__ int win_chunk(int pos, int wp) { return (((pos & 1) << 1) | (pos >> 1)) ^ (((wp >> 2) & 1) << 1); }

// DMA of K tile kt's W tile into ring slot `slot` (a device function, not a lambda in the kernel: with a lambda the
// host pass drops the kernel's launch stub)
// (buffer loads from the tile's W rows: the per-lane part of the address is a 32-bit offset, the K offset rides in
// soffset — no 64-bit per-lane pointers live across the K loop)
typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int BN, int BH>
__device__ __forceinline__ void stage_w(char* wring, int slot, int wave, __amdgpu_buffer_rsrc_t wr, const int* w_off,
                                        int koff) {
  using C = HCfg<BN, BH>;
  char* dst = wring + slot * C::WT + wave * 1024;
#pragma unroll
  for (int i = 0; i < C::NWG; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_ptr_t)(dst + i * 8192), 16, w_off[i], koff, 0, 0);
}
// DMA of the input window of the 32 physical channels starting at `ch` into window buffer `buf` (dummy: the zero
// page into that buffer — the uniform group past the last slice, which nothing reads)
// wsrc[r]: element offset of this thread's piece r from abase (-1: outside the map, the zero page)
template <bool WIDE> struct WinOff { typedef int type; };
template <> struct WinOff<true> { typedef int64_t type; };
template <int BN, int BH, typename OffT>
__device__ __forceinline__ void stage_win_t(const char* abase, char* wins, int buf, int64_t ch, int wave,
                                            const OffT* wsrc, bool dummy) {
  using C = HCfg<BN, BH>;
  const char* zero = reinterpret_cast<const char*>(g_mapa_zero_page);
  if (dummy) ch = 0;
  char* wd = wins + buf * C::WBYTES + wave * 1024;
#pragma unroll
  for (int r = 0; r < C::WROUNDS; ++r)
    __builtin_amdgcn_global_load_lds(wsrc[r] >= 0 && !dummy ? abase + (wsrc[r] + ch) * 2 : zero, wd + r * (HT * 16), 16,
                                     0, 0);
}
// 2-D blocks: the window lies in one image; a buffer descriptor over that image, a 32-bit byte offset per piece
// (pieces outside the map carry an offset past the descriptor's range: the buffer load returns zeros) and the
// channel offset in soffset
template <int BN, int BH>
__device__ __forceinline__ void stage_win(__amdgpu_buffer_rsrc_t ir, char* wins, int buf, int64_t ch, int wave,
                                          const int* wsrc, bool dummy) {
  using C = HCfg<BN, BH>;
  char* wd = wins + buf * C::WBYTES + wave * 1024;
  const int so = dummy ? 0 : (int)ch * 2;
#pragma unroll
  for (int r = 0; r < C::WROUNDS; ++r)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ir, (lds_ptr_t)(wd + r * (HT * 16)), 16, wsrc[r], so, 0, 0);
}
template <int BN, int BH>
__device__ __forceinline__ void stage_win(const char* abase, char* wins, int buf, int64_t ch, int wave,
                                          const int64_t* wsrc, bool dummy) {
  stage_win_t<BN, BH, int64_t>(abase, wins, buf, ch, wave, wsrc, dummy);
}

// F16: fp16 operands (the TF32-equivalent heads' MAPA_F16X2 split rows against f16 weights); same staging and tiles
template <int BN, bool HO = false, int BH = 16, bool FLAT = false, bool F16 = false>
__global__ void __launch_bounds__(HT, (2 * HCfg<BN, BH>::MINB)) conv_halo_kernel(GemmArgs p, HeadOut ho, HSplit sp) {
  using C = HCfg<BN, BH>;
  static_assert(!FLAT || (BN == 128 && BH == 16 && !HO), "flat blocks: 128-wide tiles of 256 positions");
  __shared__ __attribute__((aligned(1024))) char lds[C::LDS];
  char* const wring = lds;
  char* const wins = lds + C::S * C::WT;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  // ---- tile: (img, block row, block col, column tile), XCD-contiguous ranges of neighbouring blocks; FLAT: (flat
  // block, column tile, K part)
  const int ntn = p.N / BN;
  const int imgs = p.M / (p.cv_OH * p.cv_OW);
  const int Wp = p.cv_OW + 1, Hp = p.cv_OH + 1;  // FLAT raster geometry
  int img = 0, by = 0, bx = 0, tn, fb = 0, kp = 0;
  if constexpr (FLAT) {
    mapa_idx::halo_flat_tile(blockIdx.x, sp.nblk, ntn, sp.nsplit, fb, tn, kp);
  } else {
    const int nbx = (p.cv_OW + BW - 1) / BW, nby = (p.cv_OH + BH - 1) / BH;
    mapa_idx::halo_block(blockIdx.x, imgs, nby, nbx, ntn, img, by, bx, tn);
  }
  const int bn = tn * BN;
  const int nk = p.K / 32;  // 9 taps x (logical channels / 32)
  const int nslice = nk / 9;
  // this workgroup's slices [s_lo, s_hi): all of them, or K part kp of nsplit
  const int s_lo = FLAT ? (int)((int64_t)kp * nslice / sp.nsplit) : 0;
  const int s_hi = FLAT ? (int)((int64_t)(kp + 1) * nslice / sp.nsplit) : nslice;

  // ---- window staging geometry (this thread's WROUNDS pieces; pixel offsets are slice-invariant)
  // FLAT windows span images (offsets from A); a 2-D block's window lies in one image: 32-bit offsets from its base
  typename WinOff<FLAT>::type wsrc[C::WROUNDS];
  const char* abase = reinterpret_cast<const char*>(p.A) +
                      (FLAT ? 0 : (int64_t)img * p.cv_IH * p.cv_IW * p.cv_Cp * 2);
  const int img_bytes = FLAT ? 0 : p.cv_IH * p.cv_IW * p.cv_Cp * 2;  // < 2^31 (launch_conv_halo checks)
  const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc((void*)abase, 0, img_bytes, 0x00020000);
#pragma unroll
  for (int r = 0; r < C::WROUNDS; ++r) {
    const int q = r * HT + tid;
    const int wp = q >> 2, cl = q & 3;
    const int cs = win_chunk(cl, wp);  // LDS position cl holds channel chunk cs
    if constexpr (FLAT) {
      int im, iy, ix;  // window position wp = raster position fb*256 - Wp - 1 + wp
      const bool ok = wp < 256 + 2 * Wp + 2 &&
                      mapa_idx::flat_pixel(fb * 256 - Wp - 1 + wp, Wp, Hp, p.cv_OH, p.cv_OW, imgs, im, iy, ix);
      wsrc[r] = ok ? ((int64_t)(im * p.cv_IH + iy) * p.cv_IW + ix) * p.cv_Cp + cs * 8 : -1;
    } else {
      const int wy = wp / WE, wx = wp - wy * WE;
      const int iy = by * BH - 1 + wy, ix = bx * BW - 1 + wx;
      const bool ok = q < C::WPIECES && iy >= 0 && iy < p.cv_IH && ix >= 0 && ix < p.cv_IW;
      wsrc[r] = ok ? ((iy * p.cv_IW + ix) * p.cv_Cp + cs * 8) * 2 : 0x7ff00000;  // bytes in the image; past it: 0
    }
  }
  // ---- W staging geometry: instruction i of this wave covers ring rows (i*8 + wave)*16 + [0, 16)
  int w_src[C::NWG];  // byte offsets from the tile's first W row
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<const char*>(p.W) + (int64_t)bn * p.ldw * 2), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int i = 0; i < C::NWG; ++i) {
    const int r = (i * 8 + wave) * 16 + (lane >> 2);
    const int sc = (lane & 3) ^ swz64(r);
    w_src[i] = (r * (int)p.ldw + sc * 8) * 2;
  }
  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef bf16x8 b8;  // raw 16-bit operand words (bf16, or fp16 with F16)
  const int g = lane >> 4, r16 = lane & 15;
  // B fragment j of this lane: ring row rb = wn*TN + j*16 + r16; the swizzle depends on bits 2-3 of rb only, so
  // fragment j sits at b_off + j*1024 (an immediate offset of one address)
  const int rb0 = wn * C::TN + r16;
  const int b_off = rb0 * 64 + ((g ^ swz64(rb0)) << 4);
  // window pixel of (block row wm*FM, px = r16) at tap (0, 0); FLAT: of position (wm*FM)*16 + r16
  const int wp0 = (wm * C::FM) * (FLAT ? BW : WE) + r16;
  // A fragment of window pixel wp0 + c: byte (wp0 + c)*64 + win_pos(g, wp0 + c)*16, and bit 2 of wp0 + c depends on
  // c mod 8 only -> a_off[c % 8] + c*64, an immediate offset for every (tap, row) pair.  FLAT: the tap shift
  // dy*Wp + dx is a runtime value, so each tap gets one address (+ i*1024 per block row i: 16 positions on)

  // K loop over A-slices (the 32 physical channels one window holds), the K steps of a slice unrolled, so the tap
  // shift, the vmcnt depth of every step and which steps stage a window are compile-time constants.  Each step
  // consumes one W tile from ring slot `so`; the DMA group issued at step q is W step q+S-1 (+ the next A-slice's
  // window when q+S-1 starts it).  Every step issues exactly one group, also past the end (the last slice re-stages
  // the last W tile and a dummy window into slots / the buffer nobody reads any more), so the counted waits hold in
  // every slice with no last-slice branch: a peeled last slice spilled VGPRs, and scratch traffic inside a
  // counted-vmcnt region breaks the count (a spill store can retire before an older LDS-DMA).
  //  * plain operands (and the flat-raster split-K parts): A-slice = logical slice s, 9 steps (one per tap), W step
  //    q at K column (s_lo*9 + q)*32;
  //  * split-precision operands (the fp32-exact heads: logical K blocks [hi | hi | lo] against W [hi | lo | hi]): the
  //    NH hi slices first, each window staged ONCE for both of its logical slices — 18 steps, (tap, w_hi) then (tap,
  //    w_lo), the A fragments read at the first and reused at the second (a third fewer window DMAs and a quarter
  //    fewer LDS fragment reads than visiting the hi slice twice) — then the NH lo slices, 9 steps each.  Same MFMAs
  //    per output, accumulated in another order.
  const bool paired = !FLAT && p.sp_half != 0x7fffffff;
  const int NH = paired ? p.sp_half / 32 : 0;
  const int n_aslice = paired ? 2 * NH : s_hi - s_lo;
  const int64_t kfirst = (int64_t)s_lo * 9 * 64;
  const int64_t klast = ((int64_t)s_hi * 9 - 1) * 64;
  // W source offsets (bytes), branch-free inside the unrolled bodies: step r of A-slice a stages from
  // base(a) + (r & 1) * odd(a) + (r >> 1) * pair(a) — a paired hi slice: base a*576, odd = the w_lo block (NH*576),
  // pair = 64 (one tap); a 9-step slice: base (its logical slice)*576, odd 64, pair 128 (r * 64); past the last
  // slice: the last W tile again (dummy groups).
  const int hop = NH * 576;
  const int kfirst32 = s_lo * 576, klast32 = (s_hi * 9 - 1) * 64;  // K byte offsets fit 32 bits (K <= 9 * 2^12)
  // the W step sequence of A-slice a: {base, odd, pair} as above (a >= n_aslice: the dummy groups past the end)
  auto wbase = [&](int a) __attribute__((always_inline)) -> int {
    return a >= n_aslice ? klast32 : a < NH ? a * 576 : paired ? (a + NH) * 576 : kfirst32 + a * 576;
  };
  // physical channel of A-slice a (its window)
  auto aslice_ch = [&](int a) __attribute__((always_inline)) -> int64_t {
    return paired ? (int64_t)a * 32 : (int64_t)split_col(p, (s_lo + a) * 32);
  };
  {
    const int b0 = wbase(0);
    const int odd0 = NH > 0 ? hop : 64, pair0 = NH > 0 ? 64 : 128;
    stage_w<BN, BH>(wring, 0, wave, wr, w_src, b0);  // group 0: the first W tile + the first A-slice's window
    if constexpr (FLAT) stage_win<BN, BH>(abase, wins, 0, aslice_ch(0), wave, wsrc, false);
    else stage_win<BN, BH>(ir, wins, 0, aslice_ch(0), wave, wsrc, false);
#pragma unroll
    for (int s0 = 1; s0 < C::S - 1; ++s0) stage_w<BN, BH>(wring, s0, wave, wr, w_src, b0 + (s0 & 1) * odd0 + (s0 >> 1) * pair0);
  }
  int so = 0;
  auto slice_body = [&](int a, auto steps_tag) __attribute__((always_inline)) {
    constexpr int STEPS = decltype(steps_tag)::value;
    constexpr bool PAIRED = STEPS == 18;
    // W offsets: this slice (its type is this body's) and the next (paired, 9-step or past the end)
    const int bc = wbase(a), bn_ = wbase(a + 1);
    const bool nlast = a + 1 >= n_aslice, npair = a + 1 < NH;
    const int odd_n = nlast ? 0 : npair ? hop : 64, pair_n = nlast ? 0 : npair ? 64 : 128;
    // recomputed per slice (8 VGPRs live in the slice loop, not 8 more hoisted across it): the empty asm hides
    // wp0's loop invariance from LICM
    int wpl = wp0;
    asm volatile("" : "+v"(wpl));
    const int woff = (int)(wins - lds) + (a & 1) * C::WBYTES;
    int a_off[8];
    if constexpr (!FLAT) {
#pragma unroll
      for (int r = 0; r < 8; ++r) a_off[r] = wpl * 64 + (win_pos(g, wpl + r) << 4) + woff;
    }
#pragma unroll
    for (int st = 0; st < STEPS; ++st) {
      const int tap = PAIRED ? st >> 1 : st;
      // groups issued after this step's W tile, still allowed in flight: W tiles +1 .. +S-2, plus the window riding
      // with the next A-slice's first step (issued at step STEPS - S + 1)
      vm_wait(C::NWG * (C::S - 2) + (st >= STEPS - C::S + 2 ? C::WROUNDS : 0));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // this tile landed everywhere; every wave is done with the last (re-staged next)
      __builtin_amdgcn_sched_barrier(0);
      {
        const int r = st + C::S - 1;  // the W step this group stages: in this slice, or r - STEPS in the next
        int ko;
        if (r < STEPS) ko = bc + (PAIRED ? (r & 1) * hop + (r >> 1) * 64 : r * 64);
        else ko = bn_ + ((r - STEPS) & 1) * odd_n + ((r - STEPS) >> 1) * pair_n;
        stage_w<BN, BH>(wring, so == 0 ? C::S - 1 : so - 1, wave, wr, w_src, ko);
      }
      if (st == STEPS - C::S + 1) {
        const int64_t nch = a + 1 < n_aslice ? aslice_ch(a + 1) : 0;
        if constexpr (FLAT) stage_win<BN, BH>(abase, wins, (a + 1) & 1, nch, wave, wsrc, a + 1 == n_aslice);
        else stage_win<BN, BH>(ir, wins, (a + 1) & 1, nch, wave, wsrc, a + 1 == n_aslice);
      }
      const char* Ws = wring + so * C::WT + b_off;
      so = so + 1 == C::S ? 0 : so + 1;
      b8 b[C::FN];
#pragma unroll
      for (int j = 0; j < C::FN; ++j) b[j] = *reinterpret_cast<const b8*>(Ws + j * 1024);
      const char* at = lds;
      if constexpr (FLAT) {
        const int wt = wpl + (tap / 3) * Wp + tap % 3;  // window position of (tap, block row 0)
        at = lds + wt * 64 + (win_pos(g, wt) << 4) + woff;
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i) {
        b8 ai;
        if constexpr (FLAT) {
          ai = *reinterpret_cast<const b8*>(at + i * 1024);
        } else {
          const int c = (tap / 3 + i) * WE + tap % 3;  // window pixel offset of (tap, block row i)
          ai = *reinterpret_cast<const b8*>(lds + a_off[c & 7] + c * 64);
        }
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
          acc[i][j] = mfma16x16x32<F16>(ai, b[j], acc[i][j]);
      }
    }
  };
  int a = 0;
  if constexpr (!FLAT) {
#pragma unroll 1
    for (; a < NH; ++a) slice_body(a, std::integral_constant<int, 18>());
  }
#pragma unroll 1
  for (; a < n_aslice; ++a) slice_body(a, std::integral_constant<int, 9>());
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // LDS becomes the epilogue staging area

  if constexpr (FLAT) {
    if (sp.nsplit > 1) {
      // ---- split K: publish this part's partial sums; the last arriver sums every part's slab in part order
      constexpr int SLAB = 256 * BN;
      const int tile = fb * ntn + tn;
      const int voff = lane * 16;
      {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(sp.slabs + ((int64_t)tile * sp.nsplit + kp) * SLAB, 0,
                                                          SLAB * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
          for (int j = 0; j < C::FN; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, voff,
                                                   ((wave * C::FM + i) * C::FN + j) * 1024, 16);  // sc1
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
      __syncthreads();
      int* last_word = reinterpret_cast<int*>(lds + C::LDS - 16);  // above the epilogue staging rows
      if (tid == 0) {
        const int ticket = __hip_atomic_fetch_add(&sp.tickets[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = ticket == sp.nsplit - 1;
        if (last) __hip_atomic_store(&sp.tickets[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last_word = last;
      }
      __syncthreads();
      const int last = *last_word;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the slab loads below the ticket
      if (!last) return;
      for (int b = 0; b < sp.nsplit; ++b) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(sp.slabs + ((int64_t)tile * sp.nsplit + b) * SLAB, 0,
                                                          SLAB * 4, 0x00020000);
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // half a slab in flight at a time
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
              a = b == 0 ? v[i][j] : a + v[i][j];
            }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  }

  if constexpr (HO) {
    // ---- fused regressor tail.  Lane (r16, g) holds relu(acc + bias) of pixels g*4 + r of block rows wm*FM + i at
    // channels wn*64 + j*16 + r16: per block row it forms the 6 partial dot products of its 4 pixels over its 4
    // channels, a reduce-scatter over the 16 lanes of its group (then a pairwise sum) leaves 3 of them per lane
    // pair, and the two channel halves (waves wn = 0, 1) meet in LDS.
    static_assert(BN == 128 && BH == 16 && C::FM == 4 && C::FN == 4, "head-out tail: 128-wide 16x16 tiles");
    float* part = reinterpret_cast<float*>(lds);  // [256 pixels][2 halves][6]
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // one block row (16 pixels of which this lane group holds 4) at a time
      float v[24];
#pragma unroll
      for (int k = 0; k < 24; ++k) v[k] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = wn * 64 + j * 16 + r16;
        const float bj = p.bias[ch];
        float wv[6];
#pragma unroll
        for (int o = 0; o < 6; ++o) wv[o] = ho.w6[o * 128 + ch];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = fmaxf(acc[i][j][r] + bj, 0.f);
#pragma unroll
          for (int o = 0; o < 6; ++o) v[r * 6 + o] += x * wv[o];
        }
      }
#define HO_STAGE(M, HALF)                                                \
  {                                                                      \
    const bool up = (r16 & (M)) != 0;                                    \
    _Pragma("unroll") for (int t = 0; t < (HALF); ++t) {                 \
      const float mine = up ? v[(HALF) + t] : v[t];                      \
      const float other = up ? v[t] : v[(HALF) + t];                     \
      v[t] = mine + __shfl_xor(other, (M), 64);                          \
    }                                                                    \
  }
      HO_STAGE(8, 12) HO_STAGE(4, 6) HO_STAGE(2, 3)
#undef HO_STAGE
      // lanes r16 and r16 ^ 1 hold partial sums of the same 3 values: segment s = r16 >> 1 (row s >> 1, outputs
      // (s & 1)*3 ..) of this block row
#pragma unroll
      for (int t = 0; t < 3; ++t) v[t] += __shfl_xor(v[t], 1, 64);
      if ((r16 & 1) == 0) {
        const int sgm = r16 >> 1;
        const int pix = wm * 64 + i * 16 + g * 4 + (sgm >> 1);
        float* dst = part + (pix * 2 + wn) * 6 + (sgm & 1) * 3;
        dst[0] = v[0];
        dst[1] = v[1];
        dst[2] = v[2];
      }
    }
    __syncthreads();
    if (tid < 256) {
      const int py = tid >> 4, px = tid & 15;
      const int oy = by * BH + py, ox = bx * BW + px;
      if (oy < p.cv_OH && ox < p.cv_OW) {
        float raw[6];
#pragma unroll
        for (int o = 0; o < 6; ++o) raw[o] = ho.b6[o] + part[(tid * 2) * 6 + o] + part[(tid * 2 + 1) * 6 + o];
        const int64_t q = ((int64_t)img * p.cv_OH + oy) * p.cv_OW + ox;
        dense_head_pixel(raw, ho.pose + img * 19, ho.scale[img / ho.vps], q, ho.pts3d, ho.pts3d_cam, ho.rays, ho.depth, ho.conf,
                         ho.logits, ho.mask);
      }
    }
  } else {
  // ---- epilogue: 32 rows (two block rows) x 64 fp32 per wave per pass through LDS, 8 columns per lane
  float* ep = reinterpret_cast<float*>(lds) + wave * 32 * H_ELD;
  const int c8 = (lane & 7) * 8;
  const int n0 = bn + wn * C::TN + c8;
  const EpiCol8 ec = epi_col_setup8(p, n0);
#pragma unroll
  for (int part = 0; part < C::FM / 2; ++part) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) ep[(i * 16 + g * 4 + r) * H_ELD + j * 16 + r16] = acc[part * 2 + i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 2
    for (int pass = 0; pass < 4; ++pass) {
      const int rloc = pass * 8 + (lane >> 3);  // row of the 32-row pass: block row wm*FM + part*2 + rloc/16, px rloc%16
      int m = -1;
      if constexpr (FLAT) {
        int im, oy, ox;
        if (mapa_idx::flat_pixel(fb * 256 + (wm * C::FM + part * 2) * BW + rloc, Wp, Hp, p.cv_OH, p.cv_OW, imgs, im,
                                 oy, ox))
          m = (im * p.cv_OH + oy) * p.cv_OW + ox;
      } else {
        const int oy = by * BH + wm * C::FM + part * 2 + (rloc >> 4), ox = bx * BW + (rloc & 15);
        if (oy < p.cv_OH && ox < p.cv_OW) m = (img * p.cv_OH + oy) * p.cv_OW + ox;
      }
      if (m >= 0)
        epi_store_row8<bf16_t>(p, ec, m, *reinterpret_cast<const f32x4*>(ep + rloc * H_ELD + c8),
                               *reinterpret_cast<const f32x4*>(ep + rloc * H_ELD + c8 + 4));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  }
}

}  // namespace

// bn: 256 or 128 output channels per tile (0 = 256 when N % 256 == 0, else 128); bh: block rows (16, or 8 with
// bn 256).  Needs a bf16 (or f16: a.lp_f16) stride-1 conv in the
// channel-block-major K order with 32-channel slices (conv_kblock == 32); returns false otherwise.
// one image of the A operand must be addressable by the window's 32-bit buffer offsets
static bool halo_img_ok(const GemmArgs& a) { return (int64_t)a.cv_IH * a.cv_IW * a.cv_Cp * 2 < 0x7ff00000LL; }

bool launch_conv_halo(const GemmArgs& a, int bn, hipStream_t stream, int bh) {
  if (a.cv_kb != 32 || a.cv_stride != 1 || a.cv_OH != a.cv_IH || a.cv_OW != a.cv_IW || a.K != 9 * a.cv_C) return false;
  if (!halo_img_ok(a)) return false;
  if (bn == 0) bn = a.N % 256 == 0 ? 256 : 128;
  // 256-wide tiles only with 8-row blocks (the 148^2 DPT convs): 16-row 256-wide tiles measured slower than 128-wide
  // ones everywhere (kbench, round 2), and their epilogue no longer unrolls into registers (scratch), so they are gone
  if ((bh == 8) != (bn == 256)) return false;
  if (a.N % bn != 0 || (a.sp_half != 0x7fffffff && a.sp_half % 32 != 0)) return false;
  const int hw = a.cv_OH * a.cv_OW;
  const int64_t tiles = (int64_t)(a.M / hw) * ((a.cv_OH + bh - 1) / bh) * ((a.cv_OW + BW - 1) / BW) * (a.N / bn);
  if (tiles >= (int64_t(1) << 31)) return false;
  const HeadOut none{};
  const HSplit one{1, 0, nullptr, nullptr};
  void (*k)(GemmArgs, HeadOut, HSplit);
  if (a.lp_f16)
    k = bh == 8 ? conv_halo_kernel<256, false, 8, false, true> : conv_halo_kernel<128, false, 16, false, true>;
  else
    k = bh == 8 ? conv_halo_kernel<256, false, 8> : conv_halo_kernel<128>;
  hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(HT), 0, stream, a, none, one);
  return true;
}

// ---- flat-raster blocks with split K
static bool flat_ok(const GemmArgs& a) {
  return a.cv_kb == 32 && a.cv_stride == 1 && a.cv_OH == a.cv_IH && a.cv_OW == a.cv_IW && a.K == 9 * a.cv_C &&
         a.cv_OW + 1 <= FLAT_MAX_WP && a.N % 128 == 0 && (a.sp_half == 0x7fffffff || a.sp_half % 32 == 0);
}
static int64_t flat_blocks(const GemmArgs& a) {
  return ((int64_t)(a.M / (a.cv_OH * a.cv_OW)) * (a.cv_OH + 1) * (a.cv_OW + 1) + 255) / 256;
}

int conv_halo_flat_split(const GemmArgs& a, int slots, int force) {
  if (!flat_ok(a)) return 0;
  const int64_t tiles = flat_blocks(a) * (a.N / 128);
  const int nslice = a.K / 288;
  if (force > 0) return force < nslice ? force : nslice;
  // one block per CU (slots = 2 per CU), with at least two slices (18 K steps) per part and at most 8 parts: the
  // last arriver sums the parts' 128-KiB slabs alone, and a second, partly filled round of blocks costs more than
  // the extra parts win (flat_sweep.py, 8 views, round 5: the 37^2 convs' 92 tiles take 2 parts — binary16 rn3@37
  // 41.2 -> 32.3 us, l3rn@37 48.9 -> 39.2 against 4 / 5 parts; split bf16 rn3@37 59.5 -> 57.3, l3rn@37 74.0 -> 78.6;
  // the 19^2 convs' 26 tiles keep 8 / 4 parts: l4rn@19 83.6 us on stream-K, 55.8 with 8 parts)
  int64_t s = (slots / 2) / (tiles > 0 ? tiles : 1);
  int cap = nslice / 2 > 1 ? nslice / 2 : 1;
  if (cap > 8) cap = 8;
  if (s > cap) s = cap;
  return s < 1 ? 1 : (int)s;
}

int64_t conv_halo_flat_workspace_bytes(const GemmArgs& a, int nsplit, int64_t ticket_bytes) {
  if (!flat_ok(a) || nsplit <= 1) return 0;
  const int64_t tiles = flat_blocks(a) * (a.N / 128);
  // more tiles than ticket words (the top LN_TICKET_WORDS are the LayerNorm-fused GEMM's): not this kernel
  if ((tiles + LN_TICKET_WORDS) * 4 > ticket_bytes) return -1;
  return ticket_bytes + tiles * nsplit * 256 * 128 * 4;
}

bool launch_conv_halo_flat(const GemmArgs& a, int nsplit, void* ws, int64_t ws_bytes, int64_t ticket_bytes,
                           hipStream_t stream) {
  if (!flat_ok(a) || nsplit < 1) return false;
  const int64_t nblk = flat_blocks(a), tiles = nblk * (a.N / 128);
  if (tiles * nsplit >= (int64_t(1) << 31)) return false;
  HSplit sp{nsplit, (int)nblk, nullptr, nullptr};
  if (nsplit > 1) {
    const int64_t need = conv_halo_flat_workspace_bytes(a, nsplit, ticket_bytes);
    if (need <= 0 || !ws || ws_bytes < need) return false;
    sp.tickets = reinterpret_cast<int*>(ws);
    sp.slabs = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + ticket_bytes);
  }
  const HeadOut none{};
  if (a.lp_f16)
    hipLaunchKernelGGL((conv_halo_kernel<128, false, 16, true, true>), dim3((unsigned)(tiles * nsplit)), dim3(HT), 0,
                       stream, a, none, sp);
  else
    hipLaunchKernelGGL((conv_halo_kernel<128, false, 16, true>), dim3((unsigned)(tiles * nsplit)), dim3(HT), 0, stream,
                       a, none, sp);
  return true;
}

bool launch_conv_halo_headout(const GemmArgs& a, const float* w6, const float* b6, const float* pose,
                              const float* scale, int vps, float* pts3d, float* pts3d_cam, float* rays, float* depth,
                              float* conf, float* logits, uint8_t* mask, hipStream_t stream) {
  if (a.cv_kb != 32 || a.cv_stride != 1 || a.cv_OH != a.cv_IH || a.cv_OW != a.cv_IW || a.K != 9 * a.cv_C) return false;
  if (a.N != 128 || !a.bias || a.act != MAPA_ACT_RELU || (a.sp_half != 0x7fffffff && a.sp_half % 32 != 0)) return false;
  if (!halo_img_ok(a)) return false;
  const int hw = a.cv_OH * a.cv_OW;
  const int64_t tiles = (int64_t)(a.M / hw) * ((a.cv_OH + 15) / 16) * ((a.cv_OW + BW - 1) / BW);
  if (tiles >= (int64_t(1) << 31)) return false;
  HeadOut h;
  if (vps <= 0) return false;
  h.w6 = w6; h.b6 = b6; h.pose = pose; h.scale = scale; h.vps = vps;
  h.pts3d = pts3d; h.pts3d_cam = pts3d_cam; h.rays = rays; h.depth = depth; h.conf = conf; h.logits = logits;
  h.mask = mask;
  if (a.lp_f16)
    hipLaunchKernelGGL((conv_halo_kernel<128, true, 16, false, true>), dim3((unsigned)tiles), dim3(HT), 0, stream, a, h,
                       HSplit{1, 0, nullptr, nullptr});
  else
    hipLaunchKernelGGL((conv_halo_kernel<128, true>), dim3((unsigned)tiles), dim3(HT), 0, stream, a, h,
                       HSplit{1, 0, nullptr, nullptr});
  return true;
}

}  // namespace mapa_gemm_impl
