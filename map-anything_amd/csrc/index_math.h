// Index math shared by the kernels and by the host-side bounds / coverage check (tools/index_check.cpp, built with
// g++ -fsanitize=address,undefined by tests/test_index_math.py): every mapping from a workgroup id to the work it
// owns — XCD remap, GEMM tile order, stream-K iteration ranges and slab slots, attention task / K-chunk split,
// halo-conv block decode, conv K-column decode — lives here once, so the check exercises the same code the device
// runs.  Plain integer arithmetic only (no HIP types), callable from host and device.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MAPA_HD __host__ __device__ __forceinline__
#else
#define MAPA_HD inline
#endif

namespace mapa_idx {

MAPA_HD int imin(int a, int b) { return a < b ? a : b; }
MAPA_HD int imax(int a, int b) { return a > b ? a : b; }

// Blocks b, b+8, ... share an XCD (round-robin dispatch over the 8 XCDs); give each XCD a contiguous id range.
// Bijective on [0, nblk) for every nblk (the guide's non-bijective simple form breaks when nblk % 8 != 0).
MAPA_HD int xcd_remap(int b, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Linear tile index t -> (tile row, tile col), walked in groups of GM tile-rows so the ~32 tiles an XCD runs at
// once form a GM x (32/GM) patch: its A row-blocks and W column-blocks are re-read from that XCD's L2.
MAPA_HD void group_coords_rt(int t, int gm, int ntm, int ntn, int& tm, int& tn) {
  const int group = t / (gm * ntn);
  const int first = group * gm;
  const int rows = imin(gm, ntm - first);
  const int in = t - group * gm * ntn;
  tm = first + in % rows;
  tn = in / rows;
}
template <int GM>
MAPA_HD void group_coords(int t, int ntm, int ntn, int& tm, int& tn) {
  group_coords_rt(t, GM, ntm, ntn, tm, tn);
}

// Output tile of workgroup b of a data-parallel GEMM grid of ntm * ntn tiles.
template <int GM>
MAPA_HD void tile_coords(int b, int ntm, int ntn, int& tm, int& tn) {
  group_coords<GM>(xcd_remap(b, ntm * ntn), ntm, ntn, tm, tn);
}
// The same with the group height chosen at run time (mapa_gemm_tune MAPA_TUNE_TILE_GROUP; gm >= 1).
MAPA_HD void tile_coords_rt(int b, int gm, int ntm, int ntn, int& tm, int& tn) {
  group_coords_rt(xcd_remap(b, ntm * ntn), gm, ntm, ntn, tm, tn);
}

// ---- persistent data-parallel GEMM (gemm_pers.hip): round r holds tiles [r*G, min((r+1)*G, tiles)); block b takes
// the round's xcd_remap(b, n_r)-th tile (n_r = that round's tile count; blocks b >= n_r sit the round out), so in every
// round — the last, partial one included — each XCD's blocks walk one contiguous range of the GM-row tile order.
MAPA_HD bool pers_tile(int b, int G, int r, int tiles, int gm, int ntm, int ntn, int& tm, int& tn) {
  const int base = r * G;
  const int n = imin(G, tiles - base);
  if (b >= n) return false;
  group_coords_rt(base + xcd_remap(b, n), gm, ntm, ntn, tm, tn);
  return true;
}

// ---- LayerNorm-fused residual GEMM (gemm_big.hip, LNF): the row statistics of a LayerNorm over N combine across the
// ntn column tiles of a tile row ("band") inside the launch, so every band's tiles must run together.  The bands are
// dealt to the 8 XCDs in contiguous ranges and each XCD walks its bands band-major (a band's ntn tiles consecutive in
// that XCD's dispatch order): a band never straddles XCDs, its A rows are fetched into one L2, and a band whose tiles
// wait for each other is always the oldest incomplete one on its XCD.  Grid = lnf_grid blocks; the blocks past an
// XCD's last band (XCDs with one band fewer) are idle.
MAPA_HD int lnf_grid(int ntm, int ntn) { return 8 * ((ntm + 7) / 8) * ntn; }
MAPA_HD bool lnf_coords(int b, int ntm, int ntn, int& tm, int& tn) {
  const int x = b % 8, j = b / 8;
  const int q = ntm / 8, r = ntm % 8;
  const int lo = x * q + imin(x, r), cnt = q + (x < r ? 1 : 0);
  const int band = j / ntn;
  if (band >= cnt) return false;
  tm = lo + band;
  tn = j - band * ntn;
  return true;
}

// ---- stream-K (gemm_big.hip gemm_sk_kernel): data-parallel whole tiles first, then K-iteration ranges
struct SkPlan {
  int dp_tiles;  // tiles 0 .. dp_tiles-1: whole tiles, tile t on block t % G (data-parallel part)
  int base;      // dp_tiles * nk: first stream-K iteration
  int total;     // tiles * nk
  int per;       // stream-K iterations per workgroup
  int nk;        // K iterations per tile
};

// Plan for `tiles` output tiles of nk K-iterations on g resident workgroup slots (g slab pairs in the workspace).
// tail_only: every full wave of tiles data-parallel, only the last partial wave's iterations spread in chunks of
// >= nk/4 (a split tile has at most 4 contributors).  Otherwise data-parallel whole tiles for all but the last one to
// two waves (dp = false: pure stream-K), the rest spread evenly with at least a tenth of a tile's K per block (past
// ~10 contributors the last arriver's serial slab sum dominates); per_env > 0 only coarsens.  Returns the grid size
// G (<= g: every block's slab pair exists).
MAPA_HD int sk_make_plan(int64_t tiles, int nk, int g, bool tail_only, bool dp, int per_env, SkPlan& s) {
  s.nk = nk;
  s.total = (int)(tiles * nk);
  if (tail_only) {
    s.dp_tiles = (int)((tiles / g) * g);
    s.base = s.dp_tiles * s.nk;
    const int rem = s.total - s.base;
    s.per = imax((rem + g - 1) / g, imax(1, s.nk / 4));
    return g;  // blocks past the stream-K ranges only take data-parallel tiles
  }
  s.dp_tiles = (dp && tiles >= 2 * (int64_t)g) ? (int)((tiles / g - 1) * g) : 0;
  s.base = s.dp_tiles * s.nk;
  s.per = (s.total - s.base + g - 1) / g;
  s.per = imax(s.per, s.nk / 10);
  if (per_env > s.per) s.per = per_env;
  return (s.total - s.base + s.per - 1) / s.per;
}

// Block vb's iteration cursor: call sk_next until it returns false; each call yields one (tile, k0, k1) piece.
struct SkCursor {
  int dp_t, it, r1;
};
MAPA_HD SkCursor sk_begin(const SkPlan& s, int vb) {
  SkCursor c;
  c.dp_t = vb;
  c.it = s.base + vb * s.per;
  c.r1 = imin(c.it + s.per, s.total);
  return c;
}
MAPA_HD bool sk_next(const SkPlan& s, int grid, SkCursor& c, int& t, int& k0, int& k1) {
  if (c.dp_t < s.dp_tiles) {
    t = c.dp_t;
    k0 = 0;
    k1 = s.nk;
    c.dp_t += grid;
    return true;
  }
  if (c.it < c.r1) {
    t = c.it / s.nk;
    k0 = c.it - t * s.nk;
    k1 = imin(s.nk, c.r1 - t * s.nk);
    c.it = t * s.nk + k1;
    return true;
  }
  return false;
}
// The stream-K blocks whose ranges touch tile t: [lo, hi] (lo == hi: the tile is not split).
MAPA_HD void sk_contributors(const SkPlan& s, int t, int& lo, int& hi) {
  const int tb = t * s.nk;
  lo = t < s.dp_tiles ? 0 : (tb - s.base) / s.per;
  hi = t < s.dp_tiles ? 0 : (tb + s.nk - 1 - s.base) / s.per;
}
// Slab slot of block b's partial for the tile starting at iteration tb: slot 0 holds the segment its range starts
// with, slot 1 the one it ends with (a range touches at most two split tiles).
MAPA_HD int64_t sk_slab(int b, int tb, const SkPlan& s) {
  return (int64_t)b * 2 + (s.base + b * s.per >= tb ? 0 : 1);
}

// ---- attention (attention.hip attn_fwd_bf16): n_dp whole tasks, then the remaining tasks cut into `chunks`
// contiguous K/V tile ranges (the last, partial wave spread over all slots).
MAPA_HD void attn_split_plan(int ntask, int nkt, int slots, int& n_dp, int& chunks) {
  const int rem = ntask % slots;
  const int c = rem ? imin(slots / rem, imax(1, nkt / 4)) : 1;
  if (c > 1) {
    n_dp = ntask - rem;
    chunks = c;
  } else {
    n_dp = ntask;
    chunks = 1;
  }
}
// Work of grid block bid: task, K/V tile range [k0, k1), and the partial slot (-1 for whole tasks).
MAPA_HD void attn_block_work(int bid, int n_dp, int chunks, int nkt, int& task, int& k0, int& k1, int& slot) {
  if (bid < n_dp) {  // whole task; consecutive tasks (same batch/head: shared K/V) on one XCD
    task = xcd_remap(bid, n_dp);
    k0 = 0;
    k1 = nkt;
    slot = -1;
  } else {
    slot = bid - n_dp;
    task = n_dp + slot / chunks;
    const int ch = slot % chunks;
    k0 = (int)((int64_t)ch * nkt / chunks);
    k1 = (int)((int64_t)(ch + 1) * nkt / chunks);
  }
}

// ---- halo conv (conv_halo.hip): block id -> (image, block row, block col, column tile)
MAPA_HD void halo_block(int bid, int imgs, int nby, int nbx, int ntn, int& img, int& by, int& bx, int& tn) {
  int t = xcd_remap(bid, imgs * nby * nbx * ntn);
  tn = t % ntn;
  t /= ntn;
  bx = t % nbx;
  t /= nbx;
  by = t % nby;
  img = t / nby;
}

// ---- flat-raster halo conv (conv_halo.hip FLAT): the images laid end to end as one raster of rows of OW + 1
// positions (the last a zero column: the left and right neighbour of the next / previous row's edge pixels) and
// OH + 1 rows per image (the last a zero row, likewise shared), cut into blocks of 256 consecutive positions.  Every
// 3x3 tap of a position is then a constant shift, dy*(OW+1) + dx, inside one 1-D window of 256 + 2*(OW+1) + 2.
// Position P -> pixel (img, r, j); false for the pad positions and for P outside the raster.
MAPA_HD bool flat_pixel(int P, int Wp, int Hp, int OH, int OW, int imgs, int& img, int& r, int& j) {
  if (P < 0) return false;
  const int R = P / Wp;
  j = P - R * Wp;
  img = R / Hp;
  r = R - img * Hp;
  return img < imgs && r < OH && j < OW;
}
// block id -> (flat block, column tile, K part) over nblk * ntn * nsplit workgroups: XCD-contiguous ranges with the
// K parts of one tile adjacent, so the parts' partial-sum slabs meet in one L2
MAPA_HD void halo_flat_tile(int bid, int nblk, int ntn, int nsplit, int& fb, int& tn, int& kp) {
  int t = xcd_remap(bid, nblk * ntn * nsplit);
  kp = t % nsplit;
  t /= nsplit;
  tn = t % ntn;
  fb = t / ntn;
}

// ---- 3x3 conv as implicit GEMM: logical K column kc -> tap (0..8) and logical input channel, in the K order of
// mapa_gemm_desc.conv_kblock (0: tap-major k = tap*C + c; kb: channel-block-major k = (c/kb)*9kb + tap*kb + c%kb)
MAPA_HD void conv_kmap_logical(int kc, int kb, int C, int& tap, int& c) {
  if (kb == 32) {  // the head convs' block: divisions by constants
    const int blk = kc / 288, r = kc - blk * 288;
    tap = r >> 5;
    c = blk * 32 + (r & 31);
  } else if (kb > 0) {
    const int span = 9 * kb;
    const int blk = kc / span, r = kc - blk * span;
    tap = r / kb;
    c = blk * kb + (r - tap * kb);
  } else {
    tap = kc / C;
    c = kc - tap * C;
  }
}

// ---- grid-stride step in 64-bit, clamped to `total` (postprocess.hip: a 32-bit `e += stride` overflows when
// total is within one grid of 2^31)
MAPA_HD int grid_step(int e, int total, int64_t stride) {
  const int64_t n = (int64_t)e + stride;
  return n < total ? (int)n : total;
}

}  // namespace mapa_idx
