// Host-side bounds / coverage check of the kernels' work-assignment index math (csrc/index_math.h — the same
// functions the device code calls).  Built with g++ -fsanitize=address,undefined (tests/test_index_math.py), so
// any signed overflow or out-of-range table access in the mapping itself aborts the run.  Checked, over every shape
// of the MapAnything path (8 / 100 / 250-view encoder, transformer and head GEMMs, attention layouts up to the
// 2 738 001-key configs[4] layer) plus randomised ones:
//   * xcd_remap is a bijection of [0, nblk);
//   * tile_coords<GM> visits every output tile of a grid exactly once, in range; the LayerNorm-fused grid
//     (lnf_coords) too, with each band's tiles on one XCD at consecutive dispatch positions;
//   * stream-K: every (tile, k) iteration is computed by exactly one block, the blocks touching a split tile are
//     exactly sk_contributors' range, slab slots stay inside the g slab pairs of the workspace, the grid fits g;
//   * attention: every task's K/V tile range [0, nkt) is covered exactly once by its chunks, chunks are non-empty,
//     partial slots stay inside the workspace's `slots` rows;
//   * the halo-conv block decode visits every (image, block row, block col, column tile) once;
//   * the conv K-column decode is a bijection onto (tap, channel) for every K order;
//   * the clamped grid-stride step never passes `total`, even one grid short of 2^31.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../map-anything_amd/csrc/index_math.h"

using namespace mapa_idx;

static long g_checks = 0;
#define REQUIRE(c, ...)                                                   \
  do {                                                                    \
    ++g_checks;                                                           \
    if (!(c)) {                                                           \
      fprintf(stderr, "index check failed: %s (%s:%d): ", #c, __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                                       \
      fprintf(stderr, "\n");                                              \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

static void check_xcd(int nblk) {
  std::vector<char> seen(nblk, 0);
  for (int b = 0; b < nblk; ++b) {
    const int t = xcd_remap(b, nblk);
    REQUIRE(t >= 0 && t < nblk, "nblk %d b %d -> %d", nblk, b, t);
    REQUIRE(!seen[t], "nblk %d: %d hit twice", nblk, t);
    seen[t] = 1;
  }
}

template <int GM>
static void check_tiles(int ntm, int ntn) {
  std::vector<char> seen((size_t)ntm * ntn, 0);
  for (int b = 0; b < ntm * ntn; ++b) {
    int tm, tn;
    tile_coords<GM>(b, ntm, ntn, tm, tn);
    REQUIRE(tm >= 0 && tm < ntm && tn >= 0 && tn < ntn, "GM %d grid %dx%d b %d -> (%d,%d)", GM, ntm, ntn, b, tm, tn);
    char& s = seen[(size_t)tm * ntn + tn];
    REQUIRE(!s, "GM %d grid %dx%d: tile (%d,%d) twice", GM, ntm, ntn, tm, tn);
    s = 1;
  }
}

// LayerNorm-fused grid: every tile exactly once; a band's ntn tiles on one XCD (block % 8) at consecutive positions
// of that XCD's dispatch order (block / 8); the blocks past an XCD's bands are idle.
static void check_lnf(int ntm, int ntn) {
  std::vector<int> owner((size_t)ntm * ntn, -1);
  const int grid = lnf_grid(ntm, ntn);
  for (int b = 0; b < grid; ++b) {
    int tm, tn;
    if (!lnf_coords(b, ntm, ntn, tm, tn)) continue;
    REQUIRE(tm >= 0 && tm < ntm && tn >= 0 && tn < ntn, "lnf %dx%d b %d -> (%d,%d)", ntm, ntn, b, tm, tn);
    int& o = owner[(size_t)tm * ntn + tn];
    REQUIRE(o < 0, "lnf %dx%d: tile (%d,%d) twice", ntm, ntn, tm, tn);
    o = b;
  }
  for (int tm = 0; tm < ntm; ++tm)
    for (int tn = 0; tn < ntn; ++tn) {
      const int b = owner[(size_t)tm * ntn + tn], b0 = owner[(size_t)tm * ntn];
      REQUIRE(b >= 0, "lnf %dx%d: tile (%d,%d) never visited", ntm, ntn, tm, tn);
      REQUIRE(b % 8 == b0 % 8 && b / 8 == b0 / 8 + tn, "lnf %dx%d: band %d not consecutive on one XCD", ntm, ntn, tm);
    }
}

static void check_streamk(int64_t tiles, int nk, int g, bool tail, bool dp, int per_env) {
  SkPlan s;
  const int G = sk_make_plan(tiles, nk, g, tail, dp, per_env, s);
  REQUIRE(G >= 1 && G <= g, "tiles %lld nk %d g %d: grid %d", (long long)tiles, nk, g, G);
  std::vector<int> owner((size_t)tiles * nk, -1);
  std::vector<int> tlo(tiles, 1 << 30), thi(tiles, -1);
  for (int vb = 0; vb < G; ++vb) {
    SkCursor c = sk_begin(s, vb);
    int t, k0, k1, guard = 0;
    while (sk_next(s, G, c, t, k0, k1)) {
      REQUIRE(++guard <= tiles + nk + 2, "block %d does not terminate", vb);
      REQUIRE(t >= 0 && t < tiles && k0 >= 0 && k0 < k1 && k1 <= nk, "block %d piece t %d [%d,%d)", vb, t, k0, k1);
      for (int k = k0; k < k1; ++k) {
        int& o = owner[(size_t)t * nk + k];
        REQUIRE(o < 0, "tile %d k %d computed by blocks %d and %d", t, k, o, vb);
        o = vb;
      }
      if (t >= s.dp_tiles) {
        tlo[t] = tlo[t] < vb ? tlo[t] : vb;
        thi[t] = thi[t] > vb ? thi[t] : vb;
        const int64_t slab = sk_slab(vb, t * nk, s);
        REQUIRE(slab >= 0 && slab < 2LL * g, "slab %lld of %d pairs", (long long)slab, g);
      }
    }
  }
  for (size_t i = 0; i < owner.size(); ++i) REQUIRE(owner[i] >= 0, "iteration %zu (tile %zu) never computed", i, i / nk);
  for (int64_t t = s.dp_tiles; t < tiles; ++t) {
    int lo, hi;
    sk_contributors(s, (int)t, lo, hi);
    REQUIRE(lo == tlo[t] && hi == thi[t], "tile %lld contributors [%d,%d] vs actual [%d,%d]", (long long)t, lo, hi,
            tlo[t], thi[t]);
  }
}

static void check_attention(int ntask, int nkt, int slots) {
  int n_dp, chunks;
  attn_split_plan(ntask, nkt, slots, n_dp, chunks);
  REQUIRE(n_dp >= 0 && n_dp <= ntask && chunks >= 1, "plan ntask %d nkt %d", ntask, nkt);
  const int grid = n_dp + (ntask - n_dp) * chunks;
  std::vector<int> covered((size_t)ntask, 0);
  std::vector<int> next_k((size_t)ntask, 0);
  for (int bid = 0; bid < grid; ++bid) {
    int task, k0, k1, slot;
    attn_block_work(bid, n_dp, chunks, nkt, task, k0, k1, slot);
    REQUIRE(task >= 0 && task < ntask, "bid %d task %d", bid, task);
    REQUIRE(0 <= k0 && k0 < k1 && k1 <= nkt, "bid %d chunk [%d,%d) of %d", bid, k0, k1, nkt);
    if (slot >= 0) REQUIRE(slot < slots, "partial slot %d >= %d workspace rows", slot, slots);
    REQUIRE(next_k[task] == k0, "task %d chunk starts at %d, expected %d", task, k0, next_k[task]);
    next_k[task] = k1;
  }
  for (int t = 0; t < ntask; ++t) REQUIRE(next_k[t] == nkt, "task %d covered to %d of %d", t, next_k[t], nkt);
}

static void check_halo(int imgs, int nby, int nbx, int ntn) {
  const int n = imgs * nby * nbx * ntn;
  std::vector<char> seen(n, 0);
  for (int b = 0; b < n; ++b) {
    int img, by, bx, tn;
    halo_block(b, imgs, nby, nbx, ntn, img, by, bx, tn);
    REQUIRE(img >= 0 && img < imgs && by >= 0 && by < nby && bx >= 0 && bx < nbx && tn >= 0 && tn < ntn, "halo %d", b);
    char& s = seen[((img * nby + by) * nbx + bx) * ntn + tn];
    REQUIRE(!s, "halo block twice");
    s = 1;
  }
}

// flat-raster halo conv: (a) the workgroup -> (block, column tile, K part) map is a bijection, (b) over the blocks'
// positions every pixel of every image is produced exactly once, and (c) every 3x3 neighbour of a pixel sits at its
// position + dy*Wp + dx, inside the block's window [P0 - Wp - 1, P0 + 256 + Wp + 1) and <= 384 positions long, and
// reads a zero (a pad position) exactly where the conv's zero padding is
static void check_flat(int imgs, int OH, int OW, int ntn, int nsplit) {
  const int Wp = OW + 1, Hp = OH + 1;
  const int nblk = (int)(((int64_t)imgs * Hp * Wp + 255) / 256);
  REQUIRE(256 + 2 * Wp + 2 <= 384, "window %d", 256 + 2 * Wp + 2);
  const int n = nblk * ntn * nsplit;
  std::vector<char> seen((size_t)n, 0);
  for (int b = 0; b < n; ++b) {
    int fb, tn, kp;
    halo_flat_tile(b, nblk, ntn, nsplit, fb, tn, kp);
    REQUIRE(fb >= 0 && fb < nblk && tn >= 0 && tn < ntn && kp >= 0 && kp < nsplit, "flat %d", b);
    char& s = seen[((size_t)fb * ntn + tn) * nsplit + kp];
    REQUIRE(!s, "flat tile twice");
    s = 1;
  }
  std::vector<char> pix((size_t)imgs * OH * OW, 0);
  for (int P = 0; P < nblk * 256; ++P) {
    int img, r, j;
    if (!flat_pixel(P, Wp, Hp, OH, OW, imgs, img, r, j)) continue;
    REQUIRE(img < imgs && r >= 0 && r < OH && j >= 0 && j < OW, "P %d", P);
    char& s = pix[((size_t)img * OH + r) * OW + j];
    REQUIRE(!s, "pixel twice");
    s = 1;
    const int P0 = P / 256 * 256;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int Q = P + dy * Wp + dx;
        REQUIRE(Q >= P0 - Wp - 1 && Q < P0 + 256 + Wp + 1, "tap outside the window");
        int i2, r2, j2;
        const bool real = flat_pixel(Q, Wp, Hp, OH, OW, imgs, i2, r2, j2);
        const bool inside = r + dy >= 0 && r + dy < OH && j + dx >= 0 && j + dx < OW;
        REQUIRE(real == inside, "tap (%d,%d) of (%d,%d,%d): real %d inside %d", dy, dx, img, r, j, real, inside);
        if (real) REQUIRE(i2 == img && r2 == r + dy && j2 == j + dx, "tap lands on the wrong pixel");
      }
  }
  for (char c : pix) REQUIRE(c, "pixel never produced");
}

static void check_kmap(int C, int kb) {
  std::vector<char> seen((size_t)9 * C, 0);
  for (int kc = 0; kc < 9 * C; ++kc) {
    int tap, c;
    conv_kmap_logical(kc, kb, C, tap, c);
    REQUIRE(tap >= 0 && tap < 9 && c >= 0 && c < C, "kb %d C %d kc %d -> tap %d c %d", kb, C, kc, tap, c);
    char& s = seen[(size_t)tap * C + c];
    REQUIRE(!s, "kb %d C %d: (tap %d, c %d) twice", kb, C, tap, c);
    s = 1;
  }
}

static void check_grid_step(int total, int64_t stride) {
  int steps = 0;
  for (int e = 0; e < total; e = grid_step(e, total, stride)) {
    REQUIRE(e >= 0 && e < total, "e %d total %d", e, total);
    REQUIRE(++steps <= total / stride + 2, "no progress");
  }
}

int main() {
  std::mt19937 rng(12345);
  for (int n = 1; n <= 20000; ++n) check_xcd(n);

  // GEMM tile grids of the path (M = views * tokens; 256/192/128-row tiles; N / 128, 192, 256 columns) + sweeps
  const int rows[] = {256 * 2 + 2, 8 * 1370, 8 * 1369 + 1, 100 * 1370, 13 * 1369 + 1, 250 * 1370, 32 * 1370,
                      8 * 21904, 8 * 87616, 8 * 268324, 8 * 361, 8 * 1369, 2 * 256, 3 * 257};
  const int tile_rows[] = {256, 192, 128};
  const int cols[] = {768, 1024, 2304, 3072, 4096, 96, 192, 384, 256, 128, 784, 1536, 16 * 96, 4 * 192};
  const int tile_cols[] = {128, 192, 256};
  for (int M : rows)
    for (int bm : tile_rows)
      for (int N : cols)
        for (int bn : tile_cols) {
          const int ntm = (M + bm - 1) / bm, ntn = (N + bn - 1) / bn;
          if ((int64_t)ntm * ntn > 400000) continue;
          check_tiles<4>(ntm, ntn);
          check_tiles<8>(ntm, ntn);
        }
  for (int ntm = 1; ntm <= 70; ++ntm)
    for (int ntn = 1; ntn <= 40; ++ntn) {
      check_tiles<4>(ntm, ntn);
      check_tiles<8>(ntm, ntn);
      check_lnf(ntm, ntn);
    }
  for (int M : rows)
    for (int ntn : {3, 4, 5, 6, 8}) check_lnf((M + 191) / 192, ntn);

  // stream-K: the head convs (M = views * pixels, K = 9 * 3C logical split columns / 32-deep steps) + random
  const int sk_g[] = {256, 512, 1024};
  const int64_t sk_tiles[] = {46, 92, 12, 200, 511, 512, 513, 1032, 1537, 3};
  const int sk_nk[] = {648, 1944, 2304, 216, 96, 32, 7, 1};
  for (int g : sk_g)
    for (int64_t t : sk_tiles)
      for (int nk : sk_nk)
        for (int mode = 0; mode < 3; ++mode) check_streamk(t, nk, g, mode == 2, mode == 0, 0);
  for (int i = 0; i < 300; ++i) {
    const int g = 1 + rng() % 1024;
    check_streamk(1 + rng() % 3000, 1 + rng() % 700, g, rng() % 3 == 0, rng() % 2, rng() % 5 == 0 ? rng() % 300 : 0);
  }

  // attention: tasks = ceil(seq_q / 128) * heads * batch; keys in 64-row tiles
  const int slots[] = {512, 256, 1024};
  struct A { int seq_q, heads, batch, seq_kv; };
  const A att[] = {{1370, 16, 8, 1370}, {1369, 12, 8, 1369}, {10953, 12, 1, 10953}, {136901, 12, 1, 136901},
                   {13 * 1369 + 1, 12, 1, 136901}, {250 * 1369 + 1, 12, 1, 2738001}, {2048, 12, 1, 2738001},
                   {8192, 12, 1, 2738001}, {16384, 12, 1, 136901}, {300, 12, 1, 1111}, {1, 1, 1, 1},
                   {65, 3, 2, 65}, {257, 12, 32, 257}, {43809, 12, 1, 43809}};
  for (int sl : slots)
    for (const A& a : att) check_attention(((a.seq_q + 127) / 128) * a.heads * a.batch, (a.seq_kv + 63) / 64, sl);
  for (int i = 0; i < 3000; ++i) check_attention(1 + rng() % 6000, 1 + rng() % 50000, 1 + rng() % 1200);

  // halo conv blocks: 16x16 (or 8x16) pixel blocks of the 518 / 296 / 148 maps, 128 / 256-wide column tiles
  const int maps[] = {518, 296, 148, 74, 37};
  for (int hw : maps)
    for (int bh : {8, 16})
      for (int ntn : {1, 2})
        for (int imgs : {1, 2, 8}) check_halo(imgs, (hw + bh - 1) / bh, (hw + 15) / 16, ntn);

  for (int hw : {37, 19, 5, 61, 1})
    for (int imgs : {1, 2, 8, 3})
      for (int ntn : {1, 2, 6})
        for (int nsplit : {1, 5, 12}) check_flat(imgs, hw, hw, ntn, nsplit);
  check_flat(2, 37, 29, 2, 3);
  check_flat(3, 13, 21, 1, 1);
  check_flat(250, 37, 37, 2, 1);

  // conv K orders: logical (split) channel counts of the path convs
  const int convC[] = {96 * 3, 192 * 3, 384 * 3, 768 * 3, 256 * 3, 128 * 3, 96, 192, 256, 768, 588, 3 * 592};
  for (int C : convC) {
    check_kmap(C, 0);
    if (C % 32 == 0) check_kmap(C, 32);
    if (C % 16 == 0) check_kmap(C, 16);
    if (C % 64 == 0) check_kmap(C, 64);
  }

  check_grid_step(1000, 7);
  check_grid_step(2147483647 - 5, 65536LL * 256);
  check_grid_step(2147483647, 2147483647LL);
  printf("index math ok: %ld checks\n", g_checks);
  return 0;
}
