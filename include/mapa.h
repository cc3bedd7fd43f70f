/* mapa.h — C ABI of the MI355X-native MapAnything hot path (libmapa.so, gfx950).
 *
 * The reference has no native code on this path: every op below replaces a PyTorch ATen call of the
 * reference's feed-forward `MapAnything.forward` (mapanything/models/mapanything/model.py:1657-2152) and is
 * bound from Python with ctypes by the host mirror `map-anything_amd/mapanything/_native.py`
 * (INTEGRATION.md shows the binding).  Conventions:
 *   - every pointer is a device pointer owned by the caller; the library never allocates or frees;
 *   - all work is enqueued on `stream`; no host synchronisation inside any call (graph-capturable);
 *   - return 0 on success, non-zero on a rejected argument or a failed launch; `mapa_last_error()` then
 *     returns a thread-local message;
 *   - activations are row-major "token x channel" (NHWC for images); weights keep nn.Linear's [out][in]
 *     layout (convs re-packed once to [out][ky][kx][in]).
 */
#ifndef MAPA_H
#define MAPA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* mapa_stream_t; /* == hipStream_t */

/* MAPA_BF16X3: split-precision bf16 operand rows [hi | lo] (2x the logical width; see mapa_split_bf16x3),
 * accepted as an OUTPUT dtype by mapa_layernorm (y_lp) and mapa_bilinear_ac */
/* MAPA_F16: IEEE binary16 operands (the fp16 autocast recipe, infer(amp_dtype="fp16")); accepted by mapa_gemm (dense
 * A), mapa_attention, mapa_attn_merge, and as an output dtype of mapa_layernorm / mapa_patchify / mapa_convert_rows */
/* MAPA_F16 as the TF32-equivalent heads' operand (round 5 default): binary16 activations and weights have exactly
 * TF32's 11 significant bits, so an f16 mapa_gemm / conv with fp32 accumulation is the reference's TF32 arithmetic for
 * values in binary16's normal range; mapa_gemm's out_lp / out_lp_relu of an f16 GEMM, mapa_layernorm, mapa_bilinear_ac
 * (from f32) and mapa_convert_rows write such rows and raise MAPA_FAULT_F16_RANGE on values outside the range.
 * MAPA_F16X2: TF32-equivalent head operand rows [hi | lo] of binary16 (2x the logical width): v = hi + lo, hi = f16(v),
 * lo = f16(v - hi).  Read by mapa_gemm with dtype MAPA_F16 as a plain 2C-wide operand against f16 weights packed
 * [w | w] (the conv's channels doubled), written by mapa_gemm's out_s3 / out_s3_relu when dtype is MAPA_F16, and
 * accepted as an output dtype by mapa_layernorm, mapa_bilinear_ac and mapa_split_rows.  A value outside binary16's
 * range (|v| > 65504, or not finite) sets MAPA_FAULT_F16_RANGE. */
enum { MAPA_F32 = 0, MAPA_BF16 = 1, MAPA_BF16X3 = 2, MAPA_F16 = 3, MAPA_F16X2 = 4 };
enum { MAPA_A_DENSE = 0, MAPA_A_CONV3X3 = 1 };
enum { MAPA_OUT_ROWMAJOR = 0, MAPA_OUT_PIXSHUF = 1 };
/* GELU is the exact-erf form (nn.GELU()), erf evaluated branch-free to within 1.2 ulp of fp32 erff (two minimax
 * pieces, csrc/mapa_common.h erf_fast; tools/erf_check.py). */
enum { MAPA_ACT_NONE = 0, MAPA_ACT_GELU = 1, MAPA_ACT_RELU = 2, MAPA_ACT_GELU_POST = 3 };

const char* mapa_last_error(void);
int mapa_version(void);
/* 1 if a gfx950 device is visible and the code object loads on it, else 0 (message in mapa_last_error). */
int mapa_device_check(int device);
/* Debug / serialize mode: synchronise `stream` and report any device error as the failure of `what` (0 = ok).
 * The Python binding calls it after every launch when MAPA_SERIALIZE=1 (or AMD_SERIALIZE_KERNEL /
 * HIP_LAUNCH_BLOCKING is set) — SURVEY.md §5's race-detection / serialize row; no reference counterpart. */
int mapa_stream_check(mapa_stream_t stream, const char* what);

/* Device-side fault channel (round 5).  Kernels that can detect a failed assumption at run time set a bit of the
 * library's sticky fault word (below) instead of hanging or failing silently; today one: MAPA_FAULT_LN_BARRIER, a
 * LayerNorm-fused GEMM band barrier (mapa_gemm_desc.ln_out) that did not complete within its bounded wait — that
 * launch's LayerNorm rows are invalid.
 *   mapa_fault_slot_create: 64 bytes of coherent, device-mapped pinned host memory (the one allocation the library
 *     makes; free with mapa_fault_slot_destroy); *host for the CPU, *dev for mapa_fault_publish.
 *   mapa_fault_publish: enqueue on `stream` a one-lane kernel that writes dev_slot[0] = 1 | (fault word << 1) once
 *     every earlier launch on the stream has completed (graph-capturable).  The host zeroes slot[0], enqueues the
 *     work and the publish, and polls slot[0] != 0 — no stream synchronisation, so the GPU keeps running the work
 *     queued after the publish (MapAnything.infer publishes after the transformer and checks before returning).
 *   mapa_fault_reset: enqueue on `stream` a kernel that clears the fault word once every earlier launch on the
 *     stream has completed (graph-capturable); MapAnything.infer / forward start every call with it, so a publish
 *     reports only faults of its own call.
 *   mapa_fault_status: synchronous read of the fault word (and reset to 0 when `reset`); -1 on a HIP error.
 *   mapa_stream_check also reports and clears it.
 * The word is per device and per calling host thread (round 6: a thread's word is fixed at its first library call;
 * 64 words, threads beyond share round robin): every launch, reset, publish and status call of a thread uses its own
 * word, so concurrent callers on different streams of one process (one thread each) neither see nor clear each
 * other's faults.  A captured graph keeps the word of the thread that captured it.  The library's cached device
 * properties (CU counts, co-resident slot counts of the LayerNorm-fused GEMM) are kept per device too, so one process
 * may drive several devices. */
/* MAPA_FAULT_F16_RANGE: a MAPA_F16 / MAPA_F16X2 producer met a value outside binary16's range (the TF32-equivalent
 * heads' operands); the outputs of that forward are not trustworthy: MapAnything.infer / forward re-run the call with
 * the fp32-exact split-precision heads (MapAnything._range_fallback) instead of returning them. */
enum { MAPA_FAULT_LN_BARRIER = 1, MAPA_FAULT_F16_RANGE = 2 };
int mapa_fault_slot_create(uint32_t** host, uint32_t** dev);
int mapa_fault_slot_destroy(uint32_t* host);
int mapa_fault_publish(uint32_t* dev_slot, mapa_stream_t stream);
int mapa_fault_reset(mapa_stream_t stream);
int mapa_fault_status(int reset);

/* ---------------------------------------------------------------------------------------------------------
 * GEMM / implicit-GEMM convolution: C[M,N] = A[M,K] * W[N,K]^T, fused epilogue
 *   v = acc + bias[n % bias_mod]; v = act(v); v *= gamma[n]; v += resid1[o] + resid2[o];
 *   (act MAPA_ACT_GELU_POST: v = gelu(acc + bias + resid1 + resid2), gamma must be NULL — ResidualBlock,
 *   dense_rep_encoder.py:44-52)
 *   out_f32[o] = v; out_lp[o] = lowp(v); out_lp_relu[o] = lowp(max(v,0)); out_s3 / out_s3_relu: split operand
 * Replaces nn.Linear (transformer_blocks.py:65-212, dinov2 layers/block.py:93-118, mlp_head.py, pose_head.py),
 * nn.Conv2d 1x1/3x3 (dpt.py:94-311, dpt_block.py:114-177, pose_head.py:18-48, dense_rep_encoder.py:31-287),
 * nn.ConvTranspose2d k=s (dpt.py:101-131; out_mode PIXSHUF) and the 14x14/14 patch-embed conv.
 * dtype BF16: A, W, out_lp bf16 (fp32 accumulate); dtype F32: everything fp32 (exact-fp32 parity mode).
 * ------------------------------------------------------------------------------------------------------- */
typedef struct {
  int dtype;
  int M, N, K;
  const void* A;
  int64_t lda;
  const void* W;
  int64_t ldw;
  int a_mode; /* MAPA_A_DENSE or MAPA_A_CONV3X3 (A = NHWC [img][IH][IW][C], K = 9*C, pad 1) */
  int conv_C, conv_IH, conv_IW, conv_OH, conv_OW, conv_stride;
  const float* bias;
  int bias_mod; /* 0 -> N */
  const float* gamma;
  int act;
  const float* resid1;
  const float* resid2;
  float* out_f32;
  void* out_lp;
  void* out_lp_relu;
  int64_t ldo;
  int out_mode; /* MAPA_OUT_ROWMAJOR or MAPA_OUT_PIXSHUF (n = (ky*s+kx)*cout + co, m = img*h*w + y*w + x) */
  int ps_s, ps_h, ps_w, ps_cout;
  /* Optional scratch for the stream-K schedule (bf16 shapes whose tile count divides badly over the CUs) and for
   * the split-K flat-raster halo conv (the 19^2 / 37^2 convs) and for the LayerNorm-fused residual linears (ln_out):
   * device memory, ZERO-FILLED before its first use, used by one stream at a time, never written by the caller
   * afterwards.  Its 256 KiB head holds the ticket words (returned to zero when each call completes) and, in its top
   * 64 KiB, the LayerNorm bands' generation words (they count up from call to call); the rest holds fp32 partial-sum
   * slabs / row-statistics granules (scratch data) afterwards.  LayerNorm-fused calls (ln_out) should get a
   * workspace of their own, not shared with stream-K / split-K calls: their granule slots are then written only by
   * their own band with that band's monotonic epoch tags (with a shared workspace, slab data left in a slot is
   * rejected by the {epoch, ~epoch} tags alone).  The Python binding keeps one of each per stream.
   * Size: mapa_gemm_workspace_bytes.  NULL / too small -> a data-parallel schedule, or the GEMM followed by
   * mapa_layernorm (same results to rounding). */
  void* workspace;
  int64_t workspace_bytes;
  /* Split-precision operand outputs (dtype BF16 only; NULL = off): row r of out_s3 is 2*ld bf16 wide (ld = ldo, or
   * ps_cout in PIXSHUF mode) and holds [hi | lo] of the output row, hi = bf16(v), lo = bf16(v - hi) — the
   * mapa_split_bf16x3 layout, so the next GEMM/conv (a_split, conv_C = 3*C, weights [hi | lo | hi] per tap) computes
   * the fp32 product to ~2^-16.  out_s3_relu: the same of max(v, 0).  Used for the downstream heads, which the
   * reference runs with autocast disabled (model.py:1774). */
  void* out_s3;
  void* out_s3_relu;
  /* a_split != 0: A is a split-precision operand stored compact, [hi | lo] (2C bf16 per row, or per pixel in conv
   * mode), read as the logical K layout [hi | hi | lo] (K = 3C for dense A with lda >= 2C; conv_C = 3C per tap)
   * against weights packed [hi | lo | hi] — what out_s3 / mapa_split_bf16x3 / the split LayerNorm and bilinear
   * outputs store.  C % 8 == 0. */
  int a_split;
  /* conv K order (MAPA_A_CONV3X3): 0 = tap-major, k = tap*C + c; B > 0 (B % 8 == 0, C % B == 0) = channel-block-major,
   * k = (c / B)*9B + tap*B + c % B, with W's columns packed in the same order.  Consecutive K tiles then walk the 9
   * taps of one B-channel slice, so the slice of the input window stays L2-resident across the taps instead of being
   * re-fetched per tap (the head convs' fabric traffic: 9-20x their algorithmic bytes tap-major). */
  int conv_kblock;
  /* Fused LayerNorm of the output rows (ln_out NULL = off; round 4): after the epilogue, every row of out_f32 (the
   * updated fp32 residual stream; N = the LayerNorm width, 256 / 512 / 768 / 1024) is normalised with ln_w / ln_b
   * (fp32 [N]) and ln_eps and stored to ln_out in the GEMM's 16-bit dtype (fp32 for MAPA_F32), row stride ln_ldo —
   * the next sub-block's nn.LayerNorm fused into the residual linear (dinov2 layers/block.py:93-118,
   * transformer_blocks.py:452-469).  Needs out_f32, row-major.  For bf16 residual linears (out_f32 = resid1 +
   * gamma * (acc + bias), nothing else; N a multiple of 192 or 256) and with a workspace of
   * mapa_gemm_workspace_bytes, the statistics combine across the row's column tiles inside the launch (two-pass per
   * tile, Chan's merge across tiles: the standalone result up to fp32 rounding of mean / variance); otherwise the
   * GEMM is followed by mapa_layernorm on the same stream.  The fused kernel never has more workgroups in flight
   * than the device holds at once (larger problems run as several launches of whole bands), so its band barrier
   * does not depend on dispatch order; a barrier that still does not complete within its bounded wait sets
   * MAPA_FAULT_LN_BARRIER in the fault word (mapa_fault_publish / mapa_fault_status) instead of hanging. */
  const float* ln_w;
  const float* ln_b;
  float ln_eps;
  void* ln_out;
  int64_t ln_ldo;
} mapa_gemm_desc;

int mapa_gemm(const mapa_gemm_desc* d, mapa_stream_t stream);
/* Workspace bytes mapa_gemm would use for this problem (0 if its schedule needs none). */
int64_t mapa_gemm_workspace_bytes(const mapa_gemm_desc* d);
/* Tuning / test hook: force one kernel variant for every later mapa_gemm call (0 = automatic per-shape choice,
 * the default; env MAPA_GEMM_VARIANT sets the initial value).  Codes: 643/644/1282/1283 = 128x128 tiles,
 * 2560..2574 = 256-row tiles, 2580/2581 = stream-K, 2582 = tail-only stream-K (these need a workspace; without one
 * the automatic choice runs), 2584..2586 / 2588 = LDS halo-window conv, 2589 = the same on flat-raster blocks with
 * split K (needs a workspace when it splits), 2587 = 192x192 tiles; timing diagnostics with wrong results (dense A):
 * 2591 / 2592 / 2593 = the 256x128 2-per-CU kernel compute-only / loads-only / without its epilogue, 2594 / 2595 /
 * 2596 = the same for the 192x256 kernel.  (The round-2 opt-in
 * main-loop experiments — phase-interleaved and four-wave tiles — measured slower on every path shape and were
 * removed from the library) */
int mapa_gemm_set_variant(int variant);
/* The regressor tail in one launch (DPTRegressionProcessor conv2 + the dense head, dpt.py:285-311 and model.py:
 * 1865-2150): d describes the 3x3 conv 128 -> 128 (bf16, stride 1, conv_kblock 32, act MAPA_ACT_RELU, bias; no
 * outputs of its own); its ReLU'd hidden map never leaves the chip — the epilogue applies the 1x1 conv w6 [6][128] +
 * b6, the ray / depth / confidence / mask adaptors and the output assembly of mapa_dense_head_out (pose_out: the
 * launch's views' rows, scale: the metric scales, image i of the launch using scale[i / views_per_scale] —
 * views_per_scale = the launch's image count for one scene, 1 with one scale per image for batched scenes; outputs as
 * there).  Replaces mapa_gemm + mapa_dense_head_out. */
int mapa_regressor_head_out(const mapa_gemm_desc* d, const float* w6, const float* b6, const float* pose_out,
                            const float* scale, int views_per_scale, float* pts3d, float* pts3d_cam, float* rays, float* depth,
                            float* conf, float* logits, uint8_t* mask, mapa_stream_t stream);

/* Tuning / A-B hooks of the automatic kernel choice (process-wide):
 *   MAPA_TUNE_CONV_HALO (default 1): stride-1 bf16 convs in the 32-channel-slice K order (conv_kblock = 32) run on
 *     the LDS halo-window conv (N = 256: 8x16-pixel blocks, 256-wide tiles; else 16x16 blocks); 2 keeps 16x16
 *     blocks for every N; 3 is the default without the flat-raster blocks below; 0 keeps them on the implicit GEMM
 *     (variants 2584 / 2585 / 2586 / 2588 force one);
 *     With the default, the stride-1 convs too small for 16x16 blocks (up to 62 pixels wide: the 19^2 / 37^2 DPT
 *     convs) run the halo conv on flat-raster blocks with their 32-channel slices split over several workgroups per
 *     tile (variant 2589 forces it; needs the workspace mapa_gemm_workspace_bytes reports);
 *   MAPA_TUNE_TAIL_STREAMK (default 0): dense bf16 GEMMs whose 256x128 tiles leave a nearly empty last wave use
 *     the tail-only stream-K schedule (2582) when a workspace is passed;
 *   MAPA_TUNE_HALO_SPLIT (default 0 = automatic): the K part count of the flat-raster halo conv (1..64).
 *   MAPA_TUNE_TILE_GROUP (default 0 = 4): the 256-row data-parallel GEMM kernels walk each XCD's tile range in
 *     groups of this many tile rows (all tile columns of a group before the next group).
 *   MAPA_TUNE_LN_FUSE (default 2, or the environment's MAPA_LN_FUSE): 2 = ln_out requests run on the LayerNorm-fused
 *     kernel whatever the automatic tile choice of the shape; 1 = only where that choice is the 192-row kernel; 3 =
 *     only N % 256 == 0 (the 192x256-tile form); 0 = always as a separate mapa_layernorm launch (A/B).
 *   MAPA_TUNE_LN_SPIN (default 0 = 2^22): polls of the fused LayerNorm's band barrier before it gives up.
 *   MAPA_TUNE_LN_TEST_SKIP (test hook, default 0): the next `value` LayerNorm-fused launches each have one tile
 *     (band 0, column tile 0) skip its statistics publish, so band 0 times out and raises MAPA_FAULT_LN_BARRIER.
 *   MAPA_TUNE_PERS (default 1, or the environment's MAPA_GEMM_PERS): the dense 16-bit linears with a transformer
 *     epilogue (act -> 16-bit output, or the in-place fp32 residual update) and no ln_out run on the persistent
 *     register-epilogue kernel; 1 = its automatic tile shape, 2..5 = tile shape 0..3 (256x128, 192x256, 256x256,
 *     192x128), 0 = off (the data-parallel tile kernels).  Variants 2600..2608 force a shape (4..6: diagnostics;
 *     7, 8: 4-wave 192x128 / 256x128 forms, measured slower).
 *   MAPA_TUNE_PERS_LN (default 0, or the environment's MAPA_GEMM_PERS_LN): 1 = ln_out requests that the LayerNorm-
 *     fused kernel takes run on the persistent register-epilogue form (192x128 tiles, 2 per CU, whole 192-row bands
 *     per round, all co-resident); 2 = that form where K <= 1024 only; 0 = the 192-row LNF tile kernel (measured
 *     fastest inside the model).  Every form keys its row statistics on the same 192-row bands and per-band
 *     generation words, so they may alternate on one workspace.
 *   MAPA_TUNE_PERS_STAGGER (default 0 = off, or the environment's MAPA_GEMM_STAGGER): the persistent kernel's
 *     workgroups that get one tile fewer start `value` 100-MHz ticks (10 ns) late, so the chip's epilogue store bursts
 *     do not coincide (up to 100000); -1 = automatic: half a tile's time where those workgroups are < 40 % of the
 *     grid, else none.  Results are bitwise the same either way.
 *   MAPA_TUNE_DIAG_GRID (timing diagnostic, default 0): the data-parallel 256-row / 192-row tile kernels launch only
 *     their first `value` workgroups (0 = every tile); outputs of the other tiles are left unwritten. */
enum { MAPA_TUNE_CONV_HALO = 0, MAPA_TUNE_TAIL_STREAMK = 1, MAPA_TUNE_HALO_SPLIT = 2, MAPA_TUNE_TILE_GROUP = 3,
       MAPA_TUNE_LN_FUSE = 4, MAPA_TUNE_LN_SPIN = 5, MAPA_TUNE_LN_TEST_SKIP = 6, MAPA_TUNE_DIAG_GRID = 7,
       MAPA_TUNE_PERS = 8, MAPA_TUNE_PERS_LN = 9, MAPA_TUNE_PERS_STAGGER = 10 };
int mapa_gemm_tune(int key, int value);

/* ---------------------------------------------------------------------------------------------------------
 * Flash attention forward, head_dim 64, non-causal, softmax scale `scale` (default 1/8; F.scaled_dot_product_attention at
 * dinov2.py:136 and transformer_blocks.py:198-201).  Element (b, h, i, d) of Q lives at
 *   q + b*q_bstride + i*q_rstride + h*64 + d   (same for k, v, o), so the packed qkv GEMM output is read in place.
 * Q rows [0, seq_q) attend to K/V rows [0, seq_kv) of the same batch; o receives the per-head outputs.
 * lse (optional, f32 [batch][heads][seq_q]) receives log-sum-exp of the scaled scores for chunk merging.
 * kv_nseg > 0: the seq_kv logical keys live in kv_nseg row segments of K/V (physical rows
 * [kv_seg_start[s], kv_seg_start[s] + kv_seg_len[s])), e.g. the padded per-rank slots of an RCCL all-gather;
 * seq_kv must equal the sum of the lengths.
 * ------------------------------------------------------------------------------------------------------- */
#define MAPA_MAX_KV_SEGMENTS 16
typedef struct {
  int dtype;
  int batch, heads, seq_q, seq_kv;
  const void* q;
  const void* k;
  const void* v;
  void* o;
  int64_t q_bstride, q_rstride, k_bstride, k_rstride, v_bstride, v_rstride, o_bstride, o_rstride;
  float* lse;
  int kv_nseg;
  int kv_seg_start[MAPA_MAX_KV_SEGMENTS];
  int kv_seg_len[MAPA_MAX_KV_SEGMENTS];
  /* optional scratch (bf16 only, mapa_attention_workspace_bytes() bytes): the 128-row query blocks left over after
   * the full waves of the device's resident workgroups are split into K/V chunks (partials merged by LSE);
   * without it one workgroup per block */
  void* workspace;
  int64_t workspace_bytes;
  /* softmax scale on q.k (0 = 1/sqrt(64), SDPA's default); variants fold their logit scaling into it
   * (entropy scaling / scalable softmax, transformer_blocks.py:185-196) */
  float scale;
} mapa_attn_desc;

int mapa_attention(const mapa_attn_desc* d, mapa_stream_t stream);
int64_t mapa_attention_workspace_bytes(const mapa_attn_desc* d);

/* Merge two attention partials of the same queries over disjoint key sets using their LSEs (the sharded global
 * layer overlaps its K/V all-gather with the local-key partial): o = (e^{lse_a} o_a + e^{lse_b} o_b) /
 * (e^{lse_a} + e^{lse_b}).  o_* [rows][heads*64] (row stride ld, bf16 or f32 per dtype; o_out may alias o_a),
 * lse_* [heads][rows] natural-log f32 as mapa_attention writes them (batch 1); lse_out optional. */
int mapa_attn_merge(const void* o_a, const float* lse_a, const void* o_b, const float* lse_b, void* o_out,
                    float* lse_out, int dtype, int rows, int heads, int64_t ld, mapa_stream_t stream);

/* LayerNorm over the last dim (nn.LayerNorm eps=1e-6): y = (x-mean)/sqrt(var+eps)*w + b.
 * x: f32 rows (row stride ldx); outputs optional: y_f32 (ldy), y_lp (bf16 or f32 per lp_dtype, ldy; MAPA_BF16X3:
 * split rows of 2*ldy bf16).
 * Output row r reads input row (in_group > 0 ? (r / in_group) * in_group_stride + r % in_group : r) + in_row_off
 * (e.g. drop the DINOv2 cls row of every view: group T, stride T+1, offset 1). */
int mapa_layernorm(const float* x, int64_t ldx, int rows, int dim, const float* w, const float* b, float eps,
                   float* y_f32, void* y_lp, int lp_dtype, int64_t ldy, int in_group, int64_t in_group_stride,
                   int in_row_off, mapa_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------
 * Elementwise / layout kernels of the path
 * ------------------------------------------------------------------------------------------------------- */
/* img NCHW f32 [n][3][H][W] -> patches [n*(H/14)*(W/14)][kpad] (k = c*196 + ky*14 + kx, zero for k >= 588),
 * dtype bf16 or f32 (vision_transformer.py:244-249 PatchEmbed as GEMM). */
int mapa_patchify(const float* img, int n, int H, int W, void* out, int dtype, int kpad, mapa_stream_t stream);

/* x[v][0] = cls + pos[0]; x[v][1+t] = patch[v*T+t] + pos[1+t]  (vision_transformer.py:250-252) */
int mapa_assemble_tokens(const float* patch, const float* cls, const float* pos, int n, int T, int dim, float* x,
                         mapa_stream_t stream);

/* rows r in [r0, r1): x[r][:] += vec[:]   (ref-view PE, alternating_attention_transformer.py:618-626) */
int mapa_add_rowvec(float* x, int64_t ldx, int r0, int r1, int dim, const float* vec, mapa_stream_t stream);

/* Bilinear resize, align_corners=True, NHWC.  Output grid is the full (OHf, OWf) grid of F.interpolate; only
 * rows < OH and cols < OW are written (fused crop, dpt.py:213).  in: f32 or bf16 (in_dtype), out: out_dtype
 * (MAPA_BF16X3: split rows [hi | lo] of 2*C bf16 per pixel). */
int mapa_bilinear_ac(const void* in, int in_dtype, int n, int IH, int IW, int C, int OHf, int OWf, int OH, int OW,
                     void* out, int out_dtype, mapa_stream_t stream);

/* mean over `tokens` rows per image: x [n][tokens][C] f32 -> y [n][C] (AdaptiveAvgPool2d(1), pose_head.py:150).
 * work: n*32*C floats of scratch (deterministic two-pass reduction). */
int mapa_mean_tokens(const float* x, int n, int tokens, int C, float* y, void* work, mapa_stream_t stream);

/* small fp32 linear for M <= 64 rows: y[m][n] = act(sum_k x[m][k] w[n][k] + b[n])  (pose/scale MLPs) */
int mapa_linear_small(const float* x, int M, int K, const float* w, const float* b, int N, int act, float* y,
                      mapa_stream_t stream);

/* per view: pose raw (7) -> t, unit quat, R; scale raw -> s = clip(exp(.), 1e-8)   (adaptors.py:171-212, 586-732)
 * pose_out[v] = {t(3) * s, q(4), R(9), t(3) raw} (19 floats); poses44[v] (optional) = 4x4 [R | t*s];
 * scale_out[b] = s.  Rows are view-major: v = view * batch + b. */
int mapa_pose_scale_finalize(const float* pose_raw, const float* scale_raw, int nviews, int batch, float* pose_out,
                             float* scale_out, float* poses44, mapa_stream_t stream);

/* Dense head tail: conv1x1 128->6 on the ReLU'd hidden map + adaptors + output assembly (dpt.py:306-310,
 * adaptors.py:393-523/1012-1133/1740-1796, model.py:1871-1923/2116-2150, geometry.py:855-907).
 * hidden: [n][H*W][128] (bf16 or f32, dtype); w6 [6][128] f32, b6 [6]; pose_out/scale from finalize.
 * Outputs (NHWC f32, [n][H][W][c]): pts3d(3) pts3d_cam(3) rays(3) depth(1) conf(1) logits(1) mask(u8). */
int mapa_dense_head_out(const void* hidden, int dtype, int n, int HW, const float* w6, const float* b6,
                        const float* pose_out, const float* scale, int batch, float* pts3d,
                        float* pts3d_cam, float* rays, float* depth, float* conf, float* logits, uint8_t* mask,
                        mapa_stream_t stream);

/* Image normalisation of the input pipeline (image.py:270-275 / 466-470: torchvision ToTensor + Normalize):
 * hwc u8 [n][H][W][3] (decoded, resized, cropped on the host) -> out f32 [n][3][H][W] = (u8 / 255 - mean) / std,
 * IEEE float32 division and subtraction in torch's order.  mean3 / std3: HOST arrays of 3 floats. */
int mapa_normalize_image(const uint8_t* hwc, int n, int H, int W, const float* mean3, const float* std3, float* out,
                         mapa_stream_t stream);

/* GPU resize of the input pipeline, bit-exact with PIL's Image.resize on 8-bit RGB (the reference's
 * crop_resize_if_necessary: cropping.py:188-280 / 385-465, called from image.py:283-303), fused with the crop and
 * ToTensor + Normalize.  Replaces the host Image.resize(LANCZOS | BICUBIC) + crop + mapa_normalize_image chain.
 * Two steps, so a host can place the weights where it wants:
 *  1. mapa_resize_plan_build (HOST only, no device): Pillow's float64 window weights -> 22-bit fixed point
 *     (Resample.c precompute_coeffs + normalize_coeffs_8bpc, Pillow 12.2.0) for an in_w x in_h -> rs_w x rs_h
 *     resize followed by the crop box (crop_left, crop_top, +out_w, +out_h) of the resized image, into `plan`
 *     (mapa_resize_plan_bytes bytes: a mapa_resize_plan header + int32 tables);
 *  2. copy the plan to device memory, then mapa_resize_normalize: src u8 [in_h][src_row_bytes] (HWC RGB, device)
 *     -> out f32 [3][out_h][out_w] = (u8 / 255 - mean) / std (torchvision's order, like mapa_normalize_image) and/or
 *     out_u8 [out_h][out_w][3] (either may be NULL).  plan_host: the host plan (launch geometry), plan_dev: its device
 *     copy (weights); workspace: mapa_resize_workspace_bytes(plan_host) bytes of device scratch (the 8-bit
 *     intermediate image of the horizontal pass).
 * filter: MAPA_RESAMPLE_* (PIL.Image.Resampling numbering). */
enum { MAPA_RESAMPLE_LANCZOS = 1, MAPA_RESAMPLE_BILINEAR = 2, MAPA_RESAMPLE_BICUBIC = 3 };
typedef struct mapa_resize_plan {
  int32_t in_w, in_h, rs_w, rs_h, crop_left, crop_top, out_w, out_h, filter;
  int32_t need_h, need_v;      /* a pass runs only when its size changes (Resample.c need_horizontal / need_vertical) */
  int32_t kh, kv;              /* window sizes (fixed-point weights per output column / row) */
  int32_t row0, nrows;         /* input rows the kept output rows read */
  int32_t off_hb, off_hk, off_vb, off_vk;  /* int32 offsets of the bounds {xmin, count} / weight tables */
  int32_t int32s;              /* plan size in int32s */
} mapa_resize_plan;
int64_t mapa_resize_plan_bytes(int in_w, int in_h, int rs_w, int rs_h, int filter);
int mapa_resize_plan_build(int in_w, int in_h, int rs_w, int rs_h, int crop_left, int crop_top, int out_w, int out_h,
                           int filter, void* plan, int64_t plan_bytes);
int64_t mapa_resize_workspace_bytes(const void* plan_host);
int mapa_resize_normalize(const uint8_t* src, int64_t src_row_bytes, const void* plan_host, const void* plan_dev,
                          const float* mean3, const float* std3, float* out, uint8_t* out_u8, void* workspace,
                          int64_t workspace_bytes, mapa_stream_t stream);

/* Dense adaptor on its own (RayDirectionsPlusDepthWithConfidenceAndMaskAdaptor, adaptors.py:1898-1951 ->
 * 1740-1796, 393-523, 1012-1073, 1114-1133), for the module-level API (model.dense_adaptor): raw [n][HW][6] f32
 * (the regressor's conv1x1 output rows) -> NCHW f32 planes value [n][4][HW] = (ray / max(|ray|, 1e-8), exp(depth)),
 * conf [n][HW] = 1 + exp(c), logits [n][HW], mask [n][HW] = sigmoid(logits). */
int mapa_dense_adaptor(const float* raw, int n, int64_t HW, float* value, float* conf, float* logits, float* mask,
                       mapa_stream_t stream);

/* infer() post-processing (inference.py:407-480): mask_out = mask_in & ~(depth_edge & normal_edge) per view
 * (geometry.py:1788-1853 points_to_normals, 2102-2145 depth_edge, 2200-2258 normals_edge), bit-exact with the
 * reference's numpy.  pts3d/pts3d_cam [n][H][W][3] f32 (depth_z = pts3d_cam z), masks u8 [n][H][W].
 * normal_cos_thr: normals_edge's angle threshold as the float32 dot-product boundary (a window entry is an edge
 * iff n_c . n_w < normal_cos_thr), from mapa_normal_cos_threshold(edge_normal_threshold) or a host arccos of the
 * caller's choice.  work: n*H*W*17 bytes of scratch when use_edges. */
int mapa_postprocess_mask(const float* pts3d, const float* pts3d_cam, const uint8_t* mask_in, uint8_t* mask_out,
                          int n, int H, int W, float normal_cos_thr, float depth_rtol, int use_edges, void* work,
                          mapa_stream_t stream);
/* Host-only helper: the float32 boundary c with (float32 arccos(d) > deg2rad(tol_deg)) <=> d < c over d in
 * [-1, 1] (arccos in double rounded to float32); -1 if no angle exceeds tol, 2 if every angle (also 0) does. */
float mapa_normal_cos_threshold(double tol_deg);

/* apply_confidence_mask (inference.py:455-470): per view thr = quantile(conf, q) (torch.quantile's linear
 * interpolation), mask_out = mask_in & (conf > thr).  conf [n][HW] f32, masks u8 [n][HW] (may alias). */
int mapa_confidence_mask(const float* conf, const uint8_t* mask_in, uint8_t* mask_out, int n, int64_t HW, float q,
                         mapa_stream_t stream);

/* infer geometry zeroing (inference.py:486-500): pts3d, pts3d_cam ([npix][3]) and depth_along_ray ([npix]) are
 * multiplied in place by mask (u8 0/1, [npix]). */
int mapa_apply_mask(float* pts3d, float* pts3d_cam, float* depth_along_ray, const uint8_t* mask, int64_t npix,
                    mapa_stream_t stream);

/* recover_pinhole_intrinsics_from_ray_directions (geometry.py:304-447, <= 1 MPix branch): rays [n][H][W][3]
 * unit directions -> K [n][3][3]. */
int mapa_recover_intrinsics(const float* rays, int n, int H, int W, float* K, mapa_stream_t stream);

/* rgb() of image.py:93-131: img NCHW [n][3][H][W] -> clip(img*std+mean, 0, 1) as NHWC [n][H][W][3]. */
int mapa_denorm_image(const float* img, int n, int H, int W, const float* mean, const float* stdv, float* out,
                      mapa_stream_t stream);

/* Copy/convert a strided row block: dst[r][c] = src[r][c] (f32 -> bf16/f32). */
int mapa_convert_rows(const float* src, int64_t lds, int rows, int cols, void* dst, int dst_dtype, int64_t ldd,
                      mapa_stream_t stream);

/* Split-precision operand of fp32 rows (the fp32-exact geometric encoders and heads in bf16 mode): x fp32
 * [rows][cols] (row stride ldx) -> y bf16 [rows][2*cols_padded] = [hi | lo] blocks (hi = bf16(x), lo = bf16(x - hi),
 * zero past cols); read by mapa_gemm with a_split as the logical K blocks [hi | hi | lo] against weights packed
 * [hi | lo | hi], a bf16 GEMM over K = 3*cols_padded gives the fp32 product to ~2^-16.
 * Replaces the fp32 conv/linear operands of DenseRepresentationEncoder (dense_rep_encoder.py:234-287). */
int mapa_split_bf16x3(const float* x, int64_t ldx, int64_t rows, int cols, int cols_padded, void* y,
                      mapa_stream_t stream);
/* The same for either split form: dtype MAPA_BF16X3 (as mapa_split_bf16x3) or MAPA_F16X2 (the TF32-equivalent heads:
 * y binary16 [rows][2*cols_padded] = [hi | lo], hi = f16(x), lo = f16(x - hi); range faults: MAPA_FAULT_F16_RANGE). */
int mapa_split_rows(const float* x, int64_t ldx, int64_t rows, int cols, int cols_padded, void* y, int dtype,
                    mapa_stream_t stream);

/* Deterministic synthetic weights on device: out[i] = (2*u_i - 1)*half + mid, u_i = splitmix64 stream of
 * `seed` (bit-identical to mapanything/utils/synthetic.py). */
int mapa_fill_splitmix(float* out, int64_t n, uint64_t seed, float half, float mid, mapa_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------
 * Optional geometric inputs (model.py:792-1289; dense_rep_encoder.py:234-287; global_rep_encoder.py:85-104).
 * The encoders' convolutions / linears run through mapa_gemm (fp32, as the reference's autocast-disabled block).
 * ------------------------------------------------------------------------------------------------------- */
/* nn.PixelUnshuffle(r) from NHWC f32 [n][H][W][C] to token rows out[(v*h+py)*w+px][c*r*r+i*r+j] (ldo), f32/bf16.
 * lognorm != 0 applies the depth-encoder input transform first: x /= view_div[v]; x = x/max(|x|,1e-8)*log1p(|x|)
 * (normalize_depth_using_non_zero_pixels + apply_log_to_norm, geometry.py:1594-1626, 1737-1750). */
int mapa_pixel_unshuffle(const float* in, int n, int H, int W, int C, int r, const float* view_div, int lognorm,
                         void* out, int out_dtype, int64_t ldo, mapa_stream_t stream);

/* Per view: nf = clip(sum(d[d>0]) / (count(d>0) + 1e-8), 1e-8); log_nf (optional) = log(nf + 1e-8).
 * depth [n][HW] f32; work: n*128 floats of scratch (deterministic two-pass reduction). */
int mapa_depth_norm_factors(const float* depth, int n, int HW, float* nf, float* log_nf, void* work,
                            mapa_stream_t stream);

/* Camera inputs of all V views in view 0's frame (model.py:792-896, geometry.py:745-852), identity where
 * cam_mask[v] == 0, translations normalised by their mean non-zero norm (geometry.py:1629-1666).
 * quats [V][4] (x,y,z,w), trans [V][3] -> out_q [V][4], out_t [V][3], out_log_nf [V] = log(nf + 1e-8). */
int mapa_pose_inputs(const float* quats, const float* trans, const uint8_t* cam_mask, int V, float* out_q,
                     float* out_t, float* out_log_nf, mapa_stream_t stream);

/* x[v*T+t][c] += sum_j scales[j*nviews+v] * vecs[(j*nviews+v)*C + c]  (per-view global features, C % 4 == 0) */
int mapa_add_view_vectors(float* x, int T, int C, int nviews, const float* vecs, const float* scales, int nvec,
                          mapa_stream_t stream);

/* preprocess_input_views_for_inference per pixel (inference.py:222-311): rays [n][H][W][3] = unit rays from
 * pinhole K [n][3][3] (get_rays_in_camera_frame, geometry.py:186-241) or rays_in / (|rays_in| + 1e-8); with depth_z
 * [n][H][W]: depth_along_ray = |depth_z * rays / rays_z|.  Exactly one of K / rays_in. */
int mapa_view_rays(const float* K, const float* rays_in, const float* depth_z, int n, int H, int W, float* rays,
                   float* depth_along_ray, mapa_stream_t stream);

/* RoPE-2D in place (uniception croco RoPE2D / cuRoPE2D forward: pos_embed.py:101-155, curope/kernels.cu:17-82):
 * tokens (B, H, N, D) bf16 or f32 with element strides sb, sh, sn (head dim contiguous, D % 16 == 0), positions
 * int64 (B, N, 2) = (y, x).  Head dim [u_y | v_y | u_x | v_x] (quarters Q = D/4); pair j of each half rotates by
 * pos * f0 / base^(j/Q): u' = u cos - v sin, v' = v cos + u sin (fp32 math).  Also usable on the packed qkv buffer
 * (sn = 3*C, sh = 64) before the attention. */
int mapa_rope2d(void* tokens, int dtype, int B, int H, int N, int D, int64_t sb, int64_t sh, int64_t sn,
                const int64_t* positions, float base, float f0, mapa_stream_t stream);

/* dst[i] += src[i] (n % 4 == 0) */
int mapa_add_f32(float* dst, const float* src, int64_t n, mapa_stream_t stream);

/* ---------------------------------------------------------------------------------------------------------
 * Collectives of the view-sharded forward (csrc/comm.cpp): one process per GPU, RCCL over xGMI.
 * Replaces the reference's torch.distributed setup for multi-GPU runs (mapanything/utils/train_tools.py:389-402) for
 * the two exchanges the sharded path has — each global-attention layer's K/V slot all-gather
 * (alternating_attention_transformer.py:657-661 attends over every view's tokens) and the scale-token broadcast.
 * RCCL is dlopen'ed at first use (/opt/rocm/lib/librccl.so.1, or env MAPA_RCCL_LIB): no link-time dependency.
 *   mapa_comm_unique_id_bytes / mapa_comm_get_unique_id: rank 0 makes the id; the host hands it to every rank by its
 *     own channel (a TCP store, MPI, a file).
 *   mapa_comm_init: non-blocking communicator set-up polled against timeout_s (<= 0: 600 s) on `device`; a peer that
 *     never arrives or fails returns an error (the half-built communicator is aborted), never a hang.
 *   mapa_comm_allgather_kv: in place, slot `rank` of `full` ([world][slot_bytes]) goes to every rank (enqueued on
 *     `stream`, graph-capturable).  mapa_comm_broadcast: in place from `root`.
 *   mapa_comm_check: 0, or -1 after an asynchronous error (the communicator is then aborted).
 *   mapa_comm_destroy: finalize + destroy (abort != 0: ncclCommAbort, for a failed or timed-out peer). */
typedef struct mapa_comm mapa_comm;
int mapa_comm_unique_id_bytes(void);
int mapa_comm_get_unique_id(void* id_out);
int mapa_comm_init(mapa_comm** comm, int world, int rank, const void* id, int device, double timeout_s);
int mapa_comm_allgather_kv(mapa_comm* comm, void* full, int64_t slot_bytes, mapa_stream_t stream);
int mapa_comm_broadcast(mapa_comm* comm, void* buf, int64_t bytes, int root, mapa_stream_t stream);
int mapa_comm_check(mapa_comm* comm);
int mapa_comm_destroy(mapa_comm* comm, int abort);

#ifdef __cplusplus
}
#endif
#endif /* MAPA_H */
