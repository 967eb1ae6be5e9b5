/*
 * unetseg_hip.h -- C ABI of libunetseg_hip.so, the MI355X (gfx950) hot path of U-Net segmentation
 * training: conv fwd/dgrad/wgrad on MFMA, BatchNorm, pooling, bilinear upsampling, the attention
 * gate, the fused losses (Lovasz hinge, BCE-with-logits, cross entropy), binary confusion counts and
 * Adam.
 *
 * The reference (TariAgentBenchmark/unet-embroidery-seg) has no FFI: its hot path sits behind the
 * nn.Module protocol (model/model_factory.py:22 build_model, train.py:48 create_model,
 * <Model>.forward, the loss callables in model/unet_training.py:205,253 and
 * model/unet_multitask.py:119).  Each entry point below replaces the PyTorch/ATen operator the
 * reference calls at the cited line; the Python mirror (unet-embroidery-seg_amd/unetseg_hip/*.py)
 * binds them with ctypes and keeps the reference's module names, state_dict keys and errors.
 *
 * Conventions
 *  - All pointers are DEVICE pointers borrowed from the caller (PyTorch's caching allocator); the
 *    library allocates nothing.  `stream` is a hipStream_t (NULL = legacy default stream).
 *  - Activations are NHWC with an explicit pixel stride `ld*` (elements between consecutive pixels),
 *    so a tensor may be a channel slice of a wider buffer (virtual concat).  `M` = n*h*w pixels.
 *  - `dtype`: 0 = fp32, 1 = bf16 (activations).  Weights arrive fp32 and are packed by
 *    unetseg_pack_conv_weight; statistics, biases, BN parameters and losses are always fp32.
 *  - Return value 0 = ok; non-zero = error, message via unetseg_last_error() (thread-local).
 *    Launches are asynchronous: device faults surface at the caller's next synchronisation.
 */
#ifndef UNETSEG_HIP_H
#define UNETSEG_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library ------------------------------------------------------------------------------ */
const char* unetseg_last_error(void);
int unetseg_abi_version(void);
int unetseg_device_arch(char* buf, int n);

/* ---- convolution (nn.Conv2d: model/resnet_backbone.py:19,33,126,167; model/unet_resnet.py:17,19,
 *      72,74,78; model/unet_plain.py:9,12,69; model/unet_attention.py:16,20,24,76;
 *      model/unet_multitask.py:17,18,62,64,69) and the concat feeding it
 *      (torch.cat: model/unet_resnet.py:34, model/unet_plain.py:46, model/unet_attention.py:54) --- */

/* fp32 [K][C][R][S] -> wk dtype [K][R][S][Cpad] (fwd) and, if wt != NULL, wt dtype [C][R][S][K] (dgrad) */
int unetseg_pack_conv_weight(int dtype, const float* w, int K, int C, int R, int S, int Cpad, void* wk, void* wt,
                             void* stream);
/* one conv of a batched pack; `desc` arrays of these live in DEVICE memory */
typedef struct UnetsegPackDesc {
  const float* w;  /* fp32 [K][C][R][S] */
  void* wk;        /* dtype [K][R][S][Cpad] */
  void* wt;        /* dtype [C][R][S][Kld] or NULL (columns K..Kld-1 untouched: a zeroed padded image) */
  long long start; /* first tile of this conv (ascending, desc[0].start == 0; unetseg_pack_tiles tiles) */
  int K, C, R, S, Cpad, Kld; /* Kld: wt row length, 0 = K (the 64-padded dgrad image of a narrow 1x1 conv) */
} UnetsegPackDesc;
/* blocks unetseg_pack_conv_weights spends on one conv: desc[i+1].start = desc[i].start + this */
int unetseg_pack_tiles(int K, int Cpad, int taps);
/* every conv weight of a model in one launch (total = number of tiles) */
int unetseg_pack_conv_weights(int dtype, const void* desc, int n, long total, void* stream);
/* legacy generic row tile (kept for ABI v1 callers) */
int unetseg_conv_tile_m(void);
/* row tile of the BN partial statistics unetseg_conv2d_fwd writes for this shape */
int unetseg_conv2d_fwd_tile_m(int dtype, int c1, int ldc1, int c2, int ldc2, int n, int h, int w, int cout, int r,
                              int s, int stride, int pad);
/* y[n,p,q,cout] = conv(cat(x1[.., c1], x2[.., c2]), wk) (+bias) (ReLU); stats (may be NULL):
 * fp32 [ceil(M/tile)][2][cout] = per-tile (sum, M2 about the tile mean) of the rounded y (BN train) */
int unetseg_conv2d_fwd(int dtype, const void* x1, int c1, int ldc1, const void* x2, int c2, int ldc2, int n, int h,
                       int w, const void* wk, int cout, int r, int s, int stride, int pad, const float* bias, int relu,
                       void* y, int ldy, float* stats, void* stream);
/* 1x1 stride-1 conv reading relu(x1 * in_sc[c] + in_sh[c]) -- the producer's BN-ReLU output, never
 * stored (model/resnet_backbone.py:58-62 bn2 -> ReLU -> conv3); epilogue as unetseg_conv2d_fwd. bf16 */
int unetseg_conv2d_fwd_bnrelu_in(int dtype, const void* x1, int c1, int ldc1, int n, int h, int w, const void* wk,
                                 int cout, const float* in_sc, const float* in_sh, const float* bias, int relu,
                                 void* y, int ldy, float* stats, void* stream);
/* TN configuration that call runs (host-only query, -1 = none) */
int unetseg_conv2d_fwd_bnrelu_in_config(int dtype, int c1, int ldc1, int n, int h, int w, int cout);
/* The decoder's last 3x3 conv (64 -> 64, stride 1, pad 1, bias + ReLU; reference model/unet_resnet.py:77-78)
 * with the final 1x1 conv (model/unet_resnet.py:79, 64 -> head_k in {1, 2}) fused into its epilogue:
 * y as unetseg_conv2d_fwd, logits fp32 [n][head_k][h][w] = head_b + head_w . y (the stored bf16 y).
 * Replaces the reference's Conv2d -> ReLU -> Conv2d(1x1) forward.  bf16, halo path only; the _ok
 * query (host only) says whether a shape qualifies. */
int unetseg_conv2d_fwd_head_ok(int dtype, int ldc1, int n, int h, int w, int ldy, int head_k);
int unetseg_conv2d_fwd_head(int dtype, const void* x1, int ldc1, int n, int h, int w, const void* wk,
                            const float* bias, void* y, int ldy, int head_k, const float* head_w, const float* head_b,
                            float* logits, void* stream);
/* The decoder's 512^2 up_conv conv1 (3x3, 64 -> 64, stride 1, pad 1, bias + ReLU; model/unet_resnet.py:
 * 90-97): y as unetseg_conv2d_fwd, plus the ReLU mask of the stored y packed to bits, mbits[pixel][8]
 * (bit e of byte b = y[pixel][8b + e] > 0), which its consumer's data gradient reads (post 4 of
 * unetseg_conv2d_dgrad_post) instead of the 64-channel activation.  bf16, halo path only; mbits ==
 * NULL: returns 1 when the shape qualifies, else 0 (host only, nothing launched). */
int unetseg_conv2d_fwd_mask(int dtype, const void* x1, int ldc1, int n, int h, int w, const void* wk,
                            const float* bias, void* y, int ldy, unsigned char* mbits, void* stream);
/* its weight gradient with the same input prologue (workspace: unetseg_conv2d_wgrad_workspace) */
int unetseg_conv2d_wgrad_bnrelu_in(int dtype, const void* x1, int c1, int ldc1, int n, int h, int w, const void* dy,
                                   int ldy, int cout, const float* in_sc, const float* in_sh, float* ws,
                                   size_t ws_bytes, float* dw, int dw_c, int accumulate, void* stream);
/* y = [relu](conv(x, wk) * escale[cout] + bias[cout]): eval-mode BN on the accumulator (generic kernel) */
int unetseg_conv2d_fwd_affine(int dtype, const void* x1, int c1, int ldc1, const void* x2, int c2, int ldc2, int n,
                              int h, int w, const void* wk, int cout, int r, int s, int stride, int pad,
                              const float* escale, const float* bias, int relu, void* y, int ldy, void* stream);
/* Kernel-configuration queries (host only, nothing is launched; replace no reference operator:
 * they let the parity tests assert that they exercise every kernel configuration the benchmark
 * selects).  Codes: 0 = halo3 (64-channel 3x3 kernel), 1..14 = TN tile configuration
 * (conv_fast.hip tn_config: 1 256x64, 2 256x128, 3 128x128, 4 128x128 one K step, 5 64x128,
 * 6 128x64, 7 256x128 LDS-DMA ring, 8 128x128 ring, 9 64x128 ring, 10 128x128 5-stage ring,
 * 11-14 other rings), 17 / 18 = the parity classes of a stride-2 data gradient merged into one launch
 * on 128x128 / 64x128 tiles, 19 / 20 = short-K (2-4 steps) 128x128 / 128x64 tiles on one LDS stage,
 * 21 / 22 / 23 = halo-A ring 256x128 / 256x64 / 128x128, 24 / 25 = the first two persistent (several tiles per
 * block), 100 = generic igemm kernel (fp32 / unaligned channels).  *taps_out = the
 * compile-time tap count of an LDS-DMA ring (9 or 1; 0 = generic ring or not a ring). */
int unetseg_conv2d_fwd_config(int dtype, int c1, int ldc1, int c2, int ldc2, int n, int h, int w, int cout, int r,
                              int s, int stride, int pad, int* taps_out);
/* per output-parity class of the data gradient: cfg_out/taps_out[ph*stride+pw] (-1: not launched);
 * returns the number of classes launched */
int unetseg_conv2d_dgrad_config(int dtype, int ldy, int n, int p, int q, int cout, int cin, int r, int s, int stride,
                                int pad, int ldx, int h, int w, int* cfg_out, int* taps_out);
/* weight-gradient kernel: 0 = halo3_wgrad, 1 = wgrad_fast 64x256 row-run, 2 = wgrad_fast 128x128
 * row-run, 3 / 4 = the same tiles with general pixel walks, 5 = generic; *splits_out = split-K
 * slabs (reduced by wgrad_reduce<16> from 16 slabs, <4> from 4, else <1>) */
int unetseg_conv2d_wgrad_config(int dtype, int c1, int ldc1, int c2, int ldc2, int n, int h, int w, int ldy, int cout,
                                int r, int s, int stride, int pad, int* splits_out);
/* dx[n,h,w,cin] (+)= conv_transpose(dy[n,p,q,cout], wt) */
int unetseg_conv2d_dgrad(int dtype, const void* dy, int ldy, int n, int p, int q, const void* wt, int cout, int cin,
                         int r, int s, int stride, int pad, void* dx, int ldx, int h, int w, int accumulate,
                         void* stream);
/* data gradient whose epilogue applies the producer's ReLU (post 1: aux = ReLU output) or BN-ReLU
   (post 2: aux = BN input z; psc/psh = BN affine, pmean/pinv = batch stats) mask and writes the
   first backward reduction of that op: part[rows][2][cin] = (sum d, sum d*xhat) per row tile
   (fuses model/resnet_backbone.py:95-110 ReLU+BN backward pass 1 / unet_resnet.py:37-40 ReLU+bias
   into the consumer conv's dgrad).  post 4: post 1 with the mask read from the producer's packed
   ReLU bits (aux = mbits of unetseg_conv2d_fwd_mask, ld_aux ignored; 64-channel halo path only).
   part == NULL: returns rows, or -1 when the shape has no fused path (bf16 fast kernels only). */
int unetseg_conv2d_dgrad_post(int dtype, const void* dy, int ldy, int n, int p, int q, const void* wt, int cout,
                              int cin, int r, int s, int stride, int pad, void* dx, int ldx, int h, int w, int post,
                              const void* aux, int ld_aux, const float* psc, const float* psh, const float* pmean,
                              const float* pinv, float* part, int rows, void* stream);
/* 1x1 stride-1 data gradient accumulated onto the other consumers' gradient already in dx (pixel stride
   ldx >= cin, a multiple of 8: dx may be a channel slice of a skip-concat gradient), with the residual
   BN-add-ReLU backward's first pass in its epilogue (model/resnet_backbone.py:88,110-113: the next
   block's conv1 is the last consumer of the block output): dx = mask * bf16(dgrad + dx), mask =
   the packed ReLU bits written by unetseg_bn_apply_mask, part[rows][2 or 3][cin] = (sum d,
   sum d * (y1 - mean1) * inv1 [, sum d * (y2 - mean2) * inv2]) per row tile (y2 = the downsample
   branch's BN input, NULL: none).  Replaces unetseg_bn_bwd_reduce over dx.  part == NULL: returns rows,
   or 0 when the shape has no fused kernel (bf16 only). */
int unetseg_conv2d_dgrad_post_res(int dtype, const void* dy, int ldy, int n, int p, int q, const void* wt, int cout,
                                  int cin, void* dx, int ldx, const void* y1, int ld1, const float* mean1,
                                  const float* inv1, const unsigned char* mbits, const void* y2, int ld2,
                                  const float* mean2, const float* inv2, float* part, int rows, void* stream);
size_t unetseg_conv2d_wgrad_workspace(int dtype, int n, int p, int q, int cout, int cin, int r, int s);
/* dw fp32 [cout][dw_c][r][s] (PyTorch layout) (+)= sum_pix dy x; ws of the size queried above */
int unetseg_conv2d_wgrad(int dtype, const void* x1, int c1, int ldc1, const void* x2, int c2, int ldc2, int n, int h,
                         int w, const void* dy, int ldy, int cout, int r, int s, int stride, int pad, float* ws,
                         size_t ws_bytes, float* dw, int dw_c, int accumulate, void* stream);
/* the same for one source with dw holding only the first dw_rows (<= cout) GEMM rows: a padded-K conv
   (the attention gates' theta / phi, model/unet_attention.py:12-19: cout = the 64-padded output
   channels, whose dY columns are zero) accumulates straight into its real [dw_rows][dw_c][r][s] gradient */
int unetseg_conv2d_wgrad_rows(int dtype, const void* x1, int c1, int ldc1, int n, int h, int w, const void* dy,
                              int ldy, int cout, int r, int s, int stride, int pad, float* ws, size_t ws_bytes,
                              float* dw, int dw_c, int accumulate, int dw_rows, void* stream);

/* ---- ResNet stem on the fast kernels (model/resnet_backbone.py:126-131, conv 7x7/s2/p3) -------
   xp: width-padded bf16 [n][h][w+8][8] from unetseg_pack_input_stem (image column at +3);
   wk: bf16 [K][7][64] from unetseg_stem_pack_weight (k, filter row, filter col*8 + channel) */
int unetseg_pack_input_stem(const float* x, int n, int c, int h, int w, void* xp, void* stream);
int unetseg_stem_pack_weight(const float* w, int K, int C, void* wk, void* stream);
int unetseg_stem_fwd_tile_m(int n, int h, int w, int K);
/* configuration of unetseg_stem_fwd (30 = the persistent-halo stem kernel: 64 output channels, even
   input sizes whose output tiles into 16 x 32 pixels; else a TN code, -1: unsupported) and split-K
   slabs of unetseg_stem_wgrad */
int unetseg_stem_config(int n, int h, int w, int K, int* splits_out);
int unetseg_stem_fwd(const void* xp, int n, int h, int w, const void* wk, int K, void* y, int ldy, float* stats,
                     void* stream);
size_t unetseg_stem_wgrad_workspace(int n, int h, int w, int K);
int unetseg_stem_wgrad(const void* xp, int n, int h, int w, const void* dy, int ldy, int K, float* ws,
                       size_t ws_bytes, float* dw, int C, int accumulate, void* stream);
/* NCHW fp32 input [n][c][h][w] -> NHWC dtype [n][h][w][cpad] (zero channel padding) */
int unetseg_pack_input(int dtype, const float* x, int n, int c, int h, int w, int cpad, void* y, void* stream);

/* ---- BatchNorm2d, training and eval (model/resnet_backbone.py:127,169; model/unet_plain.py:10,13;
 *      model/unet_attention.py:17,21,25) -------------------------------------------------------- */

/* Chan-merge conv partials part[G][2][C] -> batch mean/invstd, scale/shift; update running stats (momentum,
 * unbiased var) and num_batches_tracked when rmean != NULL */
int unetseg_bn_finalize(const float* part, int C, int G, long M, int tile, const float* gamma, const float* beta,
                        float* rmean, float* rvar, long long* nbt, float momentum, float eps, float* mean,
                        float* invstd, float* scale, float* shift, void* stream);
/* BN partials of an NHWC view no conv produced (model/unet_dualdense.py:9-10: BatchNorm over a dense
 * block's concatenation): part [ceil(M/tile)][2][C] = (sum, M2 about the tile mean), for bn_finalize */
int unetseg_channel_stats_tiles(long M, int tile);
int unetseg_channel_stats(int dtype, const void* x, int ldx, long M, int c, int tile, float* part, void* stream);
/* eval-mode BN folded into the conv epilogue (model/resnet_backbone.py:58-61, model/unet_plain.py:8-15
 * in .eval()): kscale = gamma / sqrt(running_var + eps), bias = beta - running_mean * kscale
 * (+ conv_bias * kscale), for unetseg_conv2d_fwd_affine */
int unetseg_bn_fold(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar, float eps,
                    const float* conv_bias, float* kscale, float* bias, void* stream);
int unetseg_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                           float eps, float* scale, float* shift, void* stream);
/* out = [relu](y*sc + sh [+ r | + r*sc2 + sh2])   res_mode 0 none, 1 identity add, 2 BN'd add */
int unetseg_bn_apply(int dtype, const void* y, int ldy, const float* sc, const float* sh, const void* r, int ldr,
                     const float* sc2, const float* sh2, int res_mode, int relu, void* out, int ldo, long M, int C,
                     void* stream);
/* unetseg_bn_apply with relu = 1 that also writes the ReLU mask of `out` packed one byte per (pixel,
 * 16-B channel vector): mbits[p * C/V + c/V] bit (c % V) = (stored out[p][c] > 0), V = 8 (bf16) / 4
 * (fp32).  The backward below reads it (A = mbits, lda = 0) instead of the activation: the residual
 * BN-add-ReLU of the ResNet bottleneck (model/resnet_backbone.py:66-76), 1/16 of the bytes. */
int unetseg_bn_apply_mask(int dtype, const void* y, int ldy, const float* sc, const float* sh, const void* r, int ldr,
                          const float* sc2, const float* sh2, int res_mode, void* out, int ldo, long M, int C,
                          unsigned char* mbits, void* stream);
/* partial-buffer geometry of the channel reductions below: returns G (row groups) */
int unetseg_reduce_tiles(int dtype, long M, int C, int* tv_out, int* ppb_out);
/* backward through [relu](BN(y1) [+ BN(y2)]): per-channel partials of dz and dz*xhat.  The ReLU
 * mask comes from the activation A, from the packed mask of unetseg_bn_apply_mask (A = mbits with
 * lda == 0), or (A == NULL, msc != NULL: no residual) is recomputed from y1 as fmaf(y1, msc, msh) > 0
 * -- the forward's BN scale/shift -- saving one tensor read.  unetseg_bn_bwd_apply likewise. */
int unetseg_bn_bwd_reduce(int dtype, const void* dA, int ldd, const void* A, int lda, const float* msc,
                          const float* msh, const void* y1, int ld1, const float* mean1, const float* inv1,
                          const void* y2, int ld2, const float* mean2, const float* inv2, long M, int C, float* part,
                          int G, void* stream);
int unetseg_bn_bwd_finalize(const float* part, int C, int G, long M, int nbranch, const float* g1, const float* inv1,
                            float* dg1, float* db1, const float* g2, const float* inv2, float* dg2, float* db2,
                            float* coef, void* stream);
int unetseg_bn_bwd_apply(int dtype, const void* dA, int ldd, const void* A, int lda, const float* msc,
                         const float* msh, const void* y1, int ld1, const float* mean1, const float* inv1, void* dy1,
                         int ldo1, const void* y2, int ld2,
                         const float* mean2, const float* inv2, void* dy2, int ldo2, const float* coef, void* dzout,
                         int ldz, int dz_acc, long M, int C, void* stream);
/* ReLU backward (mask from the activation A) + per-channel bias-grad partials */
int unetseg_relu_bwd_bias(int dtype, const void* dA, int ldd, const void* A, int lda, void* dY, int ldy, long M, int C,
                          float* part, int G, void* stream);
int unetseg_colsum_finalize(const float* part, int C, int G, float* out, int accumulate, void* stream);
/* BN backward coefficients / ReLU bias gradient from the row partials part[G][2][C] written by
   unetseg_conv2d_dgrad_post (model/resnet_backbone.py BatchNorm2d backward, unet_resnet.py ReLU) */
int unetseg_bn_bwd_finalize_rows(const float* part, int C, int G, long M, const float* g1, const float* inv1,
                                 float* dg1, float* db1, float* coef, void* stream);
/* the same for the residual post-op's part[G][1+nbranch][C] (unetseg_conv2d_dgrad_post_res): coefficients
   of both branches as unetseg_bn_bwd_finalize */
int unetseg_bn_bwd_finalize_rows_res(const float* part, int C, int G, long M, int nbranch, const float* g1,
                                     const float* inv1, float* dg1, float* db1, const float* g2, const float* inv2,
                                     float* dg2, float* db2, float* coef, void* stream);
int unetseg_colsum_rows(const float* part, int C, int G, int k, float* out, int accumulate, void* stream);
/* Row partials [G][nq][C] -> [ceil(G/16)][nq][C] (16 consecutive rows merged; nq 2 or 3), run ahead of the
   finalizes above when G is large.  tile > 0: the rows are BN statistics (sum, M2 about the row mean) of
   `tile` pixels each (the last min(tile, M - g*tile)) merged by Chan's formula (nq == 2), so the merged
   partials feed unetseg_bn_finalize with tile * 16; tile == 0: plain sums.  No reference operator: an
   internal reduction stage of BatchNorm2d's statistics / backward sums. */
int unetseg_fin_merge_rows(const float* part, int C, int G, long M, int tile, int nq, float* out, void* stream);

/* ---- pooling / resampling (nn.MaxPool2d: model/resnet_backbone.py:131, model/unet_plain.py:25,
 *      model/unet_attention.py:66-69; UpsamplingBilinear2d / Upsample / interpolate:
 *      model/unet_resnet.py:21,71, model/unet_plain.py:36, model/unet_attention.py:32,41,53) ------- */
int unetseg_maxpool_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int k, int s, int ceil_mode,
                        void* y, int ldy, uint8_t* idx, int* p_out, int* q_out, void* stream);
int unetseg_maxpool_bwd(int dtype, const void* dy, int ldy, const uint8_t* idx, int n, int h, int w, int c, int k,
                        int s, int p, int q, void* dx, int ldx, int accumulate, void* stream);
int unetseg_upsample2x_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int align_corners, void* y,
                           int ldy, void* stream);
int unetseg_upsample2x_bwd(int dtype, const void* dy, int ldy, int n, int h, int w, int c, int align_corners,
                           void* dx, int ldx, int accumulate, void* stream);
/* upsample2x_bwd with the backward of the ReLU that produced x fused in (x = A, that ReLU's output, the
 * upsample its sole consumer; reference model/unet_resnet.py:25-33 unetUp conv2 -> ReLU -> next
 * block's UpsamplingBilinear2d): dx = (A > 0) ? adjoint(dy) : 0 (no accumulate); part fp32
 * [rows][2][c], slot 0 = per-block column sums of dx (the conv's bias-gradient partials,
 * unetseg_colsum_rows); rows = unetseg_upsample2x_bwd_tiles(...) */
int unetseg_upsample2x_bwd_tiles(int dtype, int n, int h, int w, int c);
int unetseg_upsample2x_bwd_relu(int dtype, const void* dy, int ldy, int n, int h, int w, int c, int align_corners,
                                const void* a, int lda, void* dx, int ldx, float* part, int rows, void* stream);
int unetseg_add(int dtype, const void* x, int ldx, void* out, int ldo, long M, int c, void* stream);
/* general bilinear resize to (oh, ow) with ATen's source-index rule (F.interpolate(size=...):
 * model/unet_attention.py:31-33,52-53, model/unet_dualdense.py:57-58; align_corners=True for the
 * multiclass losses' logit resize, model/unet_training.py:14-15); backward is a deterministic gather */
int unetseg_resize_bilinear_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int oh, int ow,
                                int align_corners, void* y, int ldy, void* stream);
int unetseg_resize_bilinear_bwd(int dtype, const void* dy, int ldy, int n, int h, int w, int c, int oh, int ow,
                                int align_corners, void* dx, int ldx, int accumulate, void* stream);
/* zero padding x [n][h][w] into y [n][oh][ow] at (top, left) (F.pad, model/unet_plain.py:42-45) and its
 * backward dx (+)= the (top, left) window of dy */
int unetseg_pad2d_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int top, int left, int oh,
                      int ow, void* y, int ldy, void* stream);
int unetseg_pad2d_bwd(int dtype, const void* dy, int ldy, int n, int h, int w, int c, int top, int left, int oh,
                      int ow, void* dx, int ldx, int accumulate, void* stream);

/* ---- narrow 1x1 heads (final / outc / seg_head / psi: model/unet_resnet.py:78,
 *      model/unet_plain.py:69, model/unet_multitask.py:69, model/unet_attention.py:24) ------------ */
int unetseg_pw_small_tile(long M); /* pixels per tile (2048, smaller when M gives < 512 tiles) */
int unetseg_pw_small_tiles(long M);
/* y fp32 planar [n][k][hw] (k <= 2); stats (k == 1, may be NULL) [unetseg_pw_small_tiles(M)][2] */
int unetseg_pw_small_fwd(int dtype, const void* x, int ldx, long M, int hw, int c, int k, const float* w,
                         const float* b, float* y, float* stats, void* stream);
int unetseg_pw_small_bwd(int dtype, const float* dy, const void* x, int ldx, long M, int hw, int c, int k,
                         const float* w, void* dx, int lddx, int dx_acc, float* part_w, float* part_b, void* stream);
/* pw_small_bwd with the producer ReLU's backward fused (x = ReLU output, sole consumer; bf16):
 * dx = (x > 0) ? dy.W : 0; part_d [G][2][c], slot 0 = column sums of dx (replaces the
 * reference autograd's ReLU backward + conv bias grad of up_conv's last conv, model/unet_resnet.py:70-78,100-103). */
int unetseg_pw_small_bwd_relu(int dtype, const float* dy, const void* x, int ldx, long M, int hw, int c, int k,
                              const float* w, void* dx, int lddx, float* part_w, float* part_b, float* part_d,
                              void* stream);

/* ---- attention gate (AttentionGate.forward: model/unet_attention.py:28-36) -------------------- */
/* alpha = sigmoid(BN1(psi)); gated = skip * alpha */
int unetseg_attn_apply(int dtype, const void* skip, int lds_, const float* psi, const float* sc, const float* sh,
                       float* alpha, void* gated, int ldg, long M, int c, void* stream);
/* part: [2][G1] (sum dpsibn, sum dpsibn * xhat) per 128-pixel tile, G1 = unetseg_attn_bwd1_tiles(M) */
int unetseg_attn_bwd1_tiles(long M);
int unetseg_attn_bwd1(int dtype, const void* dg, int ldg, const void* skip, int lds_, const float* alpha,
                      const float* psi, const float* mean, const float* inv, void* dskip, int ldds, int ds_acc,
                      float* dpsibn, long M, int c, float* part, void* stream);
int unetseg_attn_bwd2(int dtype, const float* dpsibn, const float* psi, const float* mean, const float* inv,
                      const float* coef, const void* f, int ldf, const float* wpsi, void* dzf, int lddz, long M, int c,
                      float* part_w, float* part_b, void* stream);

/* ---- losses and metrics ---------------------------------------------------------------------- */
/* Lovasz hinge, per-image mean (model/unet_training.py:219-280) on z = o[:,1]-o[:,0] (nch 2,
 * utils/train_and_eval.py:106-113) or o[:,0] (nch 1); gz = dloss/dz; loss fp32 scalar */
size_t unetseg_lovasz_workspace(int B, long P);
int unetseg_lovasz_fwd(const float* out, int nch, const int64_t* tgt, int B, long P, void* ws, size_t ws_bytes,
                       float* gz, float* loss, void* stream);
/* per-image Lovasz over the pixels whose target is not ignore_index (model/unet_training.py:268-274) */
int unetseg_lovasz_fwd_masked(const float* out, int nch, const int64_t* tgt, int B, long P, long ignore_index, void* ws,
                              size_t ws_bytes, float* gz, float* loss, void* stream);
/* BCE-with-logits mean with optional scalar pos_weight (model/unet_training.py:205-216) */
size_t unetseg_bce_workspace(int B, long P);
int unetseg_bce_fwd(const float* out, int nch, const int64_t* tgt, int B, long P, const float* pos_weight, void* ws,
                    size_t ws_bytes, float* gz, float* loss, void* stream);
/* dout[n][ch][P] = gz * (s1*a1) [* (s2*a2)] with the two-class split of utils/train_and_eval.py:106 */
int unetseg_dz_to_dout(const float* gz, int B, long P, int nch, const float* s1, float a1, const float* s2, float a2,
                       float* scratch, float* dout, void* stream);
/* global tp/fp/fn/tn (argmax, tie -> class 0) of utils/train_and_eval.py:116-138,293 */
int unetseg_confusion(const float* out, int nch, const int64_t* tgt, int B, long P, unsigned long long* conf,
                      void* stream);
/* the same with ignore_index (utils/train_and_eval.py:125-126,172-176): pixels whose target equals
 * ignore_index are skipped by the counts and the losses.  masked loss kind 0 = BCE over the valid
 * pixels, 1 = the reference's Lovasz on the flattened valid pixels (a per-pixel hinge mean, since
 * lovasz_hinge_loss then loops over single elements: model/unet_training.py:267-276) */
int unetseg_confusion_masked(const float* out, int nch, const int64_t* tgt, int B, long P, long ignore_index,
                             unsigned long long* conf, void* stream);
size_t unetseg_masked_loss_workspace(int B, long P);
int unetseg_masked_loss_fwd(const float* out, int nch, const int64_t* tgt, int B, long P, long ignore_index, int kind,
                            const float* pos_weight, void* ws, size_t ws_bytes, float* gz, float* loss, void* stream);
/* cross entropy, mean over the batch (MultiTaskLoss: model/unet_multitask.py:119-139) */
int unetseg_ce_fwd(const float* logits, const int64_t* tgt, int B, int K, float* loss, float* dlog, void* stream);
int unetseg_scale_grad(const float* g, long n, const float* s1, float a1, const float* s2, float a2, float* out,
                       void* stream);

/* ---- multiclass task (model/unet_training.py:9-91 CE_Loss / Focal_Loss / Dice_loss;
 *      utils/train_and_eval.py:20-103 metrics; model/*.py outc/final with num_classes > 2;
 *      predict.py:79-93 post-processing).  Logits fp32 planar [B][C][P], C <= 32. ----------------- */
/* 1x1 head with 1 <= k <= 32 outputs: y fp32 [n][k][hw] = x . W^T + b (W fp32 [k][c]) */
int unetseg_pw_head_fwd(int dtype, const void* x, int ldx, long M, int hw, int c, int k, const float* w,
                        const float* b, float* y, void* stream);
int unetseg_pw_head_tiles(long M);
/* dx (may be NULL) (+)= dy . W; part_w [k][c][G], part_b [k][G] (G = unetseg_pw_head_tiles(M)); c divides 256 */
int unetseg_pw_head_bwd(int dtype, const float* dy, const void* x, int ldx, long M, int hw, int c, int k,
                        const float* w, void* dx, int lddx, int dx_acc, float* part_w, float* part_b, void* stream);
size_t unetseg_mc_loss_workspace(int B, int C, long P);
/* loss fp32[3] = (total, main, dice).  focal: main term 0 = CE (class weights cls_w or NULL, ignore_index),
 * 1 = Focal (alpha < 0: None, gamma), 2 = none; dice_t float [B][P][ct] one-hot (NULL: no Dice term) */
int unetseg_mc_loss_fwd(const float* out, const int64_t* tgt, int B, int C, long P, const float* cls_w,
                        long ignore_index, int focal, float alpha, float gamma, const float* dice_t, int ct,
                        float beta, float smooth, void* ws, size_t ws_bytes, float* loss, void* stream);
/* dout fp32 [B][C][P] = gscale[0] * d total / d out (same arguments and workspace as the forward) */
int unetseg_mc_loss_bwd(const float* out, const int64_t* tgt, int B, int C, long P, const float* cls_w,
                        long ignore_index, int focal, float alpha, float gamma, const float* dice_t, int ct,
                        float beta, float smooth, const void* ws, const float* gscale, float* dout, void* stream);
/* hist u64 [(C+1)][C] += (target row, argmax column); targets outside [0, C) count in row C */
int unetseg_mc_confusion(const float* out, const int64_t* tgt, int B, int C, long P, unsigned long long* hist,
                         void* stream);
/* one image: labels int32 [OH][OW] = argmax_c bilinear(align_corners=False)-resized softmax of the
 * logits [C][H][W] cropped to rows y0..y0+ch, cols x0..x0+cw */
int unetseg_softmax_resize_argmax(const float* logits, int C, int H, int W, int y0, int x0, int ch, int cw, int OH,
                                  int OW, int32_t* labels, void* stream);

/* ---- device augmentation of the loader (utils/hf_dataloader.py:67-105, 111-180, 183-213) -------
 * Replaces HFUnetDataset.get_random_data + preprocess + hf_unet_dataset_collate for one batch:
 * PIL BICUBIC image / NEAREST mask resize (bit-exact), flip, paste on the grey / zero canvas,
 * OpenCV-style HSV jitter (hsv flag), /255, label binarise / clamp, one-hot.
 * desc: int64 [B][20] per-sample descriptors (host copy for validation + device copy), tables:
 * int32 per-sample resize / nearest / LUT tables (host + device), src / msk: packed uint8 RGB images
 * and L masks, tmp / rsz: uint8 scratch.  Outputs: img fp32 [B][3][H][W], png int64 [B][H][W],
 * onehot fp32 [B][H][W][num_classes+1] (may be NULL). */
int unetseg_augment_tables_len(long long nw, long long nh, long long ksh, long long ksv, long long hsv);
int unetseg_augment_batch(const long long* desc_host, const long long* desc, int B, const int* tables_host,
                          const int* tables, long long n_tables, const uint8_t* src, long long src_bytes,
                          const uint8_t* msk, long long msk_bytes, uint8_t* tmp, long long tmp_bytes, uint8_t* rsz,
                          long long rsz_bytes, int H, int W, int num_classes, int binary, float* img, long long* png,
                          float* onehot, void* stream);
/* The same with the per-sample tables built on the device (aug_tables: Resample.c precompute_coeffs /
 * normalize_coeffs_8bpc, Geometry.c ImagingScaleAffine and the reference's HSV LUTs restated in
 * float64, bit-identical to utils/augment_tables.py): hsv_r float64 [B][3] (device; the drawn HSV
 * factors, hf_dataloader.py:166), tables: device int32 scratch of n_tables entries at the
 * descriptors' offsets.  The host decodes, draws and packs pixels only. */
int unetseg_augment_batch_dev(const long long* desc_host, const long long* desc, int B, const double* hsv_r,
                              int* tables, long long n_tables, const uint8_t* src, long long src_bytes,
                              const uint8_t* msk, long long msk_bytes, uint8_t* tmp, long long tmp_bytes,
                              uint8_t* rsz, long long rsz_bytes, int H, int W, int num_classes, int binary, float* img,
                              long long* png, float* onehot, void* stream);
/* the device-built tables alone (parity tests); max_tasks >= max over samples of nw + nh + 2 (+768) */
int unetseg_augment_tables_dev(const long long* desc, int B, const double* hsv_r, int* tables, int max_tasks,
                               void* stream);

/* ---- streams ---------------------------------------------------------------------------------- */
/* `waiter` waits for everything enqueued so far on `signaler` (device-scope release event; no
   reference counterpart: orders the weight-gradient stream against the compute stream) */
int unetseg_stream_wait(void* waiter, void* signaler);
/* a stream restricted to the CUs set in mask[0 .. n_words) (bit i of word w = CU 32 w + i); *out = the
   hipStream_t (no reference counterpart: keeps the weight-gradient stream's persistent kernels off
   part of the chip, UNETSEG_SIDE_CUMASK) */
int unetseg_stream_create_cumask(const unsigned* mask, int n_words, void** out);

/* ---- multitask classification head (model/unet_multitask.py:73-80) -------------------------- */
int unetseg_gap_fwd(int dtype, const void* x, int ldx, int B, int HW, int C, float* g, void* stream);
int unetseg_gap_bwd(int dtype, const float* dg, int B, int HW, int C, void* dx, int ldx, int accumulate,
                    void* stream);
/* y = [dropout(relu(.))] (x W^T + b); act 1 = ReLU+dropout(p_drop) with hashed mask from seed or mask_in */
int unetseg_linear_fwd(const float* x, const float* W, const float* bias, int B, int I, int O, int act, float p_drop,
                       unsigned long long seed, const float* mask_in, float* mask_out, float* pre, float* y,
                       void* stream);
int unetseg_linear_bwd(const float* dy, const float* pre, const float* mask, float p_drop, int act, const float* x,
                       const float* W, int B, int I, int O, float* dx, float* dW, float* db, float* scratch,
                       void* stream);

/* ---- optimizer: torch.optim.Adam with coupled weight decay (train.py:62-78) over one flat fp32
 *      arena; grad_scale (may be NULL) multiplies g first ------------------------------------------ */
int unetseg_adam(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2, float eps,
                 float wd, int step, const float* grad_scale, void* stream);
/* capturable Adam (hipGraph replay): hyper[0] = lr and *step (steps taken; advanced by one after the
   update) are read from device memory */
int unetseg_adam_dev(float* p, const float* g, float* m, float* v, long n, const float* hyper, int* step, float beta1,
                     float beta2, float eps, float wd, const float* grad_scale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UNETSEG_HIP_H */
