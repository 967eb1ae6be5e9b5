// Argument blocks of the fast bf16 conv kernels (conv_fast.hip), dispatched from conv.hip.
#pragma once
#include <hip/hip_runtime.h>

constexpr int kWgBK = 32;  // wgrad K step (pixels); 64 halves the barriers but costs a wave per SIMD: slower

struct FastTNArgs {
  const void* x1;
  const void* x2;
  unsigned x1_bytes, x2_bytes;  // buffer extents for the hardware range check
  int ldc1b, ldc2b;             // pixel strides in bytes
  int c1, cin;                  // channels from x1; total GEMM K per tap
  int H, W;                     // gather-source spatial dims
  int hc, wc;                   // GEMM-row pixel grid per image
  int istride;
  int r0, rs, nr, dh0, dhs;
  int s0, ss, ns, dw0, dws;
  int S;
  const void* wt;
  unsigned w_bytes;
  int ldwb;                     // weight row stride in bytes
  int Ng;
  int ostride, ph, pw, OH, OW;
  void* y;
  int ldy, accumulate;
  const float* bias;
  int relu;
  float* stats;
  int stats_ld;
  int M;
  // data-gradient post-op (dgrad of the consumer of a ReLU / BN-ReLU output; never with
  // accumulate): post 1 = ReLU mask from aux (the ReLU output), 2 = BN-ReLU mask from aux (the BN
  // input z: z*psc + psh > 0).  The masked gradient d is what is stored; ppart[tile][2][Ng] gets the
  // per-row-tile column sums of d and (post 2) of d * (z - pmean) * pinv.
  int post;
  const void* aux;
  int ld_aux;
  const float* psc;
  const float* psh;
  const float* pmean;
  const float* pinv;
  float* ppart;
  // post 3 (residual-BN backward, the data gradient accumulated in registers): aux = the BN input z,
  // pmean / pinv its batch statistics, mbits the packed ReLU mask of the block output (the
  // unetseg_bn_apply_mask layout [M][Ng/8]), aux2 / ld_aux2 / pmean2 / pinv2 the downsample branch's BN
  // input and statistics (aux2 NULL: none).  y holds the residual gradient already delivered; what is
  // stored is d = mask * bf16(bf16(dgrad) + y), and ppart[tile][2 or 3][Ng] = sum d, sum d * xhat1
  // [, sum d * xhat2].
  const unsigned char* mbits;
  const void* aux2;
  int ld_aux2;
  const float* pmean2;
  const float* pinv2;
  int t2d;  // rows of a 2D spatial tile (BM = t2d x 32 pixels), 0 = row-major GEMM rows (set by the launcher)
  // input prologue: x1 is the producer's BN input z, the conv reads relu(z * in_sc[c] + in_sh[c])
  // (its BN-ReLU output, never materialised); register-staged configurations only, x2 == NULL
  const float* in_sc;
  const float* in_sh;
  // fused 1x1 head (halo forward with bias + ReLU only): head_y[n][k][pixel] = head_b[k] +
  // sum_c bf16(y[pixel][c]) * head_w[k][c], k < head_k (1 or 2), fp32 planar NCHW logits
  const float* head_w;
  const float* head_b;
  float* head_y;
  int head_k;
  // issue-order options of the LDS-DMA ring (set by the launcher; UNETSEG_TN_SCHED): bit 0 = the
  // waves of the second SIMD pair issue their K step's DMAs after the first K half's MFMAs
  int sched;
  // a TN configuration chosen by the caller instead of tn_config's rule (0: the rule) -- the stem's
  // experiments (UNETSEG_STEM_CFG)
  int force_cfg;
  // halo forward with bias + ReLU: also store the output's ReLU mask as bits, [M][Ng/8] (bit e of byte
  // b = channel 8b + e > 0); post 4 = post 1 with the mask read from such bits (mbits, halo path only)
  unsigned char* mbits_out;
};

struct FastWgradArgs {
  const void* x1;
  const void* x2;
  unsigned x1_bytes, x2_bytes;
  int ldc1b, ldc2b, c1, cin;
  int H, W, P, Q, stride, pad, S;
  int padw;                     // column padding (== pad except for the width-packed stem)
  const void* dy;
  unsigned dy_bytes;
  int ldyb, Cout, Ng;
  long Kpix;
  int kt_per_split;
  float* ws;
  const float* in_sc;  // as FastTNArgs: X = relu(x1 * in_sc[c] + in_sh[c]) on load (x2 == NULL)
  const float* in_sh;
  int xcd_map;  // ring kernel: XCD-contiguous work order (set by the launcher)
};

// 3x3 / stride 1 / pad 1 weight gradient on the halo path (conv_halo.hip)
struct HaloWgradArgs {
  const void* x1;
  const void* x2;
  unsigned x1_bytes, x2_bytes;
  int ldc1b, ldc2b, c1, cin;
  int N, H, W;
  const void* dy;
  unsigned dy_bytes;
  int ldyb, Cout;
  float* ws;
};

// kernel-configuration codes reported by the unetseg_conv2d_*_config queries (include/unetseg_hip.h)
// 1..14: TN tile configurations of tn_config (conv_fast.hip); 17 / 18: stride-2 dgrad parity classes
// merged into one launch on 128x128 / 64x128 register-staged tiles (launch_tn_multi); 19 / 20: short K
// (2-4 steps) on one LDS stage, 128x128 / 128x64; 21-23: halo-A rings 256x128 / 256x64 / 128x128; 24 / 25:
// the 256x128 / 256x64 halo-A rings persistent (tn_halo_persist_kernel, several tiles per block)
enum { kCfgHalo = 0, kCfgMulti128 = 17, kCfgMulti64 = 18, kCfgStemHalo = 30, kCfgFirst3x3 = 31, kCfgGeneric = 100 };
enum { kWgHalo = 0, kWgFastRow64x256 = 1, kWgFastRow128 = 2, kWgFast64x256 = 3, kWgFast128 = 4, kWgGeneric = 5,
       kWgRing64x256 = 6, kWgRing128 = 7 };

bool tn_fast_ok(const FastTNArgs& a);
int tn_fast_config(const FastTNArgs& a, int* taps_out);  // kCfgHalo or a TN configuration 1..14
int launch_tn_fast(const FastTNArgs& a, hipStream_t st);
// 2-4 independent GEMMs (stride-2 dgrad parity classes) in one launch: the shared row tile (64 /
// 128), or -1 if they cannot be merged; launch_tn_multi returns -1 without launching in that case
int tn_multi_tile_m(const FastTNArgs* fs, int n);
int launch_tn_multi(const FastTNArgs* fs, int n, hipStream_t st);
int tn_fast_tile_m(const FastTNArgs& a);
int tn_fast_post_rows(const FastTNArgs& a);  // partial rows (ppart) a launch_tn_fast call writes
bool tn_fast_post_res_ok(const FastTNArgs& a);  // the configuration has a post-3 (residual) instantiation
int halo3_blocks(const FastTNArgs& a);
bool halo3_ok(const FastTNArgs& a);
int launch_halo3(const FastTNArgs& a, hipStream_t st);
int halo_tile_m();
// the ResNet stem forward on the persistent-halo kernel (conv_halo.hip): eligibility, BN-stat tiles
// (stats [tiles][2][64], stem_halo_tile_m() pixels each) and launch
bool stem_halo_ok(int n, int h, int w, int K, int ldy);
int stem_halo_tiles(int n, int h, int w);
int stem_halo_tile_m();
int launch_stem_halo(const void* xp, int n, int h, int w, const void* wk, void* y, int ldy, float* stats,
                     hipStream_t st);
bool halo3_wgrad_ok(const HaloWgradArgs& a);
int halo3_wgrad_splits(const HaloWgradArgs& a);
int launch_halo3_wgrad(const HaloWgradArgs& a, int G_per, hipStream_t st);
bool wgrad_fast_ok(const FastWgradArgs& a);
bool wgrad_ring_ok(const FastWgradArgs& a);  // launch_wgrad_fast takes the LDS-DMA ring kernel
int launch_wgrad_ring(const FastWgradArgs& a, int splits, hipStream_t st);  // conv_wgrad_ring.hip
int wgrad_fast_splits(int Cout, int Ng, long Kpix);
int launch_wgrad_fast(FastWgradArgs a, int splits, hipStream_t st);

// the plain / attention U-Nets' first 3x3 conv on the packed image (conv_first.hip): 3 -> 64 channels,
// one K = 32 MFMA step per pixel fragment; BN partials per 8 x 32 tile (first3x3_tile_m() pixels)
bool first3x3_ok(int dtype, int c1, int ldc1, int c2, int n, int h, int w, int cout, int r, int s, int stride, int pad,
                 int ldy);
int first3x3_tile_m();
int launch_first3x3(const void* x, int ldx, const void* wk, const float* bias, int relu, void* y, int ldy, float* stats,
                    int n, int h, int w, hipStream_t st);
