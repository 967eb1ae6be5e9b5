// The first 3x3 convolution of the plain / attention U-Nets: 3 -> 64 channels, stride 1, pad 1, on
// the packed image (NHWC bf16, channels 3..7 zero: unetseg_pack_input), with the BN partial
// statistics of its rounded output (model/unet_plain.py:8-15 DoubleConv; model/unet_attention.py:65
// `inc`).  The generic implicit GEMM spent 264 us per call at attention_unet 512^2 B=8 on this
// shape: its K loop walks 9 taps x one 8-channel chunk through 64-wide tiles.  Here the whole 3x3 x 8
// receptive field (72 products; the image's channels 3..7 are zero, their weights too) is three
// K = 32 MFMA steps, K slot j = tap * 8 + channel:
//   * one block per 8 x 32 output tile, 4 waves x (2 rows x 32 columns); the tile's (8+2) x (32+2)
//     input halo (16 B per pixel) is staged in LDS once;
//   * weights = A (16 output channels x K 96, in registers for the block's life), pixels = B: a lane's
//     8 K values of one step are the 8 channels of ONE tap pixel -- one ds_read_b128 -- and a
//     fragment feeds 4 MFMAs (64 output channels);
//   * epilogue as the TN kernels: each lane holds 4 consecutive output channels of one pixel -> one
//     8-B store; BN partials (sum, M2 about the tile mean) of the bf16-rounded outputs per tile.
// The kernel is bound by its output writes (128 B per pixel).
#include "common.h"
#include "conv_fast.h"
#include "fast_util.h"

namespace {

constexpr int F1_TH = 8, F1_TW = 32;            // output tile
constexpr int F1_HP = (F1_TH + 2) * (F1_TW + 2);  // halo pixels (16 B each)

template <bool BIAS, bool RELU, bool STATS>
__global__ __launch_bounds__(256) void first3x3_fwd_kernel(const bf16* x, int ldx, const bf16* wk, const float* bias,
                                                          bf16* y, int ldy, float* stats, int N, int H, int W) {
  __shared__ __attribute__((aligned(16))) uint4 halo[F1_HP];
  __shared__ float red[4][64];
  __shared__ float tot[64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_w = W / F1_TW, tiles_h = H / F1_TH;
  const int b = blockIdx.x;
  const int tw = b % tiles_w, rest = b / tiles_w;
  const int th = rest % tiles_h, n = rest / tiles_h;
  const int h0 = th * F1_TH, w0 = tw * F1_TW;

  // ---- halo -> LDS (pixels outside the image are zero: the conv's padding) ----
  for (int hp = tid; hp < F1_HP; hp += 256) {
    const int hr = hp / (F1_TW + 2), hc = hp - hr * (F1_TW + 2);
    const int h = h0 - 1 + hr, w = w0 - 1 + hc;
    uint4 v = {0u, 0u, 0u, 0u};
    if (h >= 0 && h < H && w >= 0 && w < W) v = *reinterpret_cast<const uint4*>(x + ((long)(n * H + h) * W + w) * ldx);
    halo[hp] = v;
  }

  // ---- A fragments (weights): row k = fc*16 + lane%16; K step ks, slot group kq -> tap 4*ks + kq, its 8
  // channels (16 B of wk [64][9][8]); taps 9..11 of the last step are zero ----
  const int kq = lane >> 4, j16 = lane & 15;
  bf16x8 wa[3][4];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int tap = ks * 4 + kq;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) {
      uint4 v = {0u, 0u, 0u, 0u};
      if (tap < 9) v = *reinterpret_cast<const uint4*>(wk + ((fc * 16 + j16) * 9 + tap) * 8);
      wa[ks][fc] = *reinterpret_cast<const bf16x8*>(&v);
    }
  }
  // halo offset (16-B pixels) of this lane's tap in each K step relative to the output pixel's centre
  int toff[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int tap = ks * 4 + kq;
    toff[ks] = tap < 9 ? (tap / 3 - 1) * (F1_TW + 2) + (tap % 3 - 1) : 0;
  }
  __syncthreads();

  f32x4 acc[4][4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = wid * 2 + (p >> 1), col = (p & 1) * 16 + j16;
    const int centre = (r + 1) * (F1_TW + 2) + col + 1;
#pragma unroll
    for (int fc = 0; fc < 4; ++fc) acc[fc][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      // zero slots (taps 9..11) read the centre pixel: their weights are zero
      const uint4 v = halo[centre + toff[ks]];
      const bf16x8 pb = *reinterpret_cast<const bf16x8*>(&v);
#pragma unroll
      for (int fc = 0; fc < 4; ++fc) acc[fc][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][fc], pb, acc[fc][p], 0, 0, 0);
    }
  }

  // ---- epilogue: lane holds channels fc*16 + 4*kq + e of pixel p*16 + j16 (p -> row / column half) ----
  float csum[4][4];
#pragma unroll
  for (int fc = 0; fc < 4; ++fc) {
    float bv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bv[e] = BIAS ? bias[fc * 16 + kq * 4 + e] : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[fc][e] = 0.f;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      bf16 o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[fc][p][e] + bv[e];
        if (RELU) v = fmaxf(v, 0.f);
        o[e] = (bf16)v;
        acc[fc][p][e] = (float)o[e];  // BN statistics are of the stored (rounded) values
        csum[fc][e] += acc[fc][p][e];
      }
      const int r = wid * 2 + (p >> 1), col = (p & 1) * 16 + j16;
      bf16* dst = y + ((long)(n * H + h0 + r) * W + w0 + col) * ldy + fc * 16 + kq * 4;
      *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(o);
    }
  }
  if constexpr (STATS) {
#pragma unroll
    for (int fc = 0; fc < 4; ++fc)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float s = row16_sum(csum[fc][e]);
        if (j16 == 0) red[wid][fc * 16 + kq * 4 + e] = s;
      }
    __syncthreads();
    if (tid < 64) tot[tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    __syncthreads();
#pragma unroll
    for (int fc = 0; fc < 4; ++fc)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ch = fc * 16 + kq * 4 + e;
        const float mean = tot[ch] * (1.0f / (F1_TH * F1_TW));
        float q = 0.f;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float d = acc[fc][p][e] - mean;
          q += d * d;
        }
        q = row16_sum(q);
        if (j16 == 0) red[wid][ch] = q;  // sums consumed into tot above (barrier between)
      }
    __syncthreads();
    if (tid < 64) {
      stats[(long)b * 128 + tid] = tot[tid];
      stats[(long)b * 128 + 64 + tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    }
  }
}

}  // namespace

// the shape this kernel takes: bf16, an 8-channel input alone (x2 == NULL; any values), 64 outputs, 3x3,
// stride 1, pad 1, H % 8 == 0, W % 32 == 0, dense 64-channel output rows or wider
bool first3x3_ok(int dtype, int c1, int ldc1, int c2, int n, int h, int w, int cout, int r, int s, int stride, int pad,
                 int ldy) {
  static const bool off = getenv("UNETSEG_NO_FIRST3x3") != nullptr;
  return !off && dtype == DT_BF16 && c1 == 8 && ldc1 == 8 && c2 == 0 && cout == 64 && r == 3 && s == 3 &&
         stride == 1 && pad == 1 && n > 0 && h % F1_TH == 0 && w % F1_TW == 0 && ldy >= 64 && ldy % 4 == 0 &&
         (long)n * h * w < (1L << 31) / 64;
}

int first3x3_tile_m() { return F1_TH * F1_TW; }

int launch_first3x3(const void* x, int ldx, const void* wk, const float* bias, int relu, void* y, int ldy, float* stats,
                    int n, int h, int w, hipStream_t st) {
  const unsigned blocks = (unsigned)(n * (h / F1_TH) * (w / F1_TW));
  if (blocks == 0) return 0;
#define F1_LAUNCH(B, R, S)                                                                                          \
  hipLaunchKernelGGL((first3x3_fwd_kernel<B, R, S>), dim3(blocks), dim3(256), 0, st, (const bf16*)x, ldx,        \
                     (const bf16*)wk, bias, (bf16*)y, ldy, stats, n, h, w)
  const bool b = bias != nullptr, s = stats != nullptr;
  if (b && relu) { if (s) F1_LAUNCH(true, true, true); else F1_LAUNCH(true, true, false); }
  else if (b) { if (s) F1_LAUNCH(true, false, true); else F1_LAUNCH(true, false, false); }
  else if (relu) { if (s) F1_LAUNCH(false, true, true); else F1_LAUNCH(false, true, false); }
  else { if (s) F1_LAUNCH(false, false, true); else F1_LAUNCH(false, false, false); }
#undef F1_LAUNCH
  return 0;
}
