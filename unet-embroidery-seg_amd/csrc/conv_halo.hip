// 3x3 stride-1 "same" convolutions with 64 input channels (fwd and stride-1 dgrad), bf16, gfx950.
//
// These are the high-resolution, narrow layers of the U-Net decoder (up_conv at 512^2, up_concat1 at
// 256^2) and of ResNet layer1 at 128^2.  The generic implicit GEMM re-reads every input pixel once
// per tap (9x) through L2 and restages the weights per 256-pixel tile; here:
//  * weights stay resident: one block owns one 64-channel output tile for its whole life and keeps
//    all 9 taps x 64 x 64 bf16 (72 KiB) in LDS;
//  * the input arrives as a 2D halo tile: (TH+2) x 34 pixels x 64 channels (42.5 KiB) serve a
//    TH x 32 output tile for all 9 taps (1.33 reads per pixel instead of 9);
//  * persistent blocks (one per CU) walk spatial tiles; the next tile's halo streams in by
//    LDS-DMA (buffer_load ... lds) while the current one is computed -- two halo stages;
//  * within a tile there is no barrier: 9 taps x 2 K-halves of MFMA straight from LDS;
//  * output stores are explicit buffer stores so the per-wave count of memory operations after the
//    next tile's DMA is a compile-time constant: the wait for that DMA is `vmcnt(FP*FC)` and never
//    waits on this tile's stores.
// Operand roles as in the TN kernels: weights = A (16 output channels per MFMA row block),
// pixels = B, so each lane's accumulator holds 4 consecutive output channels of one pixel.
#include <cstdlib>

#include "common.h"
#include "conv_fast.h"
#include "fast_util.h"

// halo3: order of the next tile's halo DMA (see halo3_kernel; 2 = one piece per tap step from step 0)
#ifndef UNETSEG_HALO3_SPREAD
#define UNETSEG_HALO3_SPREAD 2
#endif

namespace {

constexpr int HW_TW = 32;  // output tile width (pixels)

// Halo pixel rows are read 16 at a time from an arbitrary start (the tap shift); XOR the chunk
// with hp & 7 (not (hp>>1) & 7 as for aligned rows): conflict-free ds_read_b128 for every start.
__device__ __forceinline__ int swzh(int hp, int ch) { return ch ^ (hp & 7); }


// EPI: epilogue flags fixed at compile time (kEpiBias | kEpiRelu | kEpiStats | kEpiAcc), or kEpiDyn
// to read them from the arguments; with them fixed the tile epilogue has no uniform branches and
// the bias sits in registers.
// kEpiHead1 / kEpiHead2: the model's final 1x1 conv (64 -> 1 or 2 logits) on the rounded outputs
// (model/unet_resnet.py:99-103 `final`, model/unet_multitask.py seg_head): the 512^2 activation is
// not read back by a separate head pass.
// kEpiMask: the ReLU mask of the stored output packed to bits, mbits_out[pixel][Ng/8] (bit e of byte b =
// channel 8b + e > 0) -- the consumer's data gradient (post 4) reads 1/16 of what the activation costs.
constexpr int kEpiBias = 1, kEpiRelu = 2, kEpiStats = 4, kEpiAcc = 8, kEpiDyn = 16, kEpiHead1 = 32, kEpiHead2 = 64,
              kEpiMask = 128;


// wait for half h of the HS pipeline and join the block: the vector-memory operations issued after
// half h's DMA may stay in flight -- the next two halves (D instructions each) and the aux loads (NA)
// / output stores (NS) issued in between (exact for the first three halves, whose predecessors are
// fewer).  A count below the true one only waits longer.
template <int D, int NA, int NS>
__device__ __forceinline__ void hs_wait(int h) {
  if (h == 0)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D) : "memory");
  else if (h == 1)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D + NA) : "memory");
  else if (h == 2)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D + NA + NS) : "memory");
  else if (h & 1)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D + 2 * NA + NS) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D + NA + 2 * NS) : "memory");
}

// HS: the input arrives as 32-channel half tiles through FOUR half stages (the same 85 KiB as two
// whole-tile stages): a half tile's DMA is issued three half-steps before it is consumed, so 64 KiB
// stay in flight per CU instead of the 0-43 KiB of the double-buffered whole tiles, whose wait at
// every tile end left the waves parked (the 512^2 layers ran at ~2.7 TB/s).  Half-stage rows are
// 64 B (4 chunks, chunk ^ (bit 2 of the pixel) << 1: conflict-free 16-pixel reads from any start).
template <int TH, int NW, int POST, int EPI, bool HS = false>
__global__ __launch_bounds__(64 * NW) void halo3_kernel(FastTNArgs a, int tiles_w, int tiles_h, int n_sp, int G_per,
                                                        unsigned y_bytes) {
  constexpr bool kDyn = (EPI & kEpiDyn) != 0;
  const bool has_bias = kDyn ? a.bias != nullptr : (EPI & kEpiBias) != 0;
  const bool do_relu = kDyn ? a.relu != 0 : (EPI & kEpiRelu) != 0;
  const bool do_stats = kDyn ? a.stats != nullptr : (EPI & kEpiStats) != 0;
  const bool do_acc = kDyn ? a.accumulate != 0 : (EPI & kEpiAcc) != 0;
  constexpr int HK = (EPI & kEpiHead2) ? 2 : (EPI & kEpiHead1) ? 1 : 0;  // fused head logits
  static_assert(HK == 0 || (!kDyn && POST == 0), "the fused head rides on a fixed bias + ReLU epilogue");
  constexpr bool kMask = (EPI & kEpiMask) != 0;
  static_assert(!kMask || (!kDyn && POST == 0 && HK == 0 && (EPI & kEpiRelu)), "mask bits of a ReLU output");
  // POST 4: post 1 with the ReLU mask read from packed bits (a.mbits, the kEpiMask layout)
  // wave w owns output rows [w*TH/NW, (w+1)*TH/NW)
  constexpr int RPW = TH / NW;               // rows per wave
  constexpr int FP = RPW * (HW_TW / 16);     // 16-pixel groups per wave
  constexpr int FC = 4;                      // 16-channel output groups (64 output channels)
  constexpr int HP = (TH + 2) * (HW_TW + 2); // halo pixels
  constexpr int HCH = HP * 8;                // 16-B chunks per halo stage
  constexpr int HI = (HCH + 64 * NW - 1) / (64 * NW);  // halo DMA instructions per wave
  constexpr int WCH = 9 * 64 * 8;            // 16-B chunks of resident weights
  constexpr int WI = WCH / (64 * NW);        // weight DMA instructions per wave
  static_assert(TH % NW == 0 && WCH % (64 * NW) == 0, "tile shape");
  // the spread halo DMA issues piece i at tap step i (mode 2) or 2 i + 1 (mode 1) of the 18-step loop:
  // every piece must land on a step that exists, or the next tile would read a partly loaded halo
  static_assert(HI <= 18 && (HI <= 9 || UNETSEG_HALO3_SPREAD != 1), "halo pieces exceed the tap steps");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  uint4* wl = lds;                           // [9*64 rows][8 chunks]
  uint4* hl = lds + WCH;                     // [2][HP][8]
  float* red = reinterpret_cast<float*>(hl + 2 * HCH);  // [NW][64]
  float* sbias = red + NW * 64;              // [64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = a.Ng >> 6;
  // block -> (output-channel tile, first spatial tile); spatial tiles dealt round-robin
  const int tn = blockIdx.x / G_per, slot = blockIdx.x % G_per;
  const int n0 = tn * 64;
  const int my_tiles = slot < n_sp ? (n_sp - slot + G_per - 1) / G_per : 0;
  const __amdgpu_buffer_rsrc_t rx = srd(a.x1, a.x1_bytes);
  const __amdgpu_buffer_rsrc_t rw = srd(a.wt, a.w_bytes);
  const __amdgpu_buffer_rsrc_t ry = srd(a.y, y_bytes);
  (void)ntn;
  const unsigned hw_img = (unsigned)(a.OH * a.OW);
  const __amdgpu_buffer_rsrc_t rh = srd(HK ? (const void*)a.head_y : a.y,
                                        HK ? (unsigned)(a.M / (a.OH * a.OW)) * HK * hw_img * 4u : 0u);
  const __amdgpu_buffer_rsrc_t rmb =
      srd(kMask ? (const void*)a.mbits_out : a.y, kMask ? (unsigned)a.M * (unsigned)(a.Ng >> 3) : 0u);
  const __amdgpu_buffer_rsrc_t rst =
      srd(do_stats ? (const void*)a.stats : a.y, do_stats ? (unsigned)n_sp * 2u * (unsigned)a.Ng * 4u : 0u);
  // post-op inputs: POST 4 the mask bits [M][Ng/8], POST 1 / 2 the pre-activation aux [M][ld_aux]
  const __amdgpu_buffer_rsrc_t raux =
      POST == 4 ? srd(a.mbits, (unsigned)a.M * (unsigned)(a.Ng >> 3))
                : srd(POST ? a.aux : a.y, POST ? (unsigned)a.M * (unsigned)a.ld_aux * 2u : 0u);

  if (kDyn && a.bias && tid < 64) sbias[tid] = a.bias[n0 + tid];
  // BN post-op coefficients of this block's 64 channels live in `red` (free in dgrad: no stats)
  float* pco = red;  // [4][64]: sc, sh, mean, inv
  if (POST == 2 && tid < 64) {
    pco[tid] = a.psc[n0 + tid];
    pco[64 + tid] = a.psh[n0 + tid];
    pco[128 + tid] = a.pmean[n0 + tid];
    pco[192 + tid] = a.pinv[n0 + tid];
  }

  // ---- resident weights: LDS row (jt, k) = weights of output channel n0+k at halo tap jt ----
  {
    const unsigned base = lds_addr(wl);
#pragma unroll 2
    for (int i = 0; i < WI; ++i) {
      const int inst = i * NW + wid;
      const int idx = inst * 64 + lane;
      const int row = idx >> 3, pc = idx & 7;
      const int jt = row >> 6, k = row & 63;
      const int jr = jt / 3, js = jt - jr * 3;
      const int wtap = (a.r0 + a.rs * jr) * a.S + (a.s0 + a.ss * js);
      const unsigned off = (unsigned)(n0 + k) * (unsigned)a.ldwb + (unsigned)(wtap * 128 + swz8(row, pc) * 16);
      dma16(rw, base + (unsigned)inst * 1024u, off);
    }
  }

  // ---- halo geometry of this lane's DMA slots (identical for every tile): byte offset relative to
  // the halo's top-left pixel (swizzle included) and which border of the halo the pixel lies on --
  // with hc % TH == 0 and wc % 32 == 0 only border pixels can leave the image, so a tile's load is
  // one add and one mask test per row ----
  unsigned hoff[HI], hflag[HI];
#pragma unroll
  for (int i = 0; i < HI; ++i) {
    const int idx = (i * NW + wid) * 64 + lane;
    const int hp = idx >> 3, hr = hp / (HW_TW + 2), hc = hp % (HW_TW + 2);
    hoff[i] = (unsigned)(hr * a.W + hc) * (unsigned)a.ldc1b + swzh(hp, lane & 7) * 16u;
    hflag[i] = idx >= HCH ? 16u : (hr == 0 ? 1u : 0u) | (hr == TH + 1 ? 2u : 0u) | (hc == 0 ? 4u : 0u) | (hc == HW_TW + 1 ? 8u : 0u);
  }
  // halo DMA instructions this wave issues per tile: HI, or HI - 1 for the waves with no slot in the
  // last one (issue_halo skips it)
  const bool full_dma = HCH % (64 * NW) == 0 || ((HI - 1) * NW + wid) * 64 < HCH;
  auto issue_halo = [&](int t, int stage) {
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    const int h0 = th * TH, w0 = tw * HW_TW;
    const unsigned base = __builtin_amdgcn_readfirstlane(lds_addr(hl + stage * HCH));
    // origin (h0 - 1, w0 - 1) wraps below zero on the first row / column; the edge mask sends
    // those lanes out of range
    const unsigned hb = __builtin_amdgcn_readfirstlane((unsigned)((nb * a.H + h0 - 1) * a.W + w0 - 1) * (unsigned)a.ldc1b);
    const unsigned kill = __builtin_amdgcn_readfirstlane(16u | (h0 == 0 ? 1u : 0u) | (h0 + TH >= a.H ? 2u : 0u) |
                                                         (w0 == 0 ? 4u : 0u) | (w0 + HW_TW >= a.W ? 8u : 0u));
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const unsigned off = (hflag[i] & kill) ? kOOB : hb + hoff[i];
      // only the last row can hold lanes past the halo (they must not write LDS)
      if (i < HI - 1 || HCH % (64 * NW) == 0 || hflag[i] != 16u) dma16(rx, base + (unsigned)((i * NW + wid) * 1024), off);
    }
  };

  // ---- half-stage geometry (HS): 4 chunks per halo pixel, HI2 DMA instructions per wave (the last
  // one only for the waves whose slots exist: waves 0..5 issue HI2, the rest HI2 - 1) ----
  constexpr int HCH2 = HP * 4;
  constexpr int HI2 = (HCH2 + 64 * NW - 1) / (64 * NW);
  constexpr int LASTW = (HCH2 - (HI2 - 1) * 64 * NW + 63) / 64;  // waves with slots in the last instruction
  static_assert(!HS || (HCH2 % 64 != 0 || true), "");
  unsigned hoff2[HS ? HI2 : 1], hflag2[HS ? HI2 : 1];
  if constexpr (HS) {
#pragma unroll
    for (int i = 0; i < HI2; ++i) {
      const int idx = (i * NW + wid) * 64 + lane;
      const int hp = idx >> 2, q = idx & 3;
      const int hr = hp / (HW_TW + 2), hc = hp % (HW_TW + 2);
      hoff2[i] = (unsigned)(hr * a.W + hc) * (unsigned)a.ldc1b + (unsigned)((q ^ (((hp >> 2) & 1) << 1)) * 16);
      hflag2[i] = idx >= HCH2 ? 16u : (hr == 0 ? 1u : 0u) | (hr == TH + 1 ? 2u : 0u) | (hc == 0 ? 4u : 0u) | (hc == HW_TW + 1 ? 8u : 0u);
    }
  }
  const bool last_dma = wid < LASTW;  // this wave issues the last half-stage instruction
  // half h = 2 t + kk (input channels 32 kk .. 32 kk + 31 of tile t) into half stage `stage`; halves
  // past this block's tiles load nothing (out of range) but are issued, so every wave's count is fixed
  auto issue_half = [&](int h, int stage) {
    const int t = h >> 1;
    const bool live = t < my_tiles;
    const int sp = live ? slot + t * G_per : slot;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    const int h0 = th * TH, w0 = tw * HW_TW;
    const unsigned base = __builtin_amdgcn_readfirstlane(lds_addr(hl + stage * HCH2));
    const unsigned hb = __builtin_amdgcn_readfirstlane((unsigned)((nb * a.H + h0 - 1) * a.W + w0 - 1) * (unsigned)a.ldc1b +
                                                       (unsigned)(h & 1) * 64u);
    const unsigned kill = __builtin_amdgcn_readfirstlane(16u | (h0 == 0 ? 1u : 0u) | (h0 + TH >= a.H ? 2u : 0u) |
                                                         (w0 == 0 ? 4u : 0u) | (w0 + HW_TW >= a.W ? 8u : 0u));
#pragma unroll
    for (int i = 0; i < HI2; ++i) {
      const unsigned off = (!live || (hflag2[i] & kill)) ? kOOB : hb + hoff2[i];
      if (i < HI2 - 1) {
        dma16(rx, base + (unsigned)((i * NW + wid) * 1024), off);
      } else if (last_dma) {
        if (hflag2[i] != 16u) dma16(rx, base + (unsigned)((i * NW + wid) * 1024), off);
      }
    }
  };

  f32x4 acc[FC][FP];
  // data-gradient post-op (a.post): running per-lane sums of the masked gradient over all tiles of
  // this block, reduced once at the end into ppart[blockIdx.x][2][Ng]
  float pq0[FC][4], pq1[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) pq0[c][e] = pq1[c][e] = 0.f;
  // per-wave vector-memory operations of one tile's epilogue, counted from the loops that issue them
  // (each issues its full count on every wave: inactive lanes go out of range, nothing is skipped):
  //   aux loads (post op): POST 4 one 8-B mask load per 16-pixel group, POST 1/2 one per (group, channel
  //   group); stores: FP x FC outputs, FP x HK head logits, FP mask words
  constexpr int NA_ = POST == 4 ? FP : POST ? FP * FC : 0;
  constexpr int NS_ = FP * FC + FP * HK + (kMask ? FP : 0);
  // (operations issued beyond these -- the accumulate epilogue's old-value loads -- only make a wait
  // wait longer; a count above the true one would not wait for the DMA)
  static_assert(!HS || 2 * HI2 + 2 * NA_ + 2 * NS_ <= 63, "hs_wait counts must fit vmcnt's 6 bits");
  auto half_wait = [&](int h) {
    if (last_dma) hs_wait<HI2, NA_, NS_>(h);
    else hs_wait<HI2 - 1, NA_, NS_>(h);
  };
  if constexpr (HS) {
    issue_half(0, 0);
    issue_half(1, 1);
    issue_half(2, 2);
  } else {
    if (my_tiles > 0) issue_halo(0, 0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }

  // halo tap offsets (uniform): jt -> (dh, dw)
  const int dh0 = a.dh0, dhs = a.dhs, dw0 = a.dw0, dws = a.dws;
  const int j16 = lane & 15, kg = lane >> 4;
  // fused head: this lane's 16 channels' head weights in registers (one block per CU: VGPRs are free)
  float hwr[HK > 0 ? HK : 1][FC][4], hbr[HK > 0 ? HK : 1];
#pragma unroll
  for (int k = 0; k < HK; ++k) {
    hbr[k] = a.head_b[k];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) hwr[k][c][e] = a.head_w[k * 64 + c * 16 + kg * 4 + e];
  }
  float breg[FC][4];  // this lane's 16 output channels' bias (compile-time flags only)
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) breg[c][e] = (!kDyn && has_bias) ? a.bias[n0 + c * 16 + kg * 4 + e] : 0.f;

  for (int t = 0; t < my_tiles; ++t) {
    const int stage = t & 1;
    if constexpr (HS) {
      half_wait(2 * t);
      issue_half(2 * t + 3, (2 * t + 3) & 3);
    }
    // post-op: this tile's aux values are loaded now, so their latency hides under the tap loop
    uint2 zr[FC][FP];
    uint2 zb[FP];  // POST 4: the 8 mask bytes (64 channels) of this lane's pixel
    if (!HS && POST) {
      // double buffer: the aux loads go out BEFORE the next tile's DMA, as buffer loads the compiler
      // does not track, and the epilogue waits for them with vmcnt(this wave's DMA count): waiting on
      // loads issued after the DMA (in-order counter) retired the next tile's halo inside this tile --
      // the prefetch was gone (16 x 512^2 post 4: 397 us against 281 for the plain data gradient)
      const int sp = slot + t * G_per;
      const int tw = sp % tiles_w, rest = sp / tiles_w;
      const int th = rest % tiles_h, nb = rest / tiles_h;
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int r = wid * RPW + p / (HW_TW / 16);
        const int col = (p % (HW_TW / 16)) * 16 + j16;
        const unsigned opix = (unsigned)((nb * a.OH + th * TH + r) * a.OW + tw * HW_TW + col);
        if (POST == 4) {
          zb[p] = bload64_asm(raux, opix * (unsigned)(a.Ng >> 3) + (unsigned)(n0 >> 3));
        } else {
#pragma unroll
          for (int c = 0; c < FC; ++c)
            zr[c][p] = bload64_asm(raux, (opix * (unsigned)a.ld_aux + (unsigned)(n0 + c * 16 + kg * 4)) * 2u);
        }
      }
    }
    // the next tile's halo DMA, one instruction per tap step at the first HI steps of the MFMA
    // loop below (UNETSEG_HALO3_SPREAD=2, default): issued all at once here, the eight waves spent
    // their issue cycles together at the tile start with the MFMA pipes idle (16 x 512^2 fwd
    // 313 -> 302-309 us, dgrad 311 -> 307-309; -DUNETSEG_HALO3_SPREAD=0 builds the old order).
    // Mode 1 (every other step from step 1) left the last piece fewer steps to land before the
    // tile-end wait: mode 2 measured fwd 311 -> 302 us, fwd + statistics 448 -> 433 us
    const bool dma_next = t + 1 < my_tiles;
    unsigned nx_base = 0u, nx_hb = 0u, nx_kill = 0u;
    if constexpr (!HS) {
      if (!UNETSEG_HALO3_SPREAD) {
        if (dma_next) issue_halo(t + 1, stage ^ 1);
      } else if (dma_next) {
        const int sp = slot + (t + 1) * G_per;
        const int tw = sp % tiles_w, rest = sp / tiles_w;
        const int th = rest % tiles_h, nb = rest / tiles_h;
        const int h0 = th * TH, w0 = tw * HW_TW;
        nx_base = __builtin_amdgcn_readfirstlane(lds_addr(hl + (stage ^ 1) * HCH));
        nx_hb = __builtin_amdgcn_readfirstlane((unsigned)((nb * a.H + h0 - 1) * a.W + w0 - 1) * (unsigned)a.ldc1b);
        nx_kill = __builtin_amdgcn_readfirstlane(16u | (h0 == 0 ? 1u : 0u) | (h0 + TH >= a.H ? 2u : 0u) |
                                                 (w0 == 0 ? 4u : 0u) | (w0 + HW_TW >= a.W ? 8u : 0u));
      }
    }
    auto issue_piece = [&](int i) {
      if (!UNETSEG_HALO3_SPREAD || !dma_next) return;
      const unsigned off = (hflag[i] & nx_kill) ? kOOB : nx_hb + hoff[i];
      if (i < HI - 1 || HCH % (64 * NW) == 0 || hflag[i] != 16u) dma16(rx, nx_base + (unsigned)((i * NW + wid) * 1024), off);
    };
    if (HS && POST == 4) {
      const int sp = slot + t * G_per;
      const int tw = sp % tiles_w, rest = sp / tiles_w;
      const int th = rest % tiles_h, nb = rest / tiles_h;
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int r = wid * RPW + p / (HW_TW / 16);
        const int col = (p % (HW_TW / 16)) * 16 + j16;
        const long opix = ((long)nb * a.OH + th * TH + r) * a.OW + tw * HW_TW + col;
        zb[p] = *reinterpret_cast<const uint2*>(a.mbits + opix * (a.Ng >> 3) + (n0 >> 3));
      }
    } else if (HS && POST) {
      const int sp = slot + t * G_per;
      const int tw = sp % tiles_w, rest = sp / tiles_w;
      const int th = rest % tiles_h, nb = rest / tiles_h;
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int r = wid * RPW + p / (HW_TW / 16);
        const int col = (p % (HW_TW / 16)) * 16 + j16;
        const long opix = ((long)nb * a.OH + th * TH + r) * a.OW + tw * HW_TW + col;
#pragma unroll
        for (int c = 0; c < FC; ++c)
          zr[c][p] = *reinterpret_cast<const uint2*>((const bf16*)a.aux + opix * a.ld_aux + n0 + c * 16 + kg * 4);
      }
    }
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (HS) {
      // half kk = input channels 32 kk .. 32 kk + 31: all nine taps, then the next half
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (kk == 1) {
          half_wait(2 * t + 1);
          issue_half(2 * t + 4, (2 * t + 4) & 3);
        }
        const uint4* hs2 = hl + ((2 * t + kk) & 3) * HCH2;
        const int ch = kk * 4 + kg;
#pragma unroll
        for (int jt = 0; jt < 9; ++jt) {
          const int jr = jt / 3, js = jt - jr * 3;
          const int dh = dh0 + dhs * jr, dw = dw0 + dws * js;
          bf16x8 wf[FC], pf[FP];
#pragma unroll
          for (int c = 0; c < FC; ++c) {
            const int row = jt * 64 + c * 16 + j16;
            uint4 v = wl[row * 8 + swz8(row, ch)];
            wf[c] = *reinterpret_cast<bf16x8*>(&v);
          }
#pragma unroll
          for (int p = 0; p < FP; ++p) {
            const int r = wid * RPW + p / (HW_TW / 16);
            const int col = (p % (HW_TW / 16)) * 16 + j16;
            const int hp = (r + 1 + dh) * (HW_TW + 2) + col + 1 + dw;
            uint4 v = hs2[hp * 4 + (kg ^ (((hp >> 2) & 1) << 1))];
            pf[p] = *reinterpret_cast<bf16x8*>(&v);
          }
#pragma unroll
          for (int c = 0; c < FC; ++c)
#pragma unroll
            for (int p = 0; p < FP; ++p)
              acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], pf[p], acc[c][p], 0, 0, 0);
        }
      }
    } else {
      // 18 steps (tap jt, K half kk), software-pipelined: the fragments of step s+1 are read before
      // the MFMAs of step s and sched_group_barrier pins that order -- left to itself the scheduler
      // issued each read right before its MFMAs, and with 2 MFMAs per LDS round trip the waves sat on
      // lgkmcnt (MFMA busy 45 %, SQ_LDS_IDX_ACTIVE 34 % at 512^2)
      const uint4* hs = hl + stage * HCH;
      auto frag_load = [&](int st, bf16x8 (&wf)[FC], bf16x8 (&pf)[FP]) {
        const int jt = st >> 1, kk = st & 1;
        const int jr = jt / 3, js = jt - jr * 3;
        const int dh = dh0 + dhs * jr, dw = dw0 + dws * js;
        const int ch = kk * 4 + kg;
#pragma unroll
        for (int c = 0; c < FC; ++c) {
          const int row = jt * 64 + c * 16 + j16;
          uint4 v = wl[row * 8 + swz8(row, ch)];
          wf[c] = *reinterpret_cast<bf16x8*>(&v);
        }
#pragma unroll
        for (int p = 0; p < FP; ++p) {
          const int r = wid * RPW + p / (HW_TW / 16);
          const int col = (p % (HW_TW / 16)) * 16 + j16;
          const int hp = (r + 1 + dh) * (HW_TW + 2) + col + 1 + dw;
          uint4 v = hs[hp * 8 + swzh(hp, ch)];
          pf[p] = *reinterpret_cast<bf16x8*>(&v);
        }
      };
      bf16x8 wfb[2][FC], pfb[2][FP];
      frag_load(0, wfb[0], pfb[0]);
      __builtin_amdgcn_sched_group_barrier(0x100, FC + FP, 0);
#pragma unroll
      for (int st = 0; st < 18; ++st) {
        if (st + 1 < 18) frag_load(st + 1, wfb[(st + 1) & 1], pfb[(st + 1) & 1]);
#pragma unroll
        for (int c = 0; c < FC; ++c)
#pragma unroll
          for (int p = 0; p < FP; ++p)
            acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfb[st & 1][c], pfb[st & 1][p], acc[c][p], 0, 0, 0);
#if UNETSEG_HALO3_INTERLEAVE
        // reads of step s+1 spread between the MFMAs of step s
        if (st + 1 < 18) {
#pragma unroll
          for (int i = 0; i < FC + FP; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          }
          __builtin_amdgcn_sched_group_barrier(0x008, FC * FP - (FC + FP), 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, FC * FP, 0);
        }
#else
        if (st + 1 < 18) __builtin_amdgcn_sched_group_barrier(0x100, FC + FP, 0);  // DS reads of step st+1
        __builtin_amdgcn_sched_group_barrier(0x008, FC * FP, 0);                    // MFMAs of step st
#endif
        // UNETSEG_HALO3_SPREAD 1: pieces at steps 1, 3, .. 2 HI - 1; 2: at steps 0 .. HI - 1
        if (UNETSEG_HALO3_SPREAD == 2 ? st < HI : ((st & 1) && (st >> 1) < HI))
          issue_piece(UNETSEG_HALO3_SPREAD == 2 ? st : st >> 1);
      }
    }

    // ================= epilogue =================
    if (!HS && POST) {
      // this tile's aux loads landed; the next tile's halo (this wave's DMAs, issued after them) may fly
      if (t + 1 < my_tiles) {
        if (full_dma)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HI) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HI - 1) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        if (POST == 4) {
          asm volatile("" : "+v"(zb[p]));
        } else {
#pragma unroll
          for (int c = 0; c < FC; ++c) asm volatile("" : "+v"(zr[c][p]));
        }
      }
    }
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    float csum[FC][4];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[c][e] = 0.f;
    uint2 outv[FC][FP];
    unsigned outo[FP], mko[FP], mkx[FP], mky[FP];
#pragma unroll
    for (int p = 0; p < FP; ++p) {
      const int r = wid * RPW + p / (HW_TW / 16);
      const int col = (p % (HW_TW / 16)) * 16 + j16;
      const long opix = ((long)nb * a.OH + th * TH + r) * a.OW + tw * HW_TW + col;
      outo[p] = (unsigned)(opix * a.ldy + n0) * 2u;
      mko[p] = (unsigned)(opix * (a.Ng >> 3) + (n0 >> 3));
      mkx[p] = mky[p] = 0u;
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int cb = c * 16 + kg * 4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[c][p][e] + (!has_bias ? 0.f : kDyn ? sbias[cb + e] : breg[c][e]);
          if (do_relu) v[e] = fmaxf(v[e], 0.f);
        }
        if (do_acc) {
          const bf16* ob = reinterpret_cast<const bf16*>((const char*)a.y + outo[p] + cb * 2);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)ob[e];
        }
        bf16 o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = (bf16)v[e];
          v[e] = (float)o[e];
        }
        if (POST) {  // mask with the producer's ReLU (from aux or its bits) and accumulate backward partials
          const bf16* z = reinterpret_cast<const bf16*>(&zr[c][p]);
          // POST 4: byte 2c + kg/2 of the pixel's 8, high nibble for odd kg
          const unsigned nib =
              POST == 4 ? ((c < 2 ? zb[p].x : zb[p].y) >> ((((2 * c + (kg >> 1)) & 3) * 8) + (kg & 1) * 4)) & 15u : 0u;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float zf = POST == 4 ? 0.f : (float)z[e];
            bool on = POST == 4 ? ((nib >> e) & 1u) != 0u : zf > 0.f;
            float xh = 0.f;
            if (POST == 2) {
              const int ch = cb + e;
              on = fmaf(zf, pco[ch], pco[64 + ch]) > 0.f;
              xh = (zf - pco[128 + ch]) * pco[192 + ch];
            }
            v[e] = on ? v[e] : 0.f;
            o[e] = (bf16)v[e];
            pq0[c][e] += v[e];
            if (POST == 2) pq1[c][e] += v[e] * xh;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          csum[c][e] += v[e];
          acc[c][p][e] = v[e];
        }
        outv[c][p] = *reinterpret_cast<uint2*>(o);
        if (kMask) {  // this lane's 4 channels -> its nibble of byte 2c + kg/2 (word x: c < 2, y: c >= 2)
          unsigned nb4 = 0u;
#pragma unroll
          for (int e = 0; e < 4; ++e) nb4 |= (v[e] > 0.f ? 1u : 0u) << e;
          const unsigned sh = (((2 * c + (kg >> 1)) & 3) * 8) + (kg & 1) * 4;
          if (c < 2) mkx[p] |= nb4 << sh;
          else mky[p] |= nb4 << sh;
        }
      }
    }
    if (kMask) {  // OR the four channel groups' nibbles (lanes j16 + 16 kg): disjoint bits
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        mkx[p] |= __shfl_xor(mkx[p], 16);
        mkx[p] |= __shfl_xor(mkx[p], 32);
        mky[p] |= __shfl_xor(mky[p], 16);
        mky[p] |= __shfl_xor(mky[p], 32);
      }
    }
    if (HK) {
      // head logits of this lane's pixels: 16 channels per lane, then the four channel groups
      // (lanes j16 + 16 kg) summed by cross-row shuffles; lanes kg == 0 store, the others' stores
      // go out of range (every wave issues exactly FP * HK head stores)
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int r = wid * RPW + p / (HW_TW / 16);
        const int col = (p % (HW_TW / 16)) * 16 + j16;
        const unsigned pix = (unsigned)((th * TH + r) * a.OW + tw * HW_TW + col);
#pragma unroll
        for (int k = 0; k < HK; ++k) {
          float hs = 0.f;
#pragma unroll
          for (int c = 0; c < FC; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) hs = fmaf(acc[c][p][e], hwr[k][c][e], hs);
          hs += __shfl_xor(hs, 16);
          hs += __shfl_xor(hs, 32);
          hs += hbr[k];
          bstore32(rh, kg == 0 ? ((unsigned)(nb * HK + k) * hw_img + pix) * 4u : kOOB, hs);
        }
      }
    }
    if (do_stats) {
      // per-tile BN partials over the TH*32 pixels (sum, M2 about the tile mean): each wave reduces its
      // own 16 * FP pixels to (sum, M2 about the wave mean) in registers -- the 16 channel values of a
      // lane reduced together over the row's 16 lanes (row16_sum_n) -- and wave 0 merges the NW waves
      // (Chan: M2 = sum M2_w + n_w (mean_w - mean)^2), the sums and then the M2s passing through `red`
      // (no room in LDS for both at once).  Until round 5 every lane fetched the tile mean of its 16
      // channels from LDS and the 32 row reductions ran one chain at a time: the statistics epilogue
      // cost almost half as much as the convolution (16 x 512^2: 475 vs 325 us)
      float sv[FC * 4], qv[FC * 4];
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) sv[c * 4 + e] = csum[c][e];
      row16_sum_n(sv);
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float mw = sv[c * 4 + e] * (1.0f / (16 * FP));
          float q = 0.f;
#pragma unroll
          for (int p = 0; p < FP; ++p) {
            const float d = acc[c][p][e] - mw;
            q += d * d;
          }
          qv[c * 4 + e] = q;
        }
      row16_sum_n(qv);
      if (j16 == 0)
#pragma unroll
        for (int c = 0; c < FC; ++c)
          *reinterpret_cast<float4*>(red + wid * 64 + c * 16 + kg * 4) =
              float4{sv[c * 4], sv[c * 4 + 1], sv[c * 4 + 2], sv[c * 4 + 3]};
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      float sw[NW];
      if (tid < 64)
#pragma unroll
        for (int w = 0; w < NW; ++w) sw[w] = red[w * 64 + tid];
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // sums read: reuse red for M2
      if (j16 == 0)
#pragma unroll
        for (int c = 0; c < FC; ++c)
          *reinterpret_cast<float4*>(red + wid * 64 + c * 16 + kg * 4) =
              float4{qv[c * 4], qv[c * 4 + 1], qv[c * 4 + 2], qv[c * 4 + 3]};
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      float tot = 0.f, q = 0.f;
      if (tid < 64) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          tot += sw[w];
          q += red[w * 64 + tid];
        }
        const float mean = tot * (1.0f / (TH * HW_TW));
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const float d = sw[w] * (1.0f / (16 * FP)) - mean;
          q = fmaf((float)(16 * FP) * d, d, q);
        }
      }
      // buffer stores issued by every wave (only wave 0's land), counted in the tile's closing wait:
      // as plain stores of wave 0 alone they were retired by that wait -- a full write round trip per
      // tile with the whole block parked on the barrier behind it (16 x 512^2: +140 us)
      const unsigned so = tid < 64 ? (unsigned)(sp * 2 * a.Ng + n0 + tid) * 4u : kOOB;
      bstore32(rst, so, tot);
      bstore32(rst, tid < 64 ? so + (unsigned)a.Ng * 4u : kOOB, q);
    }
    // output stores last: exactly FP*FC buffer stores per wave after the next tile's DMA
#pragma unroll
    for (int p = 0; p < FP; ++p)
#pragma unroll
      for (int c = 0; c < FC; ++c) bstore64(ry, outo[p] + (c * 16 + kg * 4) * 2, outv[c][p]);
    // mask bytes: lanes kg == 0 store the pixel's 8 bytes, the others' stores go out of range (every
    // wave issues exactly FP of them)
    if (kMask)
#pragma unroll
      for (int p = 0; p < FP; ++p) bstore64(rmb, kg == 0 ? mko[p] : kOOB, uint2{mkx[p], mky[p]});
    // next halo landed (all but this tile's stores retired) and every wave is done with both the
    // current stage (WAR for the DMA after next) and `red` (HS: the next half's wait does both)
    // (HS: the two statistics stores are not in hs_wait's counts -- it waits for them too, which is
    // only slower)
    if constexpr (!HS) {
      if (do_stats)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NS_ + 2) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NS_) : "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // HS: the past-the-end halves are still landing in the stages of other waves
  if constexpr (HS) asm volatile("s_barrier" ::: "memory");
  if (POST) {
    // lanes -> waves -> block: ppart[blockIdx.x][2][Ng] for this block's 64 output channels (the
    // halo stages are free now: every wave has passed the last tile's barrier)
    float* pr = reinterpret_cast<float*>(hl);  // [NW][2][64]
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t0 = row16_sum(pq0[c][e]), t1 = POST == 2 ? row16_sum(pq1[c][e]) : 0.f;
        if (j16 == 0) {
          pr[(wid * 2 + 0) * 64 + c * 16 + kg * 4 + e] = t0;
          pr[(wid * 2 + 1) * 64 + c * 16 + kg * 4 + e] = t1;
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tid < 128) {
      const int k = tid >> 6, ch = tid & 63;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += pr[(w * 2 + k) * 64 + ch];
      a.ppart[(long)blockIdx.x * 2 * a.Ng + k * a.Ng + n0 + ch] = t;
    }
  }
}


// ------------------------------------------------------------------------------------------
// The ResNet stem forward (model/resnet_backbone.py:126-131: 7x7 / stride 2 / pad 3, 3 -> 64) on the
// same persistent-halo plan.  The input is the width-packed xp bf16 [N][H][W+8][8] (conv.hip: image
// column w at packed column w+3, channels 3..7 and the 3+5 border columns zero), so filter row fr of
// output (p, q) is the 8 consecutive packed pixels 2q .. 2q+7 of input row 2p+fr-3: one 64-wide K
// chunk (8 taps x 8 channels, tap 7 has zero weight).  The TN stem gathered those 128 B per output
// pixel and filter row from L2 (7 x 128 B per pixel, 14x the input) and re-read its 57 KB of weights
// per 128-pixel tile; here a block keeps the weights (7 x 64 x 64 bf16) in LDS and streams one
// (2*TH+5) x 70 packed-pixel patch per TH x 32 output tile (TH = 16: 40.5 KB; each input pixel is
// fetched ~1.3 times instead of 14).  MFMA roles as in halo3_kernel: weights = A (16 output channels per MFMA row
// block), pixels = B (lane j16 + 16 kg reads packed pixel 2*col + 4*kk + kg of its patch row).
// Epilogue: the BN partial statistics of each tile (sum, M2 about the tile mean) -> stats[tile][2][64].
// ------------------------------------------------------------------------------------------
constexpr int kStemTH = 16;                  // output rows per tile (two per wave: each weight
                                             // fragment read from LDS feeds 4 pixel groups)
constexpr int kStemPR = 2 * kStemTH + 5;     // patch rows
constexpr int kStemPC = 2 * HW_TW + 6;       // patch columns (packed pixels)
// A patch row is stored even packed columns first, then odd ones: the 16 lanes of a pixel fragment
// read columns 2*col + ch (col = 16 consecutive pixels), i.e. 16 consecutive LDS units -- with the
// natural order they were 32 B apart and lanes j16 and j16 + 8 hit the same banks.
__device__ __forceinline__ int stem_pos(int hc) { return (hc & 1) ? kStemPC / 2 + (hc >> 1) : hc >> 1; }
__device__ __forceinline__ int stem_col(int pos) { return pos < kStemPC / 2 ? 2 * pos : 2 * (pos - kStemPC / 2) + 1; }

template <int NW, int NST>
__global__ __launch_bounds__(64 * NW) void stem_halo_kernel(const bf16* xp, unsigned x_bytes, const bf16* wk, int H,
                                                            int Wp, int P, int Q, int n_sp, bf16* y, int ldy,
                                                            unsigned y_bytes, float* stats) {
  constexpr int TH = kStemTH;
  constexpr int RPW = TH / NW;
  constexpr int FP = RPW * (HW_TW / 16);
  constexpr int FC = 4;
  constexpr int HP = kStemPR * kStemPC;            // 16-B units (packed pixels) per patch
  constexpr int HI = (HP + 64 * NW - 1) / (64 * NW);
  constexpr int HPP = HI * 64 * NW;                // a stage padded to whole DMA instructions: every
                                                   // wave issues exactly HI per patch (exact vmcnt)
  constexpr int ST_PER_TILE = FP * FC + 2;         // stores per wave and tile (outputs + 2 stats)
  constexpr int WCH = 7 * 64 * 8;                  // 16-B chunks of resident weights
  constexpr int WI = WCH / (64 * NW);
  static_assert(TH % NW == 0 && WCH % (64 * NW) == 0, "tile shape");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  uint4* wl = lds;                  // [7*64 rows][8 chunks]
  uint4* hl = lds + WCH;            // [NST][HPP]
  float* red = reinterpret_cast<float*>(hl + NST * HPP);  // [NW][64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slot = blockIdx.x, G_per = gridDim.x;
  const int my_tiles = slot < n_sp ? (n_sp - slot + G_per - 1) / G_per : 0;
  const int tiles_w = Q / HW_TW, tiles_h = P / TH;
  const __amdgpu_buffer_rsrc_t rx = srd(xp, x_bytes);
  const __amdgpu_buffer_rsrc_t rw = srd(wk, 64u * 7u * 128u);
  const __amdgpu_buffer_rsrc_t ry = srd(y, y_bytes);
  const __amdgpu_buffer_rsrc_t rs = srd(stats, (unsigned)n_sp * 128u * 4u);

  // resident weights: LDS row (fr, k) = wk[k][fr][0..63]
  {
    const unsigned base = lds_addr(wl);
#pragma unroll 2
    for (int i = 0; i < WI; ++i) {
      const int inst = i * NW + wid;
      const int idx = inst * 64 + lane;
      const int row = idx >> 3, pc = idx & 7;
      const int fr = row >> 6, k = row & 63;
      dma16(rw, base + (unsigned)inst * 1024u, (unsigned)(k * 7 + fr) * 128u + (unsigned)swz8(row, pc) * 16u);
    }
  }
  // patch geometry of this lane's DMA slots: offset from the patch origin and whether the unit lies in
  // the 3 rows above or the 2 rows below the image (only those can leave it; columns never do)
  unsigned hoff[HI], hflag[HI];
#pragma unroll
  for (int i = 0; i < HI; ++i) {
    const int idx = (i * NW + wid) * 64 + lane;
    const int hr = idx / kStemPC, hc = stem_col(idx - hr * kStemPC);  // LDS position -> packed column
    hoff[i] = (unsigned)(hr * Wp + hc) * 16u;
    hflag[i] = idx >= HP ? 16u : (hr < 3 ? 1u : 0u) | (hr >= 2 * TH + 3 ? 2u : 0u);
  }
  auto issue_patch = [&](int t, int stage) {
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    const int h0 = th * TH, w0 = tw * HW_TW;
    const unsigned base = __builtin_amdgcn_readfirstlane(lds_addr(hl + stage * HPP));
    // origin row 2*h0 - 3 wraps below zero on the first tile row; those lanes are killed
    const unsigned hb = __builtin_amdgcn_readfirstlane((unsigned)((nb * H + 2 * h0 - 3) * Wp + 2 * w0) * 16u);
    const unsigned kill = __builtin_amdgcn_readfirstlane(16u | (h0 == 0 ? 1u : 0u) | (h0 + TH >= P ? 2u : 0u));
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const unsigned off = (hflag[i] & kill) ? kOOB : hb + hoff[i];  // padding units: zeros
      dma16(rx, base + (unsigned)((i * NW + wid) * 1024), off);
    }
  };

  f32x4 acc[FC][FP];
  // NST-stage patch ring: patches 0 .. NST-2 in flight before the first tile, patch t + NST - 1 issued
  // as tile t starts (a tile's MFMA work is ~0.8 us, far below the DMA latency under load)
#pragma unroll
  for (int q = 0; q < NST - 1; ++q)
    if (q < my_tiles) issue_patch(q, q);
  if (my_tiles >= NST - 1)  // weights and patch 0 landed (patches 1 .. NST-2 may still fly)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((NST - 2) * HI) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const int j16 = lane & 15, kg = lane >> 4;

  for (int t = 0; t < my_tiles; ++t) {
    const int stage = t % NST;
    if (t + NST - 1 < my_tiles) issue_patch(t + NST - 1, (t + NST - 1) % NST);
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
    const uint4* hs = hl + stage * HPP;
#pragma unroll
    for (int fr = 0; fr < 7; ++fr) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + kg;
        bf16x8 wf[FC], pf[FP];
#pragma unroll
        for (int c = 0; c < FC; ++c) {
          const int row = fr * 64 + c * 16 + j16;
          uint4 v = wl[row * 8 + swz8(row, ch)];
          wf[c] = *reinterpret_cast<bf16x8*>(&v);
        }
#pragma unroll
        for (int p = 0; p < FP; ++p) {
          const int r = wid * RPW + p / (HW_TW / 16);
          const int col = (p % (HW_TW / 16)) * 16 + j16;
          uint4 v = hs[(2 * r + fr) * kStemPC + stem_pos(2 * col + ch)];
          pf[p] = *reinterpret_cast<bf16x8*>(&v);
        }
#pragma unroll
        for (int c = 0; c < FC; ++c)
#pragma unroll
          for (int p = 0; p < FP; ++p)
            acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], pf[p], acc[c][p], 0, 0, 0);
      }
    }

    // epilogue: round to bf16, BN partials of the rounded values, stores last
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    float csum[FC][4];
    uint2 outv[FC][FP];
    unsigned outo[FP];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[c][e] = 0.f;
#pragma unroll
    for (int p = 0; p < FP; ++p) {
      const int r = wid * RPW + p / (HW_TW / 16);
      const int col = (p % (HW_TW / 16)) * 16 + j16;
      const long opix = ((long)nb * P + th * TH + r) * Q + tw * HW_TW + col;
      outo[p] = (unsigned)(opix * ldy) * 2u;
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        bf16 o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = (bf16)acc[c][p][e];
          const float v = (float)o[e];
          acc[c][p][e] = v;
          csum[c][e] += v;
        }
        outv[c][p] = *reinterpret_cast<uint2*>(o);
      }
    }
    // BN partials as halo3_kernel's: (sum, M2 about the wave mean) per wave in registers, merged by
    // wave 0 (Chan), the sums and then the M2s through `red`
    float sv[FC * 4], qv[FC * 4];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) sv[c * 4 + e] = csum[c][e];
    row16_sum_n(sv);
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float mw = sv[c * 4 + e] * (1.0f / (16 * FP));
        float q = 0.f;
#pragma unroll
        for (int p = 0; p < FP; ++p) {
          const float d = acc[c][p][e] - mw;
          q += d * d;
        }
        qv[c * 4 + e] = q;
      }
    row16_sum_n(qv);
    if (j16 == 0)
#pragma unroll
      for (int c = 0; c < FC; ++c)
        *reinterpret_cast<float4*>(red + wid * 64 + c * 16 + kg * 4) =
            float4{sv[c * 4], sv[c * 4 + 1], sv[c * 4 + 2], sv[c * 4 + 3]};
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float sw[NW], stot = 0.f;
    if (tid < 64)
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        sw[w] = red[w * 64 + tid];
        stot += sw[w];
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (j16 == 0)
#pragma unroll
      for (int c = 0; c < FC; ++c)
        *reinterpret_cast<float4*>(red + wid * 64 + c * 16 + kg * 4) =
            float4{qv[c * 4], qv[c * 4 + 1], qv[c * 4 + 2], qv[c * 4 + 3]};
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    {
      float q = 0.f;
      if (tid < 64) {
        const float mean = stot * (1.0f / (TH * HW_TW));
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          q += red[w * 64 + tid];
          const float d = sw[w] * (1.0f / (16 * FP)) - mean;
          q = fmaf((float)(16 * FP) * d, d, q);
        }
      }
      // every wave issues both stats stores (only wave 0's lanes land): exact per-wave counts
      const unsigned so = tid < 64 ? (unsigned)(sp * 128 + tid) * 4u : kOOB;
      bstore32(rs, so, stot);
      bstore32(rs, tid < 64 ? so + 256u : kOOB, q);
    }
#pragma unroll
    for (int p = 0; p < FP; ++p)
#pragma unroll
      for (int c = 0; c < FC; ++c) bstore64(ry, outo[p] + (c * 16 + kg * 4) * 2, outv[c][p]);
    // patch t + 1 landed and every wave is done with the current stage and `red`.  In the steady
    // state (patch t + 1 issued inside the loop, patches t + 2 .. t + NST - 1 issued) exactly
    // (NST - 2) patches and (NST - 1) tiles' stores were issued after it; near either end, wait for
    // all but this tile's stores (conservative)
    if (t >= NST - 2 && t + NST - 1 < my_tiles)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"((NST - 2) * HI + (NST - 1) * ST_PER_TILE)
                   : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(ST_PER_TILE) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------------
// wgrad of the same convolutions: dW[k][tap][c] = sum_pix dY[pix][k] * X[pix + off(tap)][c].
// Block group = (64 output channels, 64 input channels); persistent over TH x 32 spatial tiles,
// each tile = dY tile (256 px x 64 ch) + X halo (340 px x 64 ch) by LDS-DMA, double buffered.
// Wave w owns input channels 16w .. 16w+15 of the 9 taps: 4 x 9 accumulators of 16x16.
// Fragments come from pixel-major LDS with ds_read_b64_tr_b16 (K = 32 pixels of one output row);
// the halo rows of a tap are the output row's pixels shifted by (dh, dw), so the same transposed
// read serves all 9 taps.  Partials go to slab[slot] in the natural [cout][tap*cin + c] layout of
// the split-K reduce.
// ------------------------------------------------------------------------------------------
// NW = 8: two waves per SIMD -- wave w owns input channels 16 (w % 4) .. of the 9 taps for output
// channels 32 (w / 4) .. 32 (w / 4) + 31 (the X fragments are read by both halves; the single wave per
// SIMD of NW = 4 left the MFMA pipe idle while its own LDS reads were in flight).
template <int TH, int NW>
__global__ __launch_bounds__(64 * NW) void halo3_wgrad_kernel(HaloWgradArgs a, int tiles_w, int tiles_h, int n_sp,
                                                              int G_per) {
  constexpr int TP = TH * HW_TW;              // output pixels per tile
  constexpr int HP = (TH + 2) * (HW_TW + 2);  // halo pixels
  constexpr int DCH = TP * 8, HCH = HP * 8;   // 16-B chunks per stage part
  constexpr int DI = DCH / (64 * NW);         // dY DMA instructions per wave
  constexpr int HI = (HCH + 64 * NW - 1) / (64 * NW);
  constexpr int STG = DCH + HCH;              // uint4 per stage
  constexpr int FM = NW == 8 ? 2 : 4, FN = 9;
  static_assert(DCH % (64 * NW) == 0, "tile shape");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid & 3, wm = NW == 8 ? wid >> 2 : 0;  // input-channel group, output-channel half
  const int mtiles = a.Cout >> 6;
  const int grp = blockIdx.x / G_per, slot = blockIdx.x % G_per;
  const int mt = grp % mtiles, ct = grp / mtiles;
  const int my_tiles = slot < n_sp ? (n_sp - slot + G_per - 1) / G_per : 0;
  const bool first = ct * 64 < a.c1;
  const __amdgpu_buffer_rsrc_t rx = first ? srd(a.x1, a.x1_bytes) : srd(a.x2, a.x2_bytes);
  const unsigned ldxb = first ? (unsigned)a.ldc1b : (unsigned)a.ldc2b;
  const unsigned xcb = (unsigned)(first ? ct * 64 : ct * 64 - a.c1) * 2u;
  const __amdgpu_buffer_rsrc_t rdy = srd(a.dy, a.dy_bytes);
  const unsigned dycb = (unsigned)mt * 128u;

  // Lane constants of the DMA rows, so that a tile's loads cost one add (+ the halo edge test) per
  // row: the byte offset relative to the tile's first pixel (dY) / its halo's top-left pixel (X),
  // swizzle included, and for the halo which border (top, bottom, left, right) the lane's pixel
  // lies on -- with H % TH == 0 and W % HW_TW == 0 only border halo pixels can leave the image.
  const int pc = lane & 7;
  unsigned doff[DI];
#pragma unroll
  for (int i = 0; i < DI; ++i) {
    const int px = ((i * NW + wid) * 64 + lane) >> 3;
    doff[i] = (unsigned)((px / HW_TW) * a.W + px % HW_TW) * (unsigned)a.ldyb + dycb + (unsigned)((pc ^ swz_tr8(px)) * 16);
  }
  unsigned hoff[HI], hflag[HI];
#pragma unroll
  for (int i = 0; i < HI; ++i) {
    const int idx = (i * NW + wid) * 64 + lane;
    const int hp = idx >> 3, hr = hp / (HW_TW + 2), hc = hp % (HW_TW + 2);
    hoff[i] = (unsigned)(hr * a.W + hc) * ldxb + xcb + (unsigned)((pc ^ swz_tr8(hp)) * 16);
    hflag[i] = idx >= HCH ? 16u : (hr == 0 ? 1u : 0u) | (hr == TH + 1 ? 2u : 0u) | (hc == 0 ? 4u : 0u) | (hc == HW_TW + 1 ? 8u : 0u);
  }
  auto issue = [&](int t, int stage) {
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    const int h0 = th * TH, w0 = tw * HW_TW;
    const unsigned base = __builtin_amdgcn_readfirstlane(lds_addr(lds + stage * STG));
    const unsigned tb = __builtin_amdgcn_readfirstlane((unsigned)((nb * a.H + h0) * a.W + w0) * (unsigned)a.ldyb);
#pragma unroll
    for (int i = 0; i < DI; ++i) dma16(rdy, base + (unsigned)((i * NW + wid) * 1024), tb + doff[i]);
    const unsigned hbase = base + DCH * 16;
    // halo origin (h0 - 1, w0 - 1): wraps below zero on the first row / column, whose lanes the
    // edge mask sends out of range
    const unsigned hb = __builtin_amdgcn_readfirstlane((unsigned)((nb * a.H + h0 - 1) * a.W + w0 - 1) * ldxb);
    const unsigned kill = __builtin_amdgcn_readfirstlane(16u | (h0 == 0 ? 1u : 0u) | (h0 + TH >= a.H ? 2u : 0u) |
                                                         (w0 == 0 ? 4u : 0u) | (w0 + HW_TW >= a.W ? 8u : 0u));
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const unsigned off = (hflag[i] & kill) ? kOOB : hb + hoff[i];
      // only the last row can hold lanes past the halo (they must not write LDS)
      if (i < HI - 1 || HCH % (64 * NW) == 0 || hflag[i] != 16u) dma16(rx, hbase + (unsigned)((i * NW + wid) * 1024), off);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (my_tiles > 0) issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  // Transposed fragment reads with no per-read address arithmetic.  A read covers image rows
  // R + 8g + qq and R + 8g + qq + 4 (lane-dependent) at 16-B chunk c; the swizzle depends on row
  // bits 1 and 3 only, so with R = B + rho (B a multiple of 16, rho = R mod 16 known at compile
  // time once the row loop is unrolled) the lane's byte offset is B * 128 (an immediate) plus a
  // per-lane value precomputed for each rho.  Wave w owns input channels 16w .. 16w+15 of all 9
  // taps, so every tap's (dh, dw) -- and with it R -- is a compile-time constant.
  auto lane_off = [&](int x, int chunk) -> unsigned {
    return (unsigned)(x * 128 + ((chunk ^ swz_tr8(x)) * 16) + (pp & 1) * 8);
  };
  unsigned pa[FM][2], pb[16][2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
#pragma unroll
    for (int i = 0; i < FM; ++i) pa[i][k] = lane_off(8 * g + qq + 4 * k, (wm * FM + i) * 2 + (pp >> 1));
#pragma unroll
    for (int r = 0; r < 16; ++r) pb[r][k] = lane_off(r + 8 * g + qq + 4 * k, wc * 2 + (pp >> 1));
  }
  auto tr2 = [&](const char* base, unsigned o0, unsigned o1) -> bf16x8 {
    s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o0));
    s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o1));
    s16x8 v = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
    return *reinterpret_cast<bf16x8*>(&v);
  };

  for (int t = 0; t < my_tiles; ++t) {
    const int stage = t & 1;
    if (t + 1 < my_tiles) issue(t + 1, stage ^ 1);
    const char* dbase = reinterpret_cast<const char*>(lds + stage * STG);
    const char* hbase = dbase + DCH * 16;
#pragma unroll
    for (int rr = 0; rr < TH; ++rr) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = tr2(dbase + rr * HW_TW * 128, pa[i][0], pa[i][1]);
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int dh = j / 3 - 1, dw = j % 3 - 1;
        const int R = (rr + 1 + dh) * (HW_TW + 2) + 1 + dw, rho = R & 15;
        bfr[j] = tr2(hbase + (R - rho) * 128, pb[rho][0], pb[rho][1]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // slab[slot][cout][tap*cin + c]
  const long Ng = 9L * a.cin;
  float* ws = a.ws + (long)slot * a.Cout * Ng;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = mt * 64 + (wm * FM + i) * 16 + g * 4 + e;
#pragma unroll
      for (int j = 0; j < FN; ++j) ws[(long)m * Ng + (long)j * a.cin + ct * 64 + wc * 16 + i16] = acc[i][j][e];
    }
}

// ------------------------------------------------------------------------------------------
// halo3r: the same convolutions with the weights resident in VGPRs instead of LDS.
//
// halo3_kernel keeps 72 KiB of weights in LDS, which leaves room for only two halo stages: one
// tile's DMA (43 KiB per CU) is in flight while the current tile computes, and the counters show the
// waves parked on that wait for a third of their cycles (SQ_WAIT_ANY 36 %, HBM at ~3.4 TB/s, MFMA
// busy 45 % at 512^2).  Here each wave holds the weights of 32 output channels x 9 taps x 64 input
// channels in registers (144 VGPRs, loaded once per block), which frees the LDS for THREE halo
// stages: tile t+2 streams in while tile t computes (87 KiB in flight per CU), and the per-MFMA LDS
// traffic drops to the pixel fragments only.
//   waves: wid & 1 = output-channel half (32 channels, FC = 2 groups of 16); wid >> 1 = pixel set
//   (FP = 32 / NW groups of 16 pixels of the 8 x 32 tile).
//   Every wave issues exactly HI halo DMAs per tile (lanes past the halo load out of range into a
//   padded stage) and, for the post-ops, exactly FC*FP aux loads, so all waits are compile-time
//   vmcnt values: the epilogue waits for this tile's aux loads (issued before tile t+2's DMA), the
//   end of a tile for tile t+1's halo; tile t+2's DMA stays in flight across the barrier.
// ------------------------------------------------------------------------------------------

template <int NW>
constexpr int halo3r_stage_chunks() {
  return ((10 * (HW_TW + 2) * 8 + 64 * NW - 1) / (64 * NW)) * 64 * NW;
}

template <int NW>
size_t halo3r_lds_bytes() {
  // [3 stages][padded halo] + red [NW/2][64] + bias [64] + post coefficients [4][64] + head [256][2]
  return (size_t)3 * halo3r_stage_chunks<NW>() * 16 + (size_t)(NW / 2) * 64 * 4 + 64 * 4 + 256 * 4 + 256 * 2 * 4;
}

template <int NW, int POST, int EPI>
__global__ __launch_bounds__(64 * NW) void halo3r_kernel(FastTNArgs a, int tiles_w, int tiles_h, int n_sp, int G_per,
                                                         unsigned y_bytes, unsigned aux_bytes) {
  constexpr int TH = 8;
  constexpr bool kDyn = (EPI & kEpiDyn) != 0;
  const bool has_bias = kDyn ? a.bias != nullptr : (EPI & kEpiBias) != 0;
  const bool do_relu = kDyn ? a.relu != 0 : (EPI & kEpiRelu) != 0;
  const bool do_stats = kDyn ? a.stats != nullptr : (EPI & kEpiStats) != 0;
  const bool do_acc = kDyn ? a.accumulate != 0 : (EPI & kEpiAcc) != 0;
  constexpr int HK = (EPI & kEpiHead2) ? 2 : (EPI & kEpiHead1) ? 1 : 0;
  static_assert(HK == 0 || (!kDyn && POST == 0), "the fused head rides on a fixed bias + ReLU epilogue");
  constexpr int NPG = NW / 2;                // pixel sets
  constexpr int FP = 16 / NPG;               // 16-pixel groups per wave
  constexpr int FC = 2;                      // 16-channel output groups per wave (32 channels)
  constexpr int HP = (TH + 2) * (HW_TW + 2); // halo pixels
  constexpr int HCH = HP * 8;                // 16-B chunks of a halo
  constexpr int HI = (HCH + 64 * NW - 1) / (64 * NW);  // halo DMA instructions per wave
  constexpr int SCH = HI * 64 * NW;          // chunks per (padded) stage
  static_assert(SCH == halo3r_stage_chunks<NW>(), "stage size");
  constexpr int NA = POST ? FP * FC : 0;     // aux loads per wave per tile
  constexpr int NS = FP * FC + FP * HK;      // stores per wave per tile
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  uint4* hl = lds;                                          // [3][SCH]
  float* red = reinterpret_cast<float*>(hl + 3 * SCH);      // [NPG][64]
  float* sbias = red + NPG * 64;                            // [64]
  float* pco = sbias + 64;                                  // [4][64]: sc, sh, mean, inv
  float* hred = pco + 256;                                  // [256 pixels][2]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wch = wid & 1, pg = wid >> 1;
  const int tn = blockIdx.x / G_per, slot = blockIdx.x % G_per;
  const int n0 = tn * 64;
  const int my_tiles = slot < n_sp ? (n_sp - slot + G_per - 1) / G_per : 0;
  const __amdgpu_buffer_rsrc_t rx = srd(a.x1, a.x1_bytes);
  const __amdgpu_buffer_rsrc_t rw = srd(a.wt, a.w_bytes);
  const __amdgpu_buffer_rsrc_t ry = srd(a.y, y_bytes);
  const __amdgpu_buffer_rsrc_t ra = srd(POST ? a.aux : a.y, POST ? aux_bytes : 0u);
  const unsigned hw_img = (unsigned)(a.OH * a.OW);
  const __amdgpu_buffer_rsrc_t rh = srd(HK ? (const void*)a.head_y : a.y,
                                        HK ? (unsigned)(a.M / (a.OH * a.OW)) * HK * hw_img * 4u : 0u);
  const int j16 = lane & 15, kg = lane >> 4;

  if (kDyn && a.bias && tid < 64) sbias[tid] = a.bias[n0 + tid];
  if (POST == 2 && tid < 64) {
    pco[tid] = a.psc[n0 + tid];
    pco[64 + tid] = a.psh[n0 + tid];
    pco[128 + tid] = a.pmean[n0 + tid];
    pco[192 + tid] = a.pinv[n0 + tid];
  }

  // ---- resident weights: wr[jt][kk][c] = output channel n0 + 32 wch + 16 c + j16, halo tap jt,
  // input channels 8 (4 kk + kg) .. +7 (the MFMA A fragment) ----
  bf16x8 wr[9][2][FC];
#pragma unroll
  for (int jt = 0; jt < 9; ++jt) {
    const int jr = jt / 3, js = jt - jr * 3;
    const int wtap = (a.r0 + a.rs * jr) * a.S + (a.s0 + a.ss * js);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int k = wch * 32 + c * 16 + j16;
        uint4 v = bload(rw, (unsigned)(n0 + k) * (unsigned)a.ldwb + (unsigned)(wtap * 128 + (kk * 4 + kg) * 16));
        wr[jt][kk][c] = *reinterpret_cast<bf16x8*>(&v);
      }
  }
  float hwr[HK > 0 ? HK : 1][FC][4], hbr[HK > 0 ? HK : 1];
#pragma unroll
  for (int k = 0; k < HK; ++k) {
    hbr[k] = a.head_b[k];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) hwr[k][c][e] = a.head_w[k * 64 + wch * 32 + c * 16 + kg * 4 + e];
  }
  float breg[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) breg[c][e] = (!kDyn && has_bias) ? a.bias[n0 + wch * 32 + c * 16 + kg * 4 + e] : 0.f;
  // the preloads above are compiler-tracked: retire them here (a pre-existing wait the compiler
  // accounts for), so no conservative vmcnt(0) lands inside the tile loop
  __builtin_amdgcn_s_waitcnt(0);

  // ---- halo DMA of tile t into stage t % 3 (see halo3_kernel); the lane geometry is recomputed per
  // issue (a few VALU) rather than held in 2 x HI VGPRs; slots past the halo load out of range into
  // the stage padding, so every wave issues exactly HI DMAs ----
  auto issue_halo = [&](int t) {
    const int stage = t % 3;
    const unsigned base = __builtin_amdgcn_readfirstlane(lds_addr(hl + stage * SCH));
    if (t >= my_tiles) {  // no such tile: the same count of DMAs, all out of range (zero fill)
#pragma unroll
      for (int i = 0; i < HI; ++i) dma16(rx, base + (unsigned)((i * NW + wid) * 1024), kOOB);
      return;
    }
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    const int h0 = th * TH, w0 = tw * HW_TW;
    const unsigned hb = __builtin_amdgcn_readfirstlane((unsigned)((nb * a.H + h0 - 1) * a.W + w0 - 1) * (unsigned)a.ldc1b);
    const unsigned kill = __builtin_amdgcn_readfirstlane(16u | (h0 == 0 ? 1u : 0u) | (h0 + TH >= a.H ? 2u : 0u) |
                                                         (w0 == 0 ? 4u : 0u) | (w0 + HW_TW >= a.W ? 8u : 0u));
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int idx = (i * NW + wid) * 64 + lane;
      const int hp = idx >> 3, hr = hp / (HW_TW + 2), hc = hp - hr * (HW_TW + 2);
      const unsigned flag = idx >= HCH ? 16u : (hr == 0 ? 1u : 0u) | (hr == TH + 1 ? 2u : 0u) | (hc == 0 ? 4u : 0u) |
                                                   (hc == HW_TW + 1 ? 8u : 0u);
      const unsigned off = (unsigned)(hr * a.W + hc) * (unsigned)a.ldc1b + swzh(hp, lane & 7) * 16u;
      dma16(rx, base + (unsigned)((i * NW + wid) * 1024), (flag & kill) ? kOOB : hb + off);
    }
  };

  // this lane's pixels: group g = pg * FP + p of the tile's 16 groups (2 per row)
  float pq0[FC][4], pq1[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) pq0[c][e] = pq1[c][e] = 0.f;
  issue_halo(0);
  issue_halo(1);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(HI) : "memory");

  // halo pixel of tap (0, 0) for each of this lane's pixel groups
  unsigned u0[FP];
#pragma unroll
  for (int p = 0; p < FP; ++p) {
    const int g = pg * FP + p;
    u0[p] = (unsigned)(((g >> 1) + 1) * (HW_TW + 2) + (g & 1) * 16 + j16 + 1);
  }
  f32x4 acc[FC][FP];
  for (int t = 0; t < my_tiles; ++t) {
    // the tap shifts pass through an opaque copy per tile: the 9 x FP fragment addresses are then
    // recomputed per tile (4 VALU each, beside the MFMAs) instead of being hoisted into 36 VGPRs
    int dh0 = a.dh0, dhs = a.dhs, dw0 = a.dw0, dws = a.dws;
    asm volatile("" : "+s"(dh0), "+s"(dhs), "+s"(dw0), "+s"(dws));
    const int sp = slot + t * G_per;
    const int tw = sp % tiles_w, rest = sp / tiles_w;
    const int th = rest % tiles_h, nb = rest / tiles_h;
    // post-op aux values of this tile: issued halfway through the tap loop (their registers live only
    // from there) and before tile t+2's DMA, so the epilogue's wait for them leaves that DMA in flight
    uint2 zr[FC][FP];
    auto issue_aux = [&]() {
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int g = pg * FP + p;
        const long opix = ((long)nb * a.OH + th * TH + (g >> 1)) * a.OW + tw * HW_TW + (g & 1) * 16 + j16;
#pragma unroll
        for (int c = 0; c < FC; ++c)
          zr[c][p] = bload64_asm(ra, (unsigned)(opix * a.ld_aux + n0 + wch * 32 + c * 16 + kg * 4) * 2u);
      }
      issue_halo(t + 2);
    };
    if (!POST) issue_halo(t + 2);
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* hs = reinterpret_cast<const char*>(hl + (t % 3) * SCH);
    // 18 steps (tap jt, K half kk), software-pipelined by hand: the pixel fragments of step s+1 are
    // read before the MFMAs of step s, and sched_group_barrier pins that order (left to itself the
    // scheduler issues each read right before its MFMAs and the waves sit on lgkmcnt)
    // byte address of halo pixel u, chunk kg (kk 0): u * 128 + ((kg ^ u) & 7) * 16 (swzh); chunk
    // 4 + kg (kk 1) differs in address bit 6 only
    auto tap_addr = [&](int jt, unsigned (&ad)[FP]) {
      const int jr = jt / 3, js = jt - jr * 3;
      const int delta = (dh0 + dhs * jr) * (HW_TW + 2) + dw0 + dws * js;  // uniform
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const unsigned u = u0[p] + (unsigned)delta;
        ad[p] = (u << 7) | (((u ^ (unsigned)kg) & 7u) << 4);
      }
    };
    auto frag_load = [&](const unsigned (&ad)[FP], int kk, bf16x8 (&pf)[FP]) {
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        uint4 v = *reinterpret_cast<const uint4*>(hs + (ad[p] ^ (kk ? 64u : 0u)));
        pf[p] = *reinterpret_cast<bf16x8*>(&v);
      }
    };
    unsigned ad[FP];
    bf16x8 pfb[2][FP];
    tap_addr(0, ad);
    frag_load(ad, 0, pfb[0]);
    __builtin_amdgcn_sched_group_barrier(0x100, FP, 0);  // step 0's reads form the first group
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      const int jt = st >> 1, kk = st & 1;
      if (st + 1 < 18) {
        if (kk == 1) tap_addr(jt + 1, ad);
        frag_load(ad, (st + 1) & 1, pfb[(st + 1) & 1]);
      }
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int p = 0; p < FP; ++p)
          acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[jt][kk][c], pfb[st & 1][p], acc[c][p], 0, 0, 0);
      if (st + 1 < 18) __builtin_amdgcn_sched_group_barrier(0x100, FP, 0);  // DS reads of step st+1
      __builtin_amdgcn_sched_group_barrier(0x008, FC * FP, 0);              // MFMAs of step st
      if (POST && st == 8) issue_aux();
    }

    // ================= epilogue =================
    if (POST) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(HI) : "memory");  // this tile's aux (tile t+2's halo may fly)
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int p = 0; p < FP; ++p) asm volatile("" : "+v"(zr[c][p]));
    }
    float csum[FC][4];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[c][e] = 0.f;
    uint2 outv[FC][FP];
    unsigned outo[FP];
#pragma unroll
    for (int p = 0; p < FP; ++p) {
      const int g = pg * FP + p;
      const long opix = ((long)nb * a.OH + th * TH + (g >> 1)) * a.OW + tw * HW_TW + (g & 1) * 16 + j16;
      outo[p] = (unsigned)(opix * a.ldy + n0) * 2u;
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int cb = wch * 32 + c * 16 + kg * 4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[c][p][e] + (!has_bias ? 0.f : kDyn ? sbias[cb + e] : breg[c][e]);
          if (do_relu) v[e] = fmaxf(v[e], 0.f);
        }
        if (do_acc) {
          const bf16* ob = reinterpret_cast<const bf16*>((const char*)a.y + outo[p] + cb * 2);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)ob[e];
        }
        bf16 o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = (bf16)v[e];
          v[e] = (float)o[e];
        }
        if (POST) {
          const bf16* z = reinterpret_cast<const bf16*>(&zr[c][p]);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float zf = (float)z[e];
            bool on = zf > 0.f;
            float xh = 0.f;
            if (POST == 2) {
              const int ch = cb + e;
              on = fmaf(zf, pco[ch], pco[64 + ch]) > 0.f;
              xh = (zf - pco[128 + ch]) * pco[192 + ch];
            }
            v[e] = on ? v[e] : 0.f;
            o[e] = (bf16)v[e];
            pq0[c][e] += v[e];
            if (POST == 2) pq1[c][e] += v[e] * xh;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          csum[c][e] += v[e];
          acc[c][p][e] = v[e];
        }
        outv[c][p] = *reinterpret_cast<uint2*>(o);
      }
    }
    if (HK) {
      // head logits: this wave's 32 channels per pixel (4 channel groups kg summed by shuffles); the
      // odd-channel-half waves hand their partial sums to the even ones through LDS
      float hsum[HK > 0 ? HK : 1][FP];
#pragma unroll
      for (int p = 0; p < FP; ++p)
#pragma unroll
        for (int k = 0; k < HK; ++k) {
          float h = 0.f;
#pragma unroll
          for (int c = 0; c < FC; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e) h = fmaf(acc[c][p][e], hwr[k][c][e], h);
          h += __shfl_xor(h, 16);
          h += __shfl_xor(h, 32);
          hsum[k][p] = h;
          if (wch == 1 && kg == 0) hred[((pg * FP + p) * 16 + j16) * 2 + k] = h;
        }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int g = pg * FP + p;
        const unsigned pix = (unsigned)((th * TH + (g >> 1)) * a.OW + tw * HW_TW + (g & 1) * 16 + j16);
#pragma unroll
        for (int k = 0; k < HK; ++k) {
          const float h = hsum[k][p] + hred[(g * 16 + j16) * 2 + k] + hbr[k];
          bstore32(rh, (wch == 0 && kg == 0) ? ((unsigned)(nb * HK + k) * hw_img + pix) * 4u : kOOB, h);
        }
      }
    }
    if (do_stats) {
      // per-tile BN partials over the 256 pixels: column sums, then M2 about the tile mean
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float s = row16_sum(csum[c][e]);
          if (j16 == 0) red[pg * 64 + wch * 32 + c * 16 + kg * 4 + e] = s;
        }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      float qv[FC][4];
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wch * 32 + c * 16 + kg * 4 + e;
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < NPG; ++w) tot += red[w * 64 + col];
          const float mean = tot * (1.0f / (TH * HW_TW));
          float q = 0.f;
#pragma unroll
          for (int p = 0; p < FP; ++p) {
            const float d = acc[c][p][e] - mean;
            q += d * d;
          }
          qv[c][e] = row16_sum(q);
        }
      float stot = 0.f;
      if (tid < 64)
#pragma unroll
        for (int w = 0; w < NPG; ++w) stot += red[w * 64 + tid];
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (j16 == 0) red[pg * 64 + wch * 32 + c * 16 + kg * 4 + e] = qv[c][e];
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (tid < 64) {
        float q = 0.f;
#pragma unroll
        for (int w = 0; w < NPG; ++w) q += red[w * 64 + tid];
        a.stats[(long)sp * 2 * a.Ng + n0 + tid] = stot;
        a.stats[(long)sp * 2 * a.Ng + a.Ng + n0 + tid] = q;
      }
    }
#pragma unroll
    for (int p = 0; p < FP; ++p)
#pragma unroll
      for (int c = 0; c < FC; ++c) bstore64(ry, outo[p] + (wch * 32 + c * 16 + kg * 4) * 2, outv[c][p]);
    // tile t+1's halo landed: after it this wave issued tile t-1's stores, tile t's aux loads, tile
    // t+2's DMA and tile t's stores (compiler-visible stats stores only add to the wait); the
    // barrier also frees stage t % 3 for tile t+3's DMA, `red` and `hred`
    constexpr int kEnd = NS + NA + HI + NS;  // vmcnt holds 6 bits: a smaller count only waits longer
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(kEnd < 63 ? kEnd : 63) : "memory");
  }
  // the zero-fill DMAs of the last two (absent) tiles may still be landing in the stages
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (POST) {
    float* pr = reinterpret_cast<float*>(hl);  // [NW][2][64]
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t0 = row16_sum(pq0[c][e]), t1 = POST == 2 ? row16_sum(pq1[c][e]) : 0.f;
        if (j16 == 0) {
          const int col = wch * 32 + c * 16 + kg * 4 + e;
          pr[(pg * 2 + 0) * 64 + col] = t0;
          pr[(pg * 2 + 1) * 64 + col] = t1;
        }
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tid < 128) {
      const int k = tid >> 6, ch = tid & 63;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NPG; ++w) t += pr[(w * 2 + k) * 64 + ch];
      a.ppart[(long)blockIdx.x * 2 * a.Ng + k * a.Ng + n0 + ch] = t;
    }
  }
}

template <int TH, int NW>
size_t halo_lds_bytes(int head_k = 0) {
  (void)head_k;
  return (size_t)9 * 64 * 128 + 2 * (size_t)(TH + 2) * (HW_TW + 2) * 128 + NW * 64 * 4 + 64 * 4;
}

}  // namespace

int halo_tile_m() { return 8 * HW_TW; }

bool halo3_ok(const FastTNArgs& a) {
  static const bool off = getenv("UNETSEG_NO_HALO") != nullptr;
  if (off) return false;
  if (a.x2 || a.c1 != 64 || a.cin != 64 || a.nr != 3 || a.ns != 3 || a.istride != 1) return false;
  if (a.dhs * a.dhs != 1 || a.dws * a.dws != 1) return false;
  const int dh_lo = a.dhs > 0 ? a.dh0 : a.dh0 - 2, dw_lo = a.dws > 0 ? a.dw0 : a.dw0 - 2;
  if (dh_lo != -1 || dw_lo != -1) return false;  // halo of one pixel on every side
  if (a.ostride != 1 || a.ph || a.pw || a.OH != a.hc || a.OW != a.wc || a.H != a.hc || a.W != a.wc) return false;
  if (a.Ng % 64 || a.hc % 8 || a.wc % HW_TW) return false;
  if ((long)a.M * a.ldy * 2 >= (1L << 31)) return false;
  if (a.post && a.post != 4 && (long)a.M * a.ld_aux * 2 >= (1L << 31)) return false;
  if (a.post == 4 && (long)a.M * (a.Ng >> 3) >= (1L << 31)) return false;
  return true;
}

template <int TH, int NW, int POST, int EPI, bool HS>
static int launch_halo3_hs(const FastTNArgs& a, hipStream_t st) {
  const int tiles_w = a.wc / HW_TW, tiles_h = a.hc / TH;
  const int n_img = a.M / (a.hc * a.wc);
  const int n_sp = n_img * tiles_h * tiles_w;
  const int ntn = a.Ng / 64;
  int G_per = 256 / ntn;
  if (G_per < 1) G_per = 1;
  if (G_per > n_sp) G_per = n_sp;
  constexpr int HK = (EPI & kEpiHead2) ? 2 : (EPI & kEpiHead1) ? 1 : 0;
  const size_t lds = halo_lds_bytes<TH, NW>(HK);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&halo3_kernel<TH, NW, POST, EPI, HS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  // experiment (UNETSEG_HALO_EXP_NOSTORE=1, wrong results): a zero-extent output descriptor -- the
  // output stores still issue (the vmcnt bookkeeping is unchanged) but the hardware drops them, so the
  // launch time without the output's HBM writes can be measured
  static const bool nostore = getenv("UNETSEG_HALO_EXP_NOSTORE") != nullptr;
  const unsigned y_bytes = nostore ? 0u : (unsigned)((long)a.M * a.ldy * 2);
  hipLaunchKernelGGL((halo3_kernel<TH, NW, POST, EPI, HS>), dim3(ntn * G_per), dim3(64 * NW), lds, st, a, tiles_w, tiles_h,
                     n_sp, G_per, y_bytes);
  return 0;
}

// The half-stage pipeline (HS) for the 8-wave kernels (UNETSEG_HALO_HS=1; default: the whole-tile
// double buffer; read per call, the parity tests run both).  Isolated, a 512^2 layer (64 tiles per
// block) is slower with it (fwd 349-363 vs 296-312 us: a second barrier per tile) and a 256^2 one
// faster (104.8 vs 124.6 us: the three-half prologue hides the first tile's load).  Round 4 (eager
// host) measured HS everywhere best in the step (C2 972.8 vs 962.1 img/s); with the replayed step plan
// of round 5 the double buffer is (C2 1016-1019 vs 1010-1011 on one box, 958-959 vs 957 on another).
template <int TH, int NW, int POST, int EPI>
static int launch_halo3_cfg(const FastTNArgs& a, hipStream_t st) {
  const char* e = getenv("UNETSEG_HALO_HS");
  const bool hs = e != nullptr && atoi(e) != 0;
  if constexpr (NW == 8) {
    if (hs) return launch_halo3_hs<TH, NW, POST, EPI, true>(a, st);
  }
  return launch_halo3_hs<TH, NW, POST, EPI, false>(a, st);
}

// blocks (= post-op partial rows) of a launch_halo3 call
int halo3_blocks(const FastTNArgs& a) {
  const int n_sp = (a.M / (a.hc * a.wc)) * (a.hc / 8) * (a.wc / HW_TW);
  const int ntn = a.Ng / 64;
  int G_per = 256 / ntn;
  if (G_per < 1) G_per = 1;
  if (G_per > n_sp) G_per = n_sp;
  return ntn * G_per;
}

template <int NW, int POST, int EPI>
static int launch_halo3r_cfg(const FastTNArgs& a, hipStream_t st) {
  constexpr int TH = 8;
  const int tiles_w = a.wc / HW_TW, tiles_h = a.hc / TH;
  const int n_img = a.M / (a.hc * a.wc);
  const int n_sp = n_img * tiles_h * tiles_w;
  const int ntn = a.Ng / 64;
  int G_per = 256 / ntn;
  if (G_per < 1) G_per = 1;
  if (G_per > n_sp) G_per = n_sp;
  const size_t lds = halo3r_lds_bytes<NW>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&halo3r_kernel<NW, POST, EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const unsigned y_bytes = (unsigned)((long)a.M * a.ldy * 2);
  const long aux_bytes = POST ? (long)a.M * a.ld_aux * 2 : 0;
  if (aux_bytes >= (1L << 31)) return -1;
  hipLaunchKernelGGL((halo3r_kernel<NW, POST, EPI>), dim3(ntn * G_per), dim3(64 * NW), lds, st, a, tiles_w, tiles_h,
                     n_sp, G_per, y_bytes, (unsigned)aux_bytes);
  return 0;
}

template <int NW>
static int launch_halo3r(const FastTNArgs& a, int epi, bool dyn, hipStream_t st) {
  if (a.head_y) {
    if (a.post || epi != (kEpiBias | kEpiRelu) || (a.head_k != 1 && a.head_k != 2)) return -1;
    return a.head_k == 2 ? launch_halo3r_cfg<NW, 0, kEpiBias | kEpiRelu | kEpiHead2>(a, st)
                         : launch_halo3r_cfg<NW, 0, kEpiBias | kEpiRelu | kEpiHead1>(a, st);
  }
  if (a.post == 1) return epi == 0 && !dyn ? launch_halo3r_cfg<NW, 1, 0>(a, st) : launch_halo3r_cfg<NW, 1, kEpiDyn>(a, st);
  if (a.post == 2) return epi == 0 && !dyn ? launch_halo3r_cfg<NW, 2, 0>(a, st) : launch_halo3r_cfg<NW, 2, kEpiDyn>(a, st);
  if (!dyn) switch (epi) {
      case kEpiBias | kEpiRelu: return launch_halo3r_cfg<NW, 0, kEpiBias | kEpiRelu>(a, st);
      case kEpiStats: return launch_halo3r_cfg<NW, 0, kEpiStats>(a, st);
      case 0: return launch_halo3r_cfg<NW, 0, 0>(a, st);
      case kEpiAcc: return launch_halo3r_cfg<NW, 0, kEpiAcc>(a, st);
      default: break;
    }
  return launch_halo3r_cfg<NW, 0, kEpiDyn>(a, st);
}

int launch_halo3(const FastTNArgs& a, hipStream_t st) {
  // UNETSEG_HALO_R=1: the register-resident-weight kernel (UNETSEG_HALO_R_NW=4: one wave per SIMD)
  static const bool v1 = getenv("UNETSEG_HALO_R") == nullptr;
  static const int rnw = getenv("UNETSEG_HALO_R_NW") ? atoi(getenv("UNETSEG_HALO_R_NW")) : 8;
  if (!v1) {
    static const bool dyn_r = getenv("UNETSEG_HALO_EPI_DYN") != nullptr;
    const int epi_r = (a.bias ? kEpiBias : 0) | (a.relu ? kEpiRelu : 0) | (a.stats ? kEpiStats : 0) |
                      (a.accumulate ? kEpiAcc : 0);
    return rnw == 4 ? launch_halo3r<4>(a, epi_r, dyn_r, st) : launch_halo3r<8>(a, epi_r, dyn_r, st);
  }
  static const int nw = getenv("UNETSEG_HALO_W4") ? 4 : 8;
  // fused dgrad post-ops are separate instantiations: their registers must not cost the plain path
  static const bool dyn = getenv("UNETSEG_HALO_EPI_DYN") != nullptr;
  const int epi = (a.bias ? kEpiBias : 0) | (a.relu ? kEpiRelu : 0) | (a.stats ? kEpiStats : 0) |
                  (a.accumulate ? kEpiAcc : 0);
  if (a.head_y) {  // fused head: bias + ReLU epilogue only (checked by the caller)
    if (a.post || epi != (kEpiBias | kEpiRelu) || (a.head_k != 1 && a.head_k != 2)) return -1;
    return a.head_k == 2 ? launch_halo3_cfg<8, 8, 0, kEpiBias | kEpiRelu | kEpiHead2>(a, st)
                         : launch_halo3_cfg<8, 8, 0, kEpiBias | kEpiRelu | kEpiHead1>(a, st);
  }
  if (a.mbits_out) {  // ReLU mask bits: bias + ReLU epilogue only (checked by the caller)
    if (a.post || epi != (kEpiBias | kEpiRelu)) return -1;
    return launch_halo3_cfg<8, 8, 0, kEpiBias | kEpiRelu | kEpiMask>(a, st);
  }
  if (a.post == 4) return epi == 0 ? launch_halo3_cfg<8, 8, 4, 0>(a, st) : -1;
  // fused dgrad post-ops come with a plain epilogue (no bias / ReLU / stats / accumulate)
  if (a.post == 1) return epi == 0 && !dyn ? launch_halo3_cfg<8, 8, 1, 0>(a, st) : launch_halo3_cfg<8, 8, 1, kEpiDyn>(a, st);
  if (a.post == 2) return epi == 0 && !dyn ? launch_halo3_cfg<8, 8, 2, 0>(a, st) : launch_halo3_cfg<8, 8, 2, kEpiDyn>(a, st);
  if (nw == 4) return launch_halo3_cfg<8, 4, 0, kEpiDyn>(a, st);
  // the epilogues the U-Net runs: conv+bias+ReLU (decoder), conv with BN statistics (encoder),
  // plain data gradient, accumulated data gradient
  if (!dyn) switch (epi) {
      case kEpiBias | kEpiRelu: return launch_halo3_cfg<8, 8, 0, kEpiBias | kEpiRelu>(a, st);
      case kEpiStats: return launch_halo3_cfg<8, 8, 0, kEpiStats>(a, st);
      case 0: return launch_halo3_cfg<8, 8, 0, 0>(a, st);
      case kEpiAcc: return launch_halo3_cfg<8, 8, 0, kEpiAcc>(a, st);
      default: break;
    }
  return launch_halo3_cfg<8, 8, 0, kEpiDyn>(a, st);
}

// the stem forward on stem_halo_kernel: 64 output channels, even input sizes with P % 16 == 0 and
// Q % 32 == 0 (UNETSEG_STEM_TN=1: the TN stem)
bool stem_halo_ok(int n, int h, int w, int K, int ldy) {
  if (getenv("UNETSEG_STEM_TN")) return false;
  if (K != 64 || ldy < 64 || ldy % 4 || n <= 0 || h % 2 || w % 2) return false;
  const int P = h / 2, Q = w / 2;
  if (P % kStemTH || Q % HW_TW) return false;
  return (long)n * h * (w + 8) * 16 < (1L << 31) && (long)n * P * Q * ldy * 2 < (1L << 31);
}

int stem_halo_tiles(int n, int h, int w) { return n * (h / 2 / kStemTH) * (w / 2 / HW_TW); }
int stem_halo_tile_m() { return kStemTH * HW_TW; }

int launch_stem_halo(const void* xp, int n, int h, int w, const void* wk, void* y, int ldy, float* stats,
                     hipStream_t st) {
  constexpr int NW = 8, NST = 2;
  const int P = h / 2, Q = w / 2, Wp = w + 8;
  const int n_sp = stem_halo_tiles(n, h, w);
  const int blocks = n_sp < 256 ? n_sp : 256;
  constexpr int HPP = (kStemPR * kStemPC + 64 * NW - 1) / (64 * NW) * (64 * NW);
  const size_t lds = (size_t)7 * 64 * 128 + (size_t)NST * HPP * 16 + NW * 64 * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&stem_halo_kernel<NW, NST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((stem_halo_kernel<NW, NST>), dim3(blocks), dim3(64 * NW), lds, st, (const bf16*)xp,
                     (unsigned)((long)n * h * Wp * 16), (const bf16*)wk, h, Wp, P, Q, n_sp, (bf16*)y, ldy,
                     (unsigned)((long)n * P * Q * ldy * 2), stats);
  return 0;
}

bool halo3_wgrad_ok(const HaloWgradArgs& a) {
  static const bool off = getenv("UNETSEG_NO_HALO") != nullptr;
  if (off) return false;
  return a.cin % 64 == 0 && a.c1 % 64 == 0 && a.Cout % 64 == 0 && a.H % 8 == 0 && a.W % HW_TW == 0;
}

// Blocks per (cout, cin) group: one persistent block per CU at a time (152 KiB LDS), so the
// makespan is ceil(groups*G / 256) rounds of ceil(n_sp / G) tiles, plus the split-K reduce that
// reads G slabs.  Pick the G that minimises that estimate (tile ~1 us with 8 waves, reduce ~4 TB/s;
// A/B against the 4-wave kernel's 2 us: +0.3-0.9 %).
int halo3_wgrad_splits(const HaloWgradArgs& a) {
  const int groups = (a.Cout / 64) * (a.cin / 64);
  const int n_sp = a.N * (a.H / 8) * (a.W / HW_TW);
  const double slab = 4.0 * a.Cout * 9.0 * a.cin;
  int best = 1;
  double best_t = 1e30;
  // with the weight gradients on their own stream the makespan matters less than the slab traffic
  // the reduce adds beside the compute stream: UNETSEG_HALO_WG_MAXG caps G (experiments)
  static const int maxg = getenv("UNETSEG_HALO_WG_MAXG") ? atoi(getenv("UNETSEG_HALO_WG_MAXG")) : 512;
  // seconds per (8 x 32)-pixel tile of one block (the makespan model; UNETSEG_HALO_WG_TILE_US overrides)
  static const double tile_s = (getenv("UNETSEG_HALO_WG_TILE_US") ? atof(getenv("UNETSEG_HALO_WG_TILE_US")) : 1.0) * 1e-6;
  // with several (cout, cin) groups, the blocks of one slot in different groups walk the same spatial
  // tiles in step; G a multiple of 8 would put them on one XCD (block b runs on XCD b % 8), so a tile's
  // dY or X halo came from that XCD's L2 after the first read -- but it forces G >= 8 and with it
  // G slabs of split-K partials (the 32^2 concat conv: 453 MB written and re-read by the reduce).  Any
  // G measured better in the step (round 4, three interleaved repeats: C2 979.8 vs 976.2 img/s, C4
  // 423.5 vs 418.8, C5 783.6 vs 765.9, allocator peak 8.11 vs 8.39 GiB); UNETSEG_HALO_WG_XCD=1 restores it
  static const bool xcd = getenv("UNETSEG_HALO_WG_XCD") && atoi(getenv("UNETSEG_HALO_WG_XCD")) != 0;
  const int step = (xcd && groups > 1) ? 8 : 1;
  for (int g = step; g <= maxg && g <= n_sp; g += step) {
    if (slab * g > 768.0 * (1 << 20)) break;  // workspace cap
    const double rounds = (double)((groups * g + 255) / 256);
    const double t = rounds * ((n_sp + g - 1) / g) * tile_s + slab * g / 4e12;
    if (t < best_t * 0.999) {
      best_t = t;
      best = g;
    }
  }
  return best;
}

int launch_halo3_wgrad(const HaloWgradArgs& a, int G_per, hipStream_t st) {
  constexpr int TH = 8;
  const int tiles_w = a.W / HW_TW, tiles_h = a.H / TH;
  const int n_sp = a.N * tiles_h * tiles_w;
  const int groups = (a.Cout / 64) * (a.cin / 64);
  const size_t lds = 2 * ((size_t)TH * HW_TW + (size_t)(TH + 2) * (HW_TW + 2)) * 128;
  static const bool w4 = getenv("UNETSEG_HALO_WG_W4") != nullptr;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&halo3_wgrad_kernel<TH, 8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&halo3_wgrad_kernel<TH, 4>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  if (w4)
    hipLaunchKernelGGL((halo3_wgrad_kernel<TH, 4>), dim3(groups * G_per), dim3(256), lds, st, a, tiles_w, tiles_h,
                       n_sp, G_per);
  else
    hipLaunchKernelGGL((halo3_wgrad_kernel<TH, 8>), dim3(groups * G_per), dim3(512), lds, st, a, tiles_w, tiles_h,
                       n_sp, G_per);
  return 0;
}
