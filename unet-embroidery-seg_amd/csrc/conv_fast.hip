// Fast bf16 implicit-GEMM conv kernels for gfx950 (the hot configurations of the U-Net:
// every conv whose input channels are a multiple of 64).  See conv.hip for the GEMM views.
//
// What makes them fast relative to the generic kernels in conv.hip:
//  * operands are fetched with raw buffer loads (SRD + 32-bit voffset); a padding tap or an
//    out-of-range row gets an offset past num_records, so the hardware returns zeros: no
//    branches, no 64-bit address arithmetic in the K loop;
//  * the K loop walks (tap, 64-channel chunk) as wave-uniform scalar state: the tap offset, the
//    concat source (x1 | x2) and the weight offset are SGPR values; per row only a precomputed
//    tap-validity bitmask and a pixel index remain in VGPRs;
//  * TN: MFMA operand roles are swapped (weights = A, pixels = B) so each lane's accumulator
//    holds 4 consecutive output channels of one pixel -> 8-byte stores; 256x128 / 256x64 tiles;
//  * wgrad: pixels are consumed 32 per K step along image rows (Q % 32 == 0), so (n, p, q0) of a
//    K step is scalar; fragments come from LDS with ds_read_b64_tr_b16.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "conv_fast.h"
#include "fast_util.h"


namespace {


// ------------------------------------------------------------------------------------------
// TN (fwd / dgrad).  Tile: BM pixels x BN output channels, K step 64 channels of one tap.
// ------------------------------------------------------------------------------------------
// ST: 1 = a single K step, 2 = global loads one K step ahead, 3 = two steps ahead (two register
// sets; only where the registers fit at two waves per SIMD)
// waves per SIMD each configuration is sized for (LDS allows that many blocks per CU); caps the
// register allocation so the two-step register prefetch cannot cost occupancy
// ST == 5 (short K on one LDS stage): 128x128 at three waves per SIMD, 128x64 at four
template <int BM, int BN, int NWM, int NWN, int ST = 3>
constexpr int tn_waves_per_simd() {
  return ST == 5 ? (BN == 64 ? 4 : 3) : (BM == 64 || (BM == 128 && BN == 64)) ? 3 : 2;
}

// byte offset of the input-prologue coefficients in the TN kernel's dynamic LDS: after the operand
// stages or the epilogue's transpose tiles + stats scratch, whichever is larger
// halo-A ring (HA): 16-B chunks of one (padded) halo stage -- every wave issues the same number of
// halo DMA instructions, so the stage is rounded up to whole instructions of the block
template <int BM, int NWM, int NWN>
constexpr int kHaloChunks() {
  constexpr int NT = 64 * NWM * NWN;  // rounded to instruction pairs (issued two at a time)
  return ((BM / 32 + 2) * 34 * 8 + 2 * NT - 1) / (2 * NT) * (2 * NT);
}
template <int BM, int BN, int NWM, int NWN, int ST, int HA = 0>
constexpr size_t kPreOff() {
  constexpr size_t stages = HA ? ((size_t)2 * kHaloChunks<BM, NWM, NWN>() + (size_t)(ST - 10) * BN * 8) * 16
                               : (size_t)(ST == 1 || ST == 5 ? 1 : ST >= 13 ? ST - 10 : 2) * (BM + BN) * 8 * 16;
  constexpr size_t epi = (size_t)NWM * NWN * 64 * ((BN / NWN) * 2 + 16) + 3 * NWM * BN * 4;
  return ((stages > epi ? stages : epi) + 15) / 16 * 16;
}

// TAPS (LDS-DMA ring only): the filter has exactly TAPS = nr x ns taps, known at compile time.  The
// K loop is then unrolled over the taps and every (row, tap) gather offset is precomputed, so a K
// step issues its loads with one multiply-add per row and a scalar channel offset (the generic
// ring re-derives tap deltas, validity masks and offsets every step: ~70 VALU + ~90 SALU per step
// on the 256x128 tile, which is what held its MFMA pipe at ~45 % busy).
// PRE: the input prologue of FastTNArgs (x1 = BN input z, staged as relu(z*in_sc + in_sh) between the
// global load and the LDS store); the per-channel coefficients sit in LDS after the tile stages.
// The tile body: did = this block's linear id among gx * gy tiles (gy column tiles per row tile).
// HA (halo A operand, TAPS == 9 on the LDS-DMA ring; the value = pieces the next chunk's halo DMA is
// issued in, at taps 0, 9/HA, ..): see the K loop below.
template <int BM, int BN, int NWM, int NWN, int ST, int POST, int TAPS, bool PRE, int HA = 0>
__device__ __forceinline__ void tn_fast_body(const FastTNArgs& a, const int did, const int gx, const int gy) {
  constexpr int NT = 64 * NWM * NWN;
  constexpr int WTM = BM / NWM, WTN = BN / NWN;
  constexpr int FP = WTM / 16, FC = WTN / 16;
  constexpr int RSTEP = NT / 8;
  constexpr int A_PER = BM / RSTEP, B_PER = BN / RSTEP;
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // [2 or NS][(BM+BN)*8]
  constexpr int STAGE = (BM + BN) * 8;
  constexpr bool kDMA = ST >= 13;
  static_assert(!(PRE && kDMA), "the input prologue needs register staging");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (dispatch id d -> XCD
  // d % 8), each with its own L2.  Give every XCD a contiguous range of tiles, N tiles fastest, so
  // the N tiles of one row tile and the neighbouring row tiles (the 3x3 taps re-read them) share
  // one L2.  Bijective for any tile count.
  const int ntiles = gx * gy;
  const int xq = ntiles >> 3, xr = ntiles & 7, xcd = did & 7;
  const int lin = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (did >> 3);
  const int tile_m = lin / gy, tile_n = lin - tile_m * gy;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kv = tid & 7, rb = tid >> 3;
  const int hw = a.hc * a.wc;
  // GEMM row -> linear pixel of the (hc, wc) grid.  With a.t2d = TR, a BM-row tile is a TR x 32
  // spatial block instead of BM consecutive pixels of one image row: the nine taps then re-read
  // one (TR+2) x 34 footprint, which stays in the XCD's L2 while the chunk's taps run.
  auto row_pix = [&](int m) -> int {
    if (!a.t2d) return m;
    const int TR = a.t2d, tsz = TR * 32, tpr = a.wc >> 5;
    const int t = m / tsz, i = m - t * tsz;
    const int rest = t / tpr, tw = t - rest * tpr;
    return (rest * TR + (i >> 5)) * a.wc + (tw << 5) + (i & 31);
  };

  const __amdgpu_buffer_rsrc_t r1 = srd(a.x1, a.x1_bytes);
  const __amdgpu_buffer_rsrc_t r2 = srd(a.x2 ? a.x2 : a.x1, a.x2 ? a.x2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rw = srd(a.wt, a.w_bytes);

  int pix[A_PER];
  unsigned vmask[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int m = m0 + rb + RSTEP * i;
    pix[i] = 0;
    vmask[i] = 0u;
    if (m < a.M) {
      const int pm = row_pix(m);
      const int nb = pm / hw, rem = pm - nb * hw;
      const int hh = rem / a.wc, ww = rem - hh * a.wc;
      const int ih0 = hh * a.istride, iw0 = ww * a.istride;
      pix[i] = (nb * a.H + ih0) * a.W + iw0;
      unsigned msk = 0u;
      for (int jr = 0; jr < a.nr; ++jr) {
        const int ih = ih0 + a.dh0 + a.dhs * jr;
        if (ih < 0 || ih >= a.H) continue;
        for (int js = 0; js < a.ns; ++js) {
          const int iw = iw0 + a.dw0 + a.dws * js;
          if (iw >= 0 && iw < a.W) msk |= 1u << (jr * a.ns + js);
        }
      }
      vmask[i] = msk;
    }
  }
  unsigned boff[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int n = n0 + rb + RSTEP * i;
    // the LDS-DMA variant writes lane-linearly (slot = kv), so it fetches the chunk that slot holds
    // under the XOR swizzle instead: kv ^ ((row >> 1) & 7) (row parity is the same for every i)
    const int kvs = kDMA ? (kv ^ ((rb >> 1) & 7)) : kv;
    boff[i] = n < a.Ng ? (unsigned)n * (unsigned)a.ldwb + kvs * 16 : kOOB;
  }

  const int nch = a.cin >> 6;
  const int nsteps = a.nr * a.ns * nch;
  // two register sets: the loads of K step kt+2 are issued while step kt is computed and
  // step kt+1's registers are written to LDS, so each load has two steps of MFMA to land
  uint4 ra0[A_PER], rb0[B_PER], ra1[A_PER], rb1[B_PER];
  // scalar K-step state
  int s_jr = 0, s_js = 0, s_c = 0;
  // ---- LDS-DMA ring (ST >= 13, NS = ST - 10 stages): buffer_load ... lds straight into the stage,
  // NS - 1 K steps in flight, counted vmcnt + raw barrier (no register staging) ----
  auto gload_dma = [&](int stage, bool live) {
    const int dh = a.dh0 + a.dhs * s_jr, dw = a.dw0 + a.dws * s_js;
    const int tapbit = (s_jr * a.ns + s_js) & 31;
    const int tapdelta = dh * a.W + dw;
    const unsigned wofs = (unsigned)(((a.r0 + a.rs * s_jr) * a.S + (a.s0 + a.ss * s_js)) * a.cin + s_c) * 2u;
    const unsigned sbase = lds_addr(lds) + (unsigned)(stage * STAGE * 16) + (unsigned)(wid * 8 * 128);
    const int kvs = kv ^ ((rb >> 1) & 7);
    const bool first = s_c < a.c1;
    const unsigned cb = (unsigned)(first ? s_c : s_c - a.c1) * 2u + kvs * 16;
    const unsigned ldcb = first ? (unsigned)a.ldc1b : (unsigned)a.ldc2b;
    const __amdgpu_buffer_rsrc_t rx = first ? r1 : r2;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const bool ok = live && ((vmask[i] >> tapbit) & 1u);
      const unsigned off = ok ? (unsigned)(pix[i] + tapdelta) * ldcb + cb : kOOB;
      dma16(rx, sbase + (unsigned)(RSTEP * i * 128), off);
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      dma16(rw, sbase + (unsigned)((BM + RSTEP * i) * 128), (!live || boff[i] == kOOB) ? kOOB : boff[i] + wofs);
    if (++s_js == a.ns) {
      s_js = 0;
      if (++s_jr == a.nr) {
        s_jr = 0;
        s_c += 64;
      }
    }
  };
  // live == false (a K step past the end): every offset is out of range, so the loads return
  // zeros without touching memory.  Issuing them anyway keeps the loop free of conditional loads,
  // which lets hipcc count vmcnt exactly (with conditional loads it waits for the loads of the
  // step in flight too, exposing their latency every K step).
  auto gload = [&](uint4 (&ra)[A_PER], uint4 (&rbv)[B_PER], int& kc, bool live = true) {
    kc = s_c;  // channel base of this K step (input prologue)
    const int dh = a.dh0 + a.dhs * s_jr, dw = a.dw0 + a.dws * s_js;
    const int tapbit = (s_jr * a.ns + s_js) & 31;
    const int tapdelta = dh * a.W + dw;
    const unsigned wofs = (unsigned)(((a.r0 + a.rs * s_jr) * a.S + (a.s0 + a.ss * s_js)) * a.cin + s_c) * 2u;
    if (s_c < a.c1) {
      const unsigned cb = (unsigned)s_c * 2u + kv * 16;
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const bool ok = live && ((vmask[i] >> tapbit) & 1u);
        const unsigned off = (unsigned)(pix[i] + tapdelta) * (unsigned)a.ldc1b + cb;
        ra[i] = bload(r1, ok ? off : kOOB);
      }
    } else {
      const unsigned cb = (unsigned)(s_c - a.c1) * 2u + kv * 16;
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const bool ok = live && ((vmask[i] >> tapbit) & 1u);
        const unsigned off = (unsigned)(pix[i] + tapdelta) * (unsigned)a.ldc2b + cb;
        ra[i] = bload(r2, ok ? off : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) rbv[i] = bload(rw, (!live || boff[i] == kOOB) ? kOOB : boff[i] + wofs);
    // K order: taps fastest, 64-channel chunks outer -- the nine taps of one chunk run back to
    // back over the same input footprint (L2-resident), instead of cycling through every chunk
    if (++s_js == a.ns) {
      s_js = 0;
      if (++s_jr == a.nr) {
        s_jr = 0;
        s_c += 64;
      }
    }
  };
  // input prologue coefficients: [2][cin] floats after the operand stages / epilogue scratch
  const float* pre_l = reinterpret_cast<const float*>(lds + kPreOff<BM, BN, NWM, NWN, ST>() / 16);
  if constexpr (PRE) {
    float* w = reinterpret_cast<float*>(lds + kPreOff<BM, BN, NWM, NWN, ST>() / 16);
    for (int c = tid; c < a.c1; c += NT) {
      w[c] = a.in_sc[c];
      w[a.c1 + c] = a.in_sh[c];
    }
    __syncthreads();
  }
  auto sstore = [&](int buf, const uint4 (&ra)[A_PER], const uint4 (&rbv)[B_PER], int kc) {
    uint4* L = lds + buf * STAGE;
    float psc[8], psh[8];
    if constexpr (PRE) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        psc[e] = pre_l[kc + kv * 8 + e];
        psh[e] = pre_l[a.c1 + kc + kv * 8 + e];
      }
    }
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = rb + RSTEP * i;
      uint4 v = ra[i];
      if constexpr (PRE) {  // == bn_apply: (bf16) relu(fmaf(z, sc, sh))
        v.x = bnrelu_pair(v.x, (f32x2){psc[0], psc[1]}, (f32x2){psh[0], psh[1]});
        v.y = bnrelu_pair(v.y, (f32x2){psc[2], psc[3]}, (f32x2){psh[2], psh[3]});
        v.z = bnrelu_pair(v.z, (f32x2){psc[4], psc[5]}, (f32x2){psh[4], psh[5]});
        v.w = bnrelu_pair(v.w, (f32x2){psc[6], psc[7]}, (f32x2){psh[6], psh[7]});
      }
      L[row * 8 + swz8(row, kv)] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = rb + RSTEP * i;
      L[(BM + row) * 8 + swz8(row, kv)] = rbv[i];
    }
  };

  f32x4 acc[FC][FP];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Fragment reads: row = base + p*16 + (lane & 15) and the swizzle depends on (row >> 1) & 7, i.e.
  // on the lane alone, so each (operand, K half) has one per-lane byte offset and the p / c steps are
  // immediates (p * 16 rows * 128 B); per step only the stage base is added.
  unsigned foffA[2], foffB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15, sw = ((kk * 4 + (lane >> 4)) ^ ((r >> 1) & 7)) * 16;
    foffA[kk] = (unsigned)((wm * WTM + r) * 128 + sw);
    foffB[kk] = (unsigned)((BM + wn * WTN + r) * 128 + sw);
  }
  auto frags = [&](int buf, int kk, bf16x8 (&pf)[FP], bf16x8 (&wf)[FC]) {
    const char* sb = reinterpret_cast<const char*>(lds + buf * STAGE);
    const char* pa = sb + foffA[kk];
    const char* pb = sb + foffB[kk];
#pragma unroll
    for (int p = 0; p < FP; ++p) pf[p] = *reinterpret_cast<const bf16x8*>(pa + p * 2048);
#pragma unroll
    for (int c = 0; c < FC; ++c) wf[c] = *reinterpret_cast<const bf16x8*>(pb + c * 2048);
  };
  auto mfmas = [&](const bf16x8 (&pf)[FP], const bf16x8 (&wf)[FC]) {
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int p = 0; p < FP; ++p)
        acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], pf[p], acc[c][p], 0, 0, 0);
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 pf[FP], wf[FC];
      frags(buf, kk, pf, wf);
      mfmas(pf, wf);
    }
  };

  if constexpr (HA) {
    // ---- halo-A ring: 3x3 stride-1 "same" convolutions whose BM-row tile is a TRH x 32 spatial
    // block (a.t2d == TRH).  Per 64-channel chunk the (TRH+2) x 34 halo of the tile is LDS-DMA'd
    // ONCE (double buffered, the next chunk's halo in flight during this chunk's nine taps) and the
    // nine taps read their A fragments from it at a uniform pixel shift; only the weights stream
    // through the NS-stage ring, one tap per K step.  Per chunk that is ~43 KiB of A DMA instead of
    // 9 x 32 KiB of re-gathered tap rows: 2.3x fewer DMA instructions per MFMA than the gather ring.
    static_assert(TAPS == 9 && kDMA && !PRE && (B_PER % 2 == 0 || B_PER == 1), "halo-A ring: 3x3 taps");
    constexpr int NS = ST - 10;
    constexpr int TRH = BM / 32;
    constexpr int HPIX = (TRH + 2) * 34;
    constexpr int HST = kHaloChunks<BM, NWM, NWN>();  // 16-B chunks per halo stage (padded)
    constexpr int HI = HST / NT;                       // halo DMA instructions per wave (every wave)
    constexpr int WST = BN * 8;                        // 16-B chunks per weight stage
    constexpr int WP = B_PER;                          // weight DMA instructions per wave per K step
    static_assert(HI % 2 == 0, "halo rows are issued in pairs");
    static_assert(WP * (NS - 2) + HI <= 63, "vmcnt range");
    // the next chunk's halo goes out in HA pieces (HI / HA DMA instructions each) at taps 0, 9 / HA, ..
    constexpr int HPC = HI / HA, TPER = 9 / HA;
    static_assert(HI % (2 * HA) == 0 && 9 % HA == 0, "halo pieces of whole instruction pairs");
    // this block's spatial tile (row_pix with t2d == TRH: tiles of TRH image rows x 32 columns,
    // stacked over the images; hc % TRH == 0, so a tile never straddles two images)
    const int tpr = a.wc >> 5;
    const int tt = m0 / BM;
    const int rest = tt / tpr, twi = tt - rest * tpr;
    const int hg = rest * TRH;  // first row of the tile in the stacked (N * hc) row space
    const int nb = hg / a.hc, h0 = hg - nb * a.hc, w0 = twi * 32;
    const unsigned pb1 = a.x1_bytes / (unsigned)a.ldc1b;
    const unsigned pb2 = a.x2 ? a.x2_bytes / (unsigned)a.ldc2b : 0u;
    const unsigned pbad = (pb1 > pb2 ? pb1 : pb2) + 1u;
    // this lane's halo DMA slots: source pixel (or pbad: outside the image / past the halo) and the
    // swizzled source chunk; LDS slot (hp, lane & 7) holds chunk (lane & 7) ^ (hp & 7)
    unsigned hvp[HI], hsw[HI];
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int idx = (i * (NWM * NWN) + wid) * 64 + lane;
      const int hp = idx >> 3;
      const int hr = hp / 34, hcol = hp - hr * 34;
      const int h = h0 - 1 + hr, w = w0 - 1 + hcol;
      const bool ok = hp < HPIX && h >= 0 && h < a.H && w >= 0 && w < a.W;
      hvp[i] = ok ? (unsigned)((nb * a.H + h) * a.W + w) : pbad;
      hsw[i] = (unsigned)(((lane & 7) ^ (hp & 7)) * 16);
    }
    unsigned tw[9];  // weight byte offset of each tap
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int jr = t / 3, js = t - jr * 3;
      tw[t] = (unsigned)(((a.r0 + a.rs * jr) * a.S + (a.s0 + a.ss * js)) * a.cin) * 2u;
    }
    // A fragment p of this lane: tile pixel (row wm * WTM / 32 + p / 2, column (p & 1) * 16 + lane % 16)
    // -> halo pixel at the centre tap; a tap adds the uniform shift dh * 34 + dw
    static_assert(WTM == 64 && FP == 4, "64-row wave tiles: two image rows of 32 pixels");
    int hq[FP];
#pragma unroll
    for (int p = 0; p < FP; ++p) hq[p] = (wm * 2 + (p >> 1) + 1) * 34 + (p & 1) * 16 + (lane & 15) + 1;
    const int chA = lane >> 4;  // 16-B chunk of the first K half (the second is chA ^ 4)
    unsigned foffW[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r = lane & 15;
      foffW[kk] = (unsigned)((wn * WTN + r) * 128 + ((kk * 4 + (lane >> 4)) ^ ((r >> 1) & 7)) * 16);
    }
    const unsigned hbase = lds_addr(lds);
    const unsigned wbase = hbase + 2u * HST * 16u;
    const int nch = a.cin >> 6;
    auto issue_halo = [&](int c, int hs, int i0, int i1) {
      const bool live = c < nch;
      const int c64 = c * 64;
      const bool first = c64 < a.c1;
      const __amdgpu_buffer_rsrc_t rx = srd_u(first ? a.x1 : a.x2, !live ? 0u : first ? a.x1_bytes : a.x2_bytes);
      const unsigned ldcb = first ? (unsigned)a.ldc1b : (unsigned)a.ldc2b;
      const unsigned soff = __builtin_amdgcn_readfirstlane(live ? (unsigned)(first ? c64 : c64 - a.c1) * 2u : 0u);
      const unsigned sb = __builtin_amdgcn_readfirstlane(hbase + (unsigned)(hs * HST * 16) + (unsigned)(wid * 1024));
#pragma unroll
      for (int i = i0; i < i1; i += 2)
        dma16x2<NT * 16>(rx, sb + (unsigned)(i * NT * 16), __umul24(hvp[i], ldcb) + hsw[i],
                         __umul24(hvp[i + 1], ldcb) + hsw[i + 1], soff);
    };
    auto issue_w = [&](int c, int t, int stage) {
      const bool live = c < nch;
      const __amdgpu_buffer_rsrc_t rwx = srd_u(a.wt, live ? a.w_bytes : 0u);
      const unsigned wsoff = __builtin_amdgcn_readfirstlane(live ? tw[t] + (unsigned)(c * 64) * 2u : 0u);
      const unsigned sb = __builtin_amdgcn_readfirstlane(wbase + (unsigned)(stage * WST * 16) + (unsigned)(wid * 8 * 128));
      if constexpr (B_PER == 1) {
        dma16s(rwx, sb, boff[0], wsoff);
      } else {
#pragma unroll
        for (int i = 0; i < B_PER; i += 2)
          dma16x2<RSTEP * 128>(rwx, sb + (unsigned)(RSTEP * i * 128), boff[i], boff[i + 1], wsoff);
      }
    };
    // wait for this step's weight stage (and, at a chunk's first tap, its halo): the younger DMAs
    // still in flight are the NS-2 later weight steps plus the next chunk's halo when it was issued
    // after this step's weights (taps 1 .. NS-1 of a chunk)
    auto wait_step = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      // halo pieces issued in the NS-1 iterations since this step's weights went out (those
      // iterations' taps t-1 .. t-NS+1, mod 9)
      constexpr int n = WP * (NS - 2) + HPC * (((((t - 1) % 9 + 9) % 9) % TPER == 0 ? 1 : 0) +
                                               (NS >= 3 && ((((t - 2) % 9 + 9) % 9) % TPER == 0) ? 1 : 0) +
                                               (NS >= 4 && ((((t - 3) % 9 + 9) % 9) % TPER == 0) ? 1 : 0) +
                                               (NS >= 5 && ((((t - 4) % 9 + 9) % 9) % TPER == 0) ? 1 : 0));
      static_assert(NS <= 5, "wait count");
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(n) : "memory");
    };
    issue_halo(0, 0, 0, HI);
#pragma unroll
    for (int s0 = 0; s0 < NS - 1; ++s0) issue_w(s0 / 9, s0 % 9, s0);
    int stage = 0;
    for (int c = 0; c < nch; ++c) {
      const char* hs = reinterpret_cast<const char*>(lds) + (c & 1) * HST * 16;
      auto step = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        wait_step(tc);
        const int jr = t / 3, js = t - jr * 3;
        const int shift = (a.dh0 + a.dhs * jr) * 34 + (a.dw0 + a.dws * js);
        unsigned ab[FP];
#pragma unroll
        for (int p = 0; p < FP; ++p) {
          const int hp = hq[p] + shift;
          ab[p] = (unsigned)(hp * 128 + ((chA ^ (hp & 7)) * 16));
        }
        const char* ws = reinterpret_cast<const char*>(lds) + 2 * HST * 16 + stage * WST * 16;
        bf16x8 pf[FP], wf[FC];
#pragma unroll
        for (int p = 0; p < FP; ++p) pf[p] = *reinterpret_cast<const bf16x8*>(hs + ab[p]);
#pragma unroll
        for (int cc = 0; cc < FC; ++cc) wf[cc] = *reinterpret_cast<const bf16x8*>(ws + foffW[0] + cc * 2048);
        const int st2 = stage == 0 ? NS - 1 : stage - 1;  // (stage + NS - 1) % NS
        issue_w(c + (t + NS - 1) / 9, (t + NS - 1) % 9, st2);
        if constexpr (t % TPER == 0) issue_halo(c + 1, (c + 1) & 1, (t / TPER) * HPC, (t / TPER + 1) * HPC);
        mfmas(pf, wf);
#pragma unroll
        for (int p = 0; p < FP; ++p) pf[p] = *reinterpret_cast<const bf16x8*>(hs + (ab[p] ^ 64u));
#pragma unroll
        for (int cc = 0; cc < FC; ++cc) wf[cc] = *reinterpret_cast<const bf16x8*>(ws + foffW[1] + cc * 2048);
        mfmas(pf, wf);
        stage = stage == NS - 1 ? 0 : stage + 1;
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
      step(std::integral_constant<int, 4>{});
      step(std::integral_constant<int, 5>{});
      step(std::integral_constant<int, 6>{});
      step(std::integral_constant<int, 7>{});
      step(std::integral_constant<int, 8>{});
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else if constexpr (kDMA && TAPS > 0) {
    constexpr int NS = ST - 10, PER = A_PER + B_PER;
    static_assert(NS >= 3 && PER * (NS - 2) <= 63, "vmcnt range");
    static_assert(A_PER % 2 == 0 && (B_PER % 2 == 0 || B_PER == 1), "rows are issued in pairs");
    // (row, tap) -> gather pixel, or pbad: one past every source's last pixel, so pbad * ldcb is
    // out of range for either source (the launcher checks it cannot wrap 32 bits)
    const unsigned pb1 = a.x1_bytes / (unsigned)a.ldc1b;
    const unsigned pb2 = a.x2 ? a.x2_bytes / (unsigned)a.ldc2b : 0u;
    const unsigned pbad = (pb1 > pb2 ? pb1 : pb2) + 1u;
    unsigned vpix[A_PER][TAPS];
    unsigned tw[TAPS];  // weight byte offset of each tap
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const int jr = t / a.ns, js = t - jr * a.ns;
      const int tapdelta = (a.dh0 + a.dhs * jr) * a.W + a.dw0 + a.dws * js;
      tw[t] = (unsigned)(((a.r0 + a.rs * jr) * a.S + (a.s0 + a.ss * js)) * a.cin) * 2u;
#pragma unroll
      for (int i = 0; i < A_PER; ++i) vpix[i][t] = ((vmask[i] >> t) & 1u) ? (unsigned)(pix[i] + tapdelta) : pbad;
    }
    const unsigned kv16 = (unsigned)(kv ^ ((rb >> 1) & 7)) * 16u;
    const unsigned lbase = lds_addr(lds) + (unsigned)(wid * 8 * 128);
    const int nch = a.cin >> 6;
    // issue K step (chunk c, tap t) into stage `stage`; a chunk past the end loads through
    // zero-extent descriptors (zeros, no memory traffic) so every step issues PER loads
    auto issue = [&](int c, int t, int stage) {
      const bool live = c < nch;
      const int c64 = c * 64;
      const bool first = c64 < a.c1;
      // wave-uniform by construction; readfirstlane keeps them in SGPRs for the asm operands
      const __amdgpu_buffer_rsrc_t rx = srd_u(first ? a.x1 : a.x2, !live ? 0u : first ? a.x1_bytes : a.x2_bytes);
      const __amdgpu_buffer_rsrc_t rwx = srd_u(a.wt, live ? a.w_bytes : 0u);
      const unsigned ldcb = first ? (unsigned)a.ldc1b : (unsigned)a.ldc2b;
      const unsigned soff = __builtin_amdgcn_readfirstlane(live ? (unsigned)(first ? c64 : c64 - a.c1) * 2u : 0u);
      const unsigned wsoff = __builtin_amdgcn_readfirstlane(live ? tw[t] + (unsigned)c64 * 2u : 0u);
      const unsigned sb = __builtin_amdgcn_readfirstlane(lbase + (unsigned)(stage * STAGE * 16));
#pragma unroll
      for (int i = 0; i < A_PER; i += 2)
        dma16x2<RSTEP * 128>(rx, sb + (unsigned)(RSTEP * i * 128), __umul24(vpix[i][t], ldcb) + kv16,
                             __umul24(vpix[i + 1][t], ldcb) + kv16, soff);
      if constexpr (B_PER == 1) {
        dma16s(rwx, sb + (unsigned)(BM * 128), boff[0], wsoff);
      } else {
#pragma unroll
        for (int i = 0; i < B_PER; i += 2)
          dma16x2<RSTEP * 128>(rwx, sb + (unsigned)((BM + RSTEP * i) * 128), boff[i], boff[i + 1], wsoff);
      }
    };
#pragma unroll
    for (int s0 = 0; s0 < NS - 1; ++s0) issue(s0 / TAPS, s0 % TAPS, s0);
    int stage = 0;
    // DMA issue costs the issuing wave tens of cycles per instruction; right after the barrier every
    // wave would issue at once and leave the MFMA pipes idle.  With sched bit 0 the waves sharing a
    // SIMD (w and w + 4 of 8) split: one issues before its first K half, the other after it.
    const bool late = (a.sched & 1) && NWM * NWN == 8 && ((wid >> 2) & 1);
    for (int c = 0; c < nch; ++c) {
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PER * (NS - 2)) : "memory");
        bf16x8 pf[FP], wf[FC];
        frags(stage, 0, pf, wf);  // first fragments in flight while this step's loads issue
        const int st2 = stage == 0 ? NS - 1 : stage - 1;  // (stage + NS - 1) % NS
        if (!late) issue(c + (t + NS - 1) / TAPS, (t + NS - 1) % TAPS, st2);
        mfmas(pf, wf);
        frags(stage, 1, pf, wf);
        if (late) issue(c + (t + NS - 1) / TAPS, (t + NS - 1) % TAPS, st2);
        mfmas(pf, wf);
        stage = stage == NS - 1 ? 0 : stage + 1;
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else if constexpr (kDMA) {
    constexpr int NS = ST - 10, PER = A_PER + B_PER;
    static_assert(NS >= 3 && PER * (NS - 2) <= 63, "vmcnt range");
#pragma unroll
    for (int s0 = 0; s0 < NS - 1; ++s0) gload_dma(s0, s0 < nsteps);
    for (int kt = 0; kt < nsteps; ++kt) {
      // this wave's DMAs of step kt have landed (the NS-2 younger steps stay in flight), this
      // wave's LDS reads of step kt-1 are done; the barrier makes both true for every wave
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PER * (NS - 2)) : "memory");
      gload_dma((kt + NS - 1) % NS, kt + NS - 1 < nsteps);  // refills the stage read at kt-1
      compute(kt % NS);
    }
    // every DMA (past-the-end ones write zeros) has landed before the epilogue reuses the LDS
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else if (ST == 1) {  // one K step
    int kc0 = 0;
    if (nsteps > 0) {
      gload(ra0, rb0, kc0);
      sstore(0, ra0, rb0, kc0);
      __syncthreads();
      compute(0);
    }
    __syncthreads();
  } else if (ST == 5) {
    // short K (<= 4 steps) on ONE LDS stage: the next step's loads are in registers while this step
    // computes; two barriers per step.  The single stage (32 / 24 KiB) and the one register set let
    // 3-4 blocks share a CU, which is what hides the HBM latency of these memory-bound layers.
    int kc0 = 0;
    if (nsteps > 0) {
      gload(ra0, rb0, kc0);
      sstore(0, ra0, rb0, kc0);
      __syncthreads();
    }
    for (int kt = 0; kt < nsteps; ++kt) {
      const bool more = kt + 1 < nsteps;
      if (more) gload(ra0, rb0, kc0);
      compute(0);
      __syncthreads();
      if (more) {
        sstore(0, ra0, rb0, kc0);
        __syncthreads();
      }
    }
  } else if (ST == 2) {  // loads one step ahead (one register set)
    int kc0 = 0;
    if (nsteps > 0) {
      gload(ra0, rb0, kc0);
      sstore(0, ra0, rb0, kc0);
      __syncthreads();
    }
    for (int kt = 0; kt < nsteps; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nsteps) gload(ra0, rb0, kc0);
      compute(cur);
      if (kt + 1 < nsteps) sstore(cur ^ 1, ra0, rb0, kc0);
      __syncthreads();
    }
  } else {  // ST == 3: loads two steps ahead (two register sets)
    // Loads and LDS stores are unconditional inside the loop (past-the-end steps load zeros), so
    // the in-order vmcnt bookkeeping is the same on every path: each sstore waits only for the
    // register set it writes, while the set issued in the same half stays in flight.
    int kc0 = 0, kc1 = 0;
    if (nsteps > 0) {
      gload(ra0, rb0, kc0);
      sstore(0, ra0, rb0, kc0);
      gload(ra1, rb1, kc1, nsteps > 1);
      __syncthreads();
    }
    for (int kt = 0; kt < nsteps; kt += 2) {
      // even step: stage 0 holds kt, registers 1 hold kt+1 (in flight)
      gload(ra0, rb0, kc0, kt + 2 < nsteps);
      compute(0);
      sstore(1, ra1, rb1, kc1);
      __syncthreads();
      if (kt + 1 >= nsteps) break;
      // odd step: stage 1 holds kt+1, registers 0 hold kt+2 (in flight)
      gload(ra1, rb1, kc1, kt + 3 < nsteps);
      compute(1);
      sstore(0, ra0, rb0, kc0);
      __syncthreads();
    }
  }

  // ---- epilogue: lane holds D[cout = (lane>>4)*4 + e][pixel = lane&15] per (c, p) subtile ----
  // bias + ReLU + bf16 rounding in registers; per-wave BN partials (sum, M2 about the wave's
  // mean) by shuffles; each wave transposes its WTM x WTN tile through LDS (the operand stages are
  // free after the K loop's last barrier) and writes whole 16-B chunks of each pixel's channel
  // run; finally one barrier and a Chan merge of the row-waves' partials per output channel.
  static_assert(WTM == 64, "64 rows per wave");
  const int kg = lane >> 4, j16 = lane & 15;
  const int row0 = m0 + wm * WTM;
  const int cnt = min(WTM, a.M - row0);
  constexpr int LROW = WTN * 2 + 16;  // bytes per LDS row (padded: conflict-free 8-B writes)
  char* tl = reinterpret_cast<char*>(lds) + wid * (WTM * LROW);
  // per-wave (sum, M2) of the stats / post-op partials, after every wave's transpose tile: [2 or 3][NWM][BN]
  float* red = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + NWM * NWN * WTM * LROW);

  float csum[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[c][e] = 0.f;
  float bias[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c) {
    const int nb = n0 + wn * WTN + c * 16 + kg * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[c][e] = (a.bias && nb + e < a.Ng) ? a.bias[nb + e] : 0.f;
  }
  auto out_pix = [&](int m0_) -> long {
    const int m = row_pix(m0_);
    if (a.ostride == 1 && a.ph == 0 && a.pw == 0 && a.OW == a.wc && a.OH == a.hc) return m;
    const int nb = m / hw, rem = m - nb * hw;
    const int hh = rem / a.wc, ww = rem - hh * a.wc;
    return ((long)nb * a.OH + hh * a.ostride + a.ph) * a.OW + ww * a.ostride + a.pw;
  };
  // post-op aux values, loaded first so their latency overlaps the rounding pass
  uint2 zr[FC][FP];
  if (POST == 1) {
#pragma unroll
    for (int c = 0; c < FC; ++c) {
      const int nb = n0 + wn * WTN + c * 16 + kg * 4;
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const bool ok = nb < a.Ng && p * 16 + j16 < cnt;
        zr[c][p] = ok ? *reinterpret_cast<const uint2*>((const bf16*)a.aux + out_pix(row0 + p * 16 + j16) * a.ld_aux + nb)
                      : uint2{0u, 0u};
      }
    }
  }
#pragma unroll
  for (int p = 0; p < FP; ++p) {
    const bool mok = p * 16 + j16 < cnt;
#pragma unroll
    for (int c = 0; c < FC; ++c) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[c][p][e] + bias[c][e];
        if (a.relu) v = fmaxf(v, 0.f);
        acc[c][p][e] = mok ? (float)(bf16)v : 0.f;  // BN statistics are of the stored (rounded) values
        csum[c][e] += acc[c][p][e];
      }
    }
  }
  if (POST == 1) {
    // mask the rounded gradient with the producer's ReLU (recomputed from aux) and reduce its
    // backward partials over the wave's rows: q0 = sum d, q1 = sum d * xhat (BN) (one reduction chain
    // pair at a time: row16_sum_n over a channel group's 8 spills in the 5-stage 128x128 tile)
#pragma unroll
    for (int c = 0; c < FC; ++c) {
      const int nb = n0 + wn * WTN + c * 16 + kg * 4;
      const bool nok = nb < a.Ng;
      float sc4[4], sh4[4], mu4[4], iv4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool bn = a.post == 2 && nok;
        sc4[e] = bn ? a.psc[nb + e] : 0.f;
        sh4[e] = bn ? a.psh[nb + e] : 0.f;
        mu4[e] = bn ? a.pmean[nb + e] : 0.f;
        iv4[e] = bn ? a.pinv[nb + e] : 0.f;
      }
      float q0[4] = {0.f, 0.f, 0.f, 0.f}, q1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const bf16* z = reinterpret_cast<const bf16*>(&zr[c][p]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float zf = (float)z[e];
          const bool on = a.post == 2 ? fmaf(zf, sc4[e], sh4[e]) > 0.f : zf > 0.f;
          const float d = on ? acc[c][p][e] : 0.f;
          acc[c][p][e] = d;
          q0[e] += d;
          q1[e] += d * ((zf - mu4[e]) * iv4[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t0 = row16_sum(q0[e]), t1 = row16_sum(q1[e]);
        if (j16 == 0) {
          const int col = wn * WTN + c * 16 + kg * 4 + e;
          red[wm * BN + col] = t0;
          red[(NWM + wm) * BN + col] = t1;
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < FP; ++p)
#pragma unroll
    for (int c = 0; c < FC; ++c) {
      bf16 ob[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) ob[e] = (bf16)acc[c][p][e];  // exact: acc holds rounded values
      *reinterpret_cast<uint2*>(tl + (p * 16 + j16) * LROW + (c * 16 + kg * 4) * 2) = *reinterpret_cast<uint2*>(ob);
    }
  if (a.stats) {
    // (sum, M2 about the wave mean) of each of the lane's FC * 4 channels over the wave's rows; the
    // row reductions run together (row16_sum_n)
    float sv[FC * 4], qv[FC * 4];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) sv[c * 4 + e] = csum[c][e];
    row16_sum_n(sv);
    const float inv_cnt = 1.0f / (float)max(cnt, 1);
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float mean = sv[c * 4 + e] * inv_cnt;
        float q = 0.f;
#pragma unroll
        for (int p = 0; p < FP; ++p)
          if (p * 16 + j16 < cnt) {
            const float d = acc[c][p][e] - mean;
            q += d * d;
          }
        qv[c * 4 + e] = q;
      }
    row16_sum_n(qv);
    if (j16 == 0)
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wn * WTN + c * 16 + kg * 4 + e;
          red[wm * BN + col] = sv[c * 4 + e];
          red[(NWM + wm) * BN + col] = qv[c * 4 + e];
        }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS tile is written
  __builtin_amdgcn_wave_barrier();
  // coalesced write-out: lane -> (pixel row r = i*(64/CPR) + lane/CPR, 16-B chunk lane%CPR)
  constexpr int CPR = WTN / 8;          // 16-B chunks per pixel row of the wave tile
  constexpr int RPI = 64 / CPR;         // rows per store instruction
  const int ck = lane % CPR, rsub = lane / CPR;
  const int nc = n0 + wn * WTN + ck * 8;
  // post 3 (residual-BN backward) on the transposed tile, 8 channels x this lane's rows: d = mask *
  // bf16(dgrad + the residual gradient already in y); q0 = sum d, q1 = sum d * xhat1 [, q2 = .. xhat2]
  constexpr int NQ3 = POST == 3 ? 8 : 1;
  float q3[3][NQ3], mu3[2][NQ3], iv3[2][NQ3];
  const bool two = POST == 3 && a.aux2 != nullptr;
  if constexpr (POST == 3) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = nc + e < a.Ng;
      q3[0][e] = q3[1][e] = q3[2][e] = 0.f;
      mu3[0][e] = ok ? a.pmean[nc + e] : 0.f;
      iv3[0][e] = ok ? a.pinv[nc + e] : 0.f;
      mu3[1][e] = (ok && two) ? a.pmean2[nc + e] : 0.f;
      iv3[1][e] = (ok && two) ? a.pinv2[nc + e] : 0.f;
    }
  }
  // the write-out's global reads (the old gradient; post 3: y3 / y_ds and the mask byte) of GRP rows
  // are issued together before their stores: the stores may alias them as far as the compiler knows,
  // so loads left inside the row loop would each wait out a full memory round trip (vmcnt also counts
  // the preceding stores) -- eight serial HBM latencies per tile in these short-K layers.  Post 3 in
  // groups of four rows (its 13 registers per row beside the partials and coefficients would spill).
  constexpr int NIT = WTM / RPI;
  constexpr int GRP = (POST == 3 && NIT > 4) ? 4 : NIT;
  static_assert(NIT % GRP == 0, "row groups");
#pragma unroll
  for (int g0 = 0; g0 < NIT; g0 += GRP) {
    uint4 oldv[GRP], zv[POST == 3 ? GRP : 1], z2v[POST == 3 ? GRP : 1];
    unsigned mkv[POST == 3 ? GRP : 1];
    if (POST == 3 || a.accumulate) {
      // every load unconditional, at a valid address for the lanes whose row / chunk is absent (this
      // wave's first row, or the last row M - 1 when the wave has none -- the last tile's second
      // row-wave can start past M; the last chunk; their values are never used): a load under the lane
      // condition had its value moved across the branch and was waited on by itself -- GRP serial
      // round trips
      const bf16* aux2p = two ? (const bf16*)a.aux2 : (const bf16*)a.aux;
      const long ld2 = two ? a.ld_aux2 : a.ld_aux;
      const int ncl = nc < a.Ng ? nc : a.Ng - 8;
#pragma unroll
      for (int j = 0; j < GRP; ++j) {
        const int r = (g0 + j) * RPI + rsub;
        const long opx = out_pix(r < cnt ? row0 + r : min(row0, a.M - 1));
        oldv[j] = *reinterpret_cast<const uint4*>((const bf16*)a.y + opx * a.ldy + ncl);
        if constexpr (POST == 3) {
          zv[j] = *reinterpret_cast<const uint4*>((const bf16*)a.aux + opx * a.ld_aux + ncl);
          z2v[j] = *reinterpret_cast<const uint4*>(aux2p + opx * ld2 + ncl);
          mkv[j] = (unsigned)a.mbits[opx * (a.Ng >> 3) + (ncl >> 3)];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < GRP; ++j) {
      const int r = (g0 + j) * RPI + rsub;
      if (r >= cnt || nc >= a.Ng) continue;
      const long opx = out_pix(row0 + r);
      bf16* ptr = (bf16*)a.y + opx * a.ldy + nc;
      uint4 v = *reinterpret_cast<const uint4*>(tl + r * LROW + ck * 16);
      if constexpr (POST == 3) {
        const uint4 old = oldv[j], z = zv[j], z2 = z2v[j];
        const unsigned mk = mkv[j];
        const bf16* ob = reinterpret_cast<const bf16*>(&old);
        const bf16* zb = reinterpret_cast<const bf16*>(&z);
        const bf16* z2b = reinterpret_cast<const bf16*>(&z2);
        bf16* nv = reinterpret_cast<bf16*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bf16 sm = (bf16)((float)nv[e] + (float)ob[e]);  // == the accumulating store
          const float d = ((mk >> e) & 1u) ? (float)sm : 0.f;
          nv[e] = (bf16)d;
          q3[0][e] += d;
          q3[1][e] = fmaf(d, ((float)zb[e] - mu3[0][e]) * iv3[0][e], q3[1][e]);
          if (two) q3[2][e] = fmaf(d, ((float)z2b[e] - mu3[1][e]) * iv3[1][e], q3[2][e]);
        }
      } else if (a.accumulate) {  // dx += dgrad (two bf16 tensors summed in fp32, like autograd's accumulation)
        const uint4 old = oldv[j];
        const bf16* ob = reinterpret_cast<const bf16*>(&old);
        bf16* nv = reinterpret_cast<bf16*>(&v);
#pragma unroll
        for (int e = 0; e < 8; ++e) nv[e] = (bf16)((float)nv[e] + (float)ob[e]);
      }
      *reinterpret_cast<uint4*>(ptr) = v;
    }
  }
  if constexpr (POST == 3) {
    // sum over the lanes of this chunk column (same ck), then one lane per chunk writes the wave's
    // partials of its 8 channels to red[q][NWM][BN]
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        for (int o = CPR; o < 64; o <<= 1) q3[q][e] += __shfl_xor(q3[q][e], o, 64);
    if (rsub == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = wn * WTN + ck * 8 + e;
        red[wm * BN + col] = q3[0][e];
        red[(NWM + wm) * BN + col] = q3[1][e];
        red[(2 * NWM + wm) * BN + col] = q3[2][e];
      }
    }
  }
  if (POST) {
    // plain sums of the NWM row-waves' partials -> ppart[tile_m][nq][Ng] (nq = 3 with a second
    // residual branch, else 2)
    const int nq = (POST == 3 && a.aux2) ? 3 : 2;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int col = tid; col < BN; col += NT) {
      const int n = n0 + col;
      if (n >= a.Ng) continue;
      float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < NWM; ++w) {
        t0 += red[w * BN + col];
        t1 += red[(NWM + w) * BN + col];
        if (POST == 3) t2 += red[(2 * NWM + w) * BN + col];
      }
      a.ppart[(long)tile_m * nq * a.Ng + n] = t0;
      a.ppart[(long)tile_m * nq * a.Ng + a.Ng + n] = t1;
      if (nq == 3) a.ppart[(long)tile_m * nq * a.Ng + 2 * a.Ng + n] = t2;
    }
  }
  if (a.stats) {
    // Chan merge of the NWM row-wave partials -> one (sum, M2) per block row tile (BM rows),
    // written contiguously: stats[tile_m][2][Ng].  Raw barrier: LDS visibility only -- a
    // __syncthreads() would also wait for this block's output stores to retire.
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int col = tid; col < BN; col += NT) {
      const int n = n0 + col;
      if (n >= a.Ng) continue;
      float st = 0.f, nt = 0.f;
#pragma unroll
      for (int w = 0; w < NWM; ++w) {
        st += red[w * BN + col];
        nt += (float)max(0, min(WTM, a.M - (m0 + w * WTM)));
      }
      const float mean = st / fmaxf(nt, 1.f);
      float q = 0.f;
#pragma unroll
      for (int w = 0; w < NWM; ++w) {
        const float nw = (float)max(0, min(WTM, a.M - (m0 + w * WTM)));
        if (nw > 0.f) {
          const float d = red[w * BN + col] / nw - mean;
          q += red[(NWM + w) * BN + col] + nw * d * d;
        }
      }
      a.stats[(long)tile_m * 2 * a.Ng + n] = st;
      a.stats[(long)tile_m * 2 * a.Ng + a.Ng + n] = q;
    }
  }
}

template <int BM, int BN, int NWM, int NWN, int ST, int POST, int TAPS = 0, bool PRE = false, int HA = 0>
__global__ __launch_bounds__(64 * NWM * NWN, (tn_waves_per_simd<BM, BN, NWM, NWN, ST>())) void tn_fast_kernel(FastTNArgs a) {
  tn_fast_body<BM, BN, NWM, NWN, ST, POST, TAPS, PRE, HA>(a, blockIdx.x + gridDim.x * blockIdx.y, gridDim.x, gridDim.y);
}

// Several independent GEMMs of one configuration in one launch: the output-parity classes of a
// stride-2 data gradient (conv.hip dgrad_classes; 4 / 2 / 2 / 1 taps, a few hundred tiles each),
// which launched one after another left the chip mostly idle.  Blocks [start[k], start[k+1]) run
// GEMM k as its own gx[k] x gy[k] grid.
struct TNMulti {
  FastTNArgs c[4];
  int start[5];
  int gx[4], gy[4];
  int n;
};

template <int BM, int BN, int NWM, int NWN, int ST, int POST>
__global__ __launch_bounds__(64 * NWM * NWN, (tn_waves_per_simd<BM, BN, NWM, NWN>())) void tn_multi_kernel(TNMulti m) {
  const int b = blockIdx.x;
  int k = 0;
  while (k + 1 < m.n && b >= m.start[k + 1]) ++k;
  tn_fast_body<BM, BN, NWM, NWN, ST, POST, 0, false>(m.c[k], b - m.start[k], m.gx[k], m.gy[k]);
}

// ------------------------------------------------------------------------------------------
// Persistent halo-A ring (round 6).  The halo-A ring above runs one 256-row tile per block: each
// tile's prologue (its first chunk's halo + the first weight stages: an exposed HBM / L2 round trip)
// and its epilogue (the transpose through LDS, one barrier, the 64 KiB write-out) sit outside the
// MFMA loop, and at one block per CU nothing hides them -- the short-K 3x3 layers (2-4 chunks of 64
// channels: the decoder's conv2 forwards, the concat data gradients) ran at 34-40 % of the MFMA peak.
// Here a block runs T consecutive tiles (T * grid >= tiles; the dispatcher still balances whole
// blocks) as ONE pipeline over (tile, chunk, tap):
//  * the next chunk's halo -- at a tile's last chunk, the NEXT TILE's first chunk -- goes out in HA
//    pieces during the current chunk's taps, and the weight ring runs on across the tile boundary
//    (9 taps per chunk, 3 stages: a tap's weight stage is tap % 3 on every chunk);
//  * the epilogue is register-direct: each lane stores its fragments (4 output channels of one
//    pixel, 8 B) with buffer stores straight from the accumulators, so no LDS is needed and the
//    next tile's first halo + weight stages stay in flight through it; BN statistics / post-op
//    partials go through a 4 KiB `red` scratch;
//  * the post-op aux values of a tile (post 1 / 2) are loaded at its epilogue; bias and post-2
//    coefficients sit in LDS (no compiler-tracked global load in the loop: hipcc would wait vmcnt(0)
//    for it and drain the DMA pipeline).
// Every wave issues the same vector-memory operations in the same order (out-of-range lanes and dead
// steps go through zero-extent descriptors / kOOB offsets), so every wait is a compile-time count:
// the ops younger than the awaited weight stage (see wait_at).  Requires: 3x3 stride-1 pad-1, output
// grid == input grid, hc % 8 == 0, wc % 32 == 0 (every tile full), no input prologue.
template <int BN, int NWN>
constexpr size_t kPersistLds() {
  constexpr int HST = kHaloChunks<256, 4, NWN>();
  return (size_t)2 * HST * 16 + (size_t)3 * BN * 8 * 16 + (size_t)2 * 4 * BN * 4;  // halo x2, weights x3, red
}

template <int BN, int NWN, int POST, int HA>
__global__ __launch_bounds__(512, 2) void tn_halo_persist_kernel(FastTNArgs a, int T, int ntiles, unsigned y_bytes) {
  constexpr int BM = 256, NWM = 4, NT = 512, NS = 3;
  constexpr int WTN = BN / NWN, FP = 4, FC = WTN / 16;
  constexpr int RSTEP = NT / 8;
  constexpr int B_PER = BN / RSTEP;
  static_assert(B_PER == 1 || B_PER == 2, "weight rows per thread");
  constexpr int HST = kHaloChunks<BM, NWM, NWN>();
  constexpr int HI = HST / NT;
  constexpr int HPIX = 10 * 34;
  constexpr int WST = BN * 8;
  constexpr int WP = B_PER;                 // weight DMA instructions per wave per step
  constexpr int HPC = HI / HA, TPER = 9 / HA;
  static_assert(HI % (2 * HA) == 0 && 9 % HA == 0, "halo pieces of whole instruction pairs");
  // per-wave vector-memory operations outside the DMA stream: the epilogue's stores
  constexpr int NST = FC * FP;              // output stores
  static_assert(WP + 2 * HPC + NST + 2 <= 63, "vmcnt range");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  const int kv = tid & 7, rb = tid >> 3;
  const int kg = lane >> 4, j16 = lane & 15;
  const int gy = (a.Ng + BN - 1) / BN;
  const int tpr = a.wc >> 5;
  const int nch = a.cin >> 6;

  // LDS: [halo stage 0][halo stage 1][weight stages 0..2][red 2 x NWM x BN floats][bias | post coeffs]
  const unsigned hbase = lds_addr(lds);
  const unsigned wbase = hbase + 2u * HST * 16u;
  float* red = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + 2 * HST * 16 + 3 * WST * 16);
  float* xco = red + 2 * NWM * BN;  // bias [Ng] (fwd) or sc / sh / mean / inv [4][Ng] (post 2)
  const bool has_bias = a.bias != nullptr;
  if (has_bias)
    for (int c = tid; c < a.Ng; c += NT) xco[c] = a.bias[c];
  if (POST && a.post == 2)
    for (int c = tid; c < a.Ng; c += NT) {
      xco[c] = a.psc[c];
      xco[a.Ng + c] = a.psh[c];
      xco[2 * a.Ng + c] = a.pmean[c];
      xco[3 * a.Ng + c] = a.pinv[c];
    }
  __syncthreads();

  // this block's tiles: XCD-contiguous block order (dispatch id d runs on XCD d % 8), T tiles each,
  // output-channel tiles fastest
  const int nbk = gridDim.x, b = blockIdx.x;
  const int xq = nbk >> 3, xr = nbk & 7, xcd = b & 7;
  const int lb = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (b >> 3);
  const int tfirst = lb * T;
  const int tcount = max(0, min(T, ntiles - tfirst));

  const unsigned pb1 = a.x1_bytes / (unsigned)a.ldc1b;
  const unsigned pb2 = a.x2 ? a.x2_bytes / (unsigned)a.ldc2b : 0u;
  const unsigned pbad = (pb1 > pb2 ? pb1 : pb2) + 1u;
  // halo slot i of this lane is halo pixel hp = (i * 8 + wid) * 8 + lane / 8, chunk lane % 8: the LDS
  // slot (hp, lane & 7) holds source chunk (lane & 7) ^ (hp & 7), and hp & 7 = (lane >> 3) & 7 for every i
  const unsigned hsw = (unsigned)(((lane & 7) ^ ((lane >> 3) & 7)) * 16);
  const int kvs16 = (kv ^ ((rb >> 1) & 7)) * 16;
  // a tile: (row tile, first output channel, image, first row, first column), all wave-uniform
  struct Tile {
    int tm, n0, nb, h0, w0;
  };
  auto tile_of = [&](int j) -> Tile {
    const int tl = tfirst + j;
    Tile t;
    t.tm = tl / gy;
    t.n0 = (tl - t.tm * gy) * BN;
    const int rest = t.tm / tpr, twi = t.tm - rest * tpr;
    const int hg = rest * 8;
    t.nb = hg / a.hc;
    t.h0 = hg - t.nb * a.hc;
    t.w0 = twi * 32;
    return t;
  };
  // source pixel of halo slot i of tile t (pbad: outside the image or past the halo) -- computed at
  // issue time instead of held in registers
  auto halo_pix = [&](const Tile& t, int i) -> unsigned {
    const int hp = (i * (NWM * NWN) + wid) * 8 + (lane >> 3);
    const int hr = hp / 34, hc = hp - hr * 34;
    const int h = t.h0 - 1 + hr, w = t.w0 - 1 + hc;
    const bool ok = hp < HPIX && h >= 0 && h < a.H && w >= 0 && w < a.W;
    return ok ? (unsigned)((t.nb * a.H + h) * a.W + w) : pbad;
  };
  auto wrow = [&](const Tile& t, int i) -> unsigned {
    const int n = t.n0 + rb + RSTEP * i;
    return n < a.Ng ? (unsigned)n * (unsigned)a.ldwb + kvs16 : kOOB;
  };
  unsigned tw[9];  // weight byte offset of each tap
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int jr = t / 3, js = t - jr * 3;
    tw[t] = (unsigned)(((a.r0 + a.rs * jr) * a.S + (a.s0 + a.ss * js)) * a.cin) * 2u;
  }
  int hq[FP];
#pragma unroll
  for (int p = 0; p < FP; ++p) hq[p] = (wm * 2 + (p >> 1) + 1) * 34 + (p & 1) * 16 + j16 + 1;
  const int chA = kg;
  unsigned foffW[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = j16;
    foffW[kk] = (unsigned)((wn * WTN + r) * 128 + ((kk * 4 + kg) ^ ((r >> 1) & 7)) * 16);
  }
  // halo pieces [i0, i1) of chunk cc of the tile whose halo pixels are v, into halo stage hs
  auto issue_halo = [&](const Tile& tt, bool live, int cc, int hs, int i0, int i1) {
    const int c64 = cc * 64;
    const bool first = c64 < a.c1;
    const __amdgpu_buffer_rsrc_t rx = srd_u(first ? a.x1 : a.x2, !live ? 0u : first ? a.x1_bytes : a.x2_bytes);
    const unsigned ldcb = first ? (unsigned)a.ldc1b : (unsigned)a.ldc2b;
    const unsigned soff = __builtin_amdgcn_readfirstlane(live ? (unsigned)(first ? c64 : c64 - a.c1) * 2u : 0u);
    const unsigned sb = __builtin_amdgcn_readfirstlane(hbase + (unsigned)(hs * HST * 16) + (unsigned)(wid * 1024));
#pragma unroll
    for (int i = i0; i < i1; i += 2)
      dma16x2<NT * 16>(rx, sb + (unsigned)(i * NT * 16), __umul24(halo_pix(tt, i), ldcb) + hsw,
                       __umul24(halo_pix(tt, i + 1), ldcb) + hsw, soff);
  };
  auto issue_w = [&](const Tile& tt, bool live, int cc, int t, int stage) {
    const __amdgpu_buffer_rsrc_t rwx = srd_u(a.wt, live ? a.w_bytes : 0u);
    const unsigned wsoff = __builtin_amdgcn_readfirstlane(live ? tw[t] + (unsigned)(cc * 64) * 2u : 0u);
    const unsigned sb = __builtin_amdgcn_readfirstlane(wbase + (unsigned)(stage * WST * 16) + (unsigned)(wid * 8 * 128));
    if constexpr (B_PER == 1) {
      dma16s(rwx, sb, wrow(tt, 0), wsoff);
    } else {
      dma16x2<RSTEP * 128>(rwx, sb, wrow(tt, 0), wrow(tt, 1), wsoff);
    }
  };
  constexpr auto P_ = [](int t) { return ((((t % 9) + 9) % 9) % TPER == 0) ? HPC : 0; };

  const __amdgpu_buffer_rsrc_t ry = srd(a.y, y_bytes);
  // post-op aux values (POST) / the statistics or post-op partials [row tiles][2][Ng]
  const bool do_stats = a.stats != nullptr;
  const __amdgpu_buffer_rsrc_t raux = srd(POST ? a.aux : a.y, POST ? (unsigned)a.M * (unsigned)a.ld_aux * 2u : 0u);
  const __amdgpu_buffer_rsrc_t rq = srd(POST ? (const void*)a.ppart : do_stats ? (const void*)a.stats : a.y,
                                        (POST || do_stats) ? (unsigned)(a.M / BM) * 2u * (unsigned)a.Ng * 4u : 0u);
  const int E = NST + ((POST || do_stats) ? 2 : 0);  // stores of one epilogue (per wave)

  if (tcount <= 0) return;  // (the grid is sized so this never happens)
  Tile cur = tile_of(0);
  // prologue: chunk 0's whole halo, weight steps 0 and 1
  issue_halo(cur, true, 0, 0, 0, HI);
  issue_w(cur, true, 0, 0, 0);
  issue_w(cur, true, 0, 1, 1);

  int gc = 0;  // chunks started by this block (halo stage parity)
  for (int j = 0; j < tcount; ++j) {
    const bool has_next = j + 1 < tcount;
    const Tile nxt = has_next ? tile_of(j + 1) : cur;
    f32x4 acc[FC][FP];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint2 zr[FC][FP];
    unsigned opix[FP];
#pragma unroll
    for (int p = 0; p < FP; ++p)
      opix[p] = (unsigned)((cur.nb * a.hc + cur.h0 + wm * 2 + (p >> 1)) * a.wc + cur.w0 + (p & 1) * 16 + j16);

    for (int c = 0; c < nch; ++c, ++gc) {
      const bool last = c == nch - 1;
      const bool tstart = c == 0 && j > 0;
      // the chunk after this one: this tile's c + 1, or the next tile's chunk 0 (dead past the block's tiles)
      const bool nx_same = !last;
      const bool nx_live = nx_same || has_next;
      const int nx_c = nx_same ? c + 1 : 0;
      const char* hs = reinterpret_cast<const char*>(lds) + (gc & 1) * HST * 16;
      auto step = [&](auto tc) {
        constexpr int t = decltype(tc)::value;
        // wait for this step's weight stage (at tap 0 also the chunk's halo, issued before it): the
        // younger operations of this wave are the next step's weights, the halo pieces of the two
        // previous steps and, at a tile's first two taps, the previous tile's epilogue stores
        constexpr int base = WP + P_(t - 1) + P_(t - 2);
        if constexpr (t <= 1) {
          if (tstart) {
            if (E == NST + 2)
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(base + NST + 2) : "memory");
            else
              asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(base + NST) : "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(base) : "memory");
          }
        } else {
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(base) : "memory");
        }
        const int jr = t / 3, js = t - jr * 3;
        const int shift = (a.dh0 + a.dhs * jr) * 34 + (a.dw0 + a.dws * js);
        unsigned ab[FP];
#pragma unroll
        for (int p = 0; p < FP; ++p) {
          const int hp = hq[p] + shift;
          ab[p] = (unsigned)(hp * 128 + ((chA ^ (hp & 7)) * 16));
        }
        const char* ws = reinterpret_cast<const char*>(lds) + 2 * HST * 16 + (t % 3) * WST * 16;
        bf16x8 pf[FP], wf[FC];
#pragma unroll
        for (int p = 0; p < FP; ++p) pf[p] = *reinterpret_cast<const bf16x8*>(hs + ab[p]);
#pragma unroll
        for (int cc = 0; cc < FC; ++cc) wf[cc] = *reinterpret_cast<const bf16x8*>(ws + foffW[0] + cc * 2048);
        // weights of the step two ahead (stage (t + 2) % 3): this chunk's tap t + 2, or the next chunk's
        if constexpr (t + 2 < 9) {
          issue_w(cur, true, c, t + 2, (t + 2) % 3);
        } else {
          issue_w(nx_same ? cur : nxt, nx_live, nx_c, t + 2 - 9, (t + 2) % 3);
        }
        if constexpr (t % TPER == 0) {
          issue_halo(nx_same ? cur : nxt, nx_live, nx_c, (gc + 1) & 1, (t / TPER) * HPC, (t / TPER + 1) * HPC);
        }
#pragma unroll
        for (int cc = 0; cc < FC; ++cc)
#pragma unroll
          for (int p = 0; p < FP; ++p)
            acc[cc][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cc], pf[p], acc[cc][p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < FP; ++p) pf[p] = *reinterpret_cast<const bf16x8*>(hs + (ab[p] ^ 64u));
#pragma unroll
        for (int cc = 0; cc < FC; ++cc) wf[cc] = *reinterpret_cast<const bf16x8*>(ws + foffW[1] + cc * 2048);
#pragma unroll
        for (int cc = 0; cc < FC; ++cc)
#pragma unroll
          for (int p = 0; p < FP; ++p)
            acc[cc][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cc], pf[p], acc[cc][p], 0, 0, 0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
      step(std::integral_constant<int, 4>{});
      step(std::integral_constant<int, 5>{});
      step(std::integral_constant<int, 6>{});
      step(std::integral_constant<int, 7>{});
      step(std::integral_constant<int, 8>{});
    }

    // ================= epilogue (register-direct) =================
    if constexpr (POST) {
      // the post-op aux values of this tile (untracked loads, then every older operation retired with
      // them: the next tile's first halo and weight stages were issued during the last chunk and have
      // mostly landed).  Held across the tap loop instead (issued at its last taps) they cost the
      // 8-wave kernel its registers: 123 VGPRs spilled.
#pragma unroll
      for (int cc = 0; cc < FC; ++cc) {
        const int nb = cur.n0 + wn * WTN + cc * 16 + kg * 4;
#pragma unroll
        for (int p = 0; p < FP; ++p)
          zr[cc][p] = bload64_asm(raux, nb < a.Ng ? (opix[p] * (unsigned)a.ld_aux + (unsigned)nb) * 2u : kOOB);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int cc = 0; cc < FC; ++cc)
#pragma unroll
        for (int p = 0; p < FP; ++p) asm volatile("" : "+v"(zr[cc][p]));
    }
    // one 16-channel group at a time (bias / ReLU / rounding, post-op mask, stores, column partials):
    // the whole-tile form held acc, the aux values, the packed outputs and 32 partials at once and spilled
#pragma unroll
    for (int cc = 0; cc < FC; ++cc) {
      const int nb = cur.n0 + wn * WTN + cc * 16 + kg * 4;
      const bool nok = nb < a.Ng;
      float bias4[4], sc4[4], sh4[4], mu4[4], iv4[4], s4[4], m4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bias4[e] = (has_bias && nok) ? xco[nb + e] : 0.f;
        const bool bn = POST && a.post == 2 && nok;
        sc4[e] = bn ? xco[nb + e] : 0.f;
        sh4[e] = bn ? xco[a.Ng + nb + e] : 0.f;
        mu4[e] = bn ? xco[2 * a.Ng + nb + e] : 0.f;
        iv4[e] = bn ? xco[3 * a.Ng + nb + e] : 0.f;
        s4[e] = m4[e] = 0.f;
      }
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        bf16 o[4];
        const bf16* z = reinterpret_cast<const bf16*>(&zr[cc][p]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[cc][p][e] + bias4[e];
          if (a.relu) v = fmaxf(v, 0.f);
          v = (float)(bf16)v;  // BN statistics / post-op sums are of the stored (rounded) values
          if constexpr (POST) {
            const float zf = (float)z[e];
            const bool on = a.post == 2 ? fmaf(zf, sc4[e], sh4[e]) > 0.f : zf > 0.f;
            v = on ? v : 0.f;
            m4[e] += v * ((zf - mu4[e]) * iv4[e]);
          }
          s4[e] += v;
          acc[cc][p][e] = v;
          o[e] = (bf16)v;
        }
        uint2 ov = *reinterpret_cast<uint2*>(o);
        if (a.accumulate && nok) {  // dx += dgrad (bf16 + bf16 in fp32); hipcc drains vmcnt here: slower, correct
          const uint2 old = *reinterpret_cast<const uint2*>((const bf16*)a.y + (long)opix[p] * a.ldy + nb);
          const bf16* ob = reinterpret_cast<const bf16*>(&old);
          bf16* nv = reinterpret_cast<bf16*>(&ov);
#pragma unroll
          for (int e = 0; e < 4; ++e) nv[e] = (bf16)((float)nv[e] + (float)ob[e]);
        }
        // exactly FC * FP output stores per wave (absent channels go out of range)
        bstore64(ry, nok ? (opix[p] * (unsigned)a.ldy + (unsigned)nb) * 2u : kOOB, ov);
      }
      if (POST || do_stats) {
        // this group's column partials over the wave's 64 pixels -> red[2][NWM][BN]: (sum d, sum d xhat)
        // for the post-op, (sum, M2 about the wave mean) for the statistics
        row16_sum_n(s4);
        if (!POST) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float mean = s4[e] * (1.0f / 64.f);
            float q = 0.f;
#pragma unroll
            for (int p = 0; p < FP; ++p) {
              const float d = acc[cc][p][e] - mean;
              q += d * d;
            }
            m4[e] = q;
          }
        }
        row16_sum_n(m4);
        if (j16 == 0)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int col = wn * WTN + cc * 16 + kg * 4 + e;
            red[wm * BN + col] = s4[e];
            red[(NWM + wm) * BN + col] = m4[e];
          }
      }
    }
    if (POST || do_stats) {
      // the NWM row-waves merged per column (plain sums for the post-op, Chan for the statistics),
      // stored by buffer stores every wave issues (2 each; lanes without a column go out of range)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const int col = tid;
      const int n = cur.n0 + col;
      const bool ok = col < BN && n < a.Ng;
      float t0 = 0.f, t1 = 0.f;
      if (ok) {
        if constexpr (POST) {
#pragma unroll
          for (int w = 0; w < NWM; ++w) {
            t0 += red[w * BN + col];
            t1 += red[(NWM + w) * BN + col];
          }
        } else {
#pragma unroll
          for (int w = 0; w < NWM; ++w) t0 += red[w * BN + col];
          const float mean = t0 * (1.0f / BM);
#pragma unroll
          for (int w = 0; w < NWM; ++w) {
            const float d = red[w * BN + col] * (1.0f / 64.f) - mean;
            t1 += red[(NWM + w) * BN + col] + 64.f * d * d;
          }
        }
      }
      const unsigned so = ok ? (unsigned)(cur.tm * 2 * a.Ng + n) * 4u : kOOB;
      bstore32(rq, so, t0);
      bstore32(rq, ok ? so + (unsigned)a.Ng * 4u : kOOB, t1);
    }
    cur = nxt;
  }
  // the dead DMAs issued during the last chunk land in this block's LDS: drain them before it exits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------------
// wgrad: C[cout][(tap, c)] = sum_pix dY[pix][cout] * X[n][p*st+dh][q*st+dw][c];
// tile BM couts x BN (tap,c) columns, K step = kWgBK consecutive output pixels.  Each thread
// tracks (image, row, col) of the pixels it stages and advances them by one step at a time, so
// any output width works.
// ------------------------------------------------------------------------------------------

// ROW32 (Q % 32 == 0): the 32 pixels of a K step are one run of an output row, so (image, row,
// first column) is wave-uniform scalar state and each staged row's offset is a scalar base plus a
// per-lane constant (tap shift, column, channel): a few VALU per row instead of re-deriving the
// pixel, its bounds and its 32-bit offset every step.
// PRE: X = relu(x1 * in_sc[c] + in_sh[c]) for the rows that exist (padding / past-the-end rows
// stay zero); each thread's 8 channels are fixed, so their coefficients live in registers.
template <int BM, int BN, int NWM, int NWN, bool ROW32 = false, bool PRE = false>
__global__ __launch_bounds__(64 * NWM * NWN) void wgrad_fast_kernel(FastWgradArgs a) {
  constexpr int NT = 64 * NWM * NWN;
  constexpr int BKW = kWgBK;
  constexpr int CPA = BM / 8, CPB = BN / 8;  // 16-B chunks per LDS row
  constexpr int A_PER = BKW * CPA / NT, B_PER = BKW * CPB / NT;
  constexpr int WTM = BM / NWM, WTN = BN / NWN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int STAGE = BKW * (CPA + CPB);  // uint4
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // [2][STAGE]
  static_assert(A_PER >= 1 && B_PER >= 1, "tile too small for the block");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  const __amdgpu_buffer_rsrc_t rdy = srd(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t r1 = srd(a.x1, a.x1_bytes);
  const __amdgpu_buffer_rsrc_t r2 = srd(a.x2 ? a.x2 : a.x1, a.x2 ? a.x2_bytes : 0u);

  // A (dY) chunk: column cv fixed, rows ra_row + (NT/CPA)*i
  int a_cv[A_PER], a_row[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int id = tid + NT * i;
    a_cv[i] = id % CPA;
    a_row[i] = id / CPA;
  }
  // B (X) chunk: column fixed -> (tap, c) fixed; row -> a pixel whose (n, p, q) we track
  int b_row[B_PER], b_dh[B_PER], b_dw[B_PER], b_src[B_PER], b_cv[B_PER];
  int b_n[B_PER], b_p[B_PER], b_q[B_PER];
  unsigned b_cb[B_PER];
  const long nkt_total = (a.Kpix + BKW - 1) / BKW;
  const long kt0 = (long)blockIdx.z * a.kt_per_split;
  const long kt1 = min(nkt_total, kt0 + a.kt_per_split);
  const int PQ = a.P * a.Q;
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int id = tid + NT * i;
    const int cv = id % CPB;
    b_cv[i] = cv;
    b_row[i] = id / CPB;
    const int nn = n0 + cv * 8;
    if (nn < a.Ng) {
      const int tap = nn / a.cin, c = nn - tap * a.cin;
      const int r = tap / a.S, s = tap - r * a.S;
      b_dh[i] = r - a.pad;
      b_dw[i] = s - a.padw;
      b_src[i] = c < a.c1 ? 0 : 1;
      b_cb[i] = (unsigned)(c < a.c1 ? c : c - a.c1) * 2u;
    } else {
      b_dh[i] = -(1 << 20);  // never valid
      b_dw[i] = 0;
      b_src[i] = 0;
      b_cb[i] = 0;
    }
    const long k = kt0 * BKW + b_row[i];
    const int nb = (int)(k / PQ), rem = (int)(k - (long)nb * PQ);
    b_n[i] = nb;
    b_p[i] = rem / a.Q;
    b_q[i] = rem - b_p[i] * a.Q;
  }
  const unsigned a_colb0 = (unsigned)m0 * 2u;
  float pre_sc[PRE ? B_PER : 1][8], pre_sh[PRE ? B_PER : 1][8];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int nn = n0 + b_cv[i] * 8;
      const int c = nn < a.Ng ? nn % a.cin : 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pre_sc[i][e] = nn < a.Ng ? a.in_sc[c + e] : 0.f;
        pre_sh[i][e] = nn < a.Ng ? a.in_sh[c + e] : 0.f;
      }
    }
  }
  unsigned b_okm = 0u;  // rows of the staged X set that exist (PRE)

  uint4 ra[A_PER], rbv[B_PER];
  // ---- ROW32 addressing: lane constants and scalar (image, row, column) of the next K step ----
  unsigned a_off[A_PER], b_l1[B_PER], b_l2[B_PER];
  int b_lw[B_PER];
  bool a_ok[A_PER];
  int s_n = 0, s_p = 0, s_q = 0;
  if constexpr (ROW32) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      a_ok[i] = (m0 + a_cv[i] * 8) < a.Cout;
      a_off[i] = (unsigned)a_row[i] * (unsigned)a.ldyb + a_colb0 + a_cv[i] * 16u;
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      b_lw[i] = b_row[i] * a.stride + b_dw[i];
      const int dpix = b_dh[i] * a.W + b_lw[i];  // relative to the step's (row, first column) pixel
      b_l1[i] = (unsigned)(dpix * a.ldc1b) + b_cb[i];
      b_l2[i] = (unsigned)(dpix * a.ldc2b) + b_cb[i];
    }
    const long k = kt0 * BKW;
    s_n = (int)(k / PQ);
    const int rem = (int)(k - (long)s_n * PQ);
    s_p = rem / a.Q;
    s_q = rem - s_p * a.Q;
  }
  auto gload_row = [&](long kt) {
    const unsigned abase = (unsigned)(kt * BKW) * (unsigned)a.ldyb;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) ra[i] = bload(rdy, a_ok[i] ? abase + a_off[i] : kOOB);
    const int ihb = s_p * a.stride, iwb = s_q * a.stride;
    const int pixb = (s_n * a.H + ihb) * a.W + iwb;
    const unsigned base1 = (unsigned)pixb * (unsigned)a.ldc1b, base2 = (unsigned)pixb * (unsigned)a.ldc2b;
    b_okm = 0u;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const bool ok = (unsigned)(ihb + b_dh[i]) < (unsigned)a.H && (unsigned)(iwb + b_lw[i]) < (unsigned)a.W;
      b_okm |= ok ? 1u << i : 0u;
      if (b_src[i] == 0)
        rbv[i] = bload(r1, ok ? base1 + b_l1[i] : kOOB);
      else
        rbv[i] = bload(r2, ok ? base2 + b_l2[i] : kOOB);
    }
    s_q += BKW;
    if (s_q == a.Q) {
      s_q = 0;
      if (++s_p == a.P) {
        s_p = 0;
        ++s_n;
      }
    }
  };
  auto gload = [&](long kt) {
    if constexpr (ROW32) {
      gload_row(kt);
      return;
    }
    const long k0 = kt * BKW;  // first pixel of the step (uniform)
    b_okm = 0u;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const long k = k0 + a_row[i];
      const bool ok = k < a.Kpix && (m0 + a_cv[i] * 8) < a.Cout;
      const unsigned off = (unsigned)k * (unsigned)a.ldyb + a_colb0 + a_cv[i] * 16u;
      ra[i] = bload(rdy, ok ? off : kOOB);
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int ih = b_p[i] * a.stride + b_dh[i];
      const int iw = b_q[i] * a.stride + b_dw[i];
      const bool ok = (k0 + b_row[i]) < a.Kpix && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      b_okm |= ok ? 1u << i : 0u;
      const unsigned pixi = (unsigned)((b_n[i] * a.H + ih) * a.W + iw);
      if (b_src[i] == 0)
        rbv[i] = bload(r1, ok ? pixi * (unsigned)a.ldc1b + b_cb[i] : kOOB);
      else
        rbv[i] = bload(r2, ok ? pixi * (unsigned)a.ldc2b + b_cb[i] : kOOB);
      // advance this row's pixel by one K step
      int q = b_q[i] + BKW, p = b_p[i], nb = b_n[i];
      while (q >= a.Q) {
        q -= a.Q;
        if (++p == a.P) {
          p = 0;
          ++nb;
        }
      }
      b_q[i] = q;
      b_p[i] = p;
      b_n[i] = nb;
    }
  };
  auto sstore = [&](int buf) {
    uint4* L = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = a_row[i];
      const int sw = CPA >= 16 ? swz_tr16(row) : swz_tr8(row);
      L[row * CPA + (a_cv[i] ^ sw)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = b_row[i];
      const int sw = CPB >= 16 ? swz_tr16(row) : swz_tr8(row);
      uint4 v = rbv[i];
      if constexpr (PRE) {  // == bn_apply: (bf16) relu(fmaf(z, sc, sh)); absent rows stay zero
        if ((b_okm >> i) & 1u) {
          bf16* e8 = reinterpret_cast<bf16*>(&v);
#pragma unroll
          for (int e = 0; e < 8; ++e) e8[e] = (bf16)fmaxf(fmaf((float)e8[e], pre_sc[i][e], pre_sh[i][e]), 0.f);
        }
      }
      L[BKW * CPA + row * CPB + (b_cv[i] ^ sw)] = v;
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = (int)(kt1 - kt0);
  if (nkt > 0) {
    gload(kt0);
    sstore(0);
    __syncthreads();
  }
  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
  // per-lane byte offsets of every transposed fragment read (rows 8g+qq and +4 of the K step,
  // 16-B chunk of the fragment's columns under the row swizzle): the loop adds only the stage base
  unsigned toffA[FM][2], toffB[FN][2];
  {
    const int ra_ = 8 * g + qq, rb_ = ra_ + 4;
    auto off = [&](int cpr, int col0, int row) -> unsigned {
      const int chunk = (col0 >> 3) + (pp >> 1);
      const int sw = cpr >= 16 ? swz_tr16(row) : swz_tr8(row);
      return (unsigned)(row * (cpr * 16) + ((chunk ^ sw) * 16) + (pp & 1) * 8);
    };
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      toffA[i][0] = off(CPA, wm * WTM + i * 16, ra_);
      toffA[i][1] = off(CPA, wm * WTM + i * 16, rb_);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      toffB[j][0] = BKW * CPA * 16 + off(CPB, wn * WTN + j * 16, ra_);
      toffB[j][1] = BKW * CPA * 16 + off(CPB, wn * WTN + j * 16, rb_);
    }
  }
  static_assert(BKW == 32, "one 32-pixel K half per step");
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kt0 + kt + 1);
    const char* base = reinterpret_cast<const char*>(lds + cur * STAGE);
    auto trpair = [&](unsigned o0, unsigned o1) -> bf16x8 {
      s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o0));
      s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o1));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      s16x8 v = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
      return *reinterpret_cast<bf16x8*>(&v);
    };
    {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = trpair(toffA[i][0], toffA[i][1]);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = trpair(toffB[j][0], toffB[j][1]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nkt) sstore(cur ^ 1);
    __syncthreads();
  }
  // partial slab ws[z][cout][tap*cin + c] (coalesced; wgrad_reduce permutes into PyTorch order)
  float* ws = a.ws + (long)blockIdx.z * a.Cout * a.Ng;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + e;
      if (m >= a.Cout) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane & 15);
        if (n < a.Ng) ws[(long)m * a.Ng + n] = acc[i][j][e];
      }
    }
}

template <int BM, int BN, int NWM, int NWN, int ST, int POST = 0, int TAPS = 0, bool PRE = false, int HA = 0>
int launch_tn_cfg(const FastTNArgs& a, hipStream_t st) {
  constexpr int NT = 64 * NWM * NWN;
  // operand stages, or the epilogue's per-wave transpose tiles + stats scratch if larger; then the
  // input-prologue coefficients (PRE)
  constexpr size_t kMaxPre = 2 * 2048 * 4;
  constexpr size_t off = kPreOff<BM, BN, NWM, NWN, ST, HA>();
  const size_t lds = off + (PRE ? (size_t)2 * a.c1 * 4 : 0);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tn_fast_kernel<BM, BN, NWM, NWN, ST, POST, TAPS, PRE, HA>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)(off + (PRE ? kMaxPre : 0)));
    attr = true;
  }
  dim3 grid(ceil_div(a.M, BM), ceil_div(a.Ng, BN), 1);
  FastTNArgs b = a;
  constexpr int TR = BM / 32;
  // 2D spatial tiles measured slower than row-major tiles with the chunk-outer K order: opt-in for
  // the gather ring; the halo-A ring is built on them
  static const bool t2d = getenv("UNETSEG_T2D") != nullptr;
  b.t2d = (HA || (t2d && a.nr * a.ns > 1 && a.wc % 32 == 0 && a.wc > 32 && a.hc % TR == 0)) ? TR : 0;
  // default 1 since round 5 (with the replayed step plan: +0.1-0.2 % in the step; 0 restores the round-4 issue order)
  static const int sched = getenv("UNETSEG_TN_SCHED") ? atoi(getenv("UNETSEG_TN_SCHED")) : 1;
  b.sched = sched;
  hipLaunchKernelGGL((tn_fast_kernel<BM, BN, NWM, NWN, ST, POST, TAPS, PRE, HA>), grid, dim3(NT), lds, st, b);
  return 0;
}

template <int BM, int BN, int NWM, int NWN, int ST, int POST>
int launch_tn_multi_cfg(const FastTNArgs* fs, int n, hipStream_t st) {
  constexpr int NT = 64 * NWM * NWN;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tn_multi_kernel<BM, BN, NWM, NWN, ST, POST>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPreOff<BM, BN, NWM, NWN, ST>());
    attr = true;
  }
  TNMulti m{};
  m.n = n;
  int total = 0;
  for (int k = 0; k < n; ++k) {
    m.c[k] = fs[k];
    m.c[k].t2d = 0;
    m.c[k].sched = 0;
    m.gx[k] = ceil_div(fs[k].M, BM);
    m.gy[k] = ceil_div(fs[k].Ng, BN);
    m.start[k] = total;
    total += m.gx[k] * m.gy[k];
  }
  m.start[n] = total;
  constexpr size_t lds = kPreOff<BM, BN, NWM, NWN, ST>();
  hipLaunchKernelGGL((tn_multi_kernel<BM, BN, NWM, NWN, ST, POST>), dim3(total), dim3(NT), lds, st, m);
  return 0;
}

// Compile-time tap count for the LDS-DMA ring (0 = generic ring): 3x3 and 1x1 filters, when the
// precomputed gather offsets (pixel index < 2^24, pbad * ldcb) fit the 24-bit multiply and 32 bits.
static int tn_taps(const FastTNArgs& a) {
  static const bool off = getenv("UNETSEG_TN_NO_TAPS") != nullptr;
  static const bool off1 = getenv("UNETSEG_TN_NO_TAPS1") != nullptr;
  const int taps = a.nr * a.ns;
  if (off || (taps != 9 && taps != 1) || (taps == 1 && off1)) return 0;
  const unsigned long long p1 = a.x1_bytes / (unsigned)a.ldc1b;
  const unsigned long long p2 = a.x2 ? a.x2_bytes / (unsigned)a.ldc2b : 0ull;
  const unsigned long long pbad = (p1 > p2 ? p1 : p2) + 1ull;
  const unsigned long long ld = (unsigned)(a.ldc1b > a.ldc2b ? a.ldc1b : a.ldc2b);
  if (pbad >= (1ull << 24) || ld >= (1ull << 24) || pbad * ld + 256ull >= (1ull << 32)) return 0;
  return taps;
}

template <int BM, int BN, int NWM, int NWN, int ST>
static int launch_tn_dma(const FastTNArgs& a, hipStream_t st) {
  switch (tn_taps(a)) {
    case 9: return a.post ? launch_tn_cfg<BM, BN, NWM, NWN, ST, true, 9>(a, st) : launch_tn_cfg<BM, BN, NWM, NWN, ST, false, 9>(a, st);
    case 1: return a.post ? launch_tn_cfg<BM, BN, NWM, NWN, ST, true, 1>(a, st) : launch_tn_cfg<BM, BN, NWM, NWN, ST, false, 1>(a, st);
    default: return a.post ? launch_tn_cfg<BM, BN, NWM, NWN, ST, true>(a, st) : launch_tn_cfg<BM, BN, NWM, NWN, ST>(a, st);
  }
}

// TN configuration: 0 = halo, 19 / 20 = short-K 128x128 / 128x64 on one LDS stage, 1 = 256x64, 2 = 256x128, 3 = 128x128, 4 = 128x128 single stage
// (one K step: the prefetch stage would only cost occupancy), 5 = 64x128, 6 = 128x64;
// 7-10: the same tiles on the LDS-DMA ring.  Measured (tools/gpu_cfg_sweep.sh): the 256x128 ring
// (3 stages) beats the register-staged 256x128 by 3-8 % on every large layer; the 64x128 ring (4
// stages) is 15 % faster on deep-K small-M layers (3x3 at 16x16, 72 K steps) but slower on short K.
// The halo-A ring (configuration 21, 22 for <= 64 output channels, 23 on 128x128 tiles) serves a 3x3
// stride-1 "same" conv whose output grid tiles into 8 x 32 spatial blocks, in place of the gather
// rings 7 / 13 / 10.
static bool halo_a_ok(const FastTNArgs& a) {
  // default since the round-3 A/B (+1.8 % end to end); UNETSEG_TN_NO_HALO_RING=1 keeps the gather
  // ring -- read per call so a test can run both rings in one process
  if (getenv("UNETSEG_TN_NO_HALO_RING") != nullptr || a.in_sc || a.nr != 3 || a.ns != 3 || a.istride != 1) return false;
  if (a.dhs * a.dhs != 1 || a.dws * a.dws != 1) return false;
  const int dh_lo = a.dhs > 0 ? a.dh0 : a.dh0 - 2, dw_lo = a.dws > 0 ? a.dw0 : a.dw0 - 2;
  if (dh_lo != -1 || dw_lo != -1) return false;  // one halo pixel on every side
  if (a.H != a.hc || a.W != a.wc || a.hc % 8 || a.wc % 32) return false;
  return tn_taps(a) == 9;
}

static int tn_config_base(const FastTNArgs& a);

// Persistent halo-A ring (tn_halo_persist_kernel): tiles per block for a halo-A ring call on BN-wide
// column tiles, or 0 to keep the one-tile-per-block kernel.  UNETSEG_TN_PERSIST=0 turns it off (read per
// call, so a test can run both); UNETSEG_TN_PERSIST_ROUNDS = R: T = ceil(tiles / (R x CUs)), i.e. the
// grid covers the chip about R times (default 1: one resident block per CU runs its whole share);
// UNETSEG_TN_PERSIST_MIN_T: below this many tiles per block the plain kernel runs (default 2);
// UNETSEG_TN_PERSIST_T = T forces T (tests).  Reported as configurations 24 / 25 (tn_fast_config).
static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}
static int persist_t(const FastTNArgs& a, int bn) {
  const char* e = getenv("UNETSEG_TN_PERSIST");
  if (e && atoi(e) == 0) return 0;
  if (a.in_sc || a.post < 0 || a.post > 2 || (a.bias && a.post) || a.t2d < 0) return 0;
  if (a.ostride != 1 || a.ph || a.pw || a.OH != a.hc || a.OW != a.wc || a.M % 256) return 0;
  const size_t extra = (a.bias ? (size_t)a.Ng * 4 : 0) + (a.post == 2 ? (size_t)a.Ng * 16 : 0);
  const size_t lds = (bn == 128 ? kPersistLds<128, 2>() : kPersistLds<64, 2>()) + extra;
  if (lds > 160 * 1024) return 0;
  // 32-bit buffer offsets below kOOB
  if ((unsigned long long)a.M * (unsigned)a.ldy * 2ull >= (unsigned long long)kOOB) return 0;
  if (a.post && (unsigned long long)a.M * (unsigned)a.ld_aux * 2ull >= (unsigned long long)kOOB) return 0;
  if (a.stats && (unsigned long long)(a.M / 256) * 2ull * a.Ng * 4ull >= (unsigned long long)kOOB) return 0;
  // tiles of fewer 64-channel chunks than this keep the one-tile kernel (UNETSEG_TN_PERSIST_MIN_NCH)
  const char* mc = getenv("UNETSEG_TN_PERSIST_MIN_NCH");
  if (mc && (a.cin >> 6) < atoi(mc)) return 0;
  const long ntiles = (long)(a.M / 256) * ceil_div(a.Ng, bn);
  const char* ft = getenv("UNETSEG_TN_PERSIST_T");  // tests: a fixed T (every tile count, ragged last block)
  if (ft && atoi(ft) > 0) return atoi(ft);
  const char* r = getenv("UNETSEG_TN_PERSIST_ROUNDS");
  const int rounds = r && atoi(r) > 0 ? atoi(r) : 1;
  const char* m = getenv("UNETSEG_TN_PERSIST_MIN_T");
  const int min_t = m && atoi(m) > 0 ? atoi(m) : 2;
  const long T = (ntiles + (long)rounds * cu_count() - 1) / ((long)rounds * cu_count());
  return T >= min_t ? (int)T : 0;
}

template <int BN, int NWN, int HA>
static int launch_tn_persist(const FastTNArgs& a, hipStream_t st) {
  const int T = persist_t(a, BN);
  const size_t extra = (a.bias ? (size_t)a.Ng * 4 : 0) + (a.post == 2 ? (size_t)a.Ng * 16 : 0);
  const size_t lds = kPersistLds<BN, NWN>() + extra;
  const int ntiles = (a.M / 256) * ceil_div(a.Ng, BN);
  const int grid = ceil_div(ntiles, T);
  const unsigned y_bytes = (unsigned)((unsigned long long)a.M * (unsigned)a.ldy * 2ull);
  if (a.post) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tn_halo_persist_kernel<BN, NWN, 1, HA>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((tn_halo_persist_kernel<BN, NWN, 1, HA>), dim3(grid), dim3(512), lds, st, a, T, ntiles, y_bytes);
  } else {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tn_halo_persist_kernel<BN, NWN, 0, HA>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((tn_halo_persist_kernel<BN, NWN, 0, HA>), dim3(grid), dim3(512), lds, st, a, T, ntiles, y_bytes);
  }
  return 0;
}

static int tn_config(const FastTNArgs& a) {
  if (a.force_cfg) return a.force_cfg;
  const int c = tn_config_base(a);
  if ((c == 7 || c == 13 || (c == 10 && !getenv("UNETSEG_TN_CFG_NO23"))) && halo_a_ok(a)) return c == 7 ? 21 : c == 13 ? 22 : 23;
  return c;
}

static int tn_config_base(const FastTNArgs& a) {
  if (const char* e = getenv("UNETSEG_TN_CFG")) {  // experiments: force a configuration (1..14, 19-21)
    const int c = atoi(e);
    if (c == 21) return 7;  // the halo-A ring where it applies (tn_config), else the gather ring
    if (((c >= 1 && c <= 14) || c == 19 || c == 20) && !(a.in_sc && c >= 7 && c <= 14)) return c;
  }
  static const bool no_dma_env = getenv("UNETSEG_TN_NO_DMA") != nullptr;
  // the input prologue transforms registers between load and LDS store: register-staged tiles only
  const bool no_dma = no_dma_env || a.in_sc != nullptr;
  if (!a.in_sc && halo3_ok(a)) return 0;
  const int nsteps = a.nr * a.ns * (a.cin >> 6);
  // short K (<= 4 steps: the bottleneck 1x1 layers, HBM-bound) on one LDS stage, 3-4 blocks per CU
  // (128x128 with one step keeps its own single-step tile: as fast, fewer barriers)
  static const bool no_short1 = getenv("UNETSEG_TN_NO_SHORT1") != nullptr;
  if (!no_short1 && nsteps <= 4 && (nsteps >= 2 || a.Ng <= 64)) return a.Ng <= 64 ? 20 : 19;
  if (nsteps == 1 && a.Ng > 64) return 4;
  // 128x64 (two-step prefetch, 3 blocks/CU): 5-10 % over 256x64; deep 3x3 K on the 3-stage ring
  // with compile-time taps: ~8 % more (192->64 at 256x256: 390 -> 357 us)
  if (a.Ng <= 64) return (!no_dma && nsteps >= 18 && tn_taps(a) == 9) ? 13 : 6;
  if (nsteps <= 4) return 3;
  const long tiles_big = (long)ceil_div(a.M, 256) * ceil_div(a.Ng, 128);
  if (tiles_big >= 256) return no_dma ? 2 : 7;
  const long tiles_mid = (long)ceil_div(a.M, 128) * ceil_div(a.Ng, 128);
  // one or two 128x128 tiles per CU and a deep K: the 5-stage ring with compile-time taps (one
  // block per CU) beats the register-staged tile by ~25 % (3x3 256->256 at 32x32: 43 -> 34 us)
  if (tiles_mid >= 256) return (!no_dma && nsteps >= 16 && tn_taps(a)) ? 10 : 3;
  // 64-row tiles so that small-M layers still fill the chip
  return (!no_dma && nsteps >= 32) ? 9 : 5;
}

}  // namespace

// row tile (BM) of each TN configuration
static int tn_cfg_bm(int cfg) {
  switch (cfg) {
    case 1: case 2: case 7: case 11: case 14: case 21: case 22: return 256;
    case 23: return 128;
    case 5: case 9: return 64;
    default: return 128;
  }
}

bool tn_fast_ok(const FastTNArgs& a) {
  return a.cin % 64 == 0 && a.c1 % 64 == 0 && a.nr * a.ns <= 32 && a.Ng % 8 == 0;
}

// Row tile of the BN partial statistics = the block's rows (BM) on the TN kernels, one 8x32
// spatial tile on the halo kernel.
int tn_fast_tile_m(const FastTNArgs& a) {
  const int cfg = tn_config(a);
  return cfg == 0 ? halo_tile_m() : tn_cfg_bm(cfg);
}

int tn_fast_post_rows(const FastTNArgs& a) {
  if (a.M <= 0 || a.Ng <= 0) return 0;
  const int cfg = tn_config(a);
  return cfg == 0 ? halo3_blocks(a) : ceil_div(a.M, tn_cfg_bm(cfg));
}

int tn_fast_config(const FastTNArgs& a, int* taps_out) {
  const int cfg = tn_config(a);
  if ((cfg == 21 || cfg == 22) && !a.in_sc && a.post != 3 && a.post != 4 && persist_t(a, cfg == 21 ? 128 : 64) > 0) {
    if (taps_out) *taps_out = 0;
    return cfg + 3;  // 24 / 25: the persistent halo-A ring (tn_halo_persist_kernel)
  }
  if (taps_out) *taps_out = (cfg >= 7 && cfg <= 14) ? tn_taps(a) : 0;
  return cfg;
}

// Configurations with a post-3 (residual-BN backward) instantiation: the tiles the bottleneck conv1
// data gradients take (1x1, 1-8 K steps).
bool tn_fast_post_res_ok(const FastTNArgs& a) {
  const int cfg = tn_config(a);
  return cfg == 4 || cfg == 19 || cfg == 20 || ((cfg == 7 || cfg == 10) && tn_taps(a) == 1);
}

static int launch_tn_post_res(const FastTNArgs& a, hipStream_t st) {
  switch (tn_config(a)) {
    case 4: return launch_tn_cfg<128, 128, 2, 2, 1, 3>(a, st);
    case 19: return launch_tn_cfg<128, 128, 2, 2, 5, 3>(a, st);
    case 20: return launch_tn_cfg<128, 64, 2, 2, 5, 3>(a, st);
    case 7: return tn_taps(a) == 1 ? launch_tn_cfg<256, 128, 4, 2, 13, 3, 1>(a, st) : -1;
    case 10: return tn_taps(a) == 1 ? launch_tn_cfg<128, 128, 2, 2, 15, 3, 1>(a, st) : -1;
    default: return -1;
  }
}

int launch_tn_fast(const FastTNArgs& a, hipStream_t st) {
  if (a.M <= 0 || a.Ng <= 0) return 0;
  if (a.post == 3) return a.in_sc ? -1 : launch_tn_post_res(a, st);
  if (a.post == 4) return tn_config(a) == 0 ? launch_halo3(a, st) : -1;  // mask bits: halo path only
  if (a.in_sc) {  // input prologue (fwd only: no post-op), register-staged configurations
    switch (tn_config(a)) {
      case 1: return launch_tn_cfg<256, 64, 4, 1, 2, false, 0, true>(a, st);
      case 2: return launch_tn_cfg<256, 128, 4, 2, 3, false, 0, true>(a, st);
      case 4: return launch_tn_cfg<128, 128, 2, 2, 1, false, 0, true>(a, st);
      case 5: return launch_tn_cfg<64, 128, 1, 4, 3, false, 0, true>(a, st);
      case 6: return launch_tn_cfg<128, 64, 2, 2, 3, false, 0, true>(a, st);
      case 3: return launch_tn_cfg<128, 128, 2, 2, 3, false, 0, true>(a, st);
      case 19: return launch_tn_cfg<128, 128, 2, 2, 5, false, 0, true>(a, st);
      case 20: return launch_tn_cfg<128, 64, 2, 2, 5, false, 0, true>(a, st);
      default: return -1;
    }
  }
  switch (tn_config(a)) {
    case 0: return launch_halo3(a, st);
    case 1: return a.post ? launch_tn_cfg<256, 64, 4, 1, 2, true>(a, st) : launch_tn_cfg<256, 64, 4, 1, 2>(a, st);
    case 2: return a.post ? launch_tn_cfg<256, 128, 4, 2, 3, true>(a, st) : launch_tn_cfg<256, 128, 4, 2, 3>(a, st);
    case 4: return a.post ? launch_tn_cfg<128, 128, 2, 2, 1, true>(a, st) : launch_tn_cfg<128, 128, 2, 2, 1>(a, st);
    case 5: return a.post ? launch_tn_cfg<64, 128, 1, 4, 3, true>(a, st) : launch_tn_cfg<64, 128, 1, 4, 3>(a, st);
    case 6: return a.post ? launch_tn_cfg<128, 64, 2, 2, 3, true>(a, st) : launch_tn_cfg<128, 64, 2, 2, 3>(a, st);
    // LDS-DMA ring variants (experiments via UNETSEG_TN_CFG)
    case 7: return launch_tn_dma<256, 128, 4, 2, 13>(a, st);
    case 8: return launch_tn_dma<128, 128, 2, 2, 14>(a, st);
    case 9: return launch_tn_dma<64, 128, 1, 4, 14>(a, st);
    case 10: return launch_tn_dma<128, 128, 2, 2, 15>(a, st);
    case 11: return launch_tn_dma<256, 64, 4, 1, 13>(a, st);
    case 12: return launch_tn_dma<128, 64, 2, 2, 14>(a, st);
    case 13: return launch_tn_dma<128, 64, 2, 2, 13>(a, st);
    case 14: return launch_tn_dma<256, 64, 4, 2, 13>(a, st);
    case 19: return a.post ? launch_tn_cfg<128, 128, 2, 2, 5, true>(a, st) : launch_tn_cfg<128, 128, 2, 2, 5>(a, st);
    case 20: return a.post ? launch_tn_cfg<128, 64, 2, 2, 5, true>(a, st) : launch_tn_cfg<128, 64, 2, 2, 5>(a, st);
    case 21: {
      if (persist_t(a, 128) > 0) return launch_tn_persist<128, 2, 3>(a, st);
      // weight ring depth: 3 stages (144 KiB of LDS with the two halo stages); 4 fill all 160 KiB
      static const bool ns4 = getenv("UNETSEG_TN_HALO_NS4") != nullptr;
      // the next chunk's halo DMA in three pieces at taps 0, 3, 6 (A/B +0.3 %; UNETSEG_TN_HALO_SPLIT=1:
      // all of it at tap 0)
      static const bool split = !(getenv("UNETSEG_TN_HALO_SPLIT") && atoi(getenv("UNETSEG_TN_HALO_SPLIT")) == 1);
      if (ns4) return a.post ? launch_tn_cfg<256, 128, 4, 2, 14, true, 9, false, 1>(a, st)
                             : launch_tn_cfg<256, 128, 4, 2, 14, false, 9, false, 1>(a, st);
      if (split) return a.post ? launch_tn_cfg<256, 128, 4, 2, 13, true, 9, false, 3>(a, st)
                               : launch_tn_cfg<256, 128, 4, 2, 13, false, 9, false, 3>(a, st);
      return a.post ? launch_tn_cfg<256, 128, 4, 2, 13, true, 9, false, 1>(a, st)
                    : launch_tn_cfg<256, 128, 4, 2, 13, false, 9, false, 1>(a, st);
    }
    // 64 output channels or fewer: 256x64 (eight waves of 64x32), one weight row per wave and step
    case 22:
      if (persist_t(a, 64) > 0) return launch_tn_persist<64, 2, 1>(a, st);
      return a.post ? launch_tn_cfg<256, 64, 4, 2, 13, true, 9, false, 1>(a, st)
                           : launch_tn_cfg<256, 64, 4, 2, 13, false, 9, false, 1>(a, st);
    // in place of the 5-stage 128x128 gather ring (one or two tiles per CU): 4 x 32 spatial tiles,
    // four waves, the weights on a 5-stage ring
    case 23: return a.post ? launch_tn_cfg<128, 128, 2, 2, 15, true, 9, false, 1>(a, st)
                           : launch_tn_cfg<128, 128, 2, 2, 15, false, 9, false, 1>(a, st);
    default: return a.post ? launch_tn_cfg<128, 128, 2, 2, 3, true>(a, st) : launch_tn_cfg<128, 128, 2, 2, 3>(a, st);
  }
}

// Merged launch of 2-4 GEMMs (stride-2 data-gradient parity classes) on one register-staged tile:
// 128x128 (or 64x128 when any class would take a 64-row tile).  Returns -1 (nothing launched) when
// the classes cannot share one (input prologue, a halo class, more than 4).
static bool tn_multi_off() {
  static const bool off = getenv("UNETSEG_NO_TN_MULTI") != nullptr;
  return off;
}

int tn_multi_tile_m(const FastTNArgs* fs, int n) {
  if (tn_multi_off() || n < 2 || n > 4) return -1;
  bool bm64 = false;
  for (int k = 0; k < n; ++k) {
    if (fs[k].in_sc || fs[k].M <= 0) return -1;
    const int cfg = tn_config(fs[k]);
    if (cfg == 0) return -1;
    if (tn_cfg_bm(cfg) == 64) bm64 = true;
  }
  return bm64 ? 64 : 128;
}

int launch_tn_multi(const FastTNArgs* fs, int n, hipStream_t st) {
  const int bm = tn_multi_tile_m(fs, n);
  if (bm < 0) return -1;
  const bool post = fs[0].post != 0;
  if (bm == 64) return post ? launch_tn_multi_cfg<64, 128, 1, 4, 3, true>(fs, n, st)
                            : launch_tn_multi_cfg<64, 128, 1, 4, 3, false>(fs, n, st);
  return post ? launch_tn_multi_cfg<128, 128, 2, 2, 3, true>(fs, n, st)
              : launch_tn_multi_cfg<128, 128, 2, 2, 3, false>(fs, n, st);
}

bool wgrad_fast_ok(const FastWgradArgs& a) {
  return a.cin % 8 == 0 && a.c1 % 8 == 0 && a.Cout % 64 == 0;
}

int wgrad_fast_splits(int Cout, int Ng, long Kpix) {
  const int bm = Cout <= 64 ? 64 : 128;
  const int bn = Cout <= 64 ? 256 : 128;
  const int tiles = ceil_div(Cout, bm) * ceil_div(Ng, bn);
  const long nkt = (Kpix + kWgBK - 1) / kWgBK;
  // 256 target blocks since round 5 (replayed step: +0.1-0.2 %, smaller split-K slabs; 0 = 1024 / 512)
  static const int wscale = getenv("UNETSEG_WG_BLOCKS") ? atoi(getenv("UNETSEG_WG_BLOCKS")) : 256;
  int sp = ceil_div(wscale > 0 ? wscale : (Cout <= 64 ? 1024 : 512), tiles);  // 2-4 blocks per CU
  const long max_sp = nkt / 32 > 0 ? nkt / 32 : 1;  // >= 32 K steps per split
  if (sp > max_sp) sp = (int)max_sp;
  if (sp > 512) sp = 512;
  if (sp < 1) sp = 1;
  return sp;
}

template <int BM, int BN, int NWM, int NWN, bool ROW32, bool PRE = false>
static void launch_wgrad_cfg(const FastWgradArgs& a, int splits, hipStream_t st) {
  const size_t lds = 2 * (size_t)kWgBK * (BM / 8 + BN / 8) * 16;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_fast_kernel<BM, BN, NWM, NWN, ROW32, PRE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  dim3 grid(ceil_div(a.Cout, BM), ceil_div(a.Ng, BN), splits);
  hipLaunchKernelGGL((wgrad_fast_kernel<BM, BN, NWM, NWN, ROW32, PRE>), grid, dim3(64 * NWM * NWN), lds, st, a);
}

int launch_wgrad_fast(FastWgradArgs a, int splits, hipStream_t st) {
  const long nkt = (a.Kpix + kWgBK - 1) / kWgBK;
  a.kt_per_split = (int)((nkt + splits - 1) / splits);
  if (wgrad_ring_ok(a)) return launch_wgrad_ring(a, splits, st);
  static const bool no_row = getenv("UNETSEG_WG_NO_ROW32") != nullptr;
  // ROW32: every K step is one 32-pixel run of an output row, and the per-lane pixel deltas and
  // scalar bases fit 32-bit offsets (the caller bounds both tensors below 2^31 bytes)
  const bool row32 = !no_row && a.Q % kWgBK == 0;
  if (a.in_sc) {
    if (a.Cout <= 64) {
      if (row32) launch_wgrad_cfg<64, 256, 1, 4, true, true>(a, splits, st);
      else launch_wgrad_cfg<64, 256, 1, 4, false, true>(a, splits, st);
    } else {
      if (row32) launch_wgrad_cfg<128, 128, 2, 2, true, true>(a, splits, st);
      else launch_wgrad_cfg<128, 128, 2, 2, false, true>(a, splits, st);
    }
    return 0;
  }
  if (a.Cout <= 64) {
    if (row32) launch_wgrad_cfg<64, 256, 1, 4, true>(a, splits, st);
    else launch_wgrad_cfg<64, 256, 1, 4, false>(a, splits, st);
  } else {
    if (row32) launch_wgrad_cfg<128, 128, 2, 2, true>(a, splits, st);
    else launch_wgrad_cfg<128, 128, 2, 2, false>(a, splits, st);
  }
  return 0;
}
