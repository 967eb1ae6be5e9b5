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

#include "common.h"
#include "conv_fast.h"
#include "fast_util.h"

namespace {


// ------------------------------------------------------------------------------------------
// TN (fwd / dgrad).  Tile: BM pixels x BN output channels, K step 64 channels of one tap.
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int NWM, int NWN>
__global__ __launch_bounds__(64 * NWM * NWN) void tn_fast_kernel(FastTNArgs a) {
  constexpr int NT = 64 * NWM * NWN;
  constexpr int WTM = BM / NWM, WTN = BN / NWN;
  constexpr int FP = WTM / 16, FC = WTN / 16;
  constexpr int RSTEP = NT / 8;
  constexpr int A_PER = BM / RSTEP, B_PER = BN / RSTEP;
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // [2][(BM+BN)*8]
  constexpr int STAGE = (BM + BN) * 8;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kv = tid & 7, rb = tid >> 3;
  const int hw = a.hc * a.wc;

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
      const int nb = m / hw, rem = m - nb * hw;
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
    boff[i] = n < a.Ng ? (unsigned)n * (unsigned)a.ldwb + kv * 16 : kOOB;
  }

  const int nch = a.cin >> 6;
  const int nsteps = a.nr * a.ns * nch;
  uint4 ra[A_PER], rbv[B_PER];
  // scalar K-step state
  int s_jr = 0, s_js = 0, s_c = 0;
  auto gload = [&]() {
    const int dh = a.dh0 + a.dhs * s_jr, dw = a.dw0 + a.dws * s_js;
    const int tapbit = s_jr * a.ns + s_js;
    const int tapdelta = dh * a.W + dw;
    const unsigned wofs = (unsigned)(((a.r0 + a.rs * s_jr) * a.S + (a.s0 + a.ss * s_js)) * a.cin + s_c) * 2u;
    if (s_c < a.c1) {
      const unsigned cb = (unsigned)s_c * 2u + kv * 16;
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const bool ok = (vmask[i] >> tapbit) & 1u;
        const unsigned off = (unsigned)(pix[i] + tapdelta) * (unsigned)a.ldc1b + cb;
        ra[i] = bload(r1, ok ? off : kOOB);
      }
    } else {
      const unsigned cb = (unsigned)(s_c - a.c1) * 2u + kv * 16;
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        const bool ok = (vmask[i] >> tapbit) & 1u;
        const unsigned off = (unsigned)(pix[i] + tapdelta) * (unsigned)a.ldc2b + cb;
        ra[i] = bload(r2, ok ? off : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) rbv[i] = bload(rw, boff[i] == kOOB ? kOOB : boff[i] + wofs);
    s_c += 64;
    if (s_c >= a.cin) {
      s_c = 0;
      if (++s_js == a.ns) { s_js = 0; ++s_jr; }
    }
  };
  auto sstore = [&](int buf) {
    uint4* L = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = rb + RSTEP * i;
      L[row * 8 + swz8(row, kv)] = ra[i];
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

  if (nsteps > 0) {
    gload();
    sstore(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nsteps; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nsteps) gload();
    const uint4* As = lds + cur * STAGE;
    const uint4* Bs = As + BM * 8;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 pf[FP], wf[FC];
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int row = wm * WTM + p * 16 + (lane & 15);
        uint4 v = As[row * 8 + swz8(row, ch)];
        pf[p] = *reinterpret_cast<bf16x8*>(&v);
      }
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int row = wn * WTN + c * 16 + (lane & 15);
        uint4 v = Bs[row * 8 + swz8(row, ch)];
        wf[c] = *reinterpret_cast<bf16x8*>(&v);
      }
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int p = 0; p < FP; ++p)
          acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], pf[p], acc[c][p], 0, 0, 0);
    }
    if (kt + 1 < nsteps) sstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds D[cout = (lane>>4)*4 + e][pixel = lane&15] per (c, p) subtile ----
  bf16* y = (bf16*)a.y;
  float csum[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[c][e] = 0.f;
  float bias[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c) {
    const int nb = n0 + wn * WTN + c * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[c][e] = (a.bias && nb + e < a.Ng) ? a.bias[nb + e] : 0.f;
  }
#pragma unroll
  for (int p = 0; p < FP; ++p) {
    const int m = m0 + wm * WTM + p * 16 + (lane & 15);
    const bool mok = m < a.M;
    long opix = 0;
    if (mok) {
      if (a.ostride == 1 && a.ph == 0 && a.pw == 0 && a.OW == a.wc && a.OH == a.hc) {
        opix = m;
      } else {
        const int nb = m / hw, rem = m - nb * hw;
        const int hh = rem / a.wc, ww = rem - hh * a.wc;
        opix = ((long)nb * a.OH + hh * a.ostride + a.ph) * a.OW + ww * a.ostride + a.pw;
      }
    }
#pragma unroll
    for (int c = 0; c < FC; ++c) {
      const int nb = n0 + wn * WTN + c * 16 + (lane >> 4) * 4;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = acc[c][p][e] + bias[c][e];
        if (a.relu) v[e] = fmaxf(v[e], 0.f);
      }
      if (mok && nb < a.Ng) {
        bf16* ptr = y + opix * a.ldy + nb;
        if (a.accumulate) {
          uint2 old = *reinterpret_cast<const uint2*>(ptr);
          const bf16* ob = reinterpret_cast<const bf16*>(&old);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)ob[e];
        }
        bf16 ob[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ob[e] = (bf16)v[e];
          v[e] = (float)ob[e];
          csum[c][e] += v[e];
        }
        *reinterpret_cast<uint2*>(ptr) = *reinterpret_cast<uint2*>(ob);
      }
      // keep the rounded value for the M2 pass
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[c][p][e] = (mok && nb < a.Ng) ? v[e] : 0.f;
    }
  }
  if (!a.stats) return;
  // per-tile BN partials: column sums over the tile's pixels, then M2 about the tile mean
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // [NWM][BN] sums, then [NWM][BN] M2
  const int cnt = min(BM, a.M - m0);
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float s = csum[c][e];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      s += __shfl_xor(s, 8, 64);
      if ((lane & 15) == 0) red[wm * BN + wn * WTN + c * 16 + (lane >> 4) * 4 + e] = s;
    }
  __syncthreads();
  float m2[FC][4];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = wn * WTN + c * 16 + (lane >> 4) * 4 + e;
      float tot = 0.f;
#pragma unroll
      for (int w = 0; w < NWM; ++w) tot += red[w * BN + col];
      const float mean = tot / (float)cnt;
      float q = 0.f;
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int m = m0 + wm * WTM + p * 16 + (lane & 15);
        if (m < a.M) {
          const float d = acc[c][p][e] - mean;
          q += d * d;
        }
      }
      q += __shfl_xor(q, 1, 64);
      q += __shfl_xor(q, 2, 64);
      q += __shfl_xor(q, 4, 64);
      q += __shfl_xor(q, 8, 64);
      m2[c][e] = q;
    }
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if ((lane & 15) == 0) red[NWM * BN + wm * BN + wn * WTN + c * 16 + (lane >> 4) * 4 + e] = m2[c][e];
  __syncthreads();
  for (int col = tid; col < BN; col += NT) {
    const int n = n0 + col;
    if (n < a.Ng) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < NWM; ++w) {
        s += red[w * BN + col];
        q += red[NWM * BN + w * BN + col];
      }
      a.stats[(long)n * a.stats_ld + blockIdx.x] = s;
      a.stats[((long)a.Ng + n) * a.stats_ld + blockIdx.x] = q;
    }
  }
}

// ------------------------------------------------------------------------------------------
// wgrad: C[cout][(tap, c)] = sum_pix dY[pix][cout] * X[n][p*st+dh][q*st+dw][c];
// tile BM couts x BN (tap,c) columns, K step = 32 pixels of one image row.
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int NWM, int NWN>
__global__ __launch_bounds__(64 * NWM * NWN) void wgrad_fast_kernel(FastWgradArgs a) {
  constexpr int NT = 64 * NWM * NWN;
  constexpr int BKW = 32;
  constexpr int CPA = BM / 8, CPB = BN / 8;  // 16-B chunks per LDS row
  constexpr int A_PER = BKW * CPA / NT, B_PER = BKW * CPB / NT;
  constexpr int WTM = BM / NWM, WTN = BN / NWN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  __shared__ __attribute__((aligned(16))) uint4 lds[2][BKW * (CPA + CPB)];
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
  // B (X) chunk: column fixed -> (tap, c) fixed
  int b_row[B_PER], b_dh[B_PER], b_dw[B_PER], b_src[B_PER], b_cv[B_PER];
  unsigned b_cb[B_PER];
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
      b_dw[i] = s - a.pad;
      b_src[i] = c < a.c1 ? 0 : 1;
      b_cb[i] = (unsigned)(c < a.c1 ? c : c - a.c1) * 2u;
    } else {
      b_dh[i] = -(1 << 20);  // never valid
      b_dw[i] = 0;
      b_src[i] = 0;
      b_cb[i] = 0;
    }
  }
  const unsigned a_colb0 = (unsigned)m0 * 2u;
  const long nkt_total = (a.Kpix + BKW - 1) / BKW;
  const long kt0 = (long)blockIdx.z * a.kt_per_split;
  const long kt1 = min(nkt_total, kt0 + a.kt_per_split);
  const int PQ = a.P * a.Q;

  uint4 ra[A_PER], rbv[B_PER];
  auto gload = [&](long kt) {
    const long k0 = kt * BKW;  // first pixel of the step (uniform)
    const int nb = (int)(k0 / PQ);
    const int rem = (int)(k0 - (long)nb * PQ);
    const int p = rem / a.Q, q0 = rem - p * a.Q;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const long k = k0 + a_row[i];
      const bool ok = k < a.Kpix && (m0 + a_cv[i] * 8) < a.Cout;
      const unsigned off = (unsigned)k * (unsigned)a.ldyb + a_colb0 + a_cv[i] * 16u;
      ra[i] = bload(rdy, ok ? off : kOOB);
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int ih = p * a.stride + b_dh[i];
      const int iw = (q0 + b_row[i]) * a.stride + b_dw[i];
      const bool ok = (k0 + b_row[i]) < a.Kpix && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      const unsigned pixi = (unsigned)((nb * a.H + ih) * a.W + iw);
      if (b_src[i] == 0)
        rbv[i] = bload(r1, ok ? pixi * (unsigned)a.ldc1b + b_cb[i] : kOOB);
      else
        rbv[i] = bload(r2, ok ? pixi * (unsigned)a.ldc2b + b_cb[i] : kOOB);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = a_row[i];
      const int sw = CPA >= 16 ? swz_tr16(row) : swz_tr8(row);
      lds[buf][row * CPA + (a_cv[i] ^ sw)] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = b_row[i];
      const int sw = CPB >= 16 ? swz_tr16(row) : swz_tr8(row);
      lds[buf][BKW * CPA + row * CPB + (b_cv[i] ^ sw)] = rbv[i];
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
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kt0 + kt + 1);
    const char* base = reinterpret_cast<const char*>(&lds[cur][0]);
    auto trfrag = [&](int off_bytes, int cpr, int col0) -> bf16x8 {
      const int chunk = (col0 >> 3) + (pp >> 1);
      const int ra_ = 8 * g + qq, rb_ = 8 * g + qq + 4;
      const int swa = cpr >= 16 ? swz_tr16(ra_) : swz_tr8(ra_);
      const int swb = cpr >= 16 ? swz_tr16(rb_) : swz_tr8(rb_);
      const char* pa = base + off_bytes + ra_ * (cpr * 16) + ((chunk ^ swa) * 16) + (pp & 1) * 8;
      const char* pb = base + off_bytes + rb_ * (cpr * 16) + ((chunk ^ swb) * 16) + (pp & 1) * 8;
      s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(pa));
      s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(pb));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      s16x8 v = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
      return *reinterpret_cast<bf16x8*>(&v);
    };
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = trfrag(0, CPA, wm * WTM + i * 16);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = trfrag(BKW * CPA * 16, CPB, wn * WTN + j * 16);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
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

// ------------------------------------------------------------------------------------------
// TN v3: persistent, 3-stage LDS-DMA pipeline.
//  * operands go HBM/L2 -> LDS by buffer_load_dwordx4 ... lds (no VGPR staging); the XOR
//    swizzle of the LDS image is applied to the per-lane SOURCE offset (the DMA destination is
//    lane-linear), padding taps / out-of-range rows read past num_records -> zeros;
//  * counted `s_waitcnt vmcnt(N)` + raw s_barrier: two stages stay in flight while one is
//    consumed (never vmcnt(0) in the steady state);
//  * persistent blocks (one per CU) walk tiles; the loads of the next tile's first steps overlap
//    the current tile's epilogue.  Tiles are dealt so that the 8 XCDs each get contiguous runs
//    (neighbouring pixel rows share halos in one L2); speed-only, never correctness.
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int NWM, int NWN>
__global__ __launch_bounds__(64 * NWM * NWN) void tn_dma_kernel(FastTNArgs a, int mtiles, int ntiles) {
  constexpr int NW = NWM * NWN;
  constexpr int WTM = BM / NWM, WTN = BN / NWN;
  constexpr int FP = WTM / 16, FC = WTN / 16;
  constexpr int AI = BM / 8 / NW, BI = BN / 8 / NW;
  constexpr int INS = AI + BI;
  constexpr int STAGES = 3;
  constexpr int STAGE = (BM + BN) * 8;  // uint4 per stage
  static_assert(AI >= 1 && BI >= 1, "each wave must issue A and B DMA");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  float* red = reinterpret_cast<float*>(lds + STAGES * STAGE);  // [2][NWM][BN] stats scratch
  float* sbias = red + 2 * NWM * BN;                             // [Ng] bias

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  const int hw = a.hc * a.wc;
  const __amdgpu_buffer_rsrc_t r1 = srd(a.x1, a.x1_bytes);
  const __amdgpu_buffer_rsrc_t r2 = srd(a.x2 ? a.x2 : a.x1, a.x2 ? a.x2_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rw = srd(a.wt, a.w_bytes);
  if (a.bias)
    for (int i = tid; i < a.Ng; i += 64 * NW) sbias[i] = a.bias[i];

  // tiles of this block: XCD-grouped deal of the persistent grid
  const int G = gridDim.x;
  const int total = mtiles * ntiles;
  const int nx = G / 8;
  const int slot = (G % 8 == 0) ? ((int)blockIdx.x % 8) * nx + (int)blockIdx.x / 8 : (int)blockIdx.x;
  const int my_tiles = slot < total ? (total - slot + G - 1) / G : 0;
  const int nch = a.cin >> 6;
  const int nsteps = a.nr * a.ns * nch;
  const int total_steps = my_tiles * nsteps;

  // ---- issue-side state (scalar) and per-lane row info of the tile being issued ----
  int is_tile = 0, is_jr = 0, is_js = 0, is_c = 0;
  int pix[AI];
  unsigned vmask[AI], boff[BI];
  const int pc = lane & 7, rsub = lane >> 3;
  auto setup_rows = [&](int t) {
    const int tile = slot + t * G;
    const int tm = tile % mtiles, tn = tile / mtiles;
    const int m0 = tm * BM, n0 = tn * BN;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = (wid * AI + i) * 8 + rsub;
      const int m = m0 + row;
      pix[i] = 0;
      vmask[i] = 0u;
      if (m < a.M) {
        const int nb = m / hw, rem = m - nb * hw;
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
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int row = (wid * BI + i) * 8 + rsub;
      const int n = n0 + row;
      const int lc = swz8(row, pc);  // logical chunk held by physical chunk pc (XOR involution)
      boff[i] = n < a.Ng ? (unsigned)n * (unsigned)a.ldwb + lc * 16 : kOOB;
    }
  };
  auto issue = [&](int buf) {
    const int dh = a.dh0 + a.dhs * is_jr, dw = a.dw0 + a.dws * is_js;
    const int tapbit = is_jr * a.ns + is_js;
    const int tapdelta = dh * a.W + dw;
    const unsigned wofs = (unsigned)(((a.r0 + a.rs * is_jr) * a.S + (a.s0 + a.ss * is_js)) * a.cin + is_c) * 2u;
    const unsigned base = lds_addr(lds) + (unsigned)buf * (STAGE * 16);
    const bool first = is_c < a.c1;
    const unsigned ldcb = first ? (unsigned)a.ldc1b : (unsigned)a.ldc2b;
    const unsigned cb = (unsigned)(first ? is_c : is_c - a.c1) * 2u;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int row = (wid * AI + i) * 8 + rsub;
      const int lc = swz8(row, pc);  // logical chunk held by physical chunk pc (XOR involution)
      const bool ok = (vmask[i] >> tapbit) & 1u;
      const unsigned off = ok ? (unsigned)(pix[i] + tapdelta) * ldcb + cb + lc * 16 : kOOB;
      const unsigned dst = base + (unsigned)(wid * AI + i) * 1024u;
      if (first)
        dma16(r1, dst, off);
      else
        dma16(r2, dst, off);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const unsigned dst = base + (unsigned)(BM * 128 + (wid * BI + i) * 1024);
      dma16(rw, dst, boff[i] == kOOB ? kOOB : boff[i] + wofs);
    }
    is_c += 64;
    if (is_c >= a.cin) {
      is_c = 0;
      if (++is_js == a.ns) {
        is_js = 0;
        if (++is_jr == a.nr) {
          is_jr = 0;
          if (++is_tile < my_tiles) setup_rows(is_tile);
        }
      }
    }
  };

  f32x4 acc[FC][FP];
#pragma unroll
  for (int c = 0; c < FC; ++c)
#pragma unroll
    for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};

  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // sbias visible
  if (total_steps > 0) setup_rows(0);
  if (total_steps > 0) issue(0);
  if (total_steps > 1) issue(1);

  int ct = 0, cstep = 0, bc = 0, bi = 2;
  for (int g = 0; g < total_steps; ++g) {
    if (g + 1 < total_steps)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(INS) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (g + 2 < total_steps) {
      issue(bi);
      bi = bi == STAGES - 1 ? 0 : bi + 1;
    }
    const uint4* As = lds + bc * STAGE;
    bc = bc == STAGES - 1 ? 0 : bc + 1;
    const uint4* Bs = As + BM * 8;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 pf[FP], wf[FC];
#pragma unroll
      for (int p = 0; p < FP; ++p) {
        const int row = wm * WTM + p * 16 + (lane & 15);
        uint4 v = As[row * 8 + swz8(row, ch)];
        pf[p] = *reinterpret_cast<bf16x8*>(&v);
      }
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int row = wn * WTN + c * 16 + (lane & 15);
        uint4 v = Bs[row * 8 + swz8(row, ch)];
        wf[c] = *reinterpret_cast<bf16x8*>(&v);
      }
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int p = 0; p < FP; ++p)
          acc[c][p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], pf[p], acc[c][p], 0, 0, 0);
    }
    if (++cstep < nsteps) continue;
    // ================= epilogue of tile ct =================
    cstep = 0;
    const int tile = slot + ct * G;
    ++ct;
    const int tm = tile % mtiles, tn = tile / mtiles;
    const int m0 = tm * BM, n0 = tn * BN;
    bf16* y = (bf16*)a.y;
    float csum[FC][4];
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[c][e] = 0.f;
#pragma unroll
    for (int p = 0; p < FP; ++p) {
      const int m = m0 + wm * WTM + p * 16 + (lane & 15);
      const bool mok = m < a.M;
      long opix = 0;
      if (mok) {
        if (a.ostride == 1 && a.ph == 0 && a.pw == 0 && a.OW == a.wc && a.OH == a.hc) {
          opix = m;
        } else {
          const int nb = m / hw, rem = m - nb * hw;
          const int hh = rem / a.wc, ww = rem - hh * a.wc;
          opix = ((long)nb * a.OH + hh * a.ostride + a.ph) * a.OW + ww * a.ostride + a.pw;
        }
      }
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int nb = n0 + wn * WTN + c * 16 + (lane >> 4) * 4;
        const bool ok = mok && nb < a.Ng;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[c][p][e] + ((a.bias && ok) ? sbias[nb + e] : 0.f);
          if (a.relu) v[e] = fmaxf(v[e], 0.f);
        }
        if (ok) {
          bf16* ptr = y + opix * a.ldy + nb;
          if (a.accumulate) {
            uint2 old = *reinterpret_cast<const uint2*>(ptr);
            const bf16* ob = reinterpret_cast<const bf16*>(&old);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += (float)ob[e];
          }
          bf16 ob[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ob[e] = (bf16)v[e];
            v[e] = (float)ob[e];
            csum[c][e] += v[e];
          }
          *reinterpret_cast<uint2*>(ptr) = *reinterpret_cast<uint2*>(ob);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[c][p][e] = ok ? v[e] : 0.f;
      }
    }
    if (a.stats) {
      const int cnt = min(BM, a.M - m0);
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sm = csum[c][e];
          sm += __shfl_xor(sm, 1, 64);
          sm += __shfl_xor(sm, 2, 64);
          sm += __shfl_xor(sm, 4, 64);
          sm += __shfl_xor(sm, 8, 64);
          if ((lane & 15) == 0) red[wm * BN + wn * WTN + c * 16 + (lane >> 4) * 4 + e] = sm;
        }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
      for (int c = 0; c < FC; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int col = wn * WTN + c * 16 + (lane >> 4) * 4 + e;
          float tot = 0.f;
#pragma unroll
          for (int w = 0; w < NWM; ++w) tot += red[w * BN + col];
          const float mean = tot / (float)cnt;
          float q = 0.f;
#pragma unroll
          for (int p = 0; p < FP; ++p) {
            const int m = m0 + wm * WTM + p * 16 + (lane & 15);
            if (m < a.M) {
              const float d = acc[c][p][e] - mean;
              q += d * d;
            }
          }
          q += __shfl_xor(q, 1, 64);
          q += __shfl_xor(q, 2, 64);
          q += __shfl_xor(q, 4, 64);
          q += __shfl_xor(q, 8, 64);
          if ((lane & 15) == 0) red[NWM * BN + wm * BN + col] = q;
        }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      for (int col = tid; col < BN; col += 64 * NW) {
        const int n = n0 + col;
        if (n < a.Ng) {
          float sm = 0.f, q = 0.f;
#pragma unroll
          for (int w = 0; w < NWM; ++w) {
            sm += red[w * BN + col];
            q += red[NWM * BN + w * BN + col];
          }
          a.stats[(long)n * a.stats_ld + tm] = sm;
          a.stats[((long)a.Ng + n) * a.stats_ld + tm] = q;
        }
      }
      // protect `red` against the next tile's epilogue
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll
    for (int c = 0; c < FC; ++c)
#pragma unroll
      for (int p = 0; p < FP; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int BM, int BN, int NWM, int NWN>
int launch_tn_dma(const FastTNArgs& a, hipStream_t st) {
  constexpr int NW = NWM * NWN;
  const size_t lds = 3 * (size_t)(BM + BN) * 128 + (size_t)(2 * NWM * BN) * 4 + (size_t)a.Ng * 4;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tn_dma_kernel<BM, BN, NWM, NWN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  const int mtiles = ceil_div(a.M, BM), ntiles = ceil_div(a.Ng, BN);
  int grid = 256;  // one block per CU
  if (mtiles * ntiles < grid) grid = mtiles * ntiles;
  hipLaunchKernelGGL((tn_dma_kernel<BM, BN, NWM, NWN>), dim3(grid), dim3(64 * NW), lds, st, a, mtiles, ntiles);
  return 0;
}

template <int BM, int BN, int NWM, int NWN>
int launch_tn_cfg(const FastTNArgs& a, hipStream_t st) {
  constexpr int NT = 64 * NWM * NWN;
  const size_t lds = 2 * (size_t)(BM + BN) * 8 * 16;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tn_fast_kernel<BM, BN, NWM, NWN>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  dim3 grid(ceil_div(a.M, BM), ceil_div(a.Ng, BN), 1);
  hipLaunchKernelGGL((tn_fast_kernel<BM, BN, NWM, NWN>), grid, dim3(NT), lds, st, a);
  return 0;
}

}  // namespace

bool tn_fast_ok(const FastTNArgs& a) {
  return a.cin % 64 == 0 && a.c1 % 64 == 0 && a.nr * a.ns <= 32 && a.Ng % 8 == 0;
}

// The persistent LDS-DMA kernel is opt-in until it beats the register-staged one.
static bool use_v3() {
  static const bool on = getenv("UNETSEG_TN_V3") != nullptr;
  return on;
}

int tn_fast_tile_m(const FastTNArgs& a) {
  if (halo3_ok(a)) return halo_tile_m();
  if (a.Ng <= 64) return 256;
  const long tiles_big = (long)ceil_div(a.M, 256) * ceil_div(a.Ng, 128);
  if (use_v3()) return tiles_big >= 128 ? 256 : 128;
  return tiles_big >= 256 ? 256 : 128;
}

int launch_tn_fast(const FastTNArgs& a, hipStream_t st) {
  if (a.M <= 0 || a.Ng <= 0) return 0;
  if (halo3_ok(a)) return launch_halo3(a, st);
  // zero-tap dgrad parity classes (nr*ns == 0) only write zeros: the register-staged kernel's
  // empty K loop does that, the persistent kernel would skip the tile entirely
  if (use_v3() && a.Ng <= 64 * 2048 && a.nr * a.ns > 0) {  // bias staged in LDS
    if (a.Ng <= 64) return launch_tn_dma<256, 64, 8, 1>(a, st);
    if (tn_fast_tile_m(a) == 256) return launch_tn_dma<256, 128, 4, 2>(a, st);
    return launch_tn_dma<128, 128, 2, 4>(a, st);
  }
  if (a.Ng <= 64) return launch_tn_cfg<256, 64, 4, 1>(a, st);
  if (tn_fast_tile_m(a) == 256) return launch_tn_cfg<256, 128, 4, 2>(a, st);
  return launch_tn_cfg<128, 128, 2, 2>(a, st);
}

bool wgrad_fast_ok(const FastWgradArgs& a) {
  return a.Q % 32 == 0 && a.cin % 8 == 0 && a.c1 % 8 == 0 && a.Cout % 64 == 0;
}

int wgrad_fast_splits(int Cout, int Ng, long Kpix) {
  const int bm = Cout <= 64 ? 64 : 128;
  const int bn = Cout <= 64 ? 256 : 128;
  const int tiles = ceil_div(Cout, bm) * ceil_div(Ng, bn);
  const long nkt = (Kpix + 31) / 32;
  int sp = ceil_div(Cout <= 64 ? 1024 : 512, tiles);  // 2-4 blocks per CU
  const long max_sp = nkt / 32 > 0 ? nkt / 32 : 1;  // >= 32 K steps per split
  if (sp > max_sp) sp = (int)max_sp;
  if (sp > 512) sp = 512;
  if (sp < 1) sp = 1;
  return sp;
}

int launch_wgrad_fast(FastWgradArgs a, int splits, hipStream_t st) {
  const long nkt = (a.Kpix + 31) / 32;
  a.kt_per_split = (int)((nkt + splits - 1) / splits);
  if (a.Cout <= 64) {
    dim3 grid(ceil_div(a.Cout, 64), ceil_div(a.Ng, 256), splits);
    hipLaunchKernelGGL((wgrad_fast_kernel<64, 256, 1, 4>), grid, dim3(256), 0, st, a);
  } else {
    dim3 grid(ceil_div(a.Cout, 128), ceil_div(a.Ng, 128), splits);
    hipLaunchKernelGGL((wgrad_fast_kernel<128, 128, 2, 2>), grid, dim3(256), 0, st, a);
  }
  return 0;
}
