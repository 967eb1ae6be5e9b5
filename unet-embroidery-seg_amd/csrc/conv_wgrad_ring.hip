// Weight gradient on an LDS-DMA ring (bf16, gfx950): the 1x1 / strided / small-grid shapes of the
// wgrad_fast family (conv_fast.hip) whose K steps are whole 32-pixel runs.  Its own translation unit
// because it is built with MFMA accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form, Makefile):
// with AGPR accumulators the register allocator rotates all 64 of them through v_accvgpr_mov every
// K step (as much issue time as the step's 16 MFMAs); the other conv kernels are unaffected by
// that and keep the default.
#include <cstdlib>

#include "common.h"
#include "conv_fast.h"
#include "fast_util.h"

namespace {

// ------------------------------------------------------------------------------------------
// wgrad on an LDS-DMA ring.  wgrad_fast_kernel keeps one K step in flight in registers; at the one
// or two blocks per CU its grids give (tiles x splits ~ 256-512), every step then waits out a
// global-memory latency and a 9 GFLOP 1x1 layer takes ~50 us.  Here the operand tiles of step
// kt+NS-1 are DMA'd into LDS while step kt computes.  Same tiles, LDS layout, K order and split
// boundaries as wgrad_fast_kernel, so the partial slabs are bit-identical to its.
// The LDS position of a 16-B chunk is fixed by the lane (64 lanes -> 1 KiB), so the row swizzle is
// applied to the global chunk each lane fetches.  K steps are 32 pixels: one run of an output row
// (Q % 32 == 0) or 32/Q whole rows (32 % Q == 0), so each lane's pixel delta within a step is a
// constant and the step's (n, p, q0) is scalar state.
// PRE (1x1 / stride 1 only): the BN-ReLU input prologue on the B fragments after the LDS read
// (one column per lane, so two coefficients per fragment); no row of such a step is padding.
// Conditions: wgrad_ring_ok.
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int NWM, int NWN, int NS, bool PRE>
__global__ __launch_bounds__(64 * NWM * NWN) void wgrad_ring_kernel(FastWgradArgs a) {
  constexpr int NW = NWM * NWN;
  constexpr int BKW = kWgBK;
  constexpr int CPA = BM / 8, CPB = BN / 8;
  constexpr int AI = BKW * CPA / 64, BI = BKW * CPB / 64;  // 1-KiB DMA rows per stage part
  constexpr int A_PER = AI / NW, B_PER = BI / NW;
  static_assert(A_PER * NW == AI && B_PER * NW == BI && A_PER >= 1 && B_PER >= 1, "tile / block shape");
  constexpr int PER = A_PER + B_PER;
  static_assert(NS >= 3 && PER * (NS - 2) <= 63, "vmcnt range");
  constexpr int WTM = BM / NWM, WTN = BN / NWN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr unsigned STAGE = BKW * (CPA + CPB) * 16;  // bytes
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / NWN, wn = wid % NWN;
  // 1-D grid of (split, tile) work items, split-major.  Workgroups go to the 8 XCDs round-robin, so
  // item = (L % 8) * (T / 8) + L / 8 gives each XCD a contiguous run of items: the tiles of a split
  // read the same pixels, which are then fetched into one L2 instead of all eight
  const int ntm = a.Cout / BM, ntn = (a.Ng + BN - 1) / BN, T = (int)gridDim.x;
  const int L = blockIdx.x;
  const int item = a.xcd_map && T % 8 == 0 ? (L & 7) * (T >> 3) + (L >> 3) : L;
  const int zsp = item / (ntm * ntn), tile = item - zsp * (ntm * ntn);
  const int m0 = (tile % ntm) * BM, n0 = (tile / ntm) * BN;
  const long nkt_total = a.Kpix / BKW;
  const long kt0 = (long)zsp * a.kt_per_split;
  const int nkt = (int)max(0L, min(nkt_total, kt0 + a.kt_per_split) - kt0);

  // PRE coefficients of this lane's B columns, loaded before the first DMA is issued (the
  // compiler's vmcnt bookkeeping does not see the DMA rows)
  float pre_sc[PRE ? FN : 1], pre_sh[PRE ? FN : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * WTN + j * 16 + (lane & 15);
      pre_sc[j] = n < a.Ng ? a.in_sc[n] : 0.f;
      pre_sh[j] = n < a.Ng ? a.in_sh[n] : 0.f;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }

  // lane constants of the DMA rows: A (dY) -> byte offset within a step; B (X) -> (tap, c) and the
  // pixel delta of the lane's row within a step
  unsigned a_off[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int idx = (i * NW + wid) * 64 + lane, row = idx / CPA, pos = idx % CPA;
    const int chunk = pos ^ (CPA >= 16 ? swz_tr16(row) : swz_tr8(row));
    a_off[i] = (unsigned)row * (unsigned)a.ldyb + (unsigned)(m0 + chunk * 8) * 2u;
  }
  const bool qrun = a.Q % BKW == 0;  // else 32 % Q == 0: a step is 32/Q whole rows
  int b_dh[B_PER], b_dw[B_PER];
  unsigned b_l[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int idx = (i * NW + wid) * 64 + lane, row = idx / CPB, pos = idx % CPB;
    const int chunk = pos ^ (CPB >= 16 ? swz_tr16(row) : swz_tr8(row));
    const int nn = n0 + chunk * 8;
    const int tap = nn / a.cin, c = nn - tap * a.cin;
    const int r = tap / a.S, s = tap - r * a.S;
    const int dp = qrun ? 0 : row / a.Q, dq = qrun ? row : row % a.Q;
    const bool col = nn < a.Ng;
    b_dh[i] = col ? dp * a.stride + r - a.pad : -(1 << 20);  // never valid past Ng
    b_dw[i] = dq * a.stride + s - a.padw;
    b_l[i] = col ? (unsigned)((b_dh[i] * a.W + b_dw[i]) * a.ldc1b) + (unsigned)c * 2u : 0u;
  }
  const int PQ = a.P * a.Q;
  int s_n, s_p, s_q;  // first pixel of the next step to issue
  {
    const long k = kt0 * BKW;
    s_n = (int)(k / PQ);
    const int rem = (int)(k - (long)s_n * PQ);
    s_p = rem / a.Q;
    s_q = rem - s_p * a.Q;
  }
  const int prow = qrun ? 1 : BKW / a.Q;
  const unsigned lbase = lds_addr(lds);
  // step j of this block into stage `stage`; steps past the block's end load through zero-extent
  // descriptors (no memory traffic), so every step issues PER rows and vmcnt counts stay uniform
  auto issue = [&](int j, int stage) {
    const bool live = j < nkt;
    const __amdgpu_buffer_rsrc_t ra = srd_u(a.dy, live ? a.dy_bytes : 0u);
    const __amdgpu_buffer_rsrc_t rb = srd_u(a.x1, live ? a.x1_bytes : 0u);
    const unsigned sb = __builtin_amdgcn_readfirstlane(lbase + (unsigned)stage * STAGE);
    const unsigned soa =
        __builtin_amdgcn_readfirstlane(live ? (unsigned)((kt0 + j) * BKW) * (unsigned)a.ldyb : 0u);
#pragma unroll
    for (int i = 0; i < A_PER; ++i) dma16s(ra, sb + (unsigned)((i * NW + wid) * 1024), a_off[i], soa);
    const int ihb = s_p * a.stride, iwb = s_q * a.stride;
    const unsigned xb = (unsigned)((s_n * a.H + ihb) * a.W + iwb) * (unsigned)a.ldc1b;
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const bool ok = (unsigned)(ihb + b_dh[i]) < (unsigned)a.H && (unsigned)(iwb + b_dw[i]) < (unsigned)a.W;
      dma16(rb, sb + (unsigned)((AI + i * NW + wid) * 1024), ok ? xb + b_l[i] : kOOB);
    }
    if (qrun) {
      s_q += BKW;
      if (s_q == a.Q) {
        s_q = 0;
        ++s_p;
      }
    } else {
      s_p += prow;
    }
    if (s_p == a.P) {
      s_p = 0;
      ++s_n;
    }
  };

  const int g = lane >> 4, i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3;
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
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NS - 1; ++s0) issue(s0, s0);
  int stage = 0;
  for (int kt = 0; kt < nkt; ++kt) {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PER * (NS - 2)) : "memory");
    const char* base = reinterpret_cast<const char*>(lds) + stage * STAGE;
    auto trpair = [&](unsigned o0, unsigned o1) -> bf16x8 {
      s16x4 va = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o0));
      s16x4 vb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o1));
      typedef short s16x8 __attribute__((ext_vector_type(8)));
      s16x8 v = {va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
      return *reinterpret_cast<bf16x8*>(&v);
    };
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = trpair(toffA[i][0], toffA[i][1]);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = trpair(toffB[j][0], toffB[j][1]);
    if constexpr (PRE) {  // == bn_apply: (bf16) relu(fmaf(z, sc, sh)); one channel per fragment
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        uint4 u = __builtin_bit_cast(uint4, bfr[j]);
        const f32x2 sc2 = {pre_sc[j], pre_sc[j]}, sh2 = {pre_sh[j], pre_sh[j]};
        u.x = bnrelu_pair(u.x, sc2, sh2);
        u.y = bnrelu_pair(u.y, sc2, sh2);
        u.z = bnrelu_pair(u.z, sc2, sh2);
        u.w = bnrelu_pair(u.w, sc2, sh2);
        bfr[j] = __builtin_bit_cast(bf16x8, u);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    issue(kt + NS - 1, stage == 0 ? NS - 1 : stage - 1);  // (stage + NS - 1) % NS: read by no one now
    stage = stage == NS - 1 ? 0 : stage + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prefetch past the end has landed
  float* ws = a.ws + (long)zsp * a.Cout * a.Ng;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wm * WTM + i * 16 + (lane >> 4) * 4 + e;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WTN + j * 16 + (lane & 15);
        if (n < a.Ng) ws[(long)m * a.Ng + n] = acc[i][j][e];
      }
    }
}

template <int BM, int BN, int NWM, int NWN, int NS, bool PRE>
static void launch_wgrad_ring_cfg(const FastWgradArgs& a, int splits, hipStream_t st) {
  const size_t lds = (size_t)NS * kWgBK * (BM / 8 + BN / 8) * 16;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_ring_kernel<BM, BN, NWM, NWN, NS, PRE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int blocks = (a.Cout / BM) * ceil_div(a.Ng, BN) * splits;
  hipLaunchKernelGGL((wgrad_ring_kernel<BM, BN, NWM, NWN, NS, PRE>), dim3(blocks), dim3(64 * NWM * NWN), lds, st, a);
}

template <int NS>
static void launch_wgrad_ring_ns(FastWgradArgs a, int splits, hipStream_t st) {
  static const bool no_xcd = getenv("UNETSEG_WG_NO_XCD") != nullptr;
  a.xcd_map = !no_xcd;
  if (a.Cout <= 64) {
    if (a.in_sc) launch_wgrad_ring_cfg<64, 256, 1, 4, NS, true>(a, splits, st);
    else launch_wgrad_ring_cfg<64, 256, 1, 4, NS, false>(a, splits, st);
  } else {
    if (a.in_sc) launch_wgrad_ring_cfg<128, 128, 2, 2, NS, true>(a, splits, st);
    else launch_wgrad_ring_cfg<128, 128, 2, 2, NS, false>(a, splits, st);
  }
}

}  // namespace

// shapes of the DMA-ring wgrad: one source, whole tiles of output channels, whole 32-pixel K steps
// that never straddle an image, and (PRE) a 1x1 / stride-1 filter
bool wgrad_ring_ok(const FastWgradArgs& a) {
  static const bool off = getenv("UNETSEG_WG_NO_RING") != nullptr;
  if (off || a.x2) return false;
  const int bm = a.Cout <= 64 ? 64 : 128;
  if (a.Cout % bm || a.Kpix % kWgBK) return false;
  const bool rows = a.Q % kWgBK == 0 || (kWgBK % a.Q == 0 && ((long)a.P * a.Q) % kWgBK == 0);
  if (!rows) return false;
  if (a.in_sc && (a.S != 1 || a.Ng != a.cin || a.stride != 1 || a.pad || a.padw)) return false;
  return true;
}


int launch_wgrad_ring(const FastWgradArgs& a, int splits, hipStream_t st) {
  static const int ns = getenv("UNETSEG_WG_RING_NS") ? atoi(getenv("UNETSEG_WG_RING_NS")) : 4;
  if (ns == 6) launch_wgrad_ring_ns<6>(a, splits, st);
  else if (ns == 8 && a.Cout > 64) launch_wgrad_ring_ns<8>(a, splits, st);
  else launch_wgrad_ring_ns<4>(a, splits, st);
  return 0;
}
