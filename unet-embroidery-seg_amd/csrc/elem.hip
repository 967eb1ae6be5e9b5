// Memory-bound NHWC kernels of the U-Net hot path: BatchNorm (train/eval), ReLU, residual add,
// max-pool, bilinear x2 upsample, input packing, small-Cout 1x1 convs and the attention gate.
//
// Reference ops replaced:
//   BatchNorm2d      model/resnet_backbone.py:64-70,127,169  model/unet_plain.py:10,13
//                    model/unet_attention.py:17,21,25
//   ReLU / residual  model/resnet_backbone.py:95,100,110,113  model/unet_resnet.py:37,40,73,75
//   MaxPool2d        model/resnet_backbone.py:131 (3x3/s2 ceil)  model/unet_plain.py:25 (2x2)
//   Upsample x2      model/unet_resnet.py:21,71 (align_corners=True)  model/unet_plain.py:36 (False)
//   AttentionGate    model/unet_attention.py:30-35
//
// Layout: activations NHWC with an explicit pixel stride ("ld", elements) so channel slices of a
// concat buffer are addressed in place.  Element type T is bf16 or fp32; all arithmetic is fp32.
// Every per-channel reduction is two-stage (per-block partials -> finalize) and deterministic.
#include <algorithm>

#include "common.h"

namespace {

template <typename T>
constexpr int VE = 16 / sizeof(T);

// ------------------------------------------------------------------------------------------
// Per-channel reductions of row partials part[g][q][C] (G row tiles, q = 0 .. nq-1) -- the BN
// finalizes of the forward statistics and of the fused data-gradient post-ops.  They sit on the
// compute stream between a producer and its consumer, so they are latency kernels: one wave per
// channel (NWV = 1, four channels per block, no barrier) when G <= 512, a block of NWV = 4 waves per
// channel above that; every lane issues all its loads (kFinRPL rows x nq) before it adds, and the
// lanes' fp64 partials are combined in a fixed order (deterministic).  Never 1024-thread blocks: beside
// the weight-gradient stream's persistent kernels such a block found no CU until they drained (a
// 12 us colsum took 235 us in the bench trace); 256-thread blocks ran at their isolated speed.
// ------------------------------------------------------------------------------------------
constexpr int kFinRPL = 8;  // rows per lane per round

static inline int fin_waves(int G) { return G > 512 ? 4 : 1; }
static inline unsigned fin_blocks(int C, int nwv) { return nwv > 1 ? (unsigned)C : (unsigned)ceil_div(C, 4); }
static inline unsigned fin_threads(int nwv) { return nwv > 1 ? 64u * nwv : 256u; }
// launch KERNEL<nwv> for the row count G with the finalize geometry
#define FIN_LAUNCH(KERNEL, C, G, stream, ...)                                                                  \
  do {                                                                                                     \
    const int nwv_ = fin_waves(G);                                                                         \
    const dim3 grid_(fin_blocks(C, nwv_)), block_(fin_threads(nwv_));                                      \
    if (nwv_ == 4) hipLaunchKernelGGL(KERNEL<4>, grid_, block_, 0, (hipStream_t)(stream), __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<1>, grid_, block_, 0, (hipStream_t)(stream), __VA_ARGS__);              \
  } while (0)

// fp64 sum over the wave, the same value in every lane: row rotations on the VALU (each 64-bit value
// moved as two DPP halves) leave every lane of a 16-lane row with the row's total, then the four row
// totals are read lane-uniform and added in a fixed order.  wave_sum_d (__shfl_xor) went through
// ds_bpermute, two LDS round trips per step for a double: the finalize kernels sat on that chain
template <int CTL>
__device__ __forceinline__ double row_rot_add_d(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int lo2 = __builtin_amdgcn_update_dpp(0, lo, CTL, 0xF, 0xF, false);
  const int hi2 = __builtin_amdgcn_update_dpp(0, hi, CTL, 0xF, 0xF, false);
  return v + __hiloint2double(hi2, lo2);
}
__device__ __forceinline__ double wave_sum_d_uniform(double v) {
  v = row_rot_add_d<0x128>(v);  // row_ror:8
  v = row_rot_add_d<0x124>(v);  // row_ror:4
  v = row_rot_add_d<0x122>(v);  // row_ror:2
  v = row_rot_add_d<0x121>(v);  // row_ror:1
  const int lo = __double2loint(v), hi = __double2hiint(v);
  double t = 0.0;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    t += __hiloint2double(__builtin_amdgcn_readlane(hi, 16 * r), __builtin_amdgcn_readlane(lo, 16 * r));
  return t;
}

// sum over the channel's lanes (one wave, or the block's NWV waves through sc[NQ][NWV]); every lane
// gets the same fixed-order total
template <int NWV, int NQ>
__device__ __forceinline__ void fin_group_sum(double (&v)[NQ], double* sc) {
#pragma unroll
  for (int j = 0; j < NQ; ++j) v[j] = wave_sum_d_uniform(v[j]);
  if constexpr (NWV > 1) {
    const int wid = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int j = 0; j < NQ; ++j) sc[j * NWV + wid] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      double t = 0.0;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t += sc[j * NWV + w];
      v[j] = t;
    }
  }
}

// t[j] = sum_g part[g * ldrow + (q0 + j) * C + c] for j < nq (NQ >= nq)
template <int NWV, int NQ>
__device__ __forceinline__ void fin_row_sums(const float* part, long ldrow, int C, int c, int G, int nq, int q0,
                                             double (&t)[NQ], double* sc) {
  constexpr int NL = 64 * NWV;
  const int li = NWV == 1 ? (threadIdx.x & 63) : threadIdx.x;
#pragma unroll
  for (int j = 0; j < NQ; ++j) t[j] = 0.0;
  for (int g0 = 0; g0 < G; g0 += kFinRPL * NL) {
    // every load unconditional (a row past G re-reads row G - 1, a quantity past nq the last one) and
    // masked after it: a load under a lane condition got its own branch and a vmcnt(0) behind it, which
    // serialised all kFinRPL x NQ round trips of the lane
    float v[NQ][kFinRPL];
#pragma unroll
    for (int k = 0; k < kFinRPL; ++k) {
      const int g = min(g0 + li + k * NL, G - 1);
#pragma unroll
      for (int j = 0; j < NQ; ++j) v[j][k] = part[g * ldrow + (long)(q0 + min(j, nq - 1)) * C + c];
    }
#pragma unroll
    for (int k = 0; k < kFinRPL; ++k) {
      const bool ok = g0 + li + k * NL < G;
#pragma unroll
      for (int j = 0; j < NQ; ++j) t[j] += (ok && j < nq) ? (double)v[j][k] : 0.0;
    }
  }
  fin_group_sum<NWV, NQ>(t, sc);
}

// ------------------------------------------------------------------------------------------
// BatchNorm finalize (train): partials [G][2][C] = (sum, M2 about the tile mean) with tile
// count min(tile, M - g*tile).  Chan's parallel merge in fp64.  Updates running stats exactly as
// nn.BatchNorm2d (momentum 0.1, unbiased running var) and emits scale/shift for the apply pass.
// ------------------------------------------------------------------------------------------
template <int NWV>
__global__ __launch_bounds__(NWV > 4 ? 64 * NWV : 256) void bn_finalize_kernel(const float* part, int C, int G, long M, int tile,
                                                          const float* gamma, const float* beta, float* rmean,
                                                          float* rvar, long long* nbt, float momentum, float eps,
                                                          float* mean_out, float* invstd_out, float* scale,
                                                          float* shift) {
  __shared__ double sc[NWV];
  constexpr int NL = 64 * NWV;
  const int c = NWV == 1 ? (int)blockIdx.x * 4 + (threadIdx.x >> 6) : (int)blockIdx.x;
  if (NWV == 1 && c >= C) return;  // whole waves: no barrier in the one-wave form
  const int li = NWV == 1 ? (threadIdx.x & 63) : threadIdx.x;
  const long st = 2L * C;
  // the epilogue's operands loaded up front (behind the reductions each was a round trip)
  const float gam = gamma[c], bet = beta[c];
  const float rm0 = (rmean ? rmean : gamma)[c], rv0 = (rmean ? rvar : gamma)[c];  // unused without rmean
  // pass 1 keeps this lane's rows in registers when one round covers G (pass 2 re-reads otherwise)
  float sv[kFinRPL], qv[kFinRPL];
  double tsum[1] = {0.0};
  // unconditional loads (a row past G re-reads row G - 1), masked after: see fin_row_sums
  for (int g0 = 0; g0 < G; g0 += kFinRPL * NL) {
#pragma unroll
    for (int k = 0; k < kFinRPL; ++k) {
      const int g = min(g0 + li + k * NL, G - 1);
      sv[k] = part[g * st + c];
      qv[k] = part[g * st + C + c];
    }
#pragma unroll
    for (int k = 0; k < kFinRPL; ++k) {
      if (g0 + li + k * NL >= G) sv[k] = qv[k] = 0.f;
      tsum[0] += (double)sv[k];
    }
  }
  fin_group_sum<NWV, 1>(tsum, sc);
  const double mean = tsum[0] / (double)M;
  double m2[1] = {0.0};
  const bool one_round = G <= kFinRPL * NL;
  for (int g0 = 0; g0 < G; g0 += kFinRPL * NL) {
    if (!one_round) {
#pragma unroll
      for (int k = 0; k < kFinRPL; ++k) {
        const int g = min(g0 + li + k * NL, G - 1);
        sv[k] = part[g * st + c];
        qv[k] = part[g * st + C + c];
      }
    }
#pragma unroll
    for (int k = 0; k < kFinRPL; ++k) {
      const int g = g0 + li + k * NL;
      if (g < G) {
        const long cnt = min((long)tile, M - (long)g * tile);
        const double mg = (double)sv[k] / (double)cnt;
        m2[0] += (double)qv[k] + (double)cnt * (mg - mean) * (mg - mean);
      }
    }
  }
  fin_group_sum<NWV, 1>(m2, sc);
  if (li == 0) {
    const double m2v = m2[0];
    const double var = m2v / (double)M;
    const double inv = 1.0 / sqrt(var + (double)eps);
    mean_out[c] = (float)mean;
    invstd_out[c] = (float)inv;
    const float sca = (float)(gam * inv);
    scale[c] = sca;
    shift[c] = (float)(bet - mean * gam * inv);
    if (rmean) {
      const double unb = M > 1 ? m2v / (double)(M - 1) : var;
      rmean[c] = (float)((1.0 - momentum) * rm0 + momentum * mean);
      rvar[c] = (float)((1.0 - momentum) * rv0 + momentum * unb);
    }
    if (nbt && c == 0) nbt[0] += 1;
  }
}

// eval-mode BN folded into the preceding conv: kscale = gamma / sqrt(var + eps),
// bias = beta - mean * kscale (+ conv_bias * kscale)
__global__ void bn_fold_kernel(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                               float eps, const float* conv_bias, float* kscale, float* bias) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  // the same float expressions as bn_eval_kernel, so the folded epilogue fmaf(acc, kscale, bias)
  // equals the unfolded BN pass fmaf(y, scale, shift) bit for bit in fp32
  const float inv = 1.0f / sqrtf(rvar[c] + eps);
  const float sc = gamma[c] * inv;
  kscale[c] = sc;
  const float sh = beta[c] - rmean[c] * gamma[c] * inv;
  bias[c] = conv_bias ? sh + conv_bias[c] * sc : sh;
}

__global__ void bn_eval_kernel(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                               float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.0f / sqrtf(rvar[c] + eps);
  scale[c] = gamma[c] * inv;
  shift[c] = beta[c] - rmean[c] * gamma[c] * inv;
}

// out = act(y*sc + sh + res); res: 0 none, 1 raw tensor r, 2 r*sc2 + sh2
// mbits (may be NULL): the ReLU mask of `out` packed one byte per (pixel, V-channel vector), bit e =
// (stored out[c0 + e] > 0), [M][C/V] -- the BN backward reads it instead of the whole activation
template <typename T>
__global__ void bn_apply_kernel(const T* y, int ldy, const float* sc, const float* sh, const T* r, int ldr,
                                const float* sc2, const float* sh2, int res_mode, int relu, T* out, int ldo, long M,
                                int C, uint8_t* mbits) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const long total = M * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / cv;
    const int c0 = (int)(i - pix * cv) * V;
    float v[V], rv[V];
    load_vec(y + pix * ldy + c0, v);
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = fmaf(v[e], sc[c0 + e], sh[c0 + e]);  // == bwd mask recompute
    if (res_mode) {
      load_vec(r + pix * ldr + c0, rv);
      if (res_mode == 2) {
#pragma unroll
        for (int e = 0; e < V; ++e) rv[e] = rv[e] * sc2[c0 + e] + sh2[c0 + e];
      }
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] += rv[e];
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    store_vec(out + pix * ldo + c0, v);
    if (mbits) {
      unsigned b = 0u;
#pragma unroll
      for (int e = 0; e < V; ++e) b |= ((float)(T)v[e] > 0.f ? 1u : 0u) << e;
      mbits[i] = (uint8_t)b;  // i == pix * cv + c0 / V
    }
  }
}

// ------------------------------------------------------------------------------------------
// Channel reductions over pixels (BN backward pass 1, ReLU-backward bias gradient).
// Block = 256 threads = tv channel vectors (16 B each) x rows pixel rows; each thread walks its
// pixel rows RU at a time with every load of the group issued before any use (the loads of a
// group are independent, so a wave keeps RU x tensors 16-B requests in flight).  Per-thread sums
// are folded across the wave's pixel rows with xor-shuffles (lanes with equal tx), then across
// the 4 waves through LDS.  Partials: part[k][C][G] (k = quantity), one column per block row.
// ------------------------------------------------------------------------------------------
constexpr int RU = 4;

template <typename T>
__device__ __forceinline__ void cvt16(const uint4& raw, float (&out)[16 / sizeof(T)]) {
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int i = 0; i < 16 / (int)sizeof(T); ++i) out[i] = (float)e[i];
}

// sum over the lanes of a wave that share (lane % tv); result valid in every lane
__device__ __forceinline__ float rows_sum(float v, int tv) {
  for (int o = tv; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// NQ quantities x V channels per thread -> part[k][C][G] column blockIdx.x
template <int NQ, int V>
__device__ __forceinline__ void store_partials(float (&s)[NQ][V], int tv, int c0, int C, int G, float* part,
                                               float* red /* [4][NQ][64][V] */) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, tx = threadIdx.x % tv;
#pragma unroll
  for (int k = 0; k < NQ; ++k)
#pragma unroll
    for (int e = 0; e < V; ++e) s[k][e] = rows_sum(s[k][e], tv);
  if (lane < tv) {
#pragma unroll
    for (int k = 0; k < NQ; ++k)
#pragma unroll
      for (int e = 0; e < V; ++e) red[((w * NQ + k) * 64 + tx) * V + e] = s[k][e];
  }
  __syncthreads();
  constexpr int nw = 4;  // waves per block (256 threads)
  const int cb = c0 - tx * V;        // first channel of this block's group
  for (int idx = threadIdx.x; idx < NQ * tv * V; idx += 256) {
    const int k = idx / (tv * V), rem = idx - k * tv * V;
    const int cx = rem / V, e = rem - cx * V;
    float t = 0.f;
    for (int ww = 0; ww < nw; ++ww) t += red[((ww * NQ + k) * 64 + cx) * V + e];
    part[((long)k * C + cb + cx * V + e) * G + blockIdx.x] = t;
  }
}

// BatchNorm backward, pass 1: per-(channel, pixel tile) partials of
//   sum dz, sum dz*xhat1, sum dz*xhat2     where dz = dA * mask
// MASK: 0 none, 1 (A > 0), 2 (y1*msc + msh > 0) -- the ReLU mask recomputed exactly as bn_apply
// produced A, 3 the packed mask bn_apply wrote (A = mbits [M][C/V] bytes).  Y2: second BN branch
// (downsample shortcut) present.
template <typename T, int MASK, bool Y2>
__device__ __forceinline__ void bn_bwd_reduce_body(const T* dA, int ldd, const T* A, int lda, const float* msc,
                                                   const float* msh, const T* y1, int ld1, const float* mean1,
                                                   const float* inv1, const T* y2, int ld2, const float* mean2,
                                                   const float* inv2, long M, int C, int tv, int pix_per_block,
                                                   float* part, int G) {
  constexpr int V = VE<T>;
  constexpr int NQ = Y2 ? 3 : 2;
  __shared__ float red[4 * 3 * 64 * V];
  const int tx = threadIdx.x % tv, ty = threadIdx.x / tv, rows = 256 / tv;
  const int c0 = (blockIdx.y * tv + tx) * V;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = min(M, p0 + pix_per_block);
  float s[NQ][V], m1[V], i1[V], m2v[V], i2v[V], ms[V], mh[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) s[k][e] = 0.f;
    m1[e] = mean1[c0 + e];
    i1[e] = inv1[c0 + e];
    m2v[e] = Y2 ? mean2[c0 + e] : 0.f;
    i2v[e] = Y2 ? inv2[c0 + e] : 0.f;
    ms[e] = MASK == 2 ? msc[c0 + e] : 0.f;
    mh[e] = MASK == 2 ? msh[c0 + e] : 0.f;
  }
  const uint8_t* mb = reinterpret_cast<const uint8_t*>(A);
  const int cv = C / V;
  auto acc = [&](const uint4& rd, const uint4& rx, const uint4& ra, const uint4& r2) {
    float d[V], x[V];
    cvt16<T>(rd, d);
    cvt16<T>(rx, x);
    if (MASK == 3) {
#pragma unroll
      for (int e = 0; e < V; ++e) d[e] = (ra.x >> e) & 1u ? d[e] : 0.f;
    } else if (MASK == 1) {
      float a[V];
      cvt16<T>(ra, a);
#pragma unroll
      for (int e = 0; e < V; ++e) d[e] = a[e] > 0.f ? d[e] : 0.f;
    } else if (MASK == 2) {
#pragma unroll
      for (int e = 0; e < V; ++e) d[e] = fmaf(x[e], ms[e], mh[e]) > 0.f ? d[e] : 0.f;
    }
    // explicit fmaf: the same rounding in every MASK / Y2 instantiation (the compiler's own
    // contraction choices differed between them)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      s[0][e] += d[e];
      s[1][e] = fmaf(d[e], (x[e] - m1[e]) * i1[e], s[1][e]);
    }
    if (Y2) {
      float x2[V];
      cvt16<T>(r2, x2);
#pragma unroll
      for (int e = 0; e < V; ++e) s[NQ - 1][e] = fmaf(d[e], (x2[e] - m2v[e]) * i2v[e], s[NQ - 1][e]);
    }
  };
  long p = p0 + ty;
  for (; p + (long)(RU - 1) * rows < p1; p += (long)RU * rows) {
    uint4 rd[RU], rx[RU], ra[RU], r2[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long q = p + (long)u * rows;
      rd[u] = *reinterpret_cast<const uint4*>(dA + q * ldd + c0);
      rx[u] = *reinterpret_cast<const uint4*>(y1 + q * ld1 + c0);
      if (MASK == 1) ra[u] = *reinterpret_cast<const uint4*>(A + q * lda + c0);
      if (MASK == 3) ra[u].x = mb[q * cv + c0 / V];
      if (Y2) r2[u] = *reinterpret_cast<const uint4*>(y2 + q * ld2 + c0);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) acc(rd[u], rx[u], ra[u], r2[u]);
  }
  for (; p < p1; p += rows) {
    uint4 rd = *reinterpret_cast<const uint4*>(dA + p * ldd + c0), ra = rd, r2 = rd;
    const uint4 rx = *reinterpret_cast<const uint4*>(y1 + p * ld1 + c0);
    if (MASK == 1) ra = *reinterpret_cast<const uint4*>(A + p * lda + c0);
    if (MASK == 3) ra.x = mb[p * cv + c0 / V];
    if (Y2) r2 = *reinterpret_cast<const uint4*>(y2 + p * ld2 + c0);
    acc(rd, rx, ra, r2);
  }
  store_partials<NQ, V>(s, tv, c0, C, G, part, red);
}

#define BN_RED_PARAMS                                                                                             \
  const T *dA, int ldd, const T *A, int lda, const float *msc, const float *msh, const T *y1, int ld1,            \
      const float *mean1, const float *inv1, const T *y2, int ld2, const float *mean2, const float *inv2, long M, \
      int C, int tv, int pix_per_block, float *part, int G
#define BN_RED_ARGS dA, ldd, A, lda, msc, msh, y1, ld1, mean1, inv1, y2, ld2, mean2, inv2, M, C, tv, pix_per_block, part, G
template <typename T, int MASK, bool Y2>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BN_RED_PARAMS) {
  bn_bwd_reduce_body<T, MASK, Y2>(BN_RED_ARGS);
}
// the packed-mask variant (one branch) with a register budget of four waves per SIMD: under the
// default target the scheduler serialised its main loop -- each of the 12 loads of an RU group waited on
// before the next was issued: 19.7 -> 14.5 us (C2's call), 17.1 -> 10.2 (C5's two).  With the second
// branch (Y2) the budget measured slower (12.2 -> 13.9 us): that one keeps the plain kernel
template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 4))) void bn_bwd_reduce_bits_kernel(
    BN_RED_PARAMS) {
  bn_bwd_reduce_body<T, 3, false>(BN_RED_ARGS);
}
#undef BN_RED_PARAMS
#undef BN_RED_ARGS

// pass 2: coefficients.  For branch b (1 or 2): dgamma_b += sum dz*xhat_b, dbeta_b += sum dz;
// coef[b][0][c] = gamma_b*invstd_b, coef[b][1][c] = mean(dz), coef[b][2][c] = mean(dz*xhat_b)
__global__ void bn_bwd_finalize_kernel(const float* part, int C, int G, long M, int nbranch, const float* g1,
                                       const float* inv1, float* dg1, float* db1, const float* g2, const float* inv2,
                                       float* dg2, float* db2, float* coef) {
  __shared__ double sc[16];
  const int c = blockIdx.x;
  double t[3] = {0, 0, 0};
  for (int k = 0; k < 1 + nbranch; ++k) {
    double acc = 0.0;
    for (int g = threadIdx.x; g < G; g += blockDim.x) acc += part[((long)k * C + c) * G + g];
    t[k] = block_sum(acc, sc);
  }
  if (threadIdx.x == 0) {
    const double sdz = t[0];
    dg1[c] += (float)t[1];
    db1[c] += (float)sdz;
    coef[0 * C + c] = g1[c] * inv1[c];
    coef[1 * C + c] = (float)(sdz / (double)M);
    coef[2 * C + c] = (float)(t[1] / (double)M);
    if (nbranch == 2) {
      dg2[c] += (float)t[2];
      db2[c] += (float)sdz;
      coef[3 * C + c] = g2[c] * inv2[c];
      coef[4 * C + c] = (float)(sdz / (double)M);
      coef[5 * C + c] = (float)(t[2] / (double)M);
    }
  }
}

// pass 3: dy_b = coef_a*(dz - mean(dz) - xhat_b*mean(dz*xhat_b)); optional dzout (+)= dz.
// Same block geometry as pass 1 (fixed channels per thread): the per-channel coefficients are
// folded once into dy_b = P_b*dz + Q_b*(y_b - mean_b) + R_b and kept in registers.  DZ: 0 none, 1 store,
// 2 accumulate.
template <typename T, int MASK, bool Y2, int DZ>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* dA, int ldd, const T* A, int lda,
                                                           const float* msc, const float* msh, const T* y1, int ld1,
                                                           const float* mean1, const float* inv1, T* dy1, int ldo1,
                                                           const T* y2, int ld2, const float* mean2, const float* inv2,
                                                           T* dy2, int ldo2, const float* coef, T* dzout, int ldz,
                                                           long M, int C, int tv, int pix_per_block) {
  constexpr int V = VE<T>;
  const int tx = threadIdx.x % tv, ty = threadIdx.x / tv, rows = 256 / tv;
  const int c0 = (blockIdx.y * tv + tx) * V;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = min(M, p0 + pix_per_block);
  float P1[V], Q1[V], R1[V], M1[V], P2[V], Q2[V], R2[V], M2[V], ms[V], mh[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int c = c0 + e;
    const float k1 = coef[c], cx1 = coef[2 * C + c] * inv1[c];
    P1[e] = k1;
    Q1[e] = -k1 * cx1;
    R1[e] = -k1 * coef[C + c];
    M1[e] = mean1[c];
    if (Y2) {
      const float k2 = coef[3 * C + c], cx2 = coef[5 * C + c] * inv2[c];
      P2[e] = k2;
      Q2[e] = -k2 * cx2;
      R2[e] = -k2 * coef[4 * C + c];
      M2[e] = mean2[c];
    }
    ms[e] = MASK == 2 ? msc[c] : 0.f;
    mh[e] = MASK == 2 ? msh[c] : 0.f;
  }
  const uint8_t* mb = reinterpret_cast<const uint8_t*>(A);
  const int cv = C / V;
  auto one = [&](long q, const uint4& rd, const uint4& rx, const uint4& ra, const uint4& r2, const uint4& rz) {
    float d[V], x[V], o[V];
    cvt16<T>(rd, d);
    cvt16<T>(rx, x);
    if (MASK == 3) {
#pragma unroll
      for (int e = 0; e < V; ++e) d[e] = (ra.x >> e) & 1u ? d[e] : 0.f;
    } else if (MASK == 1) {
      float a[V];
      cvt16<T>(ra, a);
#pragma unroll
      for (int e = 0; e < V; ++e) d[e] = a[e] > 0.f ? d[e] : 0.f;
    } else if (MASK == 2) {
#pragma unroll
      for (int e = 0; e < V; ++e) d[e] = fmaf(x[e], ms[e], mh[e]) > 0.f ? d[e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = fmaf(P1[e], d[e], fmaf(Q1[e], x[e] - M1[e], R1[e]));
    store_vec(dy1 + q * ldo1 + c0, o);
    if (Y2) {
      cvt16<T>(r2, x);
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] = fmaf(P2[e], d[e], fmaf(Q2[e], x[e] - M2[e], R2[e]));
      store_vec(dy2 + q * ldo2 + c0, o);
    }
    if (DZ == 2) {
      cvt16<T>(rz, o);
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] += d[e];
      store_vec(dzout + q * ldz + c0, o);
    } else if (DZ == 1) {
      store_vec(dzout + q * ldz + c0, d);
    }
  };
  long p = p0 + ty;
  for (; p + (long)(RU - 1) * rows < p1; p += (long)RU * rows) {
    uint4 rd[RU], rx[RU], ra[RU], r2[RU], rz[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long q = p + (long)u * rows;
      rd[u] = *reinterpret_cast<const uint4*>(dA + q * ldd + c0);
      rx[u] = *reinterpret_cast<const uint4*>(y1 + q * ld1 + c0);
      if (MASK == 1) ra[u] = *reinterpret_cast<const uint4*>(A + q * lda + c0);
      if (MASK == 3) ra[u].x = mb[q * cv + c0 / V];
      if (Y2) r2[u] = *reinterpret_cast<const uint4*>(y2 + q * ld2 + c0);
      if (DZ == 2) rz[u] = *reinterpret_cast<const uint4*>(dzout + q * ldz + c0);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) one(p + (long)u * rows, rd[u], rx[u], ra[u], r2[u], rz[u]);
  }
  for (; p < p1; p += rows) {
    const uint4 rd = *reinterpret_cast<const uint4*>(dA + p * ldd + c0);
    const uint4 rx = *reinterpret_cast<const uint4*>(y1 + p * ld1 + c0);
    uint4 ra = rd, r2 = rd, rz = rd;
    if (MASK == 1) ra = *reinterpret_cast<const uint4*>(A + p * lda + c0);
    if (MASK == 3) ra.x = mb[p * cv + c0 / V];
    if (Y2) r2 = *reinterpret_cast<const uint4*>(y2 + p * ld2 + c0);
    if (DZ == 2) rz = *reinterpret_cast<const uint4*>(dzout + p * ldz + c0);
    one(p, rd, rx, ra, r2, rz);
  }
}

// dY = dA * (A > 0) and per-tile column sums of dY (bias gradient partials [C][G])
template <typename T>
__global__ __launch_bounds__(256) void relu_bwd_bias_kernel(const T* dA, int ldd, const T* A, int lda, T* dY, int ldy,
                                                            long M, int C, int tv, int pix_per_block, float* part,
                                                            int G) {
  constexpr int V = VE<T>;
  __shared__ float red[4 * 64 * V];
  const int tx = threadIdx.x % tv, ty = threadIdx.x / tv, rows = 256 / tv;
  const int c0 = (blockIdx.y * tv + tx) * V;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = min(M, p0 + pix_per_block);
  float s[1][V];
#pragma unroll
  for (int e = 0; e < V; ++e) s[0][e] = 0.f;
  auto one = [&](long q, const uint4& rd, const uint4& ra) {
    float d[V], a[V];
    cvt16<T>(rd, d);
    cvt16<T>(ra, a);
    // round like the stored gradient so db == sum of the dY actually fed to wgrad
    T tmp[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      tmp[e] = (T)(a[e] > 0.f ? d[e] : 0.f);
      s[0][e] += (float)tmp[e];
    }
    *reinterpret_cast<uint4*>(dY + q * ldy + c0) = *reinterpret_cast<uint4*>(tmp);
  };
  long p = p0 + ty;
  for (; p + (long)(RU - 1) * rows < p1; p += (long)RU * rows) {
    uint4 rd[RU], ra[RU];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long q = p + (long)u * rows;
      rd[u] = *reinterpret_cast<const uint4*>(dA + q * ldd + c0);
      ra[u] = *reinterpret_cast<const uint4*>(A + q * lda + c0);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) one(p + (long)u * rows, rd[u], ra[u]);
  }
  for (; p < p1; p += rows)
    one(p, *reinterpret_cast<const uint4*>(dA + p * ldd + c0), *reinterpret_cast<const uint4*>(A + p * lda + c0));
  store_partials<1, V>(s, tv, c0, C, G, part, red);
}

// The same coefficients from the row partials of a fused data-gradient post-op
// (unetseg_conv2d_dgrad_post): part[g][2][C] = (sum dz, sum dz*xhat) per row tile.
template <int NWV>
__global__ __launch_bounds__(NWV > 4 ? 64 * NWV : 256) void bn_bwd_finalize_rows_kernel(const float* part, int C, int G, long M,
                                                                   const float* g1, const float* inv1, float* dg1,
                                                                   float* db1, float* coef) {
  __shared__ double sc[2 * NWV];
  const int c = NWV == 1 ? (int)blockIdx.x * 4 + (threadIdx.x >> 6) : (int)blockIdx.x;
  if (NWV == 1 && c >= C) return;
  // the epilogue's operands loaded up front: behind the reduction each was another round trip
  const float pg = dg1[c], pb = db1[c], k1 = g1[c] * inv1[c];
  double t[2];
  fin_row_sums<NWV, 2>(part, 2L * C, C, c, G, 2, 0, t, sc);
  if ((NWV == 1 ? (threadIdx.x & 63) : threadIdx.x) == 0) {
    const double a0 = t[0], a1 = t[1];
    dg1[c] = pg + (float)a1;
    db1[c] = pb + (float)a0;
    coef[0 * C + c] = k1;
    coef[1 * C + c] = (float)(a0 / (double)M);
    coef[2 * C + c] = (float)(a1 / (double)M);
  }
}

// The two-branch form for the residual post-op (unetseg_conv2d_dgrad_post_res): part[g][1+nbranch][C] =
// (sum dz, sum dz*xhat1 [, sum dz*xhat2]) per row tile; coefficients as bn_bwd_finalize_kernel.
template <int NWV>
__global__ __launch_bounds__(NWV > 4 ? 64 * NWV : 256) void bn_bwd_finalize_rows_res_kernel(const float* part, int C, int G, long M,
                                                                       int nbranch, const float* g1,
                                                                       const float* inv1, float* dg1, float* db1,
                                                                       const float* g2, const float* inv2, float* dg2,
                                                                       float* db2, float* coef) {
  __shared__ double sc[3 * NWV];
  const int c = NWV == 1 ? (int)blockIdx.x * 4 + (threadIdx.x >> 6) : (int)blockIdx.x;
  if (NWV == 1 && c >= C) return;
  const int nq = 1 + nbranch;
  const float pg1 = dg1[c], pb1 = db1[c], k1 = g1[c] * inv1[c];
  float pg2 = 0.f, pb2 = 0.f, k2 = 0.f;
  if (nbranch == 2) {
    pg2 = dg2[c];
    pb2 = db2[c];
    k2 = g2[c] * inv2[c];
  }
  double t[3];
  fin_row_sums<NWV, 3>(part, (long)nq * C, C, c, G, nq, 0, t, sc);
  if ((NWV == 1 ? (threadIdx.x & 63) : threadIdx.x) == 0) {
    const double sdz = t[0];
    dg1[c] = pg1 + (float)t[1];
    db1[c] = pb1 + (float)sdz;
    coef[0 * C + c] = k1;
    coef[1 * C + c] = (float)(sdz / (double)M);
    coef[2 * C + c] = (float)(t[1] / (double)M);
    if (nbranch == 2) {
      dg2[c] = pg2 + (float)t[2];
      db2[c] = pb2 + (float)sdz;
      coef[3 * C + c] = k2;
      coef[4 * C + c] = (float)(sdz / (double)M);
      coef[5 * C + c] = (float)(t[2] / (double)M);
    }
  }
}

// out[c] (+)= sum_g part[g][k][c] for part [G][2][C] (bias gradient from the fused ReLU post-op)
template <int NWV>
__global__ __launch_bounds__(NWV > 4 ? 64 * NWV : 256) void colsum_rows_kernel(const float* part, int C, int G, int k, float* out,
                                                          int accumulate) {
  __shared__ double sc[NWV];
  const int c = NWV == 1 ? (int)blockIdx.x * 4 + (threadIdx.x >> 6) : (int)blockIdx.x;
  if (NWV == 1 && c >= C) return;
  const float prev = accumulate ? out[c] : 0.f;
  double t[1];
  if (G > 0) {
    fin_row_sums<NWV, 1>(part, 2L * C, C, c, G, 1, k, t, sc);
  } else {
    t[0] = 0.0;
  }
  if ((NWV == 1 ? (threadIdx.x & 63) : threadIdx.x) == 0) out[c] = accumulate ? prev + (float)t[0] : (float)t[0];
}

// out[c] (+)= sum_g part[c][g]   (fp64 accumulation, fixed order)
__global__ void colsum_finalize_kernel(const float* part, int C, int G, float* out, int accumulate) {
  __shared__ double sc[16];
  const int c = blockIdx.x;
  double acc = 0.0;
  for (int g = threadIdx.x; g < G; g += blockDim.x) acc += part[(long)c * G + g];
  acc = block_sum(acc, sc);
  if (threadIdx.x == 0) out[c] = accumulate ? out[c] + (float)acc : (float)acc;
}

// Row partials [G][nq][C] -> [ceil(G/R)][nq][C], R consecutive rows merged (ahead of a finalize when G
// is large: the one-channel-per-block finalize then reads strided rows on only C blocks).  CHAN: the
// rows are (sum, M2 about the row's mean) of `tile` pixels each (the last min(tile, M - g*tile)),
// merged by Chan's formula in fp64; otherwise plain fp64 sums per quantity.  One wave per output row
// and 64 channels, all R x nq loads issued before the adds (clamped, masked after).
template <bool CHAN, int NQ, int R>
__global__ __launch_bounds__(256) void fin_merge_rows_kernel(const float* part, int C, int G, long M, int tile, int nq,
                                                             float* out, int G2) {
  const int g2 = (int)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int c = (int)blockIdx.y * 64 + (threadIdx.x & 63);
  if (g2 >= G2) return;
  const int cc = min(c, C - 1);
  float v[R][NQ];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int g = min(g2 * R + r, G - 1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[r][q] = part[((long)g * nq + min(q, nq - 1)) * C + cc];
  }
  if (c >= C) return;
  if constexpr (CHAN) {
    double n = 0.0, s = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long g = (long)g2 * R + r;
      if (g < G) {
        n += (double)min((long)tile, M - g * tile);
        s += (double)v[r][0];
      }
    }
    const double mean = s / n;
    double m2 = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long g = (long)g2 * R + r;
      if (g < G) {
        const double cnt = (double)min((long)tile, M - g * tile);
        const double d = (double)v[r][0] / cnt - mean;
        m2 += (double)v[r][1] + cnt * d * d;
      }
    }
    out[(long)g2 * 2 * C + c] = (float)s;
    out[(long)g2 * 2 * C + C + c] = (float)m2;
  } else {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q >= nq) break;
      double t = 0.0;
#pragma unroll
      for (int r = 0; r < R; ++r) t += g2 * R + r < G ? (double)v[r][q] : 0.0;
      out[((long)g2 * nq + q) * C + c] = (float)t;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Max pool (pad 0), NHWC.  idx = argmax position inside the k x k window (first max wins, the
// scan order of ATen's CPU kernel), stored as uint8.
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void maxpool_fwd_kernel(const T* x, int ldx, int N, int H, int W, int C, int k, int s, int P, int Q, T* y,
                                   int ldy, uint8_t* idx) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const long total = (long)N * P * Q * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t = i;
    const int v = (int)(t % cv); t /= cv;
    const int q = (int)(t % Q); t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    const int c0 = v * V;
    float best[V];
    uint8_t bi[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int r = 0; r < k; ++r) {
      const int h = p * s + r;
      if (h >= H) break;
      for (int u = 0; u < k; ++u) {
        const int w = q * s + u;
        if (w >= W) break;
        float xv[V];
        load_vec(x + ((long)(n * H + h) * W + w) * ldx + c0, xv);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (xv[e] > best[e] || isnan(xv[e])) {
            if (!isnan(best[e])) { best[e] = xv[e]; bi[e] = (uint8_t)(r * k + u); }
          }
      }
    }
    const long opix = ((long)(n * P + p) * Q + q);
    store_vec(y + opix * ldy + c0, best);
#pragma unroll
    for (int e = 0; e < V; ++e) idx[opix * C + c0 + e] = bi[e];
  }
}

// The ResNet stem's pool (model/resnet_backbone.py:135: 3x3, stride 2, ceil mode) with the window
// compile-time: unrolled taps, 32-bit indexing, the 8 (bf16) argmax bytes of a pixel stored with one
// 8-B store.  Same comparisons in the same order as maxpool_fwd_kernel (bit-identical).
template <typename T>
__global__ void maxpool_fwd_k3s2_kernel(const T* x, int ldx, int N, int H, int W, int C, int P, int Q, T* y, int ldy,
                                        uint8_t* idx) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const int total = N * P * Q * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int t = i;
    const int v = t % cv; t /= cv;
    const int q = t % Q; t /= Q;
    const int p = t % P;
    const int n = t / P;
    const int c0 = v * V;
    float best[V];
    uint8_t bi[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int h = p * 2 + r;
      if (h >= H) break;
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int w = q * 2 + u;
        if (w >= W) break;
        float xv[V];
        load_vec(x + (size_t)((n * H + h) * W + w) * ldx + c0, xv);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (xv[e] > best[e] || isnan(xv[e])) {
            if (!isnan(best[e])) { best[e] = xv[e]; bi[e] = (uint8_t)(r * 3 + u); }
          }
      }
    }
    const size_t opix = (size_t)((n * P + p) * Q + q);
    store_vec(y + opix * ldy + c0, best);
    if constexpr (V == 8) {
      uint2 pk;
      __builtin_memcpy(&pk, bi, 8);
      *reinterpret_cast<uint2*>(idx + opix * C + c0) = pk;
    } else {
      unsigned pk;
      __builtin_memcpy(&pk, bi, 4);
      *reinterpret_cast<unsigned*>(idx + opix * C + c0) = pk;
    }
  }
}

// Its gradient: one thread per 2x2 input block (h = 2i + a, w = 2j + b) and V channels.  The windows
// that contain the block are (i-1 | i) x (j-1 | j); window (p, q) reaches row a of the block as window
// row r = a + 2 (p = i - 1, a = 0 only) or r = a (p = i), likewise columns.  Each window's dy and
// argmax bytes are loaded once per block (the per-pixel gather loaded them up to 9 times and the
// bytes one at a time); every pixel sums its windows in the same (p, q) order as maxpool_bwd_kernel.
template <typename T>
__global__ void maxpool_bwd_k3s2_kernel(const T* dy, int ldy, const uint8_t* idx, int N, int H, int W, int C, int P,
                                        int Q, T* dx, int ldx, int accumulate) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const int Hh = (H + 1) >> 1, Wh = (W + 1) >> 1;
  const int total = N * Hh * Wh * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int t = i;
    const int v = t % cv; t /= cv;
    const int bj = t % Wh; t /= Wh;
    const int bi = t % Hh;
    const int n = t / Hh;
    const int c0 = v * V;
    float acc[4][V];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < V; ++e) acc[k][e] = 0.f;
    // the four windows' dy and argmax bytes loaded first, at clamped (valid) windows: under the
    // window-range conditions each window's loads were a branch with a vmcnt(0) behind it; windows out
    // of range are skipped below, in the same (p, q) order
    uint4 graw[4];
    uint2 iraw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = min(max(bi - 1 + (k >> 1), 0), P - 1), q = min(max(bj - 1 + (k & 1), 0), Q - 1);
      const size_t opix = (size_t)((n * P + p) * Q + q);
      graw[k] = *reinterpret_cast<const uint4*>(dy + opix * ldy + c0);
      if constexpr (V == 8) iraw[k] = *reinterpret_cast<const uint2*>(idx + opix * C + c0);
      else iraw[k].x = *reinterpret_cast<const unsigned*>(idx + opix * C + c0);
    }
#pragma unroll
    for (int dp = 0; dp < 2; ++dp) {
      const int p = bi - 1 + dp;
      if (p < 0 || p >= P) continue;
#pragma unroll
      for (int dq = 0; dq < 2; ++dq) {
        const int q = bj - 1 + dq;
        if (q < 0 || q >= Q) continue;
        float g[V];
        cvt16<T>(graw[dp * 2 + dq], g);
        uint8_t ib[V];
        __builtin_memcpy(ib, &iraw[dp * 2 + dq], V);
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int r = dp ? a : a + 2;
          if (r >= 3) continue;
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int u = dq ? b : b + 2;
            if (u >= 3) continue;
            const uint8_t want = (uint8_t)(r * 3 + u);
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (ib[e] == want) acc[a * 2 + b][e] += g[e];
          }
        }
      }
    }
    uint4 oraw[4];  // the block's old gradient (accumulate), likewise loaded up front at clamped pixels
    if (accumulate)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int h = min(2 * bi + (k >> 1), H - 1), w = min(2 * bj + (k & 1), W - 1);
        oraw[k] = *reinterpret_cast<const uint4*>(dx + (size_t)((n * H + h) * W + w) * ldx + c0);
      }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int h = 2 * bi + a;
      if (h >= H) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int w = 2 * bj + b;
        if (w >= W) continue;
        T* o = dx + (size_t)((n * H + h) * W + w) * ldx + c0;
        if (accumulate) {
          float old[V];
          cvt16<T>(oraw[a * 2 + b], old);
#pragma unroll
          for (int e = 0; e < V; ++e) acc[a * 2 + b][e] += old[e];
        }
        store_vec(o, acc[a * 2 + b]);
      }
    }
  }
}

// The U-Net encoders' 2x2 / stride-2 pool (model/unet_plain.py:25, model/unet_attention.py) when the
// windows tile the input exactly (h = 2P, w = 2Q): one thread per window and V channels, the four
// loads issued together (the generic kernel's loop waited on each), the same comparisons in the same
// order as maxpool_fwd_kernel (bit-identical), the argmax bytes stored with one 8-B store.
template <typename T>
__global__ void maxpool_fwd_k2s2_kernel(const T* x, int ldx, int N, int H, int W, int C, int P, int Q, T* y, int ldy,
                                        uint8_t* idx) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const int total = N * P * Q * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int t = i;
    const int v = t % cv; t /= cv;
    const int q = t % Q; t /= Q;
    const int p = t % P;
    const int n = t / P;
    const int c0 = v * V;
    float xv[4][V];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int u = 0; u < 2; ++u) load_vec(x + (size_t)((n * H + 2 * p + r) * W + 2 * q + u) * ldx + c0, xv[r * 2 + u]);
    float best[V];
    uint8_t bi[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (xv[j][e] > best[e] || isnan(xv[j][e])) {
          if (!isnan(best[e])) { best[e] = xv[j][e]; bi[e] = (uint8_t)j; }
        }
    const size_t opix = (size_t)((n * P + p) * Q + q);
    store_vec(y + opix * ldy + c0, best);
    if constexpr (V == 8) {
      uint2 pk;
      __builtin_memcpy(&pk, bi, 8);
      *reinterpret_cast<uint2*>(idx + opix * C + c0) = pk;
    } else {
      unsigned pk;
      __builtin_memcpy(&pk, bi, 4);
      *reinterpret_cast<unsigned*>(idx + opix * C + c0) = pk;
    }
  }
}

// Its gradient: each input pixel lies in exactly one window, so one thread per window writes the
// window's four pixels from one dy load and one argmax load (the generic gather loaded the argmax
// bytes one at a time); values as maxpool_bwd_kernel's (0 + dy where the argmax matches, then + old).
template <typename T>
__global__ void maxpool_bwd_k2s2_kernel(const T* dy, int ldy, const uint8_t* idx, int N, int H, int W, int C, int P,
                                        int Q, T* dx, int ldx, int accumulate) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const int total = N * P * Q * cv;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int t = i;
    const int v = t % cv; t /= cv;
    const int q = t % Q; t /= Q;
    const int p = t % P;
    const int n = t / P;
    const int c0 = v * V;
    const size_t opix = (size_t)((n * P + p) * Q + q);
    float g[V];
    load_vec(dy + opix * ldy + c0, g);
    uint8_t ib[V];
    if constexpr (V == 8) {
      const uint2 pk = *reinterpret_cast<const uint2*>(idx + opix * C + c0);
      __builtin_memcpy(ib, &pk, 8);
    } else {
      const unsigned pk = *reinterpret_cast<const unsigned*>(idx + opix * C + c0);
      __builtin_memcpy(ib, &pk, 4);
    }
    float old[4][V];
    if (accumulate)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        load_vec(dx + (size_t)((n * H + 2 * p + (j >> 1)) * W + 2 * q + (j & 1)) * ldx + c0, old[j]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        o[e] = 0.f;
        if (ib[e] == (uint8_t)j) o[e] += g[e];
        if (accumulate) o[e] += old[j][e];
      }
      store_vec(dx + (size_t)((n * H + 2 * p + (j >> 1)) * W + 2 * q + (j & 1)) * ldx + c0, o);
    }
  }
}

// gather form: dx[h][w] (+)= sum over windows containing (h,w) whose argmax is (h,w)
template <typename T>
__global__ void maxpool_bwd_kernel(const T* dy, int ldy, const uint8_t* idx, int N, int H, int W, int C, int k, int s,
                                   int P, int Q, T* dx, int ldx, int accumulate) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const long total = (long)N * H * W * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long t = i;
    const int v = (int)(t % cv); t /= cv;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const int c0 = v * V;
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    const int plo = max(0, (h - k + s) / s), phi = min(P - 1, h / s);
    const int qlo = max(0, (w - k + s) / s), qhi = min(Q - 1, w / s);
    for (int p = plo; p <= phi; ++p) {
      const int r = h - p * s;
      if (r < 0 || r >= k) continue;
      for (int q = qlo; q <= qhi; ++q) {
        const int u = w - q * s;
        if (u < 0 || u >= k) continue;
        const long opix = ((long)(n * P + p) * Q + q);
        const uint8_t want = (uint8_t)(r * k + u);
        float g[V];
        load_vec(dy + opix * ldy + c0, g);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (idx[opix * C + c0 + e] == want) acc[e] += g[e];
      }
    }
    T* o = dx + ((long)(n * H + h) * W + w) * ldx + c0;
    if (accumulate) {
      float old[V];
      load_vec(o, old);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += old[e];
    }
    store_vec(o, acc);
  }
}

// ------------------------------------------------------------------------------------------
// Bilinear x2 upsample, NHWC (source index / weight: up_src, the blend: up_blend in common.h).
// ------------------------------------------------------------------------------------------

// Row-blocked: a block covers (pixel, 8-channel) lanes of whole output rows, kRowsPB rows in turn,
// so the per-row source index and weight are wave-uniform and the per-column ones are computed
// once per lane (the flat form spent its time in 64-bit index division).
constexpr int kUpRowsPB = 4;
// rows per block actually launched (UNETSEG_UP_ROWS = 2 or 8 overrides kUpRowsPB: experiments only)
static int up_rows_pb() {
  static const int r = [] {
    const char* e = getenv("UNETSEG_UP_ROWS");
    const int v = e ? atoi(e) : 0;
    return v == 2 || v == 8 ? v : kUpRowsPB;
  }();
  return r;
}

template <typename T>
__global__ void upsample_fwd_kernel(const T* x, int ldx, int N, int H, int W, int C, int align, T* y, int ldy,
                                    int rows_pb) {
  constexpr int V = VE<T>;
  const int cv = C / V, OH = 2 * H, OW = 2 * W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= OW * cv) return;
  const int ow = idx / cv, c0 = (idx - ow * cv) * V;
  int w0, w1;
  float lw;
  up_src(ow, W, OW, align, w0, w1, lw);
  const float wl0 = 1.f - lw;
  const int r0 = blockIdx.y * rows_pb, r1 = min(r0 + rows_pb, N * OH);
  for (int r = r0; r < r1; ++r) {
    const int n = r / OH, oh = r - n * OH;
    int h0, h1;
    float lh;
    up_src(oh, H, OH, align, h0, h1, lh);
    const T* x0 = x + (long)(n * H + h0) * W * ldx + c0;
    const T* x1 = x + (long)(n * H + h1) * W * ldx + c0;
    float a[V], b[V], c[V], d[V], o[V];
    load_vec(x0 + (long)w0 * ldx, a);
    load_vec(x0 + (long)w1 * ldx, b);
    load_vec(x1 + (long)w0 * ldx, c);
    load_vec(x1 + (long)w1 * ldx, d);
    const float hl0 = 1.f - lh;
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = up_blend(a[e], b[e], c[e], d[e], wl0, lw, hl0, lh);
    store_vec(y + ((long)r * OW + ow) * ldy + c0, o);
  }
}

// weight of output index d on input index i along one axis
__device__ __forceinline__ float up_w(int d, int i, int in, int out, int align) {
  int i0, i1;
  float l1;
  up_src(d, in, out, align, i0, i1, l1);
  float w = 0.f;
  if (i0 == i) w += 1.f - l1;
  if (i1 == i) w += l1;
  return w;
}

// candidate output range of input index i along one axis (a superset; exact weights decide)
__device__ __forceinline__ void up_range(int i, int in, int out, int align, int& lo, int& hi) {
  if (align) {
    lo = in > 1 ? (int)floorf((float)(i - 1) * (out - 1) / (float)(in - 1)) : 0;
    hi = in > 1 ? (int)ceilf((float)(i + 1) * (out - 1) / (float)(in - 1)) : out - 1;
  } else {
    lo = 2 * i - 2;
    hi = i == in - 1 ? out - 1 : 2 * i + 2;
  }
  lo = max(lo, 0);
  hi = min(hi, out - 1);
}

// Nonzero taps of input index i along one axis: the bilinear hat's support is contiguous and holds
// at most kUpK output indices at x2 in either align mode (open interval of length 4 + 2/(in-1) for
// align_corners, 4 for half-pixel) -> d0 and the weights of d0 .. d0 + kUpK - 1 (zero past the end).
constexpr int kUpK = 5;
__device__ __forceinline__ void up_taps(int i, int in, int out, int align, int& d0, float (&wt)[kUpK]) {
  int lo, hi;
  up_range(i, in, out, align, lo, hi);
  d0 = hi + 1;
  for (int d = hi; d >= lo; --d)
    if (up_w(d, i, in, out, align) != 0.f) d0 = d;
#pragma unroll
  for (int k = 0; k < kUpK; ++k) wt[k] = d0 + k <= hi ? up_w(d0 + k, i, in, out, align) : 0.f;
  if (d0 > hi) d0 = lo;
}

// Separable adjoint of the block's input rows r0 .. r0+nr-1 (r = n*H + h, nr <= R, wave-uniform):
// the dy rows J = n*OH + oh feeding them are contiguous in J (also across an image boundary), so
// each is gathered once per lane -- its column taps cw summed first (cs) -- and added to every
// block row it feeds with that row's weight: (2R+3)*4 loads per lane instead of R*16 for the
// per-pixel 2-D gather (+0.4% bench step at R = 4; R = 8 loses occupancy).  Row J+1's taps are
// loaded before row J's are consumed.  Zero weights are skipped (no 0 * inf).
template <typename T, int R, int PF = 1>
__device__ __forceinline__ void up_adjoint_rows(const T* dy, int ldy, int r0, int nr, int H, int OH, int OW,
                                                int align, int cd0, const float (&cw)[kUpK], int c0,
                                                float (&acc)[R][VE<T>]) {
  constexpr int V = VE<T>;
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int e = 0; e < V; ++e) acc[i][e] = 0.f;
  int nh[R], hh[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = r0 + min(i, nr - 1);
    nh[i] = r / H;
    hh[i] = r - nh[i] * H;
  }
  int lo, hi, t;
  up_range(hh[0], H, OH, align, lo, t);
  up_range(hh[R - 1], H, OH, align, t, hi);
  const int J0 = nh[0] * OH + lo, J1 = nh[R - 1] * OH + hi;
  auto gather = [&](int J, uint4 (&g)[kUpK]) {
    const T* row = dy + ((long)J * OW + cd0) * ldy + c0;
#pragma unroll
    for (int kw = 0; kw < kUpK; ++kw)
      g[kw] = (J <= J1 && cw[kw] != 0.f) ? *reinterpret_cast<const uint4*>(row + (long)kw * ldy)
                                         : uint4{0u, 0u, 0u, 0u};
  };
  uint4 gc[kUpK];
  gather(J0, gc);
  // PF 2: rows J+1 and J+2 in flight while row J is consumed
  uint4 gm[kUpK];
  if constexpr (PF == 2) gather(J0 + 1, gm);
  for (int J = J0; J <= J1; ++J) {
    uint4 gn[kUpK];
    gather(J + PF, gn);
    const int n = J / OH, oh = J - n * OH;
    float cs[V];
#pragma unroll
    for (int e = 0; e < V; ++e) cs[e] = 0.f;
#pragma unroll
    for (int kw = 0; kw < kUpK; ++kw)
      if (cw[kw] != 0.f) {
        float gv[V];
        cvt16<T>(gc[kw], gv);
#pragma unroll
        for (int e = 0; e < V; ++e) cs[e] += cw[kw] * gv[e];
      }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float w = (i < nr && nh[i] == n) ? up_w(oh, hh[i], H, OH, align) : 0.f;
      if (w != 0.f) {
#pragma unroll
        for (int e = 0; e < V; ++e) acc[i][e] += w * cs[e];
      }
    }
#pragma unroll
    for (int kw = 0; kw < kUpK; ++kw) {
      if constexpr (PF == 2) {
        gc[kw] = gm[kw];
        gm[kw] = gn[kw];
      } else {
        gc[kw] = gn[kw];
      }
    }
  }
}

#ifndef UNETSEG_UPBWD_PF
#define UNETSEG_UPBWD_PF 2
#endif
// gather form of the adjoint: dx[h][w] (+)= sum_{oh,ow} wh(oh,h) ww(ow,w) dy[oh][ow]; row-blocked
// like the forward (row weights wave-uniform, column weights once per lane)
template <typename T, int R>
__global__ __launch_bounds__(256) void upsample_bwd_kernel(const T* dy, int ldy, int N, int H, int W, int C, int align, T* dx, int ldx,
                                    int accumulate) {
  constexpr int V = VE<T>;
  const int cv = C / V, OH = 2 * H, OW = 2 * W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= W * cv) return;
  const int w = idx / cv, c0 = (idx - w * cv) * V;
  int cd0;
  float cw[kUpK];
  up_taps(w, W, OW, align, cd0, cw);
  const int r0 = blockIdx.y * R, nr = min(R, N * H - r0);
  float acc[R][V];
  up_adjoint_rows<T, R, UNETSEG_UPBWD_PF>(dy, ldy, r0, nr, H, OH, OW, align, cd0, cw, c0, acc);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    if (i >= nr) break;
    T* o = dx + ((long)(r0 + i) * W + w) * ldx + c0;
    if (accumulate) {
      float old[V];
      load_vec(o, old);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[i][e] += old[e];
    }
    store_vec(o, acc[i]);
  }
}

// upsample_bwd with the backward of the ReLU that produced x fused in (x = that ReLU's output, the
// upsample its sole consumer: the decoder's unetUp conv2 -> next block's Upsample,
// model/unet_resnet.py:25-33): dx = (A > 0) ? adjoint(dy) : 0, rounded to T as stored; part[g][0][c]
// = per-block column sums of the stored dx (the producer conv's bias-gradient partials, reduced by
// unetseg_colsum_rows), g = blockIdx.y * gridDim.x + blockIdx.x.  No accumulate.
template <typename T, int R>
__global__ __launch_bounds__(256) void upsample_bwd_relu_kernel(const T* dy, int ldy, int N, int H, int W, int C,
                                                                 int align, const T* A, int lda, T* dx, int ldx,
                                                                 float* part) {
  constexpr int V = VE<T>;
  __shared__ float red[256 * V];
  const int cv = C / V, OH = 2 * H, OW = 2 * W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = idx < W * cv;
  const int w = live ? idx / cv : 0, c0 = live ? (idx - w * cv) * V : 0;
  float s[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s[e] = 0.f;
  if (live) {
    int cd0;
    float cw[kUpK];
    up_taps(w, W, OW, align, cd0, cw);
    const int r0 = blockIdx.y * R, nr = min(R, N * H - r0);
    uint4 am[R];  // masks first: their latency hides under the gather
#pragma unroll
    for (int i = 0; i < R; ++i)
      am[i] = i < nr ? *reinterpret_cast<const uint4*>(A + ((long)(r0 + i) * W + w) * lda + c0) : uint4{0u, 0u, 0u, 0u};
    float acc[R][V];
    up_adjoint_rows<T, R>(dy, ldy, r0, nr, H, OH, OW, align, cd0, cw, c0, acc);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i >= nr) break;
      float a[V];
      cvt16<T>(am[i], a);
      T o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        o[e] = (T)(a[e] > 0.f ? acc[i][e] : 0.f);  // == upsample_bwd's stored value, then relu_bwd's mask
        s[e] += (float)o[e];
      }
      *reinterpret_cast<uint4*>(dx + ((long)(r0 + i) * W + w) * ldx + c0) = *reinterpret_cast<uint4*>(o);
    }
  }
  // block partials: the threads of one 8-channel group are tid % cv (256 % cv == 0, blocks start
  // at a pixel boundary)
#pragma unroll
  for (int e = 0; e < V; ++e) red[threadIdx.x * V + e] = s[e];
  __syncthreads();
  const long g = (long)blockIdx.y * gridDim.x + blockIdx.x;
  for (int i = threadIdx.x; i < cv * V; i += 256) {
    const int cx = i / V, e = i - cx * V;
    float t = 0.f;
    for (int j = cx; j < 256; j += cv) t += red[j * V + e];
    part[g * 2 * C + cx * V + e] = t;
  }
}

// Row-streaming form of upsample_bwd_relu (round 6): a block owns RS input rows of one image (RS | H)
// and walks the dy rows feeding them ONCE, top to bottom, keeping only the two input rows the current
// dy row touches (every dy row oh feeds rows i0 = floor(src) and i1 = i0 + 1, and i0 never decreases):
// a row is finished -- masked, stored, summed -- as soon as the walk passes it.  Against the R = 4
// row-blocked kernel above: (2 RS + 2) dy rows gathered per RS rows instead of (2 R + 3) per R
// (1.06x instead of 1.4x of dy re-read), K = 4 column taps where no column has a fifth (the U-Net
// sizes: up_taps_max), two rows in flight in 3 x K registers of 16 B, and the 32 accumulators of the
// R = 4 form down to 16.  Arithmetic identical to upsample_bwd (same up_taps / up_w weights, same
// per-row J order, same expressions): bit-identical dx.  part[g][0][c] as upsample_bwd_relu_kernel
// (g = blockIdx.y * gridDim.x + blockIdx.x).
// MASK false: the plain adjoint (unetseg_upsample2x_bwd: no ReLU, no partials, dx (+)= as upsample_bwd's).
template <typename T, int RS, int K, int PF, bool MASK = true>
__global__ __launch_bounds__(256, PF == 1 ? 4 : 3) void upsample_bwd_relu_stream_kernel(const T* dy, int ldy, int N, int H, int W,
                                                                        int C, int align, const T* A, int lda, T* dx,
                                                                        int ldx, float* part, int accumulate = 0) {
  constexpr int V = VE<T>;
  __shared__ float red[256 * V];
  const int cv = C / V, OH = 2 * H, OW = 2 * W;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = idx < W * cv;
  const int w = live ? idx / cv : 0, c0 = live ? (idx - w * cv) * V : 0;
  float s[V];
#pragma unroll
  for (int e = 0; e < V; ++e) s[e] = 0.f;
  if (live) {
    int cd0;
    float cw5[kUpK];
    up_taps(w, W, OW, align, cd0, cw5);
    float cw[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cw[k] = cw5[k];  // K = 4: the host checked cw5[4] == 0 for every column
    const int rb = blockIdx.y * RS;              // first stacked input row (n * H + h0), RS | H
    const int n = rb / H, h0 = rb - n * H;
    int lo, hi, t;
    up_range(h0, H, OH, align, lo, t);
    up_range(h0 + RS - 1, H, OH, align, t, hi);
    // dy through a buffer descriptor: per-lane tap offsets are constants (kOOB for a zero tap), the
    // dy row's offset is scalar -- no 64-bit address per tap and row
    const __amdgpu_buffer_rsrc_t rdy =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(dy), (short)0, (int)((long)N * OH * OW * ldy * (long)sizeof(T)), 0x00020000);
    unsigned toff[K];
#pragma unroll
    for (int k = 0; k < K; ++k) toff[k] = cw[k] != 0.f ? (unsigned)(((cd0 + k) * ldy + c0) * (int)sizeof(T)) : 0x80000000u;
    auto gather = [&](int oh, uint4 (&g)[K]) {
      const int ohc = oh <= hi ? oh : hi;  // past the block's last dy row: a re-read, never consumed
      const int soff = (int)(((long)n * OH + ohc) * OW * ldy * (long)sizeof(T));
#pragma unroll
      for (int k = 0; k < K; ++k) {
        typedef int i32x4_t __attribute__((ext_vector_type(4)));
        i32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rdy, (int)toff[k], soff, 0);
        g[k] = *reinterpret_cast<uint4*>(&v);
      }
    };
    const T* An = A + ((long)n * H * W + w) * lda + c0;
    T* dxn = dx + ((long)n * H * W + w) * ldx + c0;
    auto amask = [&](int r) -> uint4 {
      if constexpr (!MASK) return uint4{0u, 0u, 0u, 0u};
      return (r >= h0 && r < h0 + RS) ? *reinterpret_cast<const uint4*>(An + (long)r * W * lda) : uint4{0u, 0u, 0u, 0u};
    };
    // finish input row r (acc = its adjoint): mask, round as stored, partial sums
    auto finish = [&](int r, const float (&acc)[V], const uint4& am) {
      if (r < h0 || r >= h0 + RS) return;
      if constexpr (!MASK) {
        T* o = dxn + (long)r * W * ldx;
        float v[V];
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] = acc[e];
        if (accumulate) {
          float old[V];
          load_vec(o, old);
#pragma unroll
          for (int e = 0; e < V; ++e) v[e] += old[e];
        }
        store_vec(o, v);
        return;
      }
      float a[V];
      cvt16<T>(am, a);
      T o[V];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        o[e] = (T)(a[e] > 0.f ? acc[e] : 0.f);
        s[e] += (float)o[e];
      }
      *reinterpret_cast<uint4*>(dxn + (long)r * W * ldx) = *reinterpret_cast<uint4*>(o);
    };
    int i0, i1;
    float l1;
    up_src(lo, H, OH, align, i0, i1, l1);
    int ra = i0;  // rows ra (accA) and ra + 1 (accB)
    float accA[V], accB[V];
#pragma unroll
    for (int e = 0; e < V; ++e) accA[e] = accB[e] = 0.f;
    uint4 mA = amask(ra), mB = amask(ra + 1);
    // PF dy rows in flight beyond the one being consumed (1 or 2)
    uint4 gc[K], gm[PF == 2 ? K : 1];
    gather(lo, gc);
    if constexpr (PF == 2) gather(lo + 1, gm);
    for (int oh = lo; oh <= hi; ++oh) {
      uint4 gn[K];
      gather(oh + PF, gn);
      up_src(oh, H, OH, align, i0, i1, l1);
      if (i0 > ra) {  // row ra has had its last dy row (i0 advances by at most one per dy row)
        finish(ra, accA, mA);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          accA[e] = accB[e];
          accB[e] = 0.f;
        }
        mA = mB;
        ++ra;
        mB = amask(ra + 1);
      }
      float cs[V];
#pragma unroll
      for (int e = 0; e < V; ++e) cs[e] = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k)
        if (cw[k] != 0.f) {
          float gv[V];
          cvt16<T>(gc[k], gv);
#pragma unroll
          for (int e = 0; e < V; ++e) cs[e] += cw[k] * gv[e];
        }
      // the weights of upsample_bwd (up_w: rows i0 and i1, summed where they coincide)
      const float wA = up_w(oh, ra, H, OH, align), wB = up_w(oh, ra + 1, H, OH, align);
      if (wA != 0.f) {
#pragma unroll
        for (int e = 0; e < V; ++e) accA[e] += wA * cs[e];
      }
      if (wB != 0.f) {
#pragma unroll
        for (int e = 0; e < V; ++e) accB[e] += wB * cs[e];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if constexpr (PF == 2) {
          gc[k] = gm[k];
          gm[k] = gn[k];
        } else {
          gc[k] = gn[k];
        }
      }
    }
    finish(ra, accA, mA);
    finish(ra + 1, accB, mB);
  }
  if constexpr (!MASK) return;
#pragma unroll
  for (int e = 0; e < V; ++e) red[threadIdx.x * V + e] = s[e];
  __syncthreads();
  const long g = (long)blockIdx.y * gridDim.x + blockIdx.x;
  for (int i = threadIdx.x; i < cv * V; i += 256) {
    const int cx = i / V, e = i - cx * V;
    float t = 0.f;
    for (int j = cx; j < 256; j += cv) t += red[j * V + e];
    part[g * 2 * C + cx * V + e] = t;
  }
}

// NCHW fp32 [N][3][H][W] -> NHWC T [N][H][W][Cpad] (zero padded)
template <typename T>
__global__ void pack_input_kernel(const float* x, int N, int C, int H, int W, int Cpad, T* y) {
  const long total = (long)N * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / ((long)H * W), hw = i - n * H * W;
    T* o = y + i * Cpad;
    for (int c = 0; c < Cpad; ++c) o[c] = (T)(c < C ? x[(n * C + c) * (long)H * W + hw] : 0.f);
  }
}

// ------------------------------------------------------------------------------------------
// 1x1 conv with tiny Cout (final 64->2, seg_head 64->1, attention psi inter->1).
// Forward: one wave per 64/ (C/V) pixels; output fp32 planar [N][K][HW] (== [M] for K=1);
// optional BN partial stats of channel 0 per block (for psi: [G][2][1], tile = pixels/block).
// ------------------------------------------------------------------------------------------
template <typename T, int K>
__global__ void pw_small_fwd_kernel(const T* x, int ldx, long M, int HW, int C, const float* w, const float* b,
                                    float* y, float* stats, int pix_per_block) {
  constexpr int V = VE<T>;
  __shared__ double sred[16];
  const int cv = C / V;  // lanes per pixel (C/V <= 64, power of two)
  const int ppw = 64 / cv;  // pixels per wave pass
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int sub = lane / cv, v = lane % cv;
  const int ppb = pix_per_block < 0 ? -pix_per_block : pix_per_block;
  const long p0 = (long)blockIdx.x * ppb;
  const long p1 = min(M, p0 + ppb);
  float wv[K][V];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int e = 0; e < V; ++e) wv[k][e] = w[k * C + v * V + e];
  double lsum = 0.0;
  if (cv == 8 && !stats && pix_per_block > 0) {
    // 8 lanes per pixel: four pixel groups per iteration (four 16-B loads in flight per lane),
    // 8-lane sums by DPP (xor 1, xor 2 within quads, then row_half_mirror: lane 0 of each 8-lane
    // group adds lane 7, i.e. the other quad's sum) instead of LDS-routed shuffles
    constexpr int U = 4;
    for (long pbase = p0 + (long)wid * 8 * U; pbase < p1; pbase += (long)nw * 8 * U) {
      float acc[U][K];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // unconditional (clamped) load: a load under the lane condition got a branch and a vmcnt(0)
        // of its own, which serialised the four groups; past-the-end pixels are never stored
        const long pc = min(pbase + u * 8 + sub, p1 - 1);
        float xv[V];
        load_vec(x + pc * ldx + v * V, xv);
#pragma unroll
        for (int k = 0; k < K; ++k) {
          float a0 = 0.f;
#pragma unroll
          for (int e = 0; e < V; ++e) a0 += xv[e] * wv[k][e];
          acc[u][k] = a0;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) {
          float t = acc[u][k];
          t += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, t), 0xB1, 0xF, 0xF, false));
          t += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, t), 0x4E, 0xF, 0xF, false));
          t += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, t), 0x141, 0xF, 0xF, false));
          acc[u][k] = t;
        }
      if (v == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long p = pbase + u * 8 + sub;
          if (p < p1) {
            const long n = p / HW, hw = p - n * HW;
#pragma unroll
            for (int k = 0; k < K; ++k) y[(n * K + k) * HW + hw] = acc[u][k] + (b ? b[k] : 0.f);
          }
        }
      }
    }
    return;
  }
  // pass 1: outputs.  Four wave passes per iteration with their loads issued first at clamped (valid)
  // pixels: the one load under `p < p1` got a branch and a vmcnt(0) of its own, one exposed round trip
  // per pass (the attention psi conv at 8 x 512^2: 57 us for 142 MB).  The dot products are spelled out
  // as the one-pass loop compiled them -- rounded products (v_pk_mul_f32), then adds in channel order --
  // so the outputs stay bit-identical whatever the unrolled code would have been contracted to
  // (the bias is loaded once up front: read under the store's lane condition it was another branch
  // with a vmcnt(0) behind it)
  constexpr int U = 4;
  const long wstep = (long)nw * ppw;
  float bk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) bk[k] = b ? b[k] : 0.f;
  for (long pbase = p0 + (long)wid * ppw; pbase < p1; pbase += U * wstep) {
    uint4 raw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long pc = min(pbase + u * wstep + sub, p1 - 1);
      raw[u] = *reinterpret_cast<const uint4*>(x + pc * ldx + v * V);
    }
    // keep the four loads together: the scheduler otherwise started unpacking the first one before the
    // others were issued (a vmcnt(0) right behind it)
    __builtin_amdgcn_sched_barrier(0);
    float xv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) cvt16<T>(raw[u], xv[u]);
    float acc[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < K; ++k) {
#pragma clang fp contract(off)
        acc[u][k] = 0.f;
#pragma unroll
        for (int e = 0; e < V; ++e) acc[u][k] += xv[u][e] * wv[k][e];
      }
    for (int o = 1; o < cv; o <<= 1)
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[u][k] += __shfl_xor(acc[u][k], o, 64);
    if (v == 0)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = pbase + u * wstep + sub;
        if (p < p1) {
          const long n = p / HW, hw = p - n * HW;
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const float val = acc[u][k] + bk[k];
            y[(n * K + k) * HW + hw] = val;
            if (k == 0) lsum += val;
          }
        }
      }
  }
  if (!stats) return;
  const double tot = block_sum(lsum, sred);
  const long cnt = p1 - p0;
  const double mean = tot / (double)cnt;
  __syncthreads();
  double lm2 = 0.0;
  for (long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const long n = p / HW, hw = p - n * HW;
    const double d = (double)y[(n * K) * HW + hw] - mean;
    lm2 += d * d;
  }
  const double m2 = block_sum(lm2, sred);
  if (threadIdx.x == 0) {
    stats[2 * blockIdx.x] = (float)tot;  // [G][2][1]
    stats[2 * blockIdx.x + 1] = (float)m2;
  }
}

// Backward of the tiny-Cout 1x1 conv.  dy fp32 planar [N][K][HW].
//   dx (+)= dy . W  (T, NHWC, ld), partials for dW [K][C][G] and db [K][G]
// MASK: x is the output of a ReLU whose backward is fused here (this conv is x's sole consumer):
// dx = (x > 0) ? dy . W : 0, and part_d[G][2][C] (slot 0) gets the column sums of the stored
// (rounded) dx -- the producer conv's bias-gradient partials, as the TN dgrad post-op writes them.
template <typename T, int K, bool MASK = false>
__global__ void pw_small_bwd_kernel(const float* dy, const T* x, int ldx, long M, int HW, int C, const float* w,
                                    T* dx, int lddx, int dx_acc, float* part_w, float* part_b, int G,
                                    int pix_per_block, float* part_d = nullptr) {
  constexpr int V = VE<T>;
  __shared__ float red[256][V];
  __shared__ float redb[256];
  const int cv = C / V;
  const int tv = cv, rows = blockDim.x / tv;
  const int tx = threadIdx.x % tv, ty = threadIdx.x / tv;
  const int c0 = tx * V;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = min(M, p0 + pix_per_block);
  float wv[K][V];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int e = 0; e < V; ++e) wv[k][e] = w[k * C + c0 + e];
  float sw[K][V], sb[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    sb[k] = 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) sw[k][e] = 0.f;
  }
  float sd[V];
#pragma unroll
  for (int e = 0; e < V; ++e) sd[e] = 0.f;
  for (long p = p0 + ty; p < p1; p += rows) {
    const long n = p / HW, hw = p - n * HW;
    float g[K];
#pragma unroll
    for (int k = 0; k < K; ++k) g[k] = dy[(n * K + k) * HW + hw];
    float xv[V], o[V];
    load_vec(x + p * ldx + c0, xv);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      // explicit product then fma (no contraction choice left to the compiler)
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        s = k == 0 ? g[0] * wv[0][e] : fmaf(g[k], wv[k][e], s);
        sw[k][e] += g[k] * xv[e];
      }
      o[e] = s;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) sb[k] += g[k];
    if (MASK) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        o[e] = xv[e] > 0.f ? (float)(T)o[e] : 0.f;  // the stored value, rounded
        sd[e] += o[e];
      }
    }
    if (dx) {
      T* dp = dx + p * lddx + c0;
      if (dx_acc) {
        float old[V];
        load_vec(dp, old);
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] += old[e];
      }
      store_vec(dp, o);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < V; ++e) red[threadIdx.x][e] = sw[k][e];
    redb[threadIdx.x] = sb[k];
    __syncthreads();
    if (ty == 0) {
      float s[V];
      float bs = 0.f;
#pragma unroll
      for (int e = 0; e < V; ++e) s[e] = 0.f;
      for (int r = 0; r < rows; ++r) {
#pragma unroll
        for (int e = 0; e < V; ++e) s[e] += red[r * tv + tx][e];
        bs += redb[r * tv + tx];
      }
#pragma unroll
      for (int e = 0; e < V; ++e) part_w[((long)k * C + c0 + e) * G + blockIdx.x] = s[e];
      if (tx == 0) part_b[(long)k * G + blockIdx.x] = bs;
    }
  }
  if (MASK) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < V; ++e) red[threadIdx.x][e] = sd[e];
    __syncthreads();
    if (ty == 0) {
      float s[V];
#pragma unroll
      for (int e = 0; e < V; ++e) s[e] = 0.f;
      for (int r = 0; r < rows; ++r)
#pragma unroll
        for (int e = 0; e < V; ++e) s[e] += red[r * tv + tx][e];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        part_d[(long)blockIdx.x * 2 * C + c0 + e] = s[e];
        part_d[(long)blockIdx.x * 2 * C + C + c0 + e] = 0.f;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Attention gate (model/unet_attention.py:30-35):
//   alpha = sigmoid(psi*sc + sh) (per pixel), gated = skip * alpha
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void attn_apply_kernel(const T* skip, int lds_, const float* psi, const float* sc, const float* sh,
                                  float* alpha, T* gated, int ldg, long M, int C) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const long total = M * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / cv;
    const int c0 = (int)(i - p * cv) * V;
    const float z = psi[p] * sc[0] + sh[0];
    const float al = 1.f / (1.f + expf(-z));
    if (c0 == 0) alpha[p] = al;
    float v[V];
    load_vec(skip + p * lds_ + c0, v);
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] *= al;
    store_vec(gated + p * ldg + c0, v);
  }
}

// backward 1: d_skip (+)= dg * alpha ; dpsibn[p] = (sum_c dg*skip) * alpha*(1-alpha);
// partials [2][1][G]: sum dpsibn, sum dpsibn * xhat(psi).  ACC: d_skip accumulates onto its buffer
template <typename T, bool ACC>
__global__ void attn_bwd1_kernel(const T* dg, int ldg, const T* skip, int lds_, const float* alpha, const float* psi,
                                 const float* mean, const float* inv, T* dskip, int ldds, float* dpsibn,
                                 long M, int C, int pix_per_block, float* part, int G) {
  constexpr int V = VE<T>;
  __shared__ double sred[16];
  const int cvt = C / V;                 // vectors per pixel
  const int cv = cvt < 64 ? cvt : 64;    // lanes per pixel (power of two)
  const int nchunk = cvt / cv;
  const int ppw = 64 / cv;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int sub = lane / cv, v = lane % cv;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = min(M, p0 + pix_per_block);
  const float mu = mean[0], iv = inv[0];
  double s0 = 0.0, s1 = 0.0;
  if (nchunk == 1) {
    // one vector per lane per pixel, four pixel groups per wave in flight.  Every load of the four
    // groups is unconditional (a pixel past the block's end re-reads its last one; only the stores are
    // masked) and the lane reductions of the four run interleaved: a load under a lane condition got
    // its own branch and a vmcnt(0) behind it, which serialised the groups
    constexpr int U = 4;
    const int c0 = v * V;
    const long step = (long)nw * ppw;
    for (long pb = p0 + (long)wid * ppw; pb < p1; pb += U * step) {
      float g[U][V], sk[U][V], old[U][V], al[U], ps[U], dot[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long pc = min(pb + u * step + sub, p1 - 1);
        al[u] = alpha[pc];
        ps[u] = psi[pc];
        load_vec(dg + pc * ldg + c0, g[u]);
        load_vec(skip + pc * lds_ + c0, sk[u]);
        if (ACC) load_vec(dskip + pc * ldds + c0, old[u]);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = pb + u * step + sub;
        float o[V];
        dot[u] = 0.f;
#pragma unroll
        for (int e = 0; e < V; ++e) {
          dot[u] += g[u][e] * sk[u][e];
          o[e] = ACC ? g[u][e] * al[u] + old[u][e] : g[u][e] * al[u] + 0.f;
        }
        if (p < p1) store_vec(dskip + p * ldds + c0, o);
      }
#pragma unroll
      for (int sh = 1; sh < 64; sh <<= 1)
        if (sh < cv)
#pragma unroll
          for (int u = 0; u < U; ++u) dot[u] += __shfl_xor(dot[u], sh, 64);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = pb + u * step + sub;
        if (p < p1 && v == 0) {
          const float d = dot[u] * al[u] * (1.f - al[u]);
          dpsibn[p] = d;
          s0 += d;
          s1 += (double)d * (ps[u] - mu) * iv;
        }
      }
    }
  } else
  for (long pbase = p0 + (long)wid * ppw; pbase < p1; pbase += (long)nw * ppw) {
    const long p = pbase + sub;
    float dot = 0.f;
    float al = 0.f;
    if (p < p1) {
      al = alpha[p];
      for (int ch = 0; ch < nchunk; ++ch) {
        const int c0 = (ch * cv + v) * V;
        float g[V], sk[V], o[V];
        load_vec(dg + p * ldg + c0, g);
        load_vec(skip + p * lds_ + c0, sk);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          dot += g[e] * sk[e];
          o[e] = g[e] * al;
        }
        T* dp = dskip + p * ldds + c0;
        if (ACC) {
          float old[V];
          load_vec(dp, old);
#pragma unroll
          for (int e = 0; e < V; ++e) o[e] += old[e];
        }
        store_vec(dp, o);
      }
    }
    for (int o = 1; o < cv; o <<= 1) dot += __shfl_xor(dot, o, 64);
    if (p < p1 && v == 0) {
      const float d = dot * al * (1.f - al);
      dpsibn[p] = d;
      s0 += d;
      s1 += (double)d * (psi[p] - mu) * iv;
    }
  }
  s0 = block_sum(s0, sred);
  s1 = block_sum(s1, sred);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = (float)s0;
    part[G + blockIdx.x] = (float)s1;
  }
}

// backward 2: dpsi = coef0*(dpsibn - coef1 - xhat*coef2); dz_f = dpsi * w_psi * (f > 0);
// partials: dW_psi [C][G] = sum dpsi * f, db_psi [G] = sum dpsi
template <typename T>
__global__ void attn_bwd2_kernel(const float* dpsibn, const float* psi, const float* mean, const float* inv,
                                 const float* coef, const T* f, int ldf, const float* wpsi, T* dzf, int lddz, long M,
                                 int C, int tv, int pix_per_block, float* part_w, float* part_b, int G) {
  constexpr int V = VE<T>;
  __shared__ float red[256][V];
  __shared__ float redb[256];
  const int tx = threadIdx.x % tv, ty = threadIdx.x / tv, rows = blockDim.x / tv;
  const int c0 = tx * V;
  const long p0 = (long)blockIdx.x * pix_per_block;
  const long p1 = min(M, p0 + pix_per_block);
  float wv[V], sw[V];
  float sb = 0.f;
#pragma unroll
  for (int e = 0; e < V; ++e) { wv[e] = wpsi[c0 + e]; sw[e] = 0.f; }
  const float mu = mean[0], iv = inv[0], k0 = coef[0], k1 = coef[1], k2 = coef[2];
  // the contractions spelled out (fmaf): unrolled, the compiler packed some products into
  // v_pk_mul_f32 + add, which rounds twice where the one-pixel loop's fma rounded once
  auto one = [&](long p, float ps, float db, const float (&fv)[V]) {
    const float xh = (ps - mu) * iv;
    const float dp = k0 * fmaf(-xh, k2, db - k1);
    float o[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      sw[e] = fmaf(dp, fv[e], sw[e]);
      o[e] = fv[e] > 0.f ? dp * wv[e] : 0.f;
    }
    if (tx == 0) sb += dp;
    store_vec(dzf + p * lddz + c0, o);
  };
  // four pixels per thread per round, all their loads issued first (one pixel per round left each
  // round's load latency exposed); the sums run in the same pixel order as before
  constexpr int U = 4;
  long p = p0 + ty;
  for (; p + (long)(U - 1) * rows < p1; p += (long)U * rows) {
    float ps[U], db[U], fv[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long q = p + (long)u * rows;
      ps[u] = psi[q];
      db[u] = dpsibn[q];
      load_vec(f + q * ldf + c0, fv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(p + (long)u * rows, ps[u], db[u], fv[u]);
  }
  for (; p < p1; p += rows) {
    float fv[V];
    load_vec(f + p * ldf + c0, fv);
    one(p, psi[p], dpsibn[p], fv);
  }
#pragma unroll
  for (int e = 0; e < V; ++e) red[threadIdx.x][e] = sw[e];
  redb[threadIdx.x] = sb;
  __syncthreads();
  if (ty == 0) {
    float s[V];
    float bs = 0.f;
#pragma unroll
    for (int e = 0; e < V; ++e) s[e] = 0.f;
    for (int r = 0; r < rows; ++r) {
#pragma unroll
      for (int e = 0; e < V; ++e) s[e] += red[r * tv + tx][e];
      bs += redb[r * tv + tx];
    }
#pragma unroll
    for (int e = 0; e < V; ++e) part_w[(long)(c0 + e) * G + blockIdx.x] = s[e];
    if (tx == 0) part_b[blockIdx.x] = bs;
  }
}

// elementwise add of NHWC tensors: out (+)= x
template <typename T>
__global__ void add_kernel(const T* x, int ldx, T* out, int ldo, long M, int C) {
  constexpr int V = VE<T>;
  const int cv = C / V;
  const long total = M * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / cv;
    const int c0 = (int)(i - p * cv) * V;
    float a[V], b[V];
    load_vec(x + p * ldx + c0, a);
    load_vec(out + p * ldo + c0, b);
#pragma unroll
    for (int e = 0; e < V; ++e) b[e] += a[e];
    store_vec(out + p * ldo + c0, b);
  }
}

inline int grid_for(long work, int per_block = 256, int cap = 16384) {
  long b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

inline int pow2_le(int v, int cap) {
  int t = 1;
  while (t * 2 <= v && t * 2 <= cap && v % (t * 2) == 0) t *= 2;
  return t;
}

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================
#define DISPATCH_T(dtype, ...)            \
  do {                                    \
    if ((dtype) == DT_BF16) {             \
      typedef bf16 T;                     \
      __VA_ARGS__;                        \
    } else {                              \
      typedef float T;                    \
      __VA_ARGS__;                        \
    }                                     \
  } while (0)

#define CHECK_VEC(dtype, C, name)                                                                               \
  do {                                                                                                          \
    US_CHECK_DTYPE(dtype, name);                                                                                \
    US_CHECK_ARG((C) > 0 && (C) % ((dtype) == DT_BF16 ? 8 : 4) == 0,                                            \
                 "%s: channels (%d) must be a positive multiple of the 16-B vector", name, (int)(C));           \
  } while (0)

UNETSEG_API int unetseg_bn_finalize(const float* part, int C, int G, long M, int tile, const float* gamma,
                                    const float* beta, float* rmean, float* rvar, long long* nbt, float momentum,
                                    float eps, float* mean, float* invstd, float* scale, float* shift, void* stream) {
  US_CHECK_ARG(part && gamma && beta && mean && invstd && scale && shift && M > 0, "bn_finalize: bad args");
  US_CHECK_ARG(C > 0 && G > 0 && tile > 0, "bn_finalize: bad sizes");
  FIN_LAUNCH(bn_finalize_kernel, C, G, stream, part, C, G, M, tile, gamma, beta, rmean, rvar, nbt, momentum, eps, mean,
             invstd, scale, shift);
  US_LAUNCH_CHECK("bn_finalize");
  return 0;
}

UNETSEG_API int unetseg_bn_fold(int C, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                float eps, const float* conv_bias, float* kscale, float* bias, void* stream) {
  US_CHECK_ARG(C > 0 && gamma && beta && rmean && rvar && kscale && bias, "bn_fold: bad args");
  hipLaunchKernelGGL(bn_fold_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, (hipStream_t)stream, C, gamma, beta, rmean,
                     rvar, eps, conv_bias, kscale, bias);
  US_LAUNCH_CHECK("bn_fold");
  return 0;
}

UNETSEG_API int unetseg_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rmean,
                                       const float* rvar, float eps, float* scale, float* shift, void* stream) {
  hipLaunchKernelGGL(bn_eval_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, (hipStream_t)stream, C, gamma, beta, rmean,
                     rvar, eps, scale, shift);
  US_LAUNCH_CHECK("bn_eval");
  return 0;
}

UNETSEG_API int unetseg_bn_apply(int dtype, const void* y, int ldy, const float* sc, const float* sh, const void* r,
                                 int ldr, const float* sc2, const float* sh2, int res_mode, int relu, void* out,
                                 int ldo, long M, int C, void* stream) {
  CHECK_VEC(dtype, C, "bn_apply");
  US_CHECK_ARG(y && sc && sh && out && M >= 0, "bn_apply: null pointer or negative M");
  US_CHECK_ARG(res_mode >= 0 && res_mode <= 2, "bn_apply: res_mode %d (0 none, 1 identity, 2 BN'd residual)", res_mode);
  US_CHECK_ARG(res_mode == 0 || r, "bn_apply: res_mode %d needs the residual", res_mode);
  US_CHECK_ARG(res_mode != 2 || (sc2 && sh2), "bn_apply: res_mode 2 needs the residual's BN coefficients");
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for(M * C / VE<T>)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)y, ldy, sc, sh, (const T*)r, ldr, sc2, sh2,
                                       res_mode, relu, (T*)out, ldo, M, C, nullptr));
  US_LAUNCH_CHECK("bn_apply");
  return 0;
}

UNETSEG_API int unetseg_bn_apply_mask(int dtype, const void* y, int ldy, const float* sc, const float* sh,
                                      const void* r, int ldr, const float* sc2, const float* sh2, int res_mode,
                                      void* out, int ldo, long M, int C, uint8_t* mbits, void* stream) {
  CHECK_VEC(dtype, C, "bn_apply_mask");
  US_CHECK_ARG(mbits != nullptr, "bn_apply_mask: mbits required");
  DISPATCH_T(dtype, hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for(M * C / VE<T>)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)y, ldy, sc, sh, (const T*)r, ldr, sc2, sh2,
                                       res_mode, 1, (T*)out, ldo, M, C, mbits));
  US_LAUNCH_CHECK("bn_apply_mask");
  return 0;
}

// pixel-tile geometry of the per-channel kernels: ~target blocks over (pixel tiles x channel
// groups), at least 2 unrolled groups of rows per thread
static int tile_geom(int dtype, long M, int C, long target, int* tv_out, int* ppb_out) {
  const int V = dtype == DT_BF16 ? 8 : 4;
  if (C <= 0 || C % V != 0 || M < 0) {  // no 16-B channel vectors: no reduction geometry (host ASan driver)
    unetseg_set_error("reduce_tiles: C=%d must be a positive multiple of %d", C, V);
    return -1;
  }
  const int cv = C / V;
  const int tv = pow2_le(cv, 64);
  const int rows = 256 / tv;
  const int groups = cv / tv;
  target /= groups;
  if (target < 64) target = 64;
  long per = (M + rows * target - 1) / (rows * target);
  per = (per + RU - 1) / RU * RU;
  if (per < 2 * RU) per = 2 * RU;
  if (per > 256) per = 256;
  const int ppb = rows * (int)per;
  if (tv_out) *tv_out = tv;
  if (ppb_out) *ppb_out = ppb;
  return ceil_div(M, ppb);
}

static long env_target(const char* name, long dflt) {
  const char* te = getenv(name);
  return te ? atol(te) : dflt;
}

// geometry of the channel-reduction kernels (also used by the host to size partial buffers).
// ~1024 blocks: against 2048, the BN-backward reductions at the unet_resnet50 B=16 shapes took
// 39.0 -> 30.5 us (65536 x 512), 63.5 -> 58.5 (1M x 64 packed mask), the finalize reads half the
// partials (tools/gpu_elem_geom.sh).  UNETSEG_RED_TARGET (tests): another block count, i.e.
// another summation order of the same partials
UNETSEG_API int unetseg_reduce_tiles(int dtype, long M, int C, int* tv_out, int* ppb_out) {
  return tile_geom(dtype, M, C, env_target("UNETSEG_RED_TARGET", 1024), tv_out, ppb_out);
}

// the BN-backward apply pass has no partials, so it takes its own block count: ~4096 blocks
// (262144 x 256: 78.4 -> 72.3 us against 2048; 1024 gave 84.5)
static int apply_tiles(int dtype, long M, int C, int* tv_out, int* ppb_out) {
  return tile_geom(dtype, M, C, env_target("UNETSEG_APPLY_TARGET", 4096), tv_out, ppb_out);
}

UNETSEG_API int unetseg_bn_bwd_reduce(int dtype, const void* dA, int ldd, const void* A, int lda, const float* msc,
                                      const float* msh, const void* y1, int ld1, const float* mean1,
                                      const float* inv1, const void* y2, int ld2, const float* mean2,
                                      const float* inv2, long M, int C, float* part, int G, void* stream) {
  CHECK_VEC(dtype, C, "bn_bwd_reduce");
  US_CHECK_ARG(dA && y1 && mean1 && inv1 && part && M >= 0, "bn_bwd_reduce: null pointer or negative M");
  int tv, ppb;
  const int g = unetseg_reduce_tiles(dtype, M, C, &tv, &ppb);
  US_CHECK_ARG(g == G, "bn_bwd_reduce: G mismatch (%d vs %d)", G, g);
  const int V = dtype == DT_BF16 ? 8 : 4;
  dim3 grid(G, C / V / tv);
  const int mask = A ? (lda == 0 ? 3 : 1) : (msc ? 2 : 0);
  hipStream_t st = (hipStream_t)stream;
#define BN_RED_LAUNCH(MK, Y2)                                                                                     \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, MK, Y2>), grid, dim3(256), 0, st, (const T*)dA, ldd, (const T*)A, lda, \
                     msc, msh, (const T*)y1, ld1, mean1, inv1, (const T*)y2, ld2, mean2, inv2, M, C, tv, ppb, part, G)
#define BN_RED_BITS()                                                                                             \
  hipLaunchKernelGGL((bn_bwd_reduce_bits_kernel<T>), grid, dim3(256), 0, st, (const T*)dA, ldd, (const T*)A, lda, \
                     msc, msh, (const T*)y1, ld1, mean1, inv1, (const T*)y2, ld2, mean2, inv2, M, C, tv, ppb, part, G)
  DISPATCH_T(dtype, {
    if (y2) {
      if (mask == 3) BN_RED_LAUNCH(3, true);
      else if (mask == 1) BN_RED_LAUNCH(1, true);
      else if (mask == 2) BN_RED_LAUNCH(2, true);
      else BN_RED_LAUNCH(0, true);
    } else {
      if (mask == 3) BN_RED_BITS();
      else if (mask == 1) BN_RED_LAUNCH(1, false);
      else if (mask == 2) BN_RED_LAUNCH(2, false);
      else BN_RED_LAUNCH(0, false);
    }
  });
#undef BN_RED_LAUNCH
#undef BN_RED_BITS
  US_LAUNCH_CHECK("bn_bwd_reduce");
  return 0;
}

UNETSEG_API int unetseg_bn_bwd_finalize(const float* part, int C, int G, long M, int nbranch, const float* g1,
                                        const float* inv1, float* dg1, float* db1, const float* g2, const float* inv2,
                                        float* dg2, float* db2, float* coef, void* stream) {
  US_CHECK_ARG(nbranch == 1 || nbranch == 2, "bn_bwd_finalize: nbranch %d must be 1 or 2", nbranch);
  US_CHECK_ARG(part && g1 && inv1 && coef && C > 0 && G > 0 && M > 0, "bn_bwd_finalize: bad args");
  US_CHECK_ARG(nbranch == 1 || (g2 && inv2), "bn_bwd_finalize: the second branch needs its gamma / invstd");
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, part, C, G, M, nbranch, g1,
                     inv1, dg1, db1, g2, inv2, dg2, db2, coef);
  US_LAUNCH_CHECK("bn_bwd_finalize");
  return 0;
}

UNETSEG_API int unetseg_bn_bwd_apply(int dtype, const void* dA, int ldd, const void* A, int lda, const float* msc,
                                     const float* msh, const void* y1, int ld1, const float* mean1, const float* inv1,
                                     void* dy1, int ldo1,
                                     const void* y2, int ld2, const float* mean2, const float* inv2, void* dy2,
                                     int ldo2, const float* coef, void* dzout, int ldz, int dz_acc, long M, int C,
                                     void* stream) {
  CHECK_VEC(dtype, C, "bn_bwd_apply");
  int tv, ppb;
  const int G = apply_tiles(dtype, M, C, &tv, &ppb);
  const int V = dtype == DT_BF16 ? 8 : 4;
  dim3 grid(G, C / V / tv);
  const int mask = A ? (lda == 0 ? 3 : 1) : (msc ? 2 : 0);
  const int dzm = dzout ? (dz_acc ? 2 : 1) : 0;
  hipStream_t st = (hipStream_t)stream;
#define BN_APP_LAUNCH(MK, Y2, DZ)                                                                                  \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, MK, Y2, DZ>), grid, dim3(256), 0, st, (const T*)dA, ldd, (const T*)A,   \
                     lda, msc, msh, (const T*)y1, ld1, mean1, inv1, (T*)dy1, ldo1, (const T*)y2, ld2, mean2, inv2,  \
                     (T*)dy2, ldo2, coef, (T*)dzout, ldz, M, C, tv, ppb)
#define BN_APP_DZ(MK, Y2)                  \
  do {                                     \
    if (dzm == 2) BN_APP_LAUNCH(MK, Y2, 2); \
    else if (dzm == 1) BN_APP_LAUNCH(MK, Y2, 1); \
    else BN_APP_LAUNCH(MK, Y2, 0);          \
  } while (0)
  DISPATCH_T(dtype, {
    if (y2) {
      if (mask == 3) BN_APP_DZ(3, true);
      else if (mask == 1) BN_APP_DZ(1, true);
      else if (mask == 2) BN_APP_DZ(2, true);
      else BN_APP_DZ(0, true);
    } else {
      if (mask == 3) BN_APP_DZ(3, false);
      else if (mask == 1) BN_APP_DZ(1, false);
      else if (mask == 2) BN_APP_DZ(2, false);
      else BN_APP_DZ(0, false);
    }
  });
#undef BN_APP_DZ
#undef BN_APP_LAUNCH
  US_LAUNCH_CHECK("bn_bwd_apply");
  return 0;
}

UNETSEG_API int unetseg_relu_bwd_bias(int dtype, const void* dA, int ldd, const void* A, int lda, void* dY, int ldy,
                                      long M, int C, float* part, int G, void* stream) {
  CHECK_VEC(dtype, C, "relu_bwd_bias");
  int tv, ppb;
  const int g = unetseg_reduce_tiles(dtype, M, C, &tv, &ppb);
  US_CHECK_ARG(g == G, "relu_bwd_bias: G mismatch");
  const int V = dtype == DT_BF16 ? 8 : 4;
  dim3 grid(G, C / V / tv);
  DISPATCH_T(dtype, hipLaunchKernelGGL(relu_bwd_bias_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream,
                                       (const T*)dA, ldd, (const T*)A, lda, (T*)dY, ldy, M, C, tv, ppb, part, G));
  US_LAUNCH_CHECK("relu_bwd_bias");
  return 0;
}

constexpr int kFinMergeR = 16;
UNETSEG_API int unetseg_fin_merge_rows(const float* part, int C, int G, long M, int tile, int nq, float* out,
                                       void* stream) {
  US_CHECK_ARG(part && out && C > 0 && G > 0 && nq >= 1 && nq <= 3, "fin_merge_rows: bad args");
  US_CHECK_ARG(tile == 0 || (nq == 2 && M > 0), "fin_merge_rows: a statistics merge needs nq == 2 and M");
  const int G2 = ceil_div(G, kFinMergeR);
  const dim3 grid(ceil_div(G2, 4), ceil_div(C, 64));
  if (tile > 0)
    hipLaunchKernelGGL((fin_merge_rows_kernel<true, 2, kFinMergeR>), grid, dim3(256), 0, (hipStream_t)stream, part, C,
                       G, M, tile, nq, out, G2);
  else if (nq == 3)
    hipLaunchKernelGGL((fin_merge_rows_kernel<false, 3, kFinMergeR>), grid, dim3(256), 0, (hipStream_t)stream, part,
                       C, G, M, tile, nq, out, G2);
  else
    hipLaunchKernelGGL((fin_merge_rows_kernel<false, 2, kFinMergeR>), grid, dim3(256), 0, (hipStream_t)stream, part,
                       C, G, M, tile, nq, out, G2);
  US_LAUNCH_CHECK("fin_merge_rows");
  return 0;
}

UNETSEG_API int unetseg_bn_bwd_finalize_rows(const float* part, int C, int G, long M, const float* g1,
                                             const float* inv1, float* dg1, float* db1, float* coef, void* stream) {
  US_CHECK_ARG(part && g1 && inv1 && dg1 && db1 && coef && M > 0, "bn_bwd_finalize_rows: bad args");
  US_CHECK_ARG(C > 0 && G > 0, "bn_bwd_finalize_rows: bad sizes");
  FIN_LAUNCH(bn_bwd_finalize_rows_kernel, C, G, stream, part, C, G, M, g1, inv1, dg1, db1, coef);
  US_LAUNCH_CHECK("bn_bwd_finalize_rows");
  return 0;
}

UNETSEG_API int unetseg_bn_bwd_finalize_rows_res(const float* part, int C, int G, long M, int nbranch, const float* g1,
                                                 const float* inv1, float* dg1, float* db1, const float* g2,
                                                 const float* inv2, float* dg2, float* db2, float* coef, void* stream) {
  US_CHECK_ARG(part && g1 && inv1 && dg1 && db1 && coef && M > 0 && C > 0 && G > 0 && (nbranch == 1 || nbranch == 2),
               "bn_bwd_finalize_rows_res: bad args");
  US_CHECK_ARG(nbranch == 1 || (g2 && inv2 && dg2 && db2), "bn_bwd_finalize_rows_res: branch 2 needs its pointers");
  FIN_LAUNCH(bn_bwd_finalize_rows_res_kernel, C, G, stream, part, C, G, M, nbranch, g1, inv1, dg1, db1, g2, inv2, dg2,
             db2, coef);
  US_LAUNCH_CHECK("bn_bwd_finalize_rows_res");
  return 0;
}

UNETSEG_API int unetseg_colsum_rows(const float* part, int C, int G, int k, float* out, int accumulate, void* stream) {
  US_CHECK_ARG(part && out && C > 0 && G >= 0 && (k == 0 || k == 1), "colsum_rows: bad args");
  FIN_LAUNCH(colsum_rows_kernel, C, G, stream, part, C, G, k, out, accumulate);
  US_LAUNCH_CHECK("colsum_rows");
  return 0;
}

UNETSEG_API int unetseg_colsum_finalize(const float* part, int C, int G, float* out, int accumulate, void* stream) {
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, part, C, G, out, accumulate);
  US_LAUNCH_CHECK("colsum_finalize");
  return 0;
}

UNETSEG_API int unetseg_maxpool_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int k, int s,
                                    int ceil_mode, void* y, int ldy, uint8_t* idx, int* p_out, int* q_out,
                                    void* stream) {
  CHECK_VEC(dtype, c, "maxpool_fwd");
  US_CHECK_ARG(x && y && idx, "maxpool_fwd: null pointer");
  US_CHECK_ARG(k >= 1 && k <= 16 && s >= 1 && n >= 0 && h >= k && w >= k, "maxpool_fwd: bad window k=%d s=%d on %dx%d", k,
               s, h, w);
  int p = ceil_mode ? (h - k + s - 1) / s + 1 : (h - k) / s + 1;
  int q = ceil_mode ? (w - k + s - 1) / s + 1 : (w - k) / s + 1;
  if (ceil_mode) {  // last window must start inside the input (ATen pooling_output_shape)
    if ((p - 1) * s >= h) --p;
    if ((q - 1) * s >= w) --q;
  }
  if (p_out) *p_out = p;
  if (q_out) *q_out = q;
  if (!y) return 0;  // shape query
  const bool fits = (long)n * h * w * c < (1L << 31) && (long)n * h * w * ldx < (1L << 31) &&
                    (long)n * p * q * ldy < (1L << 31) && !getenv("UNETSEG_MAXPOOL_GENERIC");
  if (k == 2 && s == 2 && h == 2 * p && w == 2 * q && fits)
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_k2s2_kernel<T>, dim3(grid_for((long)n * p * q * c / VE<T>)),
                                         dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx, n, h, w, c, p, q, (T*)y,
                                         ldy, idx));
  else if (k == 3 && s == 2 && fits)
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_k3s2_kernel<T>, dim3(grid_for((long)n * p * q * c / VE<T>)),
                                         dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx, n, h, w, c, p, q, (T*)y,
                                         ldy, idx));
  else
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(grid_for((long)n * p * q * c / VE<T>)), dim3(256),
                                         0, (hipStream_t)stream, (const T*)x, ldx, n, h, w, c, k, s, p, q, (T*)y, ldy,
                                         idx));
  US_LAUNCH_CHECK("maxpool_fwd");
  return 0;
}

UNETSEG_API int unetseg_maxpool_bwd(int dtype, const void* dy, int ldy, const uint8_t* idx, int n, int h, int w,
                                    int c, int k, int s, int p, int q, void* dx, int ldx, int accumulate,
                                    void* stream) {
  CHECK_VEC(dtype, c, "maxpool_bwd");
  US_CHECK_ARG(dy && idx && dx && k >= 1 && s >= 1 && n >= 0 && h >= 0 && w >= 0, "maxpool_bwd: bad args");
  const bool fits = (long)n * h * w * c < (1L << 31) && (long)n * h * w * ldx < (1L << 31) &&
                    (long)n * p * q * ldy < (1L << 31) && !getenv("UNETSEG_MAXPOOL_GENERIC");
  if (k == 2 && s == 2 && h == 2 * p && w == 2 * q && fits)
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_k2s2_kernel<T>, dim3(grid_for((long)n * p * q * c / VE<T>)),
                                         dim3(256), 0, (hipStream_t)stream, (const T*)dy, ldy, idx, n, h, w, c, p, q,
                                         (T*)dx, ldx, accumulate));
  else if (k == 3 && s == 2 && fits)
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel<T>,
                                         dim3(grid_for((long)n * ((h + 1) / 2) * ((w + 1) / 2) * c / VE<T>)), dim3(256),
                                         0, (hipStream_t)stream, (const T*)dy, ldy, idx, n, h, w, c, p, q, (T*)dx, ldx,
                                         accumulate));
  else
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for((long)n * h * w * c / VE<T>)), dim3(256),
                                         0, (hipStream_t)stream, (const T*)dy, ldy, idx, n, h, w, c, k, s, p, q, (T*)dx,
                                         ldx, accumulate));
  US_LAUNCH_CHECK("maxpool_bwd");
  return 0;
}

UNETSEG_API int unetseg_upsample2x_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c,
                                       int align_corners, void* y, int ldy, void* stream) {
  CHECK_VEC(dtype, c, "upsample_fwd");
  US_CHECK_ARG(x && y && n >= 0 && h >= 0 && w >= 0, "upsample_fwd: null pointer or negative size");
  DISPATCH_T(dtype, hipLaunchKernelGGL(upsample_fwd_kernel<T>,
                                       dim3(ceil_div(2 * w * (c / VE<T>), 256), ceil_div(n * 2 * h, up_rows_pb())),
                                       dim3(256), 0, (hipStream_t)stream, (const T*)x, ldx, n, h, w, c, align_corners,
                                       (T*)y, ldy, up_rows_pb()));
  US_LAUNCH_CHECK("upsample_fwd");
  return 0;
}

static int up_taps_max(int in, int align);
static int up_stream_rows(int dtype, int n, int h, int w, int c);

UNETSEG_API int unetseg_upsample2x_bwd(int dtype, const void* dy, int ldy, int n, int h, int w, int c,
                                       int align_corners, void* dx, int ldx, int accumulate, void* stream) {
  CHECK_VEC(dtype, c, "upsample_bwd");
  US_CHECK_ARG(dy && dx && n >= 0 && h >= 0 && w >= 0, "upsample_bwd: null pointer or negative size");
#define UP_BWD(R)                                                                                            \
  hipLaunchKernelGGL((upsample_bwd_kernel<T, R>), dim3(ceil_div(w * (c / VE<T>), 256), ceil_div(n * h, R)), dim3(256), \
                     0, (hipStream_t)stream, (const T*)dy, ldy, n, h, w, c, align_corners, (T*)dx, ldx, accumulate)
  const int rs = up_stream_rows(dtype, n, h, w, c);
  if (rs) {
    // the row-streaming adjoint without the mask (as upsample_bwd_relu's default), bit-identical
    const int K = up_taps_max(w, align_corners) <= 4 ? 4 : 5;
#define UP_STREAM_PLAIN(RS, KK)                                                                                  \
  hipLaunchKernelGGL((upsample_bwd_relu_stream_kernel<T, RS, KK, 1, false>),                                     \
                     dim3(ceil_div(w * (c / VE<T>), 256), n * h / RS), dim3(256), 0, (hipStream_t)stream,         \
                     (const T*)dy, ldy, n, h, w, c, align_corners, (const T*)nullptr, 0, (T*)dx, ldx, (float*)nullptr, \
                     accumulate)
    DISPATCH_T(dtype, if (rs == 16) {
      if (K == 4) UP_STREAM_PLAIN(16, 4); else UP_STREAM_PLAIN(16, 5);
    } else {
      if (K == 4) UP_STREAM_PLAIN(8, 4); else UP_STREAM_PLAIN(8, 5);
    });
#undef UP_STREAM_PLAIN
  } else {
    const int rpb = up_rows_pb();
    DISPATCH_T(dtype, if (rpb == 2) UP_BWD(2); else if (rpb == 8) UP_BWD(8); else UP_BWD(kUpRowsPB));
  }
#undef UP_BWD
  US_LAUNCH_CHECK("upsample_bwd");
  return 0;
}

// host restatement of up_taps' tap count: the most nonzero column taps any input column has (4 or 5)
static int up_taps_max(int in, int align) {
  const int out = 2 * in;
  int best = 0;
  for (int i = 0; i < in; ++i) {
    int lo, hi;
    if (align) {
      lo = in > 1 ? (int)floorf((float)(i - 1) * (out - 1) / (float)(in - 1)) : 0;
      hi = in > 1 ? (int)ceilf((float)(i + 1) * (out - 1) / (float)(in - 1)) : out - 1;
    } else {
      lo = 2 * i - 2;
      hi = i == in - 1 ? out - 1 : 2 * i + 2;
    }
    lo = std::max(lo, 0);
    hi = std::min(hi, out - 1);
    int cnt = 0;
    for (int d = lo; d <= hi; ++d) {
      float src;
      if (align) {
        const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
        src = scale * (float)d;
      } else {
        src = ((float)d + 0.5f) * 0.5f - 0.5f;
        if (src < 0.f) src = 0.f;
      }
      int i0 = (int)src;
      if (i0 > in - 1) i0 = in - 1;
      const int i1 = i0 + 1 < in ? i0 + 1 : in - 1;
      const float l1 = src - (float)i0;
      float wgt = 0.f;
      if (i0 == i) wgt += 1.f - l1;
      if (i1 == i) wgt += l1;
      if (wgt != 0.f) ++cnt;
    }
    best = std::max(best, cnt);
  }
  return best;
}

// rows per block of the row-streaming upsample backward (0: the row-blocked kernel): 16 where that
// still gives >= 2048 blocks, else 8; h must be a multiple (UNETSEG_UP_STREAM=0: off)
static int up_stream_rows(int dtype, int n, int h, int w, int c) {
  const char* e = getenv("UNETSEG_UP_STREAM");
  if (e && atoi(e) == 0) return 0;
  const int V = dtype == DT_BF16 ? 8 : 4;
  const long xb = ceil_div((long)w * (c / V), 256);
  for (int rs : {16, 8})
    if (h % rs == 0 && (xb * ((long)n * h / rs) >= 2048 || rs == 8)) return rs;
  return 0;
}

// partial rows (blocks) of unetseg_upsample2x_bwd_relu for this shape
UNETSEG_API int unetseg_upsample2x_bwd_tiles(int dtype, int n, int h, int w, int c) {
  const int V = dtype == DT_BF16 ? 8 : 4;
  const int rs = up_stream_rows(dtype, n, h, w, c);
  return ceil_div((long)w * (c / V), 256) * ceil_div((long)n * h, rs ? rs : up_rows_pb());
}

UNETSEG_API int unetseg_upsample2x_bwd_relu(int dtype, const void* dy, int ldy, int n, int h, int w, int c,
                                            int align_corners, const void* a, int lda, void* dx, int ldx, float* part,
                                            int rows, void* stream) {
  CHECK_VEC(dtype, c, "upsample_bwd_relu");
  US_CHECK_ARG(dy && a && dx && part, "upsample_bwd_relu: null pointer");
  const int V = dtype == DT_BF16 ? 8 : 4;
  US_CHECK_ARG(c / V <= 256 && 256 % (c / V) == 0, "upsample_bwd_relu: channels / vector must divide 256");
  US_CHECK_ARG(rows == unetseg_upsample2x_bwd_tiles(dtype, n, h, w, c), "upsample_bwd_relu: rows mismatch");
#define UP_BWD_RELU(R)                                                                                      \
  hipLaunchKernelGGL((upsample_bwd_relu_kernel<T, R>), dim3(ceil_div(w * (c / VE<T>), 256), ceil_div(n * h, R)),       \
                     dim3(256), 0, (hipStream_t)stream, (const T*)dy, ldy, n, h, w, c, align_corners, (const T*)a, lda, \
                     (T*)dx, ldx, part)
  const int rs = up_stream_rows(dtype, n, h, w, c);
  if (rs) {
    const int K = up_taps_max(w, align_corners) <= 4 ? 4 : 5;
    // dy rows in flight ahead of the consumed one (UNETSEG_UP_STREAM_PF=1 or 2)
    static const int pf = getenv("UNETSEG_UP_STREAM_PF") && atoi(getenv("UNETSEG_UP_STREAM_PF")) == 2 ? 2 : 1;
#define UP_STREAM(RS, KK)                                                                                      \
  {                                                                                                            \
    if (pf == 1) {                                                                                             \
      UP_STREAM_PF(RS, KK, 1);                                                                                 \
    } else {                                                                                                   \
      UP_STREAM_PF(RS, KK, 2);                                                                                 \
    }                                                                                                          \
  }
#define UP_STREAM_PF(RS, KK, PFV)                                                                              \
  hipLaunchKernelGGL((upsample_bwd_relu_stream_kernel<T, RS, KK, PFV>), dim3(ceil_div(w * (c / VE<T>), 256), n * h / RS), \
                     dim3(256), 0, (hipStream_t)stream, (const T*)dy, ldy, n, h, w, c, align_corners, (const T*)a, lda, \
                     (T*)dx, ldx, part)
#define UP_STREAM_K(RS) \
  if (K == 4) UP_STREAM(RS, 4) else UP_STREAM(RS, 5)
    DISPATCH_T(dtype, if (rs == 16) { UP_STREAM_K(16) } else { UP_STREAM_K(8) });
#undef UP_STREAM_K
#undef UP_STREAM
#undef UP_STREAM_PF
    US_LAUNCH_CHECK("upsample_bwd_relu");
    return 0;
  }
  const int rpb = up_rows_pb();
  DISPATCH_T(dtype, if (rpb == 2) UP_BWD_RELU(2); else if (rpb == 8) UP_BWD_RELU(8); else UP_BWD_RELU(kUpRowsPB));
#undef UP_BWD_RELU
  US_LAUNCH_CHECK("upsample_bwd_relu");
  return 0;
}

UNETSEG_API int unetseg_pack_input(int dtype, const float* x, int n, int c, int h, int w, int cpad, void* y,
                                   void* stream) {
  US_CHECK_DTYPE(dtype, "pack_input");
  US_CHECK_ARG(cpad >= c && c > 0 && n >= 0 && h >= 0 && w >= 0, "pack_input: bad sizes (c=%d, cpad=%d < c?)", c, cpad);
  US_CHECK_ARG(x && y, "pack_input: null pointer");
  DISPATCH_T(dtype, hipLaunchKernelGGL(pack_input_kernel<T>, dim3(grid_for((long)n * h * w)), dim3(256), 0,
                                       (hipStream_t)stream, x, n, c, h, w, cpad, (T*)y));
  US_LAUNCH_CHECK("pack_input");
  return 0;
}

// NCHW fp32 image -> width-padded stem layout bf16 [N][H][W+8][8]: image column w at packed column
// w+3, channels >= C and the 3 + 5 border columns zero (see unetseg_stem_fwd)
__global__ void pack_input_stem_kernel(const float* x, int N, int C, int H, int W, bf16* y) {
  const int WP = W + 8;
  const long total = (long)N * H * WP;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long row = i / WP;
    const int wp = (int)(i - row * WP), w = wp - 3;
    const long n = row / H, h = row - n * H;
    // all eight loads unconditional (clamped into the image; channels past C re-read channel C - 1,
    // the same cache line) and masked after: conditional loads were waited on one at a time
    const int wc = min(max(w, 0), W - 1);
    float xv[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) xv[c] = x[((n * C + min(c, C - 1)) * H + h) * (long)W + wc];
    bf16 v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = (bf16)((c < C && w >= 0 && w < W) ? xv[c] : 0.f);
    *reinterpret_cast<uint4*>(y + i * 8) = *reinterpret_cast<uint4*>(v);
  }
}

UNETSEG_API int unetseg_pack_input_stem(const float* x, int n, int c, int h, int w, void* y, void* stream) {
  US_CHECK_ARG(x && y && c >= 1 && c <= 8, "pack_input_stem: bad args");
  hipLaunchKernelGGL(pack_input_stem_kernel, dim3(grid_for((long)n * h * (w + 8))), dim3(256), 0, (hipStream_t)stream,
                     x, n, c, h, w, (bf16*)y);
  US_LAUNCH_CHECK("pack_input_stem");
  return 0;
}

// pixel tile of the small-Cout 1x1 / attention-psi kernels: 2048, halved (down to 128) while that
// leaves fewer than 512 blocks (the 64^2 gate's 32 K pixels had 16 blocks at 2048)
static long pw_tile(long M) {
  static const bool fixed = getenv("UNETSEG_PW_TILE_FIXED") != nullptr;  // A/B: always 2048
  long t = 2048;
  if (fixed) return t;
  while (t > 128 && (M + t - 1) / t < 512) t >>= 1;
  return t;
}
UNETSEG_API int unetseg_pw_small_tile(long M) { return (int)pw_tile(M); }
UNETSEG_API int unetseg_pw_small_tiles(long M) { return ceil_div(M, pw_tile(M)); }

// y fp32 planar [n][k][hw]; stats (k==1 only, may be NULL): [G][2], G = unetseg_pw_small_tiles(M), tile unetseg_pw_small_tile(M) px
UNETSEG_API int unetseg_pw_small_fwd(int dtype, const void* x, int ldx, long M, int hw, int c, int k, const float* w,
                                     const float* b, float* y, float* stats, void* stream) {
  CHECK_VEC(dtype, c, "pw_small_fwd");
  const int V = dtype == DT_BF16 ? 8 : 4;
  US_CHECK_ARG(c / V <= 64 && ((c / V) & (c / V - 1)) == 0, "pw_small_fwd: C/V must be a power of two <= 64");
  US_CHECK_ARG(k == 1 || k == 2, "pw_small_fwd: k must be 1 or 2");
  US_CHECK_ARG(!stats || k == 1, "pw_small_fwd: stats only for k==1");
  // without statistics the tile only sets the grid (every pixel's output is its own): 128-pixel blocks,
  // twice the resident waves of pw_tile's for the latency-bound head -- the attention U-Net's 64 -> 2
  // head at 8 x 512^2: 105.6 (2048) / 95.7 (512) / 87.7 (256) / 82.0 us (128).  UNETSEG_PW_FWD_TILE = T
  // sets it (0: pw_tile); the statistics' partial rows keep pw_tile, which the BN finalize is sized by
  static const long nostat_tile = getenv("UNETSEG_PW_FWD_TILE") ? atol(getenv("UNETSEG_PW_FWD_TILE")) : 128;
  const long tile = (!stats && nostat_tile > 0) ? nostat_tile : pw_tile(M);
  const int G = (int)ceil_div(M, tile);
  hipStream_t st = (hipStream_t)stream;
  static const int pw_sign = getenv("UNETSEG_PW_GENERIC") ? -1 : 1;  // A/B: generic shuffle path
  DISPATCH_T(dtype, {
    if (k == 1)
      hipLaunchKernelGGL((pw_small_fwd_kernel<T, 1>), dim3(G), dim3(256), 0, st, (const T*)x, ldx, M, hw, c, w, b, y,
                         stats, (int)tile * pw_sign);
    else
      hipLaunchKernelGGL((pw_small_fwd_kernel<T, 2>), dim3(G), dim3(256), 0, st, (const T*)x, ldx, M, hw, c, w, b, y,
                         stats, (int)tile * pw_sign);
  });
  US_LAUNCH_CHECK("pw_small_fwd");
  return 0;
}

// dx (may be NULL) (+)= dy . W ; part_w [k][c][G], part_b [k][G]  (G = unetseg_pw_small_tiles(M))
UNETSEG_API int unetseg_pw_small_bwd(int dtype, const float* dy, const void* x, int ldx, long M, int hw, int c, int k,
                                     const float* w, void* dx, int lddx, int dx_acc, float* part_w, float* part_b,
                                     void* stream) {
  CHECK_VEC(dtype, c, "pw_small_bwd");
  const int V = dtype == DT_BF16 ? 8 : 4;
  US_CHECK_ARG(c / V <= 256 && 256 % (c / V) == 0, "pw_small_bwd: bad C");
  const int G = unetseg_pw_small_tiles(M);
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (k == 1)
      hipLaunchKernelGGL((pw_small_bwd_kernel<T, 1>), dim3(G), dim3(256), 0, st, dy, (const T*)x, ldx, M, hw, c, w,
                         (T*)dx, lddx, dx_acc, part_w, part_b, G, (int)pw_tile(M));
    else
      hipLaunchKernelGGL((pw_small_bwd_kernel<T, 2>), dim3(G), dim3(256), 0, st, dy, (const T*)x, ldx, M, hw, c, w,
                         (T*)dx, lddx, dx_acc, part_w, part_b, G, (int)pw_tile(M));
  });
  US_LAUNCH_CHECK("pw_small_bwd");
  return 0;
}

// pw_small_bwd with the backward of the ReLU that produced x fused in (x = that ReLU's output, this
// conv its sole consumer): dx = (x > 0) ? dy . W : 0 (no accumulate), part_d [G][2][c] with slot 0
// = column sums of dx (the producer conv's bias-gradient partials; unetseg_colsum_rows reduces them)
UNETSEG_API int unetseg_pw_small_bwd_relu(int dtype, const float* dy, const void* x, int ldx, long M, int hw, int c,
                                          int k, const float* w, void* dx, int lddx, float* part_w, float* part_b,
                                          float* part_d, void* stream) {
  US_CHECK_ARG(dtype == DT_BF16, "pw_small_bwd_relu: bf16 only");
  CHECK_VEC(dtype, c, "pw_small_bwd_relu");
  US_CHECK_ARG(c / 8 <= 256 && 256 % (c / 8) == 0, "pw_small_bwd_relu: bad C");
  US_CHECK_ARG(k == 1 || k == 2, "pw_small_bwd_relu: k must be 1 or 2");
  US_CHECK_ARG(dx != nullptr && part_d != nullptr, "pw_small_bwd_relu: dx and part_d required");
  const int G = unetseg_pw_small_tiles(M);
  hipStream_t st = (hipStream_t)stream;
  if (k == 1)
    hipLaunchKernelGGL((pw_small_bwd_kernel<bf16, 1, true>), dim3(G), dim3(256), 0, st, dy, (const bf16*)x, ldx, M, hw,
                       c, w, (bf16*)dx, lddx, 0, part_w, part_b, G, (int)pw_tile(M), part_d);
  else
    hipLaunchKernelGGL((pw_small_bwd_kernel<bf16, 2, true>), dim3(G), dim3(256), 0, st, dy, (const bf16*)x, ldx, M, hw,
                       c, w, (bf16*)dx, lddx, 0, part_w, part_b, G, (int)pw_tile(M), part_d);
  US_LAUNCH_CHECK("pw_small_bwd_relu");
  return 0;
}

UNETSEG_API int unetseg_attn_apply(int dtype, const void* skip, int lds_, const float* psi, const float* sc,
                                   const float* sh, float* alpha, void* gated, int ldg, long M, int c, void* stream) {
  CHECK_VEC(dtype, c, "attn_apply");
  DISPATCH_T(dtype, hipLaunchKernelGGL(attn_apply_kernel<T>, dim3(grid_for(M * c / VE<T>)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)skip, lds_, psi, sc, sh, alpha, (T*)gated, ldg, M,
                                       c));
  US_LAUNCH_CHECK("attn_apply");
  return 0;
}

// 128-pixel tiles: the 64^2 x 512-channel gate has 32 K pixels, 2048-pixel tiles left 16 blocks
constexpr int kAttnBwd1Tile = 128;
UNETSEG_API int unetseg_attn_bwd1_tiles(long M) { return ceil_div(M, (long)kAttnBwd1Tile); }

UNETSEG_API int unetseg_attn_bwd1(int dtype, const void* dg, int ldg, const void* skip, int lds_, const float* alpha,
                                  const float* psi, const float* mean, const float* inv, void* dskip, int ldds,
                                  int ds_acc, float* dpsibn, long M, int c, float* part, void* stream) {
  CHECK_VEC(dtype, c, "attn_bwd1");
  const int V = dtype == DT_BF16 ? 8 : 4;
  US_CHECK_ARG(((c / V) & (c / V - 1)) == 0, "attn_bwd1: C/V must be a power of two");
  const int G = unetseg_attn_bwd1_tiles(M);
  if (ds_acc)
    DISPATCH_T(dtype, hipLaunchKernelGGL((attn_bwd1_kernel<T, true>), dim3(G), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)dg, ldg, (const T*)skip, lds_, alpha, psi, mean, inv, (T*)dskip,
                                         ldds, dpsibn, M, c, kAttnBwd1Tile, part, G));
  else
    DISPATCH_T(dtype, hipLaunchKernelGGL((attn_bwd1_kernel<T, false>), dim3(G), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)dg, ldg, (const T*)skip, lds_, alpha, psi, mean, inv, (T*)dskip,
                                         ldds, dpsibn, M, c, kAttnBwd1Tile, part, G));
  US_LAUNCH_CHECK("attn_bwd1");
  return 0;
}

UNETSEG_API int unetseg_attn_bwd2(int dtype, const float* dpsibn, const float* psi, const float* mean,
                                  const float* inv, const float* coef, const void* f, int ldf, const float* wpsi,
                                  void* dzf, int lddz, long M, int c, float* part_w, float* part_b, void* stream) {
  CHECK_VEC(dtype, c, "attn_bwd2");
  const int V = dtype == DT_BF16 ? 8 : 4;
  const int cv = c / V;
  US_CHECK_ARG(cv <= 256 && 256 % cv == 0, "attn_bwd2: bad C");
  const int G = unetseg_pw_small_tiles(M);
  DISPATCH_T(dtype, hipLaunchKernelGGL(attn_bwd2_kernel<T>, dim3(G), dim3(256), 0, (hipStream_t)stream, dpsibn, psi,
                                       mean, inv, coef, (const T*)f, ldf, wpsi, (T*)dzf, lddz, M, c, cv, (int)pw_tile(M), part_w,
                                       part_b, G));
  US_LAUNCH_CHECK("attn_bwd2");
  return 0;
}

UNETSEG_API int unetseg_add(int dtype, const void* x, int ldx, void* out, int ldo, long M, int c, void* stream) {
  CHECK_VEC(dtype, c, "add");
  US_CHECK_ARG(x && out && M >= 0 && ldx >= c && ldo >= c, "add: bad args");
  DISPATCH_T(dtype, hipLaunchKernelGGL(add_kernel<T>, dim3(grid_for(M * c / VE<T>)), dim3(256), 0, (hipStream_t)stream,
                                       (const T*)x, ldx, (T*)out, ldo, M, c));
  US_LAUNCH_CHECK("add");
  return 0;
}
