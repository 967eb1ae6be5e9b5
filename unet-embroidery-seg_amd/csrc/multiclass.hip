// Multiclass segmentation kernels: the C-way 1x1 head, the fused CE / Focal / Dice losses, the
// multiclass confusion histogram, and predict.py's softmax -> crop -> resize -> argmax.
//
// Reference ops replaced:
//   outc / final 1x1 (C > 2)   model/unet_resnet.py:78, model/unet_plain.py:69, model/unet_dualdense.py:88
//   CE_Loss / Focal_Loss / Dice_loss   model/unet_training.py:9-91
//   pixel_accuracy / mean_accuracy / mean_iou / frequency_weighted_iou   utils/train_and_eval.py:20-103
//   softmax + cv2.resize(INTER_LINEAR) + argmax   predict.py:79-93
//
// Logits are fp32 planar [B][C][P] (the reference's NCHW output); activations NHWC (bf16 / fp32).
// Every reduction is two-stage (per-block partials -> one finalize block), hence deterministic.
#include <cmath>

#include "common.h"

namespace {

constexpr int kMaxC = 32;   // classes handled in registers
constexpr int kHeadTile = 256;

// ------------------------------------------------------------------------------------------
// 1x1 head with K in (2, 32] outputs: y[n][k][hw] = sum_c x[p][c] w[k][c] + b[k] (fp32 out).
// Thread per pixel, weights in LDS (broadcast reads), K accumulators in registers.
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void pw_head_fwd_kernel(const T* x, int ldx, long M, int HW, int C, int K,
                                                          const float* w, const float* b, float* y) {
  extern __shared__ float sw[];  // [K][C]
  for (int i = threadIdx.x; i < K * C; i += blockDim.x) sw[i] = w[i];
  __syncthreads();
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= M) return;
  float acc[kMaxC];
#pragma unroll
  for (int k = 0; k < kMaxC; ++k) acc[k] = 0.f;
  constexpr int V = 16 / sizeof(T);
  for (int c0 = 0; c0 < C; c0 += V) {
    float xv[V];
    load_vec(x + p * ldx + c0, xv);
#pragma unroll
    for (int k = 0; k < kMaxC; ++k) {
      if (k < K) {
        float s = acc[k];
#pragma unroll
        for (int e = 0; e < V; ++e) s += xv[e] * sw[k * C + c0 + e];
        acc[k] = s;
      }
    }
  }
  const long n = p / HW, hw = p - n * HW;
#pragma unroll
  for (int k = 0; k < kMaxC; ++k)
    if (k < K) y[(n * K + k) * HW + hw] = acc[k] + (b ? b[k] : 0.f);
}

// Backward: dx (+)= dy . W (NHWC, T), dW / db partials part_w [K][C][G], part_b [K][G] over pixel
// tiles of ppb pixels.  Thread (tx = channel, ty = pixel row); dy in planar fp32.
template <typename T>
__global__ __launch_bounds__(256) void pw_head_bwd_kernel(const float* dy, const T* x, int ldx, long M, int HW, int C,
                                                          int K, const float* w, T* dx, int lddx, int dx_acc,
                                                          float* part_w, float* part_b, int G, int ppb) {
  extern __shared__ float sm[];  // [K][C] weights, then [256] reduction scratch
  float* swt = sm;
  float* red = sm + K * C;
  for (int i = threadIdx.x; i < K * C; i += blockDim.x) swt[i] = w[i];
  __syncthreads();
  const int rows = blockDim.x / C;  // C divides 256 (host check)
  const int tx = threadIdx.x % C, ty = threadIdx.x / C;
  const long p0 = (long)blockIdx.x * ppb, p1 = min(M, p0 + ppb);
  float sw[kMaxC], sb[kMaxC];
#pragma unroll
  for (int k = 0; k < kMaxC; ++k) sw[k] = sb[k] = 0.f;
  for (long p = p0 + ty; p < p1; p += rows) {
    const long n = p / HW, hw = p - n * HW;
    const float xv = (float)x[p * ldx + tx];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxC; ++k) {
      if (k < K) {
        const float g = dy[(n * K + k) * HW + hw];
        s += g * swt[k * C + tx];
        sw[k] += g * xv;
        sb[k] += g;
      }
    }
    if (dx) {
      T* dp = dx + p * lddx + tx;
      *dp = (T)(dx_acc ? s + (float)*dp : s);
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxC; ++k) {
    if (k < K) {  // uniform
      __syncthreads();
      red[threadIdx.x] = sw[k];
      __syncthreads();
      if (ty == 0) {
        float t = 0.f;
        for (int r = 0; r < rows; ++r) t += red[r * C + tx];
        part_w[((long)k * C + tx) * G + blockIdx.x] = t;
      }
      __syncthreads();
      red[threadIdx.x] = sb[k];
      __syncthreads();
      if (threadIdx.x == 0) {
        float t = 0.f;
        for (int r = 0; r < rows; ++r) t += red[r * C];  // column 0 threads carry the full sum
        part_b[(long)k * G + blockIdx.x] = t;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Fused multiclass loss.  Per pixel i (image b, position p), logits x_c, target t:
//   CE    (nn.CrossEntropyLoss(weight, ignore_index)): w_t (lse - x_t), mean = sum / sum w_t
//   Focal (reduction none, then alpha, gamma, mean over ALL pixels): logpt = -w_t nll (0 if ignored),
//         pt = exp(logpt), L = -(1-pt)^gamma * alpha * logpt
//   Dice  on softmax p and a float one-hot target [B][P][ct] (first C channels):
//         tp_c = sum t p, S_c = sum p, T_c = sum t; score_c = ((1+b^2) tp + s) / ((1+b^2) tp + b^2 fn + fp + s)
// Partials per block: [0] sum w*nll, [1] sum w, [2] sum focal, then tp[C], S[C], T[C].
// ------------------------------------------------------------------------------------------
struct McArgs {
  const float* out;
  const int64_t* tgt;
  const float* cls_w;   // [C] or NULL (= ones)
  const float* dice_t;  // [B][P][ct] float or NULL (no Dice)
  int B, C, ct;
  long P;
  long ignore;          // ignore_index
  int focal;            // main term: 0 CE, 1 Focal, 2 none (Dice only)
  float alpha, gamma;   // Focal (alpha < 0: None)
  float beta, smooth;   // Dice
};

__device__ __forceinline__ void softmax_pixel(const McArgs& a, long i, float (&x)[kMaxC], float& lse) {
  const long b = i / a.P, p = i - b * a.P;
  const float* base = a.out + b * a.C * a.P + p;
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < kMaxC; ++c)
    if (c < a.C) {
      x[c] = base[(long)c * a.P];
      m = fmaxf(m, x[c]);
    }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kMaxC; ++c)
    if (c < a.C) s += expf(x[c] - m);
  lse = m + logf(s);
}

__global__ __launch_bounds__(256) void mc_loss_partial_kernel(McArgs a, float* part, int G) {
  const int NP = 3 + 3 * a.C;
  __shared__ float red[256];
  float acc_wnll = 0.f, acc_w = 0.f, acc_f = 0.f;
  float tp[kMaxC], S[kMaxC], T[kMaxC];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) tp[c] = S[c] = T[c] = 0.f;
  const long total = (long)a.B * a.P;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float x[kMaxC], lse;
    softmax_pixel(a, i, x, lse);
    const long t = (a.tgt && a.focal != 2) ? a.tgt[i] : -1;
    const bool valid = t != a.ignore && t >= 0 && t < a.C;
    const float wt = valid ? (a.cls_w ? a.cls_w[t] : 1.f) : 0.f;
    float xt = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c)
      if (c == t) xt = x[c];
    const float nll = valid ? lse - xt : 0.f;
    acc_wnll += wt * nll;
    acc_w += wt;
    if (a.tgt && a.focal != 2 && t != a.ignore && !valid) {
      // a target that is neither a class nor ignore_index: nn.CrossEntropyLoss (the reference's CE_Loss
      // / Focal_Loss, model/unet_training.py:9-59) refuses it; here loss and gradient become NaN
      acc_w += __builtin_nanf("");
      acc_f += __builtin_nanf("");
    }
    if (a.focal == 1) {
      const float logpt = -(wt * nll);
      const float pt = expf(logpt);
      const float lp = a.alpha >= 0.f ? logpt * a.alpha : logpt;
      acc_f += -powf(1.f - pt, a.gamma) * lp;
    }
    if (a.dice_t) {
      const float* tt = a.dice_t + i * a.ct;
#pragma unroll
      for (int c = 0; c < kMaxC; ++c)
        if (c < a.C) {
          const float pc = expf(x[c] - lse), tc = tt[c];
          tp[c] += tc * pc;
          S[c] += pc;
          T[c] += tc;
        }
    }
  }
  auto reduce = [&](float v, int slot) {
    const float s = block_sum(v, red);
    if (threadIdx.x == 0) part[(long)blockIdx.x * NP + slot] = s;
  };
  reduce(acc_wnll, 0);
  reduce(acc_w, 1);
  reduce(acc_f, 2);
  if (a.dice_t)
    for (int c = 0; c < a.C; ++c) {
      float v0 = 0.f, v1 = 0.f, v2 = 0.f;
#pragma unroll
      for (int cc = 0; cc < kMaxC; ++cc)
        if (cc == c) v0 = tp[cc], v1 = S[cc], v2 = T[cc];
      reduce(v0, 3 + c);
      reduce(v1, 3 + a.C + c);
      reduce(v2, 3 + 2 * a.C + c);
    }
}

// sums (fp64, fixed order) -> loss[0] total, [1] main (CE or Focal), [2] Dice (0 if off);
// coef: [0] sum w (CE denominator), [1] B*P, then per class A_c, Bd_c (Dice numerator/denominator)
__global__ void mc_loss_finalize_kernel(McArgs a, const float* part, int G, float* loss, double* coef) {
  const int NP = 3 + 3 * a.C;
  __shared__ double s[3 + 3 * kMaxC];
  for (int j = threadIdx.x; j < NP; j += blockDim.x) {
    double t = 0.0;
    for (int g = 0; g < G; ++g) t += (double)part[(long)g * NP + j];
    s[j] = t;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const double n = (double)a.B * (double)a.P;
  const double main = a.focal == 2 ? 0.0 : a.focal == 1 ? s[2] / n : s[0] / s[1];
  double dice = 0.0;
  const bool bad = s[1] != s[1];  // an invalid target poisoned the weight sum (partial kernel)
  coef[0] = s[1];
  coef[1] = bad ? s[1] : n;
  if (a.dice_t) {
    const double b2 = (double)a.beta * a.beta;
    double mean = 0.0;
    for (int c = 0; c < a.C; ++c) {
      const double tp = s[3 + c], S = s[3 + a.C + c], T = s[3 + 2 * a.C + c];
      const double fp = S - tp, fn = T - tp;
      const double A = (1.0 + b2) * tp + a.smooth, D = (1.0 + b2) * tp + b2 * fn + fp + a.smooth;
      coef[2 + 2 * c] = A;
      coef[3 + 2 * c] = D;
      mean += A / D;
    }
    dice = 1.0 - mean / a.C;
  }
  loss[0] = (float)(bad ? s[1] : main + dice);
  loss[1] = (float)(bad ? s[1] : main);
  loss[2] = (float)dice;
}

// dout[b][c][p] = gscale * d(total)/dx_c
__global__ __launch_bounds__(256) void mc_loss_bwd_kernel(McArgs a, const double* coef, const float* gscale,
                                                          float* dout) {
  const long total = (long)a.B * a.P;
  const float g = gscale ? gscale[0] : 1.f;
  const float inv_w = (float)(1.0 / coef[0]), inv_n = (float)(1.0 / coef[1]);
  const float poison = 0.f * inv_n;  // NaN when an invalid target poisoned the sums, else 0
  const double b2 = (double)a.beta * a.beta;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float x[kMaxC], lse;
    softmax_pixel(a, i, x, lse);
    float pr[kMaxC];
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) pr[c] = c < a.C ? expf(x[c] - lse) : 0.f;
    const long t = (a.tgt && a.focal != 2) ? a.tgt[i] : -1;
    const bool valid = t != a.ignore && t >= 0 && t < a.C;
    const float wt = valid ? (a.cls_w ? a.cls_w[t] : 1.f) : 0.f;
    // main loss: dL/dx_c = k * (p_c - [c == t])
    float k = 0.f;
    if (valid) {
      if (a.focal == 0) {
        k = wt * inv_w;
      } else {
        float xt = 0.f;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c)
          if (c == t) xt = x[c];
        const float logpt = -(wt * (lse - xt));
        const float pt = expf(logpt);
        const float al = a.alpha >= 0.f ? a.alpha : 1.f;
        // L = -al (1-pt)^gm logpt ; dL/dlogpt = al [gm (1-pt)^(gm-1) pt logpt - (1-pt)^gm]
        const float om = 1.f - pt;
        const float dldl = al * (a.gamma * powf(om, a.gamma - 1.f) * pt * logpt - powf(om, a.gamma));
        k = -dldl * wt * inv_n;  // dlogpt/dx_c = -wt (p_c - [c==t])
      }
    }
    float d[kMaxC];
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) d[c] = k * (pr[c] - (c == t ? 1.f : 0.f)) + poison;
    if (a.dice_t) {
      const float* tt = a.dice_t + i * a.ct;
      float gp[kMaxC], dot = 0.f;
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        gp[c] = 0.f;
        if (c < a.C) {
          const double A = coef[2 + 2 * c], D = coef[3 + 2 * c];
          // d score_c / d p_c = ((1+b2) t D - A) / D^2   (D = b2 T + S + s)
          gp[c] = (float)(-((1.0 + b2) * tt[c] * D - A) / (D * D) / a.C);
          dot += gp[c] * pr[c];
        }
      }
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) d[c] += pr[c] * (gp[c] - dot);
    }
    const long b = i / a.P, p = i - b * a.P;
    float* o = dout + b * a.C * a.P + p;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c)
      if (c < a.C) o[(long)c * a.P] = g * d[c];
  }
}

// ------------------------------------------------------------------------------------------
// Multiclass confusion histogram: hist[t][pred] (+)= 1 with pred = argmax_c (first maximum, as
// torch.max) and row t clamped to C for targets outside [0, C) (ignore / void pixels still count in
// pixel_accuracy's total and in the predicted-class union of mean_iou).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mc_confusion_kernel(const float* out, const int64_t* tgt, int B, int C, long P,
                                                           unsigned long long* hist) {
  __shared__ unsigned int h[(kMaxC + 1) * kMaxC];
  const int nb = (C + 1) * C;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) h[j] = 0;
  __syncthreads();
  const long total = (long)B * P;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / P, p = i - b * P;
    const float* base = out + b * C * P + p;
    float m = base[0];
    int am = 0;
    for (int c = 1; c < C; ++c) {
      const float v = base[(long)c * P];
      if (v > m) {
        m = v;
        am = c;
      }
    }
    const long t = tgt[i];
    const int row = (t >= 0 && t < C) ? (int)t : C;
    atomicAdd(&h[row * C + am], 1u);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nb; j += blockDim.x)
    if (h[j]) atomicAdd(&hist[j], (unsigned long long)h[j]);
}

// ------------------------------------------------------------------------------------------
// predict.py:79-93 for one image: probabilities = softmax over C of logits [C][H][W], cropped to
// the letterbox window (y0, x0, ch, cw), resized bilinearly (half-pixel centres, edge clamp: cv2
// INTER_LINEAR = F.interpolate(align_corners=False) without antialias) to OH x OW, argmax (first).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void softmax_resize_argmax_kernel(const float* lg, int C, int H, int W, int y0,
                                                                    int x0, int ch, int cw, int OH, int OW,
                                                                    int32_t* labels) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)OH * OW) return;
  const int oy = (int)(i / OW), ox = (int)(i - (long)oy * OW);
  auto src = [](int d, int n_in, int n_out, int& i0, int& i1, float& l) {
    float s = ((float)d + 0.5f) * ((float)n_in / (float)n_out) - 0.5f;
    if (s < 0.f) s = 0.f;
    i0 = (int)s;
    if (i0 > n_in - 1) i0 = n_in - 1;
    i1 = i0 + (i0 < n_in - 1 ? 1 : 0);
    l = s - (float)i0;
  };
  int ya, yb, xa, xb;
  float ly, lx;
  src(oy, ch, OH, ya, yb, ly);
  src(ox, cw, OW, xa, xb, lx);
  const long HW = (long)H * W;
  const long q[4] = {(long)(y0 + ya) * W + x0 + xa, (long)(y0 + ya) * W + x0 + xb, (long)(y0 + yb) * W + x0 + xa,
                     (long)(y0 + yb) * W + x0 + xb};
  const float wq[4] = {(1.f - ly) * (1.f - lx), (1.f - ly) * lx, ly * (1.f - lx), ly * lx};
  float mx[4], den[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, lg[c * HW + q[k]]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(lg[c * HW + q[k]] - m);
    mx[k] = m;
    den[k] = s;
  }
  float best = -1.f;
  int arg = 0;
  for (int c = 0; c < C; ++c) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) v += wq[k] * (expf(lg[c * HW + q[k]] - mx[k]) / den[k]);
    if (v > best) {
      best = v;
      arg = c;
    }
  }
  labels[i] = arg;
}

inline int grid_of(long n, int per = 256, int cap = 65535 * 4) {
  long g = (n + per - 1) / per;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

#define MC_DISPATCH_T(dtype, ...) \
  do {                            \
    if ((dtype) == DT_BF16) {     \
      typedef bf16 T;             \
      __VA_ARGS__;                \
    } else {                      \
      typedef float T;            \
      __VA_ARGS__;                \
    }                             \
  } while (0)

UNETSEG_API int unetseg_pw_head_tiles(long M) { return ceil_div(M, (long)kHeadTile * 8); }

UNETSEG_API int unetseg_pw_head_fwd(int dtype, const void* x, int ldx, long M, int hw, int c, int k, const float* w,
                                    const float* b, float* y, void* stream) {
  US_CHECK_ARG(x && w && y && k >= 1 && k <= kMaxC && c > 0 && c % (dtype == DT_BF16 ? 8 : 4) == 0,
               "pw_head_fwd: bad args (k=%d <= %d, c=%d multiple of the 16-B vector)", k, kMaxC, c);
  if (M <= 0) return 0;
  const size_t lds = (size_t)k * c * sizeof(float);
  MC_DISPATCH_T(dtype, hipLaunchKernelGGL(pw_head_fwd_kernel<T>, dim3(ceil_div(M, 256)), dim3(256), lds,
                                          (hipStream_t)stream, (const T*)x, ldx, M, hw, c, k, w, b, y));
  US_LAUNCH_CHECK("pw_head_fwd");
  return 0;
}

// dx (may be NULL) (+)= dy . W ; part_w [k][c][G], part_b [k][G], G = unetseg_pw_head_tiles(M)
UNETSEG_API int unetseg_pw_head_bwd(int dtype, const float* dy, const void* x, int ldx, long M, int hw, int c, int k,
                                    const float* w, void* dx, int lddx, int dx_acc, float* part_w, float* part_b,
                                    void* stream) {
  US_CHECK_ARG(dy && x && w && part_w && part_b && k >= 1 && k <= kMaxC && c > 0 && c <= 256 && 256 % c == 0,
               "pw_head_bwd: bad args (k=%d, c=%d must divide 256)", k, c);
  if (M <= 0) return 0;
  const int G = unetseg_pw_head_tiles(M);
  const size_t lds = ((size_t)k * c + 256) * sizeof(float);
  MC_DISPATCH_T(dtype, hipLaunchKernelGGL(pw_head_bwd_kernel<T>, dim3(G), dim3(256), lds, (hipStream_t)stream, dy,
                                          (const T*)x, ldx, M, hw, c, k, w, (T*)dx, lddx, dx_acc, part_w, part_b, G,
                                          kHeadTile * 8));
  US_LAUNCH_CHECK("pw_head_bwd");
  return 0;
}

static McArgs mc_args(const float* out, const int64_t* tgt, int B, int C, long P, const float* cls_w, long ignore,
                      int focal, float alpha, float gamma, const float* dice_t, int ct, float beta, float smooth) {
  McArgs a{};
  a.out = out; a.tgt = tgt; a.cls_w = cls_w; a.dice_t = dice_t; a.B = B; a.C = C; a.ct = ct; a.P = P;
  a.ignore = ignore; a.focal = focal; a.alpha = alpha; a.gamma = gamma; a.beta = beta; a.smooth = smooth;
  return a;
}

static int mc_blocks(int B, long P) { return grid_of((long)B * P, 256, 1024); }

// workspace: per-block partials + fp64 coefficients
UNETSEG_API size_t unetseg_mc_loss_workspace(int B, int C, long P) {
  return (size_t)mc_blocks(B, P) * (3 + 3 * C) * sizeof(float) + (2 + 2 * kMaxC) * sizeof(double) + 64;
}

// loss fp32[3] = (total, main, Dice); focal selects the main term: 0 CE, 1 Focal, 2 none (Dice only,
// tgt may be NULL).  Fills the workspace's coefficients for the backward.
// cls_w [C] may be NULL; dice_t float [B][P][ct] (one-hot, ct >= C) may be NULL (no Dice term);
// alpha < 0 means Focal's alpha=None.
UNETSEG_API int unetseg_mc_loss_fwd(const float* out, const int64_t* tgt, int B, int C, long P, const float* cls_w,
                                    long ignore_index, int focal, float alpha, float gamma, const float* dice_t, int ct,
                                    float beta, float smooth, void* ws, size_t ws_bytes, float* loss, void* stream) {
  US_CHECK_ARG(out && (tgt || focal == 2) && ws && loss && B > 0 && P > 0 && C >= 1 && C <= kMaxC && focal >= 0 &&
                   focal <= 2, "mc_loss_fwd: bad args (C=%d, kind %d)", C, focal);
  US_CHECK_ARG(!dice_t || ct >= C, "mc_loss_fwd: dice target has %d < %d channels", ct, C);
  US_CHECK_ARG(ws_bytes >= unetseg_mc_loss_workspace(B, C, P), "mc_loss_fwd: workspace too small");
  const int G = mc_blocks(B, P);
  float* part = (float*)ws;
  double* coef = (double*)(((uintptr_t)(part + (size_t)G * (3 + 3 * C)) + 15) & ~(uintptr_t)15);
  McArgs a = mc_args(out, tgt, B, C, P, cls_w, ignore_index, focal, alpha, gamma, dice_t, ct, beta, smooth);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(mc_loss_partial_kernel, dim3(G), dim3(256), 0, st, a, part, G);
  hipLaunchKernelGGL(mc_loss_finalize_kernel, dim3(1), dim3(128), 0, st, a, part, G, loss, coef);
  US_LAUNCH_CHECK("mc_loss_fwd");
  return 0;
}

// dout fp32 [B][C][P] = gscale[0] (device scalar, NULL = 1) * d total / d out, from the workspace
// filled by the matching unetseg_mc_loss_fwd
UNETSEG_API int unetseg_mc_loss_bwd(const float* out, const int64_t* tgt, int B, int C, long P, const float* cls_w,
                                    long ignore_index, int focal, float alpha, float gamma, const float* dice_t, int ct,
                                    float beta, float smooth, const void* ws, const float* gscale, float* dout,
                                    void* stream) {
  US_CHECK_ARG(out && (tgt || focal == 2) && ws && dout && C >= 1 && C <= kMaxC, "mc_loss_bwd: bad args");
  const int G = mc_blocks(B, P);
  const float* part = (const float*)ws;
  const double* coef = (const double*)(((uintptr_t)(part + (size_t)G * (3 + 3 * C)) + 15) & ~(uintptr_t)15);
  McArgs a = mc_args(out, tgt, B, C, P, cls_w, ignore_index, focal, alpha, gamma, dice_t, ct, beta, smooth);
  hipLaunchKernelGGL(mc_loss_bwd_kernel, dim3(grid_of((long)B * P)), dim3(256), 0, (hipStream_t)stream, a, coef,
                     gscale, dout);
  US_LAUNCH_CHECK("mc_loss_bwd");
  return 0;
}

// hist u64 [(C+1)][C] += confusion of argmax(out) vs tgt (rows: target class, row C = any other value)
UNETSEG_API int unetseg_mc_confusion(const float* out, const int64_t* tgt, int B, int C, long P,
                                     unsigned long long* hist, void* stream) {
  US_CHECK_ARG(out && tgt && hist && C >= 1 && C <= kMaxC, "mc_confusion: bad args (C=%d)", C);
  hipLaunchKernelGGL(mc_confusion_kernel, dim3(grid_of((long)B * P, 256, 2048)), dim3(256), 0, (hipStream_t)stream, out,
                     tgt, B, C, P, hist);
  US_LAUNCH_CHECK("mc_confusion");
  return 0;
}

// labels int32 [OH][OW] for one image's logits [C][H][W] (predict.py:79-93)
UNETSEG_API int unetseg_softmax_resize_argmax(const float* logits, int C, int H, int W, int y0, int x0, int ch, int cw,
                                              int OH, int OW, int32_t* labels, void* stream) {
  US_CHECK_ARG(logits && labels && C >= 1 && ch >= 1 && cw >= 1 && y0 >= 0 && x0 >= 0 && y0 + ch <= H &&
                   x0 + cw <= W && OH >= 1 && OW >= 1,
               "softmax_resize_argmax: bad window");
  hipLaunchKernelGGL(softmax_resize_argmax_kernel, dim3(ceil_div((long)OH * OW, 256)), dim3(256), 0,
                     (hipStream_t)stream, logits, C, H, W, y0, x0, ch, cw, OH, OW, labels);
  US_LAUNCH_CHECK("softmax_resize_argmax");
  return 0;
}
