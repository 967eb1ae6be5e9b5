// Loss, metric and optimizer kernels of the U-Net hot path.
//
//   Lovasz hinge   model/unet_training.py:219-280  (per-image sort desc, Jaccard grad, dot)
//   BCE w/ logits  model/unet_training.py:205-216, utils/train_and_eval.py:155-182
//   2-class->1     utils/train_and_eval.py:106-113 (z = o1 - o0, fused into the loss kernels)
//   CE + cls head  model/unet_multitask.py:73-80,109-139
//   confusion      utils/train_and_eval.py:116-152, train.py:330-340
//   Adam           train.py:62-78 (torch.optim.Adam, coupled L2 weight decay)
//
// The Lovasz sort is a segmented, stable LSD radix sort (4 x 8-bit passes) on 32-bit keys that
// order the hinge errors descending; ties keep ascending pixel order (the reference's
// torch.sort is not stable, so only the loss VALUE is tie-order independent).
#include "common.h"

namespace {

constexpr int kTile = 4096;  // keys per radix tile (256 threads x 16)

__device__ __forceinline__ uint32_t desc_key(float f) {
  uint32_t u = __float_as_uint(f);
  uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ~asc;
}
__device__ __forceinline__ float key_to_float(uint32_t k) {
  uint32_t asc = ~k;
  uint32_t u = (asc & 0x80000000u) ? (asc & 0x7fffffffu) : ~asc;
  return __uint_as_float(u);
}

// logits source: planar fp32 [B][nch][P]; nch==2 -> z = o1 - o0, nch==1 -> z = o0
__device__ __forceinline__ float load_z(const float* out, int nch, int b, long P, long i) {
  const float* base = out + (long)b * nch * P;
  // both loads unconditional (a load under the nch branch was waited on inside it)
  const float o0 = base[i], o1 = base[nch == 2 ? P + i : i];
  return nch == 2 ? o1 - o0 : o0;
}

// has_ignore: pixels whose target is `ignore` get error -inf and label 0, so they sort after every
// valid pixel and contribute to neither the loss, the gradient nor the Jaccard counts of the valid
// prefix: the per-image Lovasz over the valid pixels (model/unet_training.py:268-274)
__global__ void lovasz_keygen_kernel(const float* out, int nch, const int64_t* tgt, int B, long P, uint32_t* keys,
                                     uint32_t* vals, int has_ignore, long ignore) {
  const long total = (long)B * P;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / P);
    const long px = i - (long)b * P;
    const float z = load_z(out, nch, b, P, px);
    const int64_t tv = tgt[i];
    const bool ign = has_ignore && tv == ignore;
    const uint32_t y = (!ign && tv == 1) ? 1u : 0u;
    const float e = ign ? -INFINITY : 1.0f - z * (2.0f * (float)y - 1.0f);
    keys[i] = desc_key(e);
    vals[i] = (uint32_t)px | (y << 31);
  }
}

__global__ void radix_hist_kernel(const uint32_t* keys, long P, int T, int shift, uint32_t* hist) {
  __shared__ uint32_t h[256];
  const int t = blockIdx.x, b = blockIdx.y;
  h[threadIdx.x] = 0;
  __syncthreads();
  const long base = (long)b * P + (long)t * kTile;
  const long n = min((long)kTile, P - (long)t * kTile);
  for (long i = threadIdx.x; i < n; i += 256) atomicAdd(&h[(keys[base + i] >> shift) & 255u], 1u);
  __syncthreads();
  hist[((long)b * 256 + threadIdx.x) * T + t] = h[threadIdx.x];
}

// exclusive scan of hist[b][256*T] (digit-major) in place; one 1024-thread block per segment.  Each
// thread owns a contiguous run of the segment, loaded once into registers; the runs' totals are
// scanned with wave shuffles and one LDS exchange of the 16 wave totals.
constexpr int kScanPer = 32;  // entries per thread held in registers (up to 128 tiles = 524288 pixels per image)
__global__ __launch_bounds__(1024) void radix_scan_kernel(uint32_t* hist, int T) {
  __shared__ uint32_t wsum[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t* h = hist + (long)b * 256 * T;
  const long n = 256L * T;
  const long per = (n + 1023) / 1024;
  const long lo = tid * per, hi = min(n, lo + per);
  const bool regs = per <= kScanPer;  // else (more than 524288 pixels per image) two passes over memory
  uint32_t v[kScanPer];
  uint32_t s = 0;
  if (regs) {
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
      v[i] = (i < per && lo + i < hi) ? h[lo + i] : 0u;
      s += v[i];
    }
  } else {
    for (long i = lo; i < hi; ++i) s += h[i];
  }
  // inclusive scan of the per-thread totals within the wave, then across the 16 waves
  uint32_t x = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t run = x - s;
  for (int w = 0; w < wid; ++w) run += wsum[w];
  if (regs) {
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
      if (i < per && lo + i < hi) h[lo + i] = run;
      run += v[i];
    }
  } else {
    for (long i = lo; i < hi; ++i) {
      const uint32_t c = h[i];
      h[i] = run;
      run += c;
    }
  }
}

// stable scatter.  The tile is ranked in 16 rounds of 256 keys (original order = round-major) into LDS
// in digit order, then written out from LDS: consecutive slots of one digit go to consecutive global
// positions, so the writes leave as runs (~16 keys per digit and tile) instead of one scattered 4-B
// store per key.
__global__ __launch_bounds__(256) void radix_scatter_kernel(const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
                                                            uint32_t* vout, long P, int T, int shift,
                                                            const uint32_t* hist) {
  __shared__ uint32_t gbase[256];  // global position of this tile's first key of each digit
  __shared__ uint32_t lstart[256];  // tile-local first slot of each digit
  __shared__ uint32_t run[256];     // keys of each digit placed so far
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t sk[kTile], sv[kTile];
  const int t = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t* hb = hist + (long)b * 256 * T;
  const long seg = (long)b * P;
  const long tbase = (long)t * kTile;
  const long n = min((long)kTile, P - tbase);
  // this tile's count of digit `tid`: the next entry of the digit-major exclusive scan minus this one
  const long hi = (long)tid * T + t;
  const uint32_t g0 = hb[hi];
  const uint32_t cnt = (hi + 1 < 256L * T ? hb[hi + 1] : (uint32_t)P) - g0;
  gbase[tid] = g0;
  // exclusive scan of the 256 counts (wave prefix sums, then the four wave totals)
  uint32_t x = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wcnt[0][wid] = x;
  __syncthreads();
  uint32_t off = 0;
  for (int w = 0; w < wid; ++w) off += wcnt[0][w];
  lstart[tid] = off + x - cnt;
  run[tid] = 0;
  __syncthreads();
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  for (int round = 0; round < kTile / 256; ++round) {
    const long i = round * 256L + tid;
    const bool ok = i < n;
#pragma unroll
    for (int w = 0; w < 4; ++w) wcnt[w][tid] = 0;
    __syncthreads();
    uint32_t key = 0, val = 0, d = 0;
    if (ok) {
      key = kin[seg + tbase + i];
      val = vin[seg + tbase + i];
      d = (key >> shift) & 255u;
    }
    unsigned long long m = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const unsigned long long bal = __ballot(ok && ((d >> bit) & 1u));
      m &= ((d >> bit) & 1u) ? bal : ~bal;
    }
    const int lrank = __popcll(m & lt_mask);
    if (ok && lrank == 0) wcnt[wid][d] = (uint32_t)__popcll(m);
    __syncthreads();
    if (ok) {
      uint32_t pos = lstart[d] + run[d] + lrank;
      for (int w = 0; w < wid; ++w) pos += wcnt[w][d];
      sk[pos] = key;
      sv[pos] = val;
    }
    __syncthreads();
    run[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
  }
  __syncthreads();
  for (int j = tid; j < n; j += 256) {
    const uint32_t key = sk[j];
    const uint32_t d = (key >> shift) & 255u;
    const uint32_t pos = gbase[d] + (uint32_t)j - lstart[d];
    kout[seg + pos] = key;
    vout[seg + pos] = sv[j];
  }
}

// positives per (image, 4096-key chunk) of the sorted order
__global__ void lovasz_count_kernel(const uint32_t* vals, long P, int T, uint32_t* cnt) {
  __shared__ uint32_t sc[4];
  const int t = blockIdx.x, b = blockIdx.y;
  const long lo = (long)t * kTile, hi = min(P, lo + kTile);
  const uint32_t* v = vals + (long)b * P;
  uint32_t c = 0;
  for (long i = lo + threadIdx.x; i < hi; i += 256) c += v[i] >> 31;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[(long)b * T + t] = sc[0] + sc[1] + sc[2] + sc[3];
}

// per chunk: Jaccard gradient over the sorted labels, loss partial = sum relu(e)*g,
// dz[pixel] = g*[e>0]*(-(2y-1))/B.  256 threads x 16 consecutive sorted keys.
__global__ void lovasz_chunk_kernel(const uint32_t* keys, const uint32_t* vals, long P, int T, const uint32_t* cnt,
                                    float inv_b, float* gz, float* part) {
  __shared__ uint32_t wsum[4];
  __shared__ double sred[16];
  const int t = blockIdx.x, b = blockIdx.y;
  const uint32_t* cb = cnt + (long)b * T;
  uint32_t G = 0, before = 0;
  for (int j = 0; j < T; ++j) {
    const uint32_t c = cb[j];
    G += c;
    if (j < t) before += c;
  }
  const long lo = (long)t * kTile + threadIdx.x * 16;
  const long hi = min(P, lo + 16);
  const uint32_t* k = keys + (long)b * P;
  const uint32_t* v = vals + (long)b * P;
  uint32_t vv[16], kk[16];
  uint32_t mine = 0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const long i = lo + e;
    vv[e] = i < hi ? v[i] : 0u;
    kk[e] = i < hi ? k[i] : 0u;
    mine += vv[e] >> 31;
  }
  // exclusive scan of `mine` over the block
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int w = 0; w < wid; ++w) woff += wsum[w];
  uint32_t cp = before + woff + incl - mine;  // positives strictly before lo
  const float Gf = (float)G;
  float jprev;
  if (lo == 0) {
    jprev = 0.f;
  } else {
    const float cn = (float)(lo - cp);
    jprev = 1.0f - (Gf - (float)cp) / (Gf + cn);
  }
  double loss = 0.0;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const long i = lo + e;
    if (i < hi) {
      const uint32_t y = vv[e] >> 31;
      cp += y;
      const float cn = (float)(i + 1 - cp);
      const float j = 1.0f - (Gf - (float)cp) / (Gf + cn);
      const float g = j - jprev;
      jprev = j;
      const float err = key_to_float(kk[e]);
      if (err > 0.f) loss += (double)err * (double)g;
      gz[(long)b * P + (vv[e] & 0x7fffffffu)] = err > 0.f ? g * (y ? -inv_b : inv_b) : 0.f;
    }
  }
  loss = block_sum(loss, sred);
  if (threadIdx.x == 0) part[(long)b * T + t] = (float)loss;
}

// loss = mean_b sum_t part[b][t]  (fixed order)
__global__ void lovasz_final_kernel(const float* part, int B, int T, float* loss) {
  __shared__ double sred[16];
  double s = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    double sb = 0.0;
    for (int t = 0; t < T; ++t) sb += part[(long)b * T + t];
    s += sb;
  }
  s = block_sum(s, sred);
  if (threadIdx.x == 0) loss[0] = B > 0 ? (float)(s / B) : 0.f;
}

__global__ void mean_kernel(const float* x, int n, float* out) {
  __shared__ double sred[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = block_sum(s, sred);
  if (threadIdx.x == 0) out[0] = n > 0 ? (float)(s / n) : 0.f;
}

// d_out for a per-pixel dz: nch==2 -> d o1 = +g, d o0 = -g ; scale = upstream[0] * factor
__global__ void dz_to_dout_kernel(const float* gz, int B, long P, int nch, const float* upstream, float factor,
                                  float* dout) {
  const float sc = (upstream ? upstream[0] : 1.f) * factor;
  const long total = (long)B * P;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / P);
    const long px = i - (long)b * P;
    const float g = gz[i] * sc;
    if (nch == 2) {
      dout[((long)b * 2 + 1) * P + px] = g;
      dout[((long)b * 2) * P + px] = -g;
    } else {
      dout[(long)b * P + px] = g;
    }
  }
}

// BCE with logits (PyTorch formulation), per-block partial sums; grad dz stored unscaled (1/count applied)
__global__ void bce_kernel(const float* out, int nch, const int64_t* tgt, int B, long P, const float* pos_weight,
                           float* gz, float* part) {
  __shared__ double sred[16];
  const long total = (long)B * P;
  const float pw = pos_weight ? pos_weight[0] : 1.0f;
  double s = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / P);
    const long px = i - (long)b * P;
    const float z = load_z(out, nch, b, P, px);
    const float y = tgt[i] == 1 ? 1.f : 0.f;
    const float lw = (pw - 1.f) * y + 1.f;
    const float sp = log1pf(expf(-fabsf(z))) + fmaxf(-z, 0.f);
    s += (double)((1.f - y) * z + lw * sp);
    const float sig_neg = 1.f / (1.f + expf(z));  // sigmoid(-z)
    if (gz) gz[i] = ((1.f - y) - lw * sig_neg) / (float)total;
  }
  s = block_sum(s, sred);
  if (threadIdx.x == 0) part[blockIdx.x] = (float)(s / (double)total);
}

__global__ void sum_kernel(const float* x, int n, float* out) {
  __shared__ double sred[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = block_sum(s, sred);
  if (threadIdx.x == 0) out[0] = (float)s;
}

// Binary loss over the pixels whose target is not ignore_index (utils/train_and_eval.py:169-176):
// kind 0 = BCE-with-logits (pos_weight); kind 1 = the reference's Lovasz on the FLATTENED valid
// pixels: lovasz_hinge_loss then iterates over single pixels (model/unet_training.py:267-276), so its
// value is the mean hinge relu(1 - z(2y-1)) with gradient -(2y-1)[e > 0].  gz gets the per-pixel
// gradient numerator (0 on ignored pixels); part [2][G] = (loss sum, valid count) per block.
__global__ void masked_loss_kernel(const float* out, int nch, const int64_t* tgt, int B, long P, long ignore, int kind,
                                   const float* pos_weight, float* gz, float* part) {
  __shared__ double sred[16];
  const long total = (long)B * P;
  const float pw = pos_weight ? pos_weight[0] : 1.0f;
  double s = 0.0, n = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / P);
    const long px = i - (long)b * P;
    const int64_t t = tgt[i];
    float g = 0.f;
    if (t != ignore) {
      const float z = load_z(out, nch, b, P, px);
      const float y = t == 1 ? 1.f : 0.f;
      if (kind == 0) {
        const float lw = (pw - 1.f) * y + 1.f;
        const float sp = log1pf(expf(-fabsf(z))) + fmaxf(-z, 0.f);
        s += (double)((1.f - y) * z + lw * sp);
        g = (1.f - y) - lw / (1.f + expf(z));
      } else {
        const float sg = 2.f * y - 1.f, e = 1.f - z * sg;
        s += (double)fmaxf(e, 0.f);
        g = e > 0.f ? -sg : 0.f;
      }
      n += 1.0;
    }
    gz[i] = g;
  }
  s = block_sum(s, sred);
  n = block_sum(n, sred);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = (float)s;
    part[gridDim.x + blockIdx.x] = (float)n;
  }
}

// loss = sum / count (count 0: NaN for BCE, as a mean over nothing; 0 for the Lovasz branch, whose
// empty loss list returns logits.sum() * 0); inv = 1 / count (0 if none)
__global__ void masked_finalize_kernel(const float* part, int G, int kind, float* loss, float* inv) {
  __shared__ double sred[16];
  double s = 0.0, n = 0.0;
  for (int i = threadIdx.x; i < G; i += blockDim.x) {
    s += part[i];
    n += part[G + i];
  }
  s = block_sum(s, sred);
  n = block_sum(n, sred);
  if (threadIdx.x == 0) {
    loss[0] = n > 0.0 ? (float)(s / n) : (kind == 0 ? __builtin_nanf("") : 0.f);
    inv[0] = n > 0.0 ? (float)(1.0 / n) : 0.f;
  }
}

__global__ void scale_by_kernel(float* x, long n, const float* s) {
  const float f = s[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= f;
}

// confusion counts: mode 2 -> pred = o1 > o0 (argmax, tie -> 0); mode 1 -> pred = sigmoid(o0) > 0.5;
// pixels whose target equals `ignore` are skipped when has_ignore (utils/train_and_eval.py:125-126)
__global__ void confusion_kernel(const float* out, int nch, const int64_t* tgt, int B, long P,
                                 unsigned long long* conf, int has_ignore, long ignore) {
  __shared__ unsigned long long sc[4][16];
  const long total = (long)B * P;
  unsigned long long c[4] = {0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    if (has_ignore && tgt[i] == ignore) continue;
    const int b = (int)(i / P);
    const long px = i - (long)b * P;
    bool pred;
    if (nch == 2) {
      const float* base = out + (long)b * 2 * P;
      pred = base[P + px] > base[px];
    } else {
      const float z = out[(long)b * P + px];
      pred = 1.0f / (1.0f + expf(-z)) > 0.5f;
    }
    const bool t = tgt[i] == 1;
    c[pred && t ? 0 : (pred ? 1 : (t ? 2 : 3))] += 1;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    unsigned long long v = c[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) sc[k][wid] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long v = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) v += sc[threadIdx.x][w];
    atomicAdd(&conf[threadIdx.x], v);
  }
}

// torch.optim.Adam single step on flat fp32 buffers (coupled L2 weight decay)
__global__ void adam_kernel(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                            float eps, float wd, float bc1, float bc2_sqrt, const float* grad_scale) {
  const float inv_scale = grad_scale ? 1.0f / grad_scale[0] : 1.0f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gr = g[i] * inv_scale;
    const float pv = p[i];
    if (wd != 0.f) gr = gr + wd * pv;
    float mv = m[i];
    mv = mv + (1.f - beta1) * (gr - mv);
    float vv = v[i] * beta2 + (1.f - beta2) * gr * gr;
    m[i] = mv;
    v[i] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    p[i] = pv - (lr / bc1) * (mv / denom);
  }
}

// Capturable form (hipGraph replay): lr and the step count live in device memory, so a replayed
// step uses the current values.  hyper[0] = lr; *step is the count of steps already taken (the
// update uses *step + 1; adam_step_commit advances it afterwards).
__global__ void adam_dev_kernel(float* p, const float* g, float* m, float* v, long n, const float* hyper,
                                const int* step, float beta1, float beta2, float eps, float wd,
                                const float* grad_scale) {
  __shared__ float k[2];
  if (threadIdx.x == 0) {
    const double t = (double)(step[0] + 1);
    const double bc1 = 1.0 - pow((double)beta1, t);
    const double bc2 = 1.0 - pow((double)beta2, t);
    k[0] = (float)bc1;
    k[1] = (float)sqrt(bc2);
  }
  __syncthreads();
  const float bc1 = k[0], bc2_sqrt = k[1], lr = hyper[0];
  const float inv_scale = grad_scale ? 1.0f / grad_scale[0] : 1.0f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gr = g[i] * inv_scale;
    const float pv = p[i];
    if (wd != 0.f) gr = gr + wd * pv;
    float mv = m[i];
    mv = mv + (1.f - beta1) * (gr - mv);
    float vv = v[i] * beta2 + (1.f - beta2) * gr * gr;
    m[i] = mv;
    v[i] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    p[i] = pv - (lr / bc1) * (mv / denom);
  }
}

__global__ void adam_step_commit_kernel(int* step) { step[0] += 1; }

// ------------------------------------------------------------------------------------------
// multitask classification head (model/unet_multitask.py:73-80)
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void gap_kernel(const T* x, int ldx, int B, int HW, int C, float* g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C;
  double s = 0.0;
  for (int p = 0; p < HW; ++p) s += (float)x[((long)b * HW + p) * ldx + c];
  g[i] = (float)(s / HW);
}

template <typename T>
__global__ void gap_bwd_kernel(const float* dg, int B, int HW, int C, T* dx, int ldx, int accumulate) {
  const long total = (long)B * HW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / C;
    const int c = (int)(i - pix * C);
    const int b = (int)(pix / HW);
    T* o = dx + pix * ldx + c;
    float v = dg[(long)b * C + c] / (float)HW;
    if (accumulate) v += (float)(*o);
    *o = (T)v;
  }
}

__device__ __forceinline__ float hash_u01(unsigned long long seed, unsigned long long i) {
  unsigned long long z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// y[b][o] = act(sum_i x[b][i] W[o][i] + bias[o]); act: 0 none, 1 relu, 2 relu + dropout(p)
// one wave per output element
__global__ void linear_fwd_kernel(const float* x, const float* W, const float* bias, int B, int I, int O, int act,
                                  float p_drop, unsigned long long seed, const float* mask_in, float* mask_out,
                                  float* pre, float* y) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wave >= B * O) return;
  const int b = wave / O, o = wave - b * O;
  float s = 0.f;
  // eight rounds' loads in flight (the plain loop waited out one round trip per 64 inputs); the
  // products are added in the same i order
  constexpr int U = 8;
  int i = lane;
  for (; i + 64 * (U - 1) < I; i += 64 * U) {
    float xv[U], wv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xv[u] = x[(long)b * I + i + 64 * u];
      wv[u] = W[(long)o * I + i + 64 * u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s = fmaf(xv[u], wv[u], s);  // explicit: as the plain loop's contraction
  }
  for (; i < I; i += 64) s += x[(long)b * I + i] * W[(long)o * I + i];
  s = wave_sum(s);
  if (lane == 0) {
    s += bias ? bias[o] : 0.f;
    if (pre) pre[wave] = s;
    if (act >= 1) s = fmaxf(s, 0.f);
    if (act == 2) {
      float keep;
      if (mask_in) keep = mask_in[wave];
      else keep = hash_u01(seed, (unsigned long long)wave) >= p_drop ? 1.f : 0.f;
      if (mask_out) mask_out[wave] = keep;
      s = s * keep / (1.f - p_drop);
    }
    y[wave] = s;
  }
}

// backward of linear (+ act): dyp = dy * act'(pre) ; dx[b][i] = sum_o dyp W[o][i] ; dW += ; db +=
__global__ void linear_act_bwd_kernel(const float* dy, const float* pre, const float* mask, float p_drop, int act,
                                      int B, int O, float* dyp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * O) return;
  float g = dy[i];
  if (act >= 1 && pre[i] <= 0.f) g = 0.f;
  if (act == 2) g = g * mask[i] / (1.f - p_drop);
  dyp[i] = g;
}

__global__ void linear_bwd_x_kernel(const float* dyp, const float* W, int B, int I, int O, float* dx) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * I) return;
  const int b = t / I, i = t - b * I;
  float s = 0.f;
  // 32 outputs' loads in flight per round (one round trip per load left the 2048 -> 512 FC's
  // backward at ~100 us); the products are added in the same o order as the plain loop
  constexpr int U = 32;
  int o = 0;
  for (; o + U <= O; o += U) {
    float d[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      d[u] = dyp[(long)b * O + o + u];
      w[u] = W[(long)(o + u) * I + i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s = fmaf(d[u], w[u], s);  // explicit: the packed-multiply form rounds twice
  }
  for (; o < O; ++o) s += dyp[(long)b * O + o] * W[(long)o * I + i];
  dx[t] = s;
}

__global__ void linear_bwd_w_kernel(const float* dyp, const float* x, int B, int I, int O, float* dW, float* db) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= O * I) return;
  const int o = t / I, i = t - o * I;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += dyp[(long)b * O + o] * x[(long)b * I + i];
  dW[t] += s;
  if (i == 0 && db) {
    float sb = 0.f;
    for (int b = 0; b < B; ++b) sb += dyp[(long)b * O + o];
    db[o] += sb;
  }
}

// cross entropy (mean) over B rows of K logits; dlog = (softmax - onehot)/B (unscaled)
// nn.CrossEntropyLoss() (mean, ignore_index -100): rows whose target is -100 contribute nothing and
// the mean runs over the others; any other target outside [0, K) makes the loss and its gradient
// NaN (torch raises; no out-of-range read here either way).
__global__ void ce_kernel(const float* logits, const int64_t* tgt, int B, int K, float* loss, float* dlog) {
  __shared__ double sred[16];
  __shared__ int cnt[2];
  if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
  __syncthreads();
  int nvalid = 0, nbad = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const long long t = tgt[b];
    nvalid += (t >= 0 && t < K) ? 1 : 0;
    nbad += (t != -100 && (t < 0 || t >= K)) ? 1 : 0;
  }
  atomicAdd(&cnt[0], nvalid);  // LDS atomics
  atomicAdd(&cnt[1], nbad);
  __syncthreads();
  const float denom = (float)max(cnt[0], 1);
  const bool bad = cnt[1] > 0;
  double s = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const float* l = logits + (long)b * K;
    const long long t = tgt[b];
    const bool ok = t >= 0 && t < K;
    float mx = l[0];
    for (int k = 1; k < K; ++k) mx = fmaxf(mx, l[k]);
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(l[k] - mx);
    const float lse = mx + logf(se);
    if (ok) s += (double)(lse - l[t]);
    for (int k = 0; k < K; ++k)
      dlog[(long)b * K + k] = bad ? NAN : ok ? (expf(l[k] - lse) - (k == t ? 1.f : 0.f)) / denom : 0.f;
  }
  s = block_sum(s, sred);
  if (threadIdx.x == 0) loss[0] = bad ? NAN : cnt[0] == 0 ? NAN : (float)(s / (double)cnt[0]);
}

// multiply a per-element gradient buffer by a device scalar: out = g * (s1[0]*a1 + s2[0]*a2)
__global__ void scale_grad_kernel(const float* g, long n, const float* s1, float a1, const float* s2, float a2,
                                  float* out) {
  const float sc = (s1 ? s1[0] * a1 : 0.f) + (s2 ? s2[0] * a2 : 0.f);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] = g[i] * sc;
}

inline int grid_for(long work, int cap = 8192) {
  long b = (work + 255) / 256;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (int)b;
}

}  // namespace

// =========================================================================================
// C ABI
// =========================================================================================

UNETSEG_API size_t unetseg_lovasz_workspace(int B, long P) {
  const long T = (P + kTile - 1) / kTile;
  return (size_t)B * P * 4 * sizeof(uint32_t) + (size_t)B * 256 * T * sizeof(uint32_t) +
         (size_t)B * T * (sizeof(uint32_t) + sizeof(float)) + 256;
}

// Lovasz hinge (per-image mean).  out: planar fp32 [B][nch][P] logits (nch 2 -> z = o1-o0);
// tgt int64 [B][P] (==1 is foreground).  Writes loss[0] and gz [B][P] = dloss/dz (already /B).
static int lovasz_impl(const float* out, int nch, const int64_t* tgt, int B, long P, int has_ignore, long ignore,
                       void* ws, size_t ws_bytes, float* gz, float* loss, void* stream);

UNETSEG_API int unetseg_lovasz_fwd(const float* out, int nch, const int64_t* tgt, int B, long P, void* ws,
                                   size_t ws_bytes, float* gz, float* loss, void* stream) {
  return lovasz_impl(out, nch, tgt, B, P, 0, 0L, ws, ws_bytes, gz, loss, stream);
}

// per-image Lovasz over the pixels whose target is not ignore_index (lovasz_hinge_loss(..., ignore_index))
UNETSEG_API int unetseg_lovasz_fwd_masked(const float* out, int nch, const int64_t* tgt, int B, long P,
                                          long ignore_index, void* ws, size_t ws_bytes, float* gz, float* loss,
                                          void* stream) {
  return lovasz_impl(out, nch, tgt, B, P, 1, ignore_index, ws, ws_bytes, gz, loss, stream);
}

static int lovasz_impl(const float* out, int nch, const int64_t* tgt, int B, long P, int has_ignore, long ignore,
                       void* ws, size_t ws_bytes, float* gz, float* loss, void* stream) {
  US_CHECK_ARG(out && tgt && ws && gz && loss, "lovasz_fwd: null pointer");
  US_CHECK_ARG(nch == 1 || nch == 2, "lovasz_fwd: nch must be 1 or 2");
  US_CHECK_ARG(P < 0x80000000L, "lovasz_fwd: too many pixels per image");
  US_CHECK_ARG(ws_bytes >= unetseg_lovasz_workspace(B, P), "lovasz_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  if (B == 0 || P == 0) {
    (void)hipMemsetAsync(loss, 0, sizeof(float), st);
    return 0;
  }
  const int T = (int)((P + kTile - 1) / kTile);
  uint32_t* k0 = (uint32_t*)ws;
  uint32_t* v0 = k0 + (long)B * P;
  uint32_t* k1 = v0 + (long)B * P;
  uint32_t* v1 = k1 + (long)B * P;
  uint32_t* hist = v1 + (long)B * P;
  uint32_t* cnt = hist + (long)B * 256 * T;
  float* part = (float*)(cnt + (long)B * T);
  hipLaunchKernelGGL(lovasz_keygen_kernel, dim3(grid_for((long)B * P)), dim3(256), 0, st, out, nch, tgt, B, P, k0, v0,
                     has_ignore, ignore);
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = pass * 8;
    hipLaunchKernelGGL(radix_hist_kernel, dim3(T, B), dim3(256), 0, st, k0, P, T, shift, hist);
    hipLaunchKernelGGL(radix_scan_kernel, dim3(B), dim3(1024), 0, st, hist, T);
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(T, B), dim3(256), 0, st, k0, v0, k1, v1, P, T, shift, hist);
    uint32_t* t;
    t = k0; k0 = k1; k1 = t;
    t = v0; v0 = v1; v1 = t;
  }
  hipLaunchKernelGGL(lovasz_count_kernel, dim3(T, B), dim3(256), 0, st, v0, P, T, cnt);
  hipLaunchKernelGGL(lovasz_chunk_kernel, dim3(T, B), dim3(256), 0, st, k0, v0, P, T, cnt, 1.0f / (float)B, gz, part);
  hipLaunchKernelGGL(lovasz_final_kernel, dim3(1), dim3(64), 0, st, part, B, T, loss);
  US_LAUNCH_CHECK("lovasz_fwd");
  return 0;
}

UNETSEG_API size_t unetseg_bce_workspace(int B, long P) { return (size_t)grid_for((long)B * P) * sizeof(float) + 256; }

// BCE-with-logits mean loss; gz (may be NULL) = dloss/dz (already /count); pos_weight fp32 scalar or NULL
UNETSEG_API int unetseg_bce_fwd(const float* out, int nch, const int64_t* tgt, int B, long P, const float* pos_weight,
                                void* ws, size_t ws_bytes, float* gz, float* loss, void* stream) {
  US_CHECK_ARG(out && tgt && ws && loss, "bce_fwd: null pointer");  // gz may be NULL (no gradient)
  US_CHECK_ARG(nch == 1 || nch == 2, "bce_fwd: nch %d must be 1 or 2", nch);
  US_CHECK_ARG(B > 0 && P > 0, "bce_fwd: empty batch");
  US_CHECK_ARG(ws_bytes >= unetseg_bce_workspace(B, P), "bce_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int G = grid_for((long)B * P);
  hipLaunchKernelGGL(bce_kernel, dim3(G), dim3(256), 0, st, out, nch, tgt, B, P, pos_weight, gz, (float*)ws);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, st, (const float*)ws, G, loss);
  US_LAUNCH_CHECK("bce_fwd");
  return 0;
}

// dout = gz * (s1[0]*a1 + s2[0]*a2) scattered to the planar logits (nch 2: +/-)
UNETSEG_API int unetseg_dz_to_dout(const float* gz, int B, long P, int nch, const float* s1, float a1, const float* s2,
                                   float a2, float* scratch, float* dout, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)B * P;
  hipLaunchKernelGGL(scale_grad_kernel, dim3(grid_for(n)), dim3(256), 0, st, gz, n, s1, a1, s2, a2, scratch);
  hipLaunchKernelGGL(dz_to_dout_kernel, dim3(grid_for(n)), dim3(256), 0, st, scratch, B, P, nch, (const float*)nullptr,
                     1.f, dout);
  US_LAUNCH_CHECK("dz_to_dout");
  return 0;
}

// conf (uint64[4]) += (tp, fp, fn, tn)
UNETSEG_API int unetseg_confusion(const float* out, int nch, const int64_t* tgt, int B, long P, unsigned long long* conf,
                                  void* stream) {
  hipLaunchKernelGGL(confusion_kernel, dim3(grid_for((long)B * P, 2048)), dim3(256), 0, (hipStream_t)stream, out, nch,
                     tgt, B, P, conf, 0, 0L);
  US_LAUNCH_CHECK("confusion");
  return 0;
}

UNETSEG_API int unetseg_adam(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2,
                             float eps, float wd, int step, const float* grad_scale, void* stream) {
  US_CHECK_ARG(p && g && m && v && n >= 0, "adam: null pointer or negative size");
  US_CHECK_ARG(step >= 1, "adam: step must be >= 1");
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n, 16384)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1,
                     beta2, eps, wd, (float)bc1, (float)sqrt(bc2), grad_scale);
  US_LAUNCH_CHECK("adam");
  return 0;
}

UNETSEG_API int unetseg_adam_dev(float* p, const float* g, float* m, float* v, long n, const float* hyper, int* step,
                                 float beta1, float beta2, float eps, float wd, const float* grad_scale,
                                 void* stream) {
  US_CHECK_ARG(hyper && step, "adam_dev: hyper and step must be device pointers");
  hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_for(n, 16384)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     hyper, step, beta1, beta2, eps, wd, grad_scale);
  hipLaunchKernelGGL(adam_step_commit_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step);
  US_LAUNCH_CHECK("adam_dev");
  return 0;
}

UNETSEG_API int unetseg_gap_fwd(int dtype, const void* x, int ldx, int B, int HW, int C, float* g, void* stream) {
  US_CHECK_DTYPE(dtype, "gap_fwd");
  US_CHECK_ARG(x && g && B > 0 && HW > 0 && C > 0 && ldx >= C, "gap_fwd: bad args");
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(gap_kernel<bf16>, dim3(ceil_div(B * C, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)x,
                       ldx, B, HW, C, g);
  else
    hipLaunchKernelGGL(gap_kernel<float>, dim3(ceil_div(B * C, 256)), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       ldx, B, HW, C, g);
  US_LAUNCH_CHECK("gap_fwd");
  return 0;
}

UNETSEG_API int unetseg_gap_bwd(int dtype, const float* dg, int B, int HW, int C, void* dx, int ldx, int accumulate,
                                void* stream) {
  US_CHECK_DTYPE(dtype, "gap_bwd");
  US_CHECK_ARG(dg && dx && B > 0 && HW > 0 && C > 0 && ldx >= C, "gap_bwd: bad args");
  const long n = (long)B * HW * C;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(gap_bwd_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dg, B, HW, C,
                       (bf16*)dx, ldx, accumulate);
  else
    hipLaunchKernelGGL(gap_bwd_kernel<float>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, dg, B, HW, C,
                       (float*)dx, ldx, accumulate);
  US_LAUNCH_CHECK("gap_bwd");
  return 0;
}

UNETSEG_API int unetseg_linear_fwd(const float* x, const float* W, const float* bias, int B, int I, int O, int act,
                                   float p_drop, unsigned long long seed, const float* mask_in, float* mask_out,
                                   float* pre, float* y, void* stream) {
  US_CHECK_ARG(x && W && y && B > 0 && I > 0 && O > 0, "linear_fwd: null pointer or empty shape");
  US_CHECK_ARG(act >= 0 && act <= 2 && (act != 2 || p_drop < 1.f), "linear_fwd: act %d / p_drop %g", act, p_drop);
  const long threads = (long)B * O * 64;
  hipLaunchKernelGGL(linear_fwd_kernel, dim3(ceil_div(threads, 256)), dim3(256), 0, (hipStream_t)stream, x, W, bias, B,
                     I, O, act, p_drop, seed, mask_in, mask_out, pre, y);
  US_LAUNCH_CHECK("linear_fwd");
  return 0;
}

// dx (may be NULL) = dyp . W ; dW += dyp^T x ; db += sum dyp ; scratch: B*O floats
UNETSEG_API int unetseg_linear_bwd(const float* dy, const float* pre, const float* mask, float p_drop, int act,
                                   const float* x, const float* W, int B, int I, int O, float* dx, float* dW, float* db,
                                   float* scratch, void* stream) {
  US_CHECK_ARG(dy && x && W && dW && db && scratch && B > 0 && I > 0 && O > 0, "linear_bwd: null pointer or empty shape");
  US_CHECK_ARG(act >= 0 && act <= 2 && (act == 0 || pre) && (act != 2 || (mask && p_drop < 1.f)),
               "linear_bwd: act %d needs pre (and the dropout mask)", act);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(linear_act_bwd_kernel, dim3(ceil_div(B * O, 256)), dim3(256), 0, st, dy, pre, mask, p_drop, act, B,
                     O, scratch);
  if (dx) hipLaunchKernelGGL(linear_bwd_x_kernel, dim3(ceil_div(B * I, 256)), dim3(256), 0, st, scratch, W, B, I, O, dx);
  hipLaunchKernelGGL(linear_bwd_w_kernel, dim3(ceil_div(O * I, 256)), dim3(256), 0, st, scratch, x, B, I, O, dW, db);
  US_LAUNCH_CHECK("linear_bwd");
  return 0;
}

UNETSEG_API int unetseg_ce_fwd(const float* logits, const int64_t* tgt, int B, int K, float* loss, float* dlog,
                               void* stream) {
  US_CHECK_ARG(logits && tgt && loss && dlog && B > 0 && K > 0, "ce_fwd: null pointer or empty shape");
  hipLaunchKernelGGL(ce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, logits, tgt, B, K, loss, dlog);
  US_LAUNCH_CHECK("ce_fwd");
  return 0;
}

// out = g * (s1[0]*a1 + s2[0]*a2)
UNETSEG_API int unetseg_scale_grad(const float* g, long n, const float* s1, float a1, const float* s2, float a2,
                                   float* out, void* stream) {
  hipLaunchKernelGGL(scale_grad_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, g, n, s1, a1, s2, a2, out);
  US_LAUNCH_CHECK("scale_grad");
  return 0;
}

// confusion counts over the pixels whose target is not ignore_index
UNETSEG_API int unetseg_confusion_masked(const float* out, int nch, const int64_t* tgt, int B, long P, long ignore_index,
                                         unsigned long long* conf, void* stream) {
  US_CHECK_ARG(out && tgt && conf && (nch == 1 || nch == 2), "confusion_masked: bad args");
  hipLaunchKernelGGL(confusion_kernel, dim3(grid_for((long)B * P, 2048)), dim3(256), 0, (hipStream_t)stream, out, nch,
                     tgt, B, P, conf, 1, ignore_index);
  US_LAUNCH_CHECK("confusion_masked");
  return 0;
}

UNETSEG_API size_t unetseg_masked_loss_workspace(int B, long P) {
  return (size_t)2 * grid_for((long)B * P) * sizeof(float) + 256;
}

// binary loss over the non-ignored pixels; kind 0 BCE (pos_weight may be NULL), 1 Lovasz (flattened,
// see masked_loss_kernel).  gz [B][P] = dloss/dz (already / count); loss fp32 scalar
UNETSEG_API int unetseg_masked_loss_fwd(const float* out, int nch, const int64_t* tgt, int B, long P, long ignore_index,
                                        int kind, const float* pos_weight, void* ws, size_t ws_bytes, float* gz,
                                        float* loss, void* stream) {
  US_CHECK_ARG(out && tgt && gz && loss && ws && (kind == 0 || kind == 1), "masked_loss_fwd: bad args");
  US_CHECK_ARG(ws_bytes >= unetseg_masked_loss_workspace(B, P), "masked_loss_fwd: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int G = grid_for((long)B * P);
  float* part = (float*)ws;
  float* inv = part + 2 * G;
  hipLaunchKernelGGL(masked_loss_kernel, dim3(G), dim3(256), 0, st, out, nch, tgt, B, P, ignore_index, kind, pos_weight,
                     gz, part);
  hipLaunchKernelGGL(masked_finalize_kernel, dim3(1), dim3(256), 0, st, part, G, kind, loss, inv);
  hipLaunchKernelGGL(scale_by_kernel, dim3(G), dim3(256), 0, st, gz, (long)B * P, inv);
  US_LAUNCH_CHECK("masked_loss_fwd");
  return 0;
}
