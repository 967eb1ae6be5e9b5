// Device data augmentation of the training / validation loader.
//
// Reference (CPU, per sample): utils/hf_dataloader.py:67-105 (__getitem__), 111-180
// (get_random_data), 183-213 (hf_unet_dataset_collate):
//   image.resize((nw, nh), BICUBIC); label.resize((nw, nh), NEAREST); optional FLIP_LEFT_RIGHT;
//   paste at (dx, dy) on a (128,128,128) / 0 canvas of the input size; in training mode an HSV
//   jitter (cv2 RGB2HSV -> three uint8 LUTs -> HSV2RGB); image / 255 (float64 -> float32 NCHW);
//   label: binary (> 0) for the binary task, values >= num_classes -> num_classes, int64, one-hot.
// Here the host decodes the files, draws the random parameters in the reference's order and builds
// per-sample tables (utils/augment_tables.py); three kernels do the pixel work for a whole batch:
//   aug_hpass   : PIL's horizontal BICUBIC pass (22-bit fixed-point taps, uint8 x int32, clip8)
//                 over the source rows the vertical pass needs -> tmp (uint8 [rows][nw][3])
//   aug_vpass   : PIL's vertical pass -> rsz (uint8 [nh][nw][3])
//   aug_compose : flip + paste + HSV jitter + /255 + NEAREST label + binary/clamp + one-hot,
//                 one thread per output pixel, writing the collated fp32 / int64 tensors directly.
// The resize is bit-exact with Pillow (same integer arithmetic); the HSV jitter follows OpenCV's
// 8-bit RGB2HSV_b (integer) / HSV2RGB_b (fp32, no contraction, round-half-even) algorithm.
#include "common.h"

namespace {

// per-sample descriptor: int64 [AUG_DESC] (layout shared with utils/hf_dataloader.py)
enum {
  D_SRC = 0, D_MSK, D_TMP, D_RSZ, D_IW, D_IH, D_NW, D_NH, D_DX, D_DY, D_FLIP, D_Y0, D_ROWS, D_KSH, D_KSV,
  D_TAB, D_HSV, D_MIW, D_MIH, AUG_DESC = 20
};

struct Tabs {  // int32 tables of one sample, consecutive from desc[D_TAB]
  const int *bh, *kh, *bv, *kv, *nx, *ny, *lut;
};

__host__ __device__ inline long long tab_len(long long nw, long long nh, long long ksh, long long ksv, long long hsv) {
  return nw * 2 + nw * ksh + nh * 2 + nh * ksv + nw + nh + (hsv ? 768 : 0);
}

__device__ inline Tabs tabs_of(const int* tables, const long long* d) {
  const long long nw = d[D_NW], nh = d[D_NH];
  Tabs t;
  t.bh = tables + d[D_TAB];
  t.kh = t.bh + nw * 2;
  t.bv = t.kh + nw * d[D_KSH];
  t.kv = t.bv + nh * 2;
  t.nx = t.kv + nh * d[D_KSV];
  t.ny = t.nx + nw;
  t.lut = t.ny + nh;
  return t;
}

constexpr int kPrecision = 22;  // Resample.c PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int clip8(int v) {
  v >>= kPrecision;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

__global__ __launch_bounds__(256) void aug_hpass(const long long* desc, const int* tables, const uint8_t* src, uint8_t* tmp) {
  const long long* d = desc + (long)blockIdx.y * AUG_DESC;
  const int nw = (int)d[D_NW], iw = (int)d[D_IW], rows = (int)d[D_ROWS], y0 = (int)d[D_Y0], ksh = (int)d[D_KSH];
  const Tabs t = tabs_of(tables, d);
  const uint8_t* s = src + d[D_SRC];
  uint8_t* o = tmp + d[D_TMP];
  const long total = (long)rows * nw;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int xx = (int)(i % nw), r = (int)(i / nw);
    const int xmin = t.bh[2 * xx], n = t.bh[2 * xx + 1];
    const int* k = t.kh + (long)xx * ksh;
    const uint8_t* row = s + ((long)(y0 + r) * iw + xmin) * 3;
    int a0 = 1 << (kPrecision - 1), a1 = a0, a2 = a0;
    for (int x = 0; x < n; ++x) {
      const int w = k[x];
      a0 += (int)row[3 * x] * w;
      a1 += (int)row[3 * x + 1] * w;
      a2 += (int)row[3 * x + 2] * w;
    }
    uint8_t* q = o + i * 3;
    q[0] = (uint8_t)clip8(a0);
    q[1] = (uint8_t)clip8(a1);
    q[2] = (uint8_t)clip8(a2);
  }
}

__global__ __launch_bounds__(256) void aug_vpass(const long long* desc, const int* tables, const uint8_t* tmp, uint8_t* rsz) {
  const long long* d = desc + (long)blockIdx.y * AUG_DESC;
  const int nw = (int)d[D_NW], nh = (int)d[D_NH], ksv = (int)d[D_KSV];
  const Tabs t = tabs_of(tables, d);
  const uint8_t* s = tmp + d[D_TMP];
  uint8_t* o = rsz + d[D_RSZ];
  const long total = (long)nh * nw * 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % 3);
    const long pix = i / 3;
    const int xx = (int)(pix % nw), yy = (int)(pix / nw);
    const int ymin = t.bv[2 * yy], n = t.bv[2 * yy + 1];
    const int* k = t.kv + (long)yy * ksv;
    const uint8_t* col = s + ((long)ymin * nw + xx) * 3 + c;
    int a = 1 << (kPrecision - 1);
    for (int y = 0; y < n; ++y) a += (int)col[(long)y * nw * 3] * k[y];
    o[i] = (uint8_t)clip8(a);
  }
}

// OpenCV RGB2HSV_b (hrange 180, hsv_shift 12): integer; the division tables are round(a / i) with
// no ties, i.e. (2a + i) / (2i) in integers
__device__ inline void rgb2hsv(int r, int g, int b, int& h, int& s, int& v) {
  v = max(max(b, g), r);
  const int vmin = min(min(b, g), r);
  const int diff = v - vmin;
  const int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
  const int sdiv = v ? (2 * (255 << 12) + v) / (2 * v) : 0;
  const int hdiv = diff ? (2 * 122880 + diff) / (2 * diff) : 0;  // (180 << 12) / (6 diff)
  s = (diff * sdiv + (1 << 11)) >> 12;
  h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
  h = (h * hdiv + (1 << 11)) >> 12;
  h += h < 0 ? 180 : 0;
  h = h < 0 ? 0 : (h > 255 ? 255 : h);
}

__device__ inline int sat_u8(float x) {
  const float r = __builtin_rintf(x);
  return r < 0.f ? 0 : (r > 255.f ? 255 : (int)r);
}

// OpenCV HSV2RGB_b: fp32 sector arithmetic (separate roundings: contraction off), then
// saturate_cast<uchar>(x * 255)
__device__ inline void hsv2rgb(int hi, int si, int vi, int& r, int& g, int& b) {
#pragma clang fp contract(off)
  const float h0 = (float)hi, s = (float)si * (1.f / 255.f), v = (float)vi * (1.f / 255.f);
  float bf, gf, rf;
  if (s == 0.f) {
    bf = gf = rf = v;
  } else {
    float h = h0 * (6.f / 180.f);
    h = fmodf(h, 6.f);
    int sector = (int)floorf(h);
    h -= (float)sector;
    if ((unsigned)sector >= 6u) {
      sector = 0;
      h = 0.f;
    }
    float tab[4];
    tab[0] = v;
    tab[1] = v * (1.f - s);
    tab[2] = v * (1.f - s * h);
    tab[3] = v * (1.f - s * (1.f - h));
    const int sd[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
    bf = tab[sd[sector][0]];
    gf = tab[sd[sector][1]];
    rf = tab[sd[sector][2]];
  }
  r = sat_u8(rf * 255.f);
  g = sat_u8(gf * 255.f);
  b = sat_u8(bf * 255.f);
}

__global__ __launch_bounds__(256) void aug_compose(const long long* desc, const int* tables, const uint8_t* rsz,
                                                   const uint8_t* msk, int H, int W, int num_classes, int binary,
                                                   float* img, long long* png, float* onehot) {
  const int n = blockIdx.y;
  const long long* d = desc + (long)n * AUG_DESC;
  const int nw = (int)d[D_NW], nh = (int)d[D_NH], dx = (int)d[D_DX], dy = (int)d[D_DY], flip = (int)d[D_FLIP];
  const int hsv = (int)d[D_HSV], miw = (int)d[D_MIW];
  const Tabs t = tabs_of(tables, d);
  const uint8_t* im = rsz + d[D_RSZ];
  const uint8_t* mk = msk + d[D_MSK];
  const long plane = (long)H * W;
  const int C1 = num_classes + 1;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < plane; p += (long)gridDim.x * blockDim.x) {
    const int x = (int)(p % W), y = (int)(p / W);
    const int sx = x - dx, sy = y - dy;
    int r = 128, g = 128, b = 128, lab = 0;
    if (sx >= 0 && sx < nw && sy >= 0 && sy < nh) {
      const int fx = flip ? nw - 1 - sx : sx;
      const uint8_t* q = im + ((long)sy * nw + fx) * 3;
      r = q[0];
      g = q[1];
      b = q[2];
      lab = mk[(long)t.ny[sy] * miw + t.nx[fx]];
    }
    if (hsv) {
      int h, s, v;
      rgb2hsv(r, g, b, h, s, v);
      hsv2rgb(t.lut[h], t.lut[256 + s], t.lut[512 + v], r, g, b);
    }
    float* o = img + (long)n * 3 * plane + p;
    o[0] = (float)((double)r / 255.0);
    o[plane] = (float)((double)g / 255.0);
    o[2 * plane] = (float)((double)b / 255.0);
    if (binary) lab = lab > 0 ? 1 : 0;
    if (lab >= num_classes) lab = num_classes;
    png[(long)n * plane + p] = lab;
    if (onehot) {
      float* oh = onehot + ((long)n * plane + p) * C1;
      for (int c = 0; c < C1; ++c) oh[c] = c == lab ? 1.f : 0.f;
    }
  }
}

int grid_for(long work) {
  long g = (work + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

// ---- the per-sample tables built on the device (utils/augment_tables.py restated in float64) ----
// Every float64 operation is the one numpy performs, in the same order, with contraction off, so the
// int32 tables are bit-identical to the host builder's (which is pinned against Pillow).
__device__ double bicubic_filter(double x) {
#pragma clang fp contract(off)
  const double a = -0.5;
  x = fabs(x);
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Resample.c precompute_coeffs + normalize_coeffs_8bpc for output coordinate i: bounds (xmin, n) and
// ksize fixed-point taps (bicubic_coeffs); `shift` is subtracted from xmin and the window clamped to
// [0, limit) (the vertical pass reads rows y0 .. y0 + rows of the horizontal pass)
__device__ void bicubic_row(int in_size, int out_size, int ksize, int i, int shift, int limit, int* bounds, int* k) {
#pragma clang fp contract(off)
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double ss = 1.0 / filterscale;
  const double center = ((double)i + 0.5) * scale;
  const double lo = center - support + 0.5;
  const long long xmin = lo < 0 ? 0 : (long long)trunc(lo);
  long long hi = (long long)trunc(center + support + 0.5);
  hi = hi < in_size ? hi : in_size;
  const long long xmax = hi - xmin;
  // two passes over the taps (the filter re-evaluated, same values): the normalising sum first, in
  // the C loop's order, then the fixed-point taps -- no per-thread array
  double ww = 0.0;
  for (int x = 0; x < ksize; ++x) ww += x < xmax ? bicubic_filter(((double)((long long)x + xmin) - center + 0.5) * ss) : 0.0;
  for (int x = 0; x < ksize; ++x) {
    const double w = x < xmax ? bicubic_filter(((double)((long long)x + xmin) - center + 0.5) * ss) : 0.0;
    const double kx = ww != 0.0 ? w / ww : w;
    const double scaled = kx * (double)(1 << kPrecision);
    k[x] = (int)trunc(kx < 0 ? -0.5 + scaled : 0.5 + scaled);
  }
  long long b0 = xmin - shift, n = xmax;
  if (b0 < 0) {
    n += b0;
    b0 = 0;
  }
  if (b0 + n > limit) n = limit - b0;
  bounds[0] = (int)b0;
  bounds[1] = (int)(n < 0 ? 0 : n);
}

// Geometry.c ImagingScaleAffine's accumulated source coordinate (nearest_index): one sequential loop
__device__ void nearest_rows(int in_size, int out_size, int* idx) {
#pragma clang fp contract(off)
  const double a = (double)in_size / (double)out_size;
  double xo = a * 0.5;
  for (int i = 0; i < out_size; ++i) {
    if (i) xo += a;
    long long v = (long long)trunc(xo);
    idx[i] = (int)(v < in_size - 1 ? v : in_size - 1);
  }
}

// one block per (sample, part): tasks [0, nw) horizontal taps, [nw, nw + nh) vertical taps, then the
// two nearest-index scans and the 768 LUT entries (hsv_luts)
__global__ __launch_bounds__(256) void aug_tables(const long long* desc, const double* hsv_r, int* tables) {
#pragma clang fp contract(off)
  const int n = blockIdx.y;
  const long long* d = desc + (long)n * AUG_DESC;
  const int iw = (int)d[D_IW], ih = (int)d[D_IH], nw = (int)d[D_NW], nh = (int)d[D_NH];
  const int ksh = (int)d[D_KSH], ksv = (int)d[D_KSV], y0 = (int)d[D_Y0], rows = (int)d[D_ROWS];
  const int hsv = (int)d[D_HSV];
  int* bh = tables + d[D_TAB];
  int* kh = bh + (long)nw * 2;
  int* bv = kh + (long)nw * ksh;
  int* kv = bv + (long)nh * 2;
  int* nx = kv + (long)nh * ksv;
  int* ny = nx + nw;
  int* lut = ny + nh;
  const long tasks = (long)nw + nh + 2 + (hsv ? 768 : 0);
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < tasks; t += (long)gridDim.x * blockDim.x) {
    if (t < nw) {
      bicubic_row(iw, nw, ksh, (int)t, 0, iw, bh + 2 * t, kh + t * ksh);
    } else if (t < (long)nw + nh) {
      const int y = (int)(t - nw);
      bicubic_row(ih, nh, ksv, y, y0, rows, bv + 2 * y, kv + (long)y * ksv);
    } else if (t == (long)nw + nh) {
      nearest_rows((int)d[D_MIW], nw, nx);
    } else if (t == (long)nw + nh + 1) {
      nearest_rows((int)d[D_MIH], nh, ny);
    } else {
      const int e = (int)(t - nw - nh - 2), c = e >> 8, x = e & 255;
      const double r = hsv_r[n * 3 + c];
      const double v = (double)x * r;
      int o;
      if (c == 0) {
        o = (int)fmod(v, 180.0);  // (x * r0) % 180, x * r0 >= 0
      } else {
        const double cv = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
        o = (int)cv;
      }
      lut[e] = o & 255;
    }
  }
}

// ksize of a BICUBIC axis (bicubic_coeffs), and the first / one-past-last source row the vertical
// pass reads (resize_plan's ybox), recomputed on the host to validate a descriptor
long long bicubic_ksize(long long in_size, long long out_size) {
  double fs = (double)in_size / (double)out_size;
  if (fs < 1.0) fs = 1.0;
  return (long long)ceil(2.0 * fs) * 2 + 1;
}

}  // namespace

UNETSEG_API int unetseg_augment_tables_len(long long nw, long long nh, long long ksh, long long ksv, long long hsv) {
  return (int)tab_len(nw, nh, ksh, ksv, hsv);
}

UNETSEG_API int unetseg_augment_batch(const long long* desc_host, const long long* desc, int B, const int* tables_host,
                                      const int* tables, long long n_tables, const uint8_t* src, long long src_bytes,
                                      const uint8_t* msk, long long msk_bytes, uint8_t* tmp, long long tmp_bytes,
                                      uint8_t* rsz, long long rsz_bytes, int H, int W, int num_classes, int binary,
                                      float* img, long long* png, float* onehot, hipStream_t stream) {
  US_CHECK_ARG(B > 0 && H > 0 && W > 0 && num_classes > 0, "augment_batch: bad sizes B=%d H=%d W=%d nc=%d", B, H, W,
               num_classes);
  US_CHECK_ARG(desc_host && desc && tables_host && tables && src && msk && tmp && rsz && img && png,
               "augment_batch: null pointer");
  long max_h = 1, max_v = 1;
  for (int i = 0; i < B; ++i) {
    const long long* d = desc_host + (long)i * AUG_DESC;
    const long long iw = d[D_IW], ih = d[D_IH], nw = d[D_NW], nh = d[D_NH], miw = d[D_MIW], mih = d[D_MIH];
    US_CHECK_ARG(iw > 0 && ih > 0 && nw > 0 && nh > 0 && miw > 0 && mih > 0 && d[D_KSH] > 0 && d[D_KSV] > 0,
                 "augment_batch: sample %d has an empty image or tables", i);
    US_CHECK_ARG(d[D_Y0] >= 0 && d[D_ROWS] > 0 && d[D_Y0] + d[D_ROWS] <= ih, "augment_batch: sample %d row window", i);
    US_CHECK_ARG(d[D_SRC] >= 0 && d[D_SRC] + iw * ih * 3 <= src_bytes, "augment_batch: sample %d image range", i);
    US_CHECK_ARG(d[D_MSK] >= 0 && d[D_MSK] + miw * mih <= msk_bytes, "augment_batch: sample %d mask range", i);
    US_CHECK_ARG(d[D_TMP] >= 0 && d[D_TMP] + d[D_ROWS] * nw * 3 <= tmp_bytes, "augment_batch: sample %d tmp range", i);
    US_CHECK_ARG(d[D_RSZ] >= 0 && d[D_RSZ] + nh * nw * 3 <= rsz_bytes, "augment_batch: sample %d rsz range", i);
    const long long len = tab_len(nw, nh, d[D_KSH], d[D_KSV], d[D_HSV]);
    US_CHECK_ARG(d[D_TAB] >= 0 && d[D_TAB] + len <= n_tables, "augment_batch: sample %d table range", i);
    // every index the kernels follow stays inside its image
    const int* bh = tables_host + d[D_TAB];
    const int* bv = bh + nw * 2 + nw * d[D_KSH];
    const int* nx = bv + nh * 2 + nh * d[D_KSV];
    const int* ny = nx + nw;
    for (long long x = 0; x < nw; ++x)
      US_CHECK_ARG(bh[2 * x] >= 0 && bh[2 * x + 1] >= 0 && bh[2 * x + 1] <= d[D_KSH] && bh[2 * x] + bh[2 * x + 1] <= iw &&
                       nx[x] >= 0 && nx[x] < miw,
                   "augment_batch: sample %d horizontal table %lld out of range", i, x);
    for (long long y = 0; y < nh; ++y)
      US_CHECK_ARG(bv[2 * y] >= 0 && bv[2 * y + 1] >= 0 && bv[2 * y + 1] <= d[D_KSV] &&
                       bv[2 * y] + bv[2 * y + 1] <= d[D_ROWS] && ny[y] >= 0 && ny[y] < mih,
                   "augment_batch: sample %d vertical table %lld out of range", i, y);
    max_h = max_h > d[D_ROWS] * nw ? max_h : (long)(d[D_ROWS] * nw);
    max_v = max_v > nh * nw * 3 ? max_v : (long)(nh * nw * 3);
  }
  aug_hpass<<<dim3(grid_for(max_h), B), 256, 0, stream>>>(desc, tables, src, tmp);
  US_LAUNCH_CHECK("aug_hpass");
  aug_vpass<<<dim3(grid_for(max_v), B), 256, 0, stream>>>(desc, tables, tmp, rsz);
  US_LAUNCH_CHECK("aug_vpass");
  aug_compose<<<dim3(grid_for((long)H * W), B), 256, 0, stream>>>(desc, tables, rsz, msk, H, W, num_classes, binary,
                                                                  img, png, onehot);
  US_LAUNCH_CHECK("aug_compose");
  return 0;
}

// The same batch with the per-sample tables built on the device (aug_tables) from the descriptors and
// the HSV factors hsv_r (float64 [B][3], device): the host only decodes, draws and packs the pixels.
// tables: device scratch of n_tables int32 laid out as desc[D_TAB] / unetseg_augment_tables_len say.
UNETSEG_API int unetseg_augment_batch_dev(const long long* desc_host, const long long* desc, int B, const double* hsv_r,
                                          int* tables, long long n_tables, const uint8_t* src, long long src_bytes,
                                          const uint8_t* msk, long long msk_bytes, uint8_t* tmp, long long tmp_bytes,
                                          uint8_t* rsz, long long rsz_bytes, int H, int W, int num_classes, int binary,
                                          float* img, long long* png, float* onehot, hipStream_t stream) {
  US_CHECK_ARG(B > 0 && H > 0 && W > 0 && num_classes > 0, "augment_batch_dev: bad sizes B=%d H=%d W=%d nc=%d", B, H,
               W, num_classes);
  US_CHECK_ARG(desc_host && desc && hsv_r && tables && src && msk && tmp && rsz && img && png,
               "augment_batch_dev: null pointer");
  long max_h = 1, max_v = 1, max_t = 1;
  for (int i = 0; i < B; ++i) {
    const long long* d = desc_host + (long)i * AUG_DESC;
    const long long iw = d[D_IW], ih = d[D_IH], nw = d[D_NW], nh = d[D_NH], miw = d[D_MIW], mih = d[D_MIH];
    US_CHECK_ARG(iw > 0 && ih > 0 && nw > 0 && nh > 0 && miw > 0 && mih > 0, "augment_batch_dev: sample %d is empty", i);
    US_CHECK_ARG(d[D_KSH] == bicubic_ksize(iw, nw) && d[D_KSV] == bicubic_ksize(ih, nh),
                 "augment_batch_dev: sample %d kernel sizes %lld / %lld", i, d[D_KSH], d[D_KSV]);
    US_CHECK_ARG(d[D_Y0] >= 0 && d[D_ROWS] > 0 && d[D_Y0] + d[D_ROWS] <= ih, "augment_batch_dev: sample %d row window",
                 i);
    US_CHECK_ARG(d[D_SRC] >= 0 && d[D_SRC] + iw * ih * 3 <= src_bytes, "augment_batch_dev: sample %d image range", i);
    US_CHECK_ARG(d[D_MSK] >= 0 && d[D_MSK] + miw * mih <= msk_bytes, "augment_batch_dev: sample %d mask range", i);
    US_CHECK_ARG(d[D_TMP] >= 0 && d[D_TMP] + d[D_ROWS] * nw * 3 <= tmp_bytes, "augment_batch_dev: sample %d tmp range",
                 i);
    US_CHECK_ARG(d[D_RSZ] >= 0 && d[D_RSZ] + nh * nw * 3 <= rsz_bytes, "augment_batch_dev: sample %d rsz range", i);
    const long long len = tab_len(nw, nh, d[D_KSH], d[D_KSV], d[D_HSV]);
    US_CHECK_ARG(d[D_TAB] >= 0 && d[D_TAB] + len <= n_tables, "augment_batch_dev: sample %d table range", i);
    max_h = max_h > d[D_ROWS] * nw ? max_h : (long)(d[D_ROWS] * nw);
    max_v = max_v > nh * nw * 3 ? max_v : (long)(nh * nw * 3);
    const long tasks = (long)(nw + nh + 2 + (d[D_HSV] ? 768 : 0));
    max_t = max_t > tasks ? max_t : tasks;
  }
  // the kernels' indices are in range by construction: every window is clamped to its image (the
  // vertical one to the row window), the nearest indices to [0, size)
  aug_tables<<<dim3(grid_for(max_t), B), 256, 0, stream>>>(desc, hsv_r, tables);
  US_LAUNCH_CHECK("aug_tables");
  aug_hpass<<<dim3(grid_for(max_h), B), 256, 0, stream>>>(desc, tables, src, tmp);
  US_LAUNCH_CHECK("aug_hpass");
  aug_vpass<<<dim3(grid_for(max_v), B), 256, 0, stream>>>(desc, tables, tmp, rsz);
  US_LAUNCH_CHECK("aug_vpass");
  aug_compose<<<dim3(grid_for((long)H * W), B), 256, 0, stream>>>(desc, tables, rsz, msk, H, W, num_classes, binary,
                                                                  img, png, onehot);
  US_LAUNCH_CHECK("aug_compose");
  return 0;
}

// the device-built tables alone (tests: compared with utils/augment_tables.py bit for bit)
UNETSEG_API int unetseg_augment_tables_dev(const long long* desc, int B, const double* hsv_r, int* tables, int max_tasks,
                                           hipStream_t stream) {
  US_CHECK_ARG(B > 0 && desc && hsv_r && tables && max_tasks > 0, "augment_tables_dev: bad args");
  aug_tables<<<dim3(grid_for(max_tasks), B), 256, 0, stream>>>(desc, hsv_r, tables);
  US_LAUNCH_CHECK("aug_tables");
  return 0;
}
