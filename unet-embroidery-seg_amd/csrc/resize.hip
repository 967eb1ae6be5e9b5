// General bilinear resize and zero padding (NHWC, bf16 / fp32), forward and backward.
//
// Reference ops replaced (inputs whose size does not halve / double exactly):
//   F.interpolate(size=..., bilinear, align_corners=False)  model/unet_attention.py:31-33,52-53,
//                                                           model/unet_dualdense.py:57-58
//   F.interpolate(..., align_corners=True) of CE/Focal/Dice  model/unet_training.py:14-15,36-37,71-72
//   F.pad (pad-then-cat)                                    model/unet_plain.py:42-45
// Source coordinates follow ATen's upsample_bilinear2d exactly (area_pixel_compute_source_index):
//   align_corners: src = dst * (in-1)/(out-1)  (0 when out == 1)
//   otherwise:     src = max(0, (dst + 0.5) * in/out - 0.5)
//   i0 = (int)src, i1 = i0 + (i0 < in-1), l1 = src - i0, l0 = 1 - l1   (fp32)
// The backward is a deterministic GATHER: every input pixel sums, in a fixed order, the output
// pixels whose source row/column pair names it, with the forward's own weights recomputed.
#include "common.h"

namespace {

struct Axis {
  int in, out;
  bool align;
  float scale;
  __device__ __forceinline__ void src(int d, int& i0, int& i1, float& l1) const {
    float s = align ? (float)d * scale : fmaxf(((float)d + 0.5f) * scale - 0.5f, 0.f);
    i0 = (int)s;
    if (i0 > in - 1) i0 = in - 1;
    i1 = i0 + (i0 < in - 1 ? 1 : 0);
    l1 = s - (float)i0;
  }
  // output indices that may name input index i (a superset; the caller checks i0/i1 exactly)
  __device__ __forceinline__ void range(int i, int& lo, int& hi) const {
    if (scale <= 0.f) {  // out == 1 with align_corners: the single output reads index 0
      lo = 0;
      hi = out - 1;
      return;
    }
    // i0(d) in {i-1, i} <=> i-1 <= src(d) < i+1
    float a = align ? (float)(i - 1) / scale : ((float)(i - 1) + 0.5f) / scale - 0.5f;
    float b = align ? (float)(i + 1) / scale : ((float)(i + 1) + 0.5f) / scale - 0.5f;
    lo = (int)floorf(a) - 1;
    hi = (int)ceilf(b) + 1;
    if (lo < 0) lo = 0;
    if (hi > out - 1) hi = out - 1;
  }
};

__host__ __device__ inline float axis_scale(int in, int out, bool align) {
  if (align) return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  return (float)in / (float)out;
}

template <typename T>
__global__ __launch_bounds__(256) void resize_fwd_kernel(const T* x, int ldx, int N, int C, Axis ay, Axis ax, T* y,
                                                         int ldy) {
  const long total = (long)N * ay.out * ax.out * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int ox = (int)(pix % ax.out);
    const long r = pix / ax.out;
    const int oy = (int)(r % ay.out);
    const int n = (int)(r / ay.out);
    int y0, y1, x0, x1;
    float ly, lx;
    ay.src(oy, y0, y1, ly);
    ax.src(ox, x0, x1, lx);
    const long b = (long)n * ay.in;
    auto at = [&](int yy, int xx) { return (float)x[((b + yy) * ax.in + xx) * (long)ldx + c]; };
    const float v = (1.f - ly) * ((1.f - lx) * at(y0, x0) + lx * at(y0, x1)) + ly * ((1.f - lx) * at(y1, x0) + lx * at(y1, x1));
    y[pix * (long)ldy + c] = (T)v;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void resize_bwd_kernel(const T* dy, int ldy, int N, int C, Axis ay, Axis ax, T* dx,
                                                         int ldx, int accumulate) {
  const long total = (long)N * ay.in * ax.in * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int ix = (int)(pix % ax.in);
    const long r = pix / ax.in;
    const int iy = (int)(r % ay.in);
    const int n = (int)(r / ay.in);
    int ylo, yhi, xlo, xhi;
    ay.range(iy, ylo, yhi);
    ax.range(ix, xlo, xhi);
    float acc = 0.f;
    for (int oy = ylo; oy <= yhi; ++oy) {
      int y0, y1;
      float ly;
      ay.src(oy, y0, y1, ly);
      // forward weight of input row iy in output row oy (both taps may name it at the border)
      if (y0 != iy && y1 != iy) continue;
      const float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      for (int ox = xlo; ox <= xhi; ++ox) {
        int x0, x1;
        float lx;
        ax.src(ox, x0, x1, lx);
        if (x0 != ix && x1 != ix) continue;
        const float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        acc += wy * wx * (float)dy[(((long)n * ay.out + oy) * ax.out + ox) * ldy + c];
      }
    }
    T* o = dx + pix * (long)ldx + c;
    *o = (T)(accumulate ? acc + (float)*o : acc);
  }
}

// y[n][oy][ox] = x[n][oy - top][ox - left] inside, 0 outside (F.pad with zeros, top/left >= 0)
template <typename T>
__global__ __launch_bounds__(256) void pad_fwd_kernel(const T* x, int ldx, int N, int H, int W, int C, int top, int left,
                                                      int OH, int OW, T* y, int ldy) {
  const long total = (long)N * OH * OW * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int ox = (int)(pix % OW);
    const long r = pix / OW;
    const int oy = (int)(r % OH);
    const int n = (int)(r / OH);
    const int iy = oy - top, ix = ox - left;
    float v = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = (float)x[(((long)n * H + iy) * W + ix) * ldx + c];
    y[pix * (long)ldy + c] = (T)v;
  }
}

// dx (+)= dy[top:top+H, left:left+W]
template <typename T>
__global__ __launch_bounds__(256) void pad_bwd_kernel(const T* dy, int ldy, int N, int H, int W, int C, int top,
                                                      int left, int OH, int OW, T* dx, int ldx, int accumulate) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int ix = (int)(pix % W);
    const long r = pix / W;
    const int iy = (int)(r % H);
    const int n = (int)(r / H);
    const float g = (float)dy[(((long)n * OH + iy + top) * OW + ix + left) * ldy + c];
    T* o = dx + pix * (long)ldx + c;
    *o = (T)(accumulate ? g + (float)*o : g);
  }
}

// Per-row-tile BatchNorm partials of an NHWC view: part[g][0][c] = sum over rows g*tile.. of x,
// part[g][1][c] = M2 about that tile's mean (the layout the conv epilogues write, merged by
// unetseg_bn_finalize).  For inputs no conv produced (the dense blocks' concatenations).
template <typename T>
__global__ __launch_bounds__(256) void channel_stats_kernel(const T* x, int ldx, long M, int C, int tile, float* part) {
  const int c = blockIdx.y * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long r0 = (long)blockIdx.x * tile, r1 = min(M, r0 + tile);
  float s = 0.f;
  for (long r = r0; r < r1; ++r) s += (float)x[r * ldx + c];
  const float mean = s / (float)(r1 - r0);
  float q = 0.f;
  for (long r = r0; r < r1; ++r) {
    const float d = (float)x[r * ldx + c] - mean;
    q += d * d;
  }
  part[(long)blockIdx.x * 2 * C + c] = s;
  part[(long)blockIdx.x * 2 * C + C + c] = q;
}

inline int grid_n(long n) {
  long g = (n + 255) / 256;
  if (g > 65535 * 8) g = 65535 * 8;
  return (int)(g < 1 ? 1 : g);
}

Axis make_axis(int in, int out, int align) {
  Axis a;
  a.in = in;
  a.out = out;
  a.align = align != 0;
  a.scale = axis_scale(in, out, a.align);
  return a;
}

}  // namespace

#define RS_DISPATCH_T(dtype, ...) \
  do {                            \
    if ((dtype) == DT_BF16) {     \
      typedef bf16 T;             \
      __VA_ARGS__;                \
    } else {                      \
      typedef float T;            \
      __VA_ARGS__;                \
    }                             \
  } while (0)

UNETSEG_API int unetseg_resize_bilinear_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int oh,
                                            int ow, int align_corners, void* y, int ldy, void* stream) {
  US_CHECK_ARG(x && y && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0 && ldx >= c && ldy >= c,
               "resize_bilinear_fwd: bad args");
  const Axis ay = make_axis(h, oh, align_corners), ax = make_axis(w, ow, align_corners);
  RS_DISPATCH_T(dtype, hipLaunchKernelGGL(resize_fwd_kernel<T>, dim3(grid_n((long)n * oh * ow * c)), dim3(256), 0,
                                          (hipStream_t)stream, (const T*)x, ldx, n, c, ay, ax, (T*)y, ldy));
  US_LAUNCH_CHECK("resize_bilinear_fwd");
  return 0;
}

UNETSEG_API int unetseg_resize_bilinear_bwd(int dtype, const void* dy, int ldy, int n, int h, int w, int c, int oh,
                                            int ow, int align_corners, void* dx, int ldx, int accumulate,
                                            void* stream) {
  US_CHECK_ARG(dy && dx && n > 0 && h > 0 && w > 0 && c > 0 && oh > 0 && ow > 0, "resize_bilinear_bwd: bad args");
  const Axis ay = make_axis(h, oh, align_corners), ax = make_axis(w, ow, align_corners);
  RS_DISPATCH_T(dtype, hipLaunchKernelGGL(resize_bwd_kernel<T>, dim3(grid_n((long)n * h * w * c)), dim3(256), 0,
                                          (hipStream_t)stream, (const T*)dy, ldy, n, c, ay, ax, (T*)dx, ldx,
                                          accumulate));
  US_LAUNCH_CHECK("resize_bilinear_bwd");
  return 0;
}

UNETSEG_API int unetseg_pad2d_fwd(int dtype, const void* x, int ldx, int n, int h, int w, int c, int top, int left,
                                  int oh, int ow, void* y, int ldy, void* stream) {
  US_CHECK_ARG(x && y && top >= 0 && left >= 0 && top + h <= oh && left + w <= ow, "pad2d_fwd: bad args");
  RS_DISPATCH_T(dtype, hipLaunchKernelGGL(pad_fwd_kernel<T>, dim3(grid_n((long)n * oh * ow * c)), dim3(256), 0,
                                          (hipStream_t)stream, (const T*)x, ldx, n, h, w, c, top, left, oh, ow, (T*)y,
                                          ldy));
  US_LAUNCH_CHECK("pad2d_fwd");
  return 0;
}

UNETSEG_API int unetseg_pad2d_bwd(int dtype, const void* dy, int ldy, int n, int h, int w, int c, int top, int left,
                                  int oh, int ow, void* dx, int ldx, int accumulate, void* stream) {
  US_CHECK_ARG(dy && dx && top >= 0 && left >= 0 && top + h <= oh && left + w <= ow, "pad2d_bwd: bad args");
  RS_DISPATCH_T(dtype, hipLaunchKernelGGL(pad_bwd_kernel<T>, dim3(grid_n((long)n * h * w * c)), dim3(256), 0,
                                          (hipStream_t)stream, (const T*)dy, ldy, n, h, w, c, top, left, oh, ow,
                                          (T*)dx, ldx, accumulate));
  US_LAUNCH_CHECK("pad2d_bwd");
  return 0;
}

UNETSEG_API int unetseg_channel_stats_tiles(long M, int tile) { return ceil_div(M, tile); }

// part fp32 [ceil(M/tile)][2][C]: (sum, M2 about the tile mean) per row tile of x (NHWC view, ld)
UNETSEG_API int unetseg_channel_stats(int dtype, const void* x, int ldx, long M, int c, int tile, float* part,
                                      void* stream) {
  US_CHECK_ARG(x && part && M > 0 && c > 0 && tile > 0 && ldx >= c, "channel_stats: bad args");
  const dim3 grid(ceil_div(M, tile), ceil_div(c, 256));
  RS_DISPATCH_T(dtype, hipLaunchKernelGGL(channel_stats_kernel<T>, grid, dim3(256), 0, (hipStream_t)stream,
                                          (const T*)x, ldx, M, c, tile, part));
  US_LAUNCH_CHECK("channel_stats");
  return 0;
}
