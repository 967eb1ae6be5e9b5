// Shared definitions for the unetseg HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#define UNETSEG_API extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

enum { DT_F32 = 0, DT_BF16 = 1 };

// ---- error handling: thread-local message, int status ------------------------------------
void unetseg_set_error(const char* fmt, ...);

#define US_CHECK_ARG(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      unetseg_set_error(__VA_ARGS__);      \
      return 1;                            \
    }                                      \
  } while (0)

// shared argument checks of the C ABI's launching entry points (exercised by tests/asan/cabi_asan.cpp)
#define US_CHECK_DTYPE(dt, name) \
  US_CHECK_ARG((dt) == DT_F32 || (dt) == DT_BF16, "%s: bad dtype %d (0 = fp32, 1 = bf16)", name, (int)(dt))
#define US_CHECK_CONV_GEOM(name, n, h, w, r, s, stride, pad)                                                   \
  US_CHECK_ARG((n) >= 0 && (h) >= 0 && (w) >= 0 && (r) >= 1 && (s) >= 1 && (stride) >= 1 && (pad) >= 0,       \
               "%s: bad geometry n=%d h=%d w=%d r=%d s=%d stride=%d pad=%d", name, n, h, w, r, s, stride, pad)

#define US_LAUNCH_CHECK(name)                                                        \
  do {                                                                               \
    hipError_t _e = hipGetLastError();                                               \
    if (_e != hipSuccess) {                                                          \
      unetseg_set_error("%s: launch failed: %s", name, hipGetErrorString(_e));       \
      return 2;                                                                      \
    }                                                                                \
  } while (0)

// ---- element conversion ------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T>
__device__ __forceinline__ T from_f(float v) { return (T)v; }

// 16-byte vector of T
template <typename T>
struct Vec {
  static constexpr int N = 16 / sizeof(T);
};

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float (&out)[16 / sizeof(T)]) {
  uint4 raw = *reinterpret_cast<const uint4*>(p);
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int i = 0; i < 16 / (int)sizeof(T); ++i) out[i] = (float)e[i];
}

template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float (&in)[16 / sizeof(T)]) {
  uint4 raw;
  T* e = reinterpret_cast<T*>(&raw);
#pragma unroll
  for (int i = 0; i < 16 / (int)sizeof(T); ++i) e[i] = (T)in[i];
  *reinterpret_cast<uint4*>(p) = raw;
}

// ---- wave / block reductions (wave64) ------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum over blockDim.x threads (multiple of 64, <= 1024); every thread gets the result
template <typename F>
__device__ __forceinline__ F block_sum(F v, F* scratch /* >= 16 entries */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  F t = 0;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// ---- bilinear x2 upsample (model/unet_resnet.py:21,71 align_corners=True; unet_plain.py:36 False) --
// source index pair and weight of output index d: align_corners=True: src = d*(in-1)/(out-1);
// False: src = max((d+0.5)/2 - 0.5, 0)  (ATen area_pixel_compute_source_index, scale 0.5)
__device__ __forceinline__ void up_src(int d, int in, int out, int align, int& i0, int& i1, float& l1) {
  float src;
  if (align) {
    const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;  // ATen area_pixel_compute_scale
    src = scale * (float)d;
  } else {
    src = ((float)d + 0.5f) * 0.5f - 0.5f;
    if (src < 0.f) src = 0.f;
  }
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + 1 < in ? i0 + 1 : in - 1;
  l1 = src - (float)i0;
}
// the blend of the four source values, as explicit products / fmas (no contraction choice left to the
// compiler: any kernel that recomputes an upsampled value gets the stored bits)
__device__ __forceinline__ float up_blend(float a, float b, float c, float d, float wl0, float lw, float hl0,
                                          float lh) {
  const float t0 = fmaf(lw, b, wl0 * a), t1 = fmaf(lw, d, wl0 * c);
  return fmaf(lh, t1, hl0 * t0);
}

// one conv weight of a batched pack (unetseg_pack_conv_weights); layout shared with the host
struct UnetsegPackDesc {
  const float* w;   // fp32 [K][C][R][S]
  void* wk;         // dtype [K][R][S][Cpad]
  void* wt;         // dtype [C][R][S][Kld] or NULL
  long long start;  // first tile of this conv in the batch (unetseg_pack_tiles tiles per conv)
  int K, C, R, S, Cpad, Kld;  // Kld: wt row length (0 = K; > K: the zeroed 64-padded image, see the header)
};

