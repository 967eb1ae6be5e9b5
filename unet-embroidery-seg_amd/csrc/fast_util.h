// Device helpers shared by the fast bf16 conv kernels (conv_fast.hip, conv_halo.hip).
#pragma once
#include "common.h"

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB = 0x80000000u;  // beyond any num_records we build (< 2^31)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return *reinterpret_cast<uint4*>(&v);
}
__device__ __forceinline__ int swz8(int row, int ch) { return ch ^ ((row >> 1) & 7); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// BN-ReLU input prologue on one packed bf16 pair: (bf16) relu(fmaf(z, sc, sh)), bn_apply's expression
// and rounding, as unpack + one packed fma (v_pk_fma_f32) + round-to-nearest-even pack + ReLU as a
// signed 16-bit max on the bf16 bit patterns (a negative bf16 is a negative int16; -0 becomes +0) --
// 3 VALU per pair fewer than the scalar form, which bound the prologue variants' VALU issue.
__device__ __forceinline__ unsigned bnrelu_pair(unsigned v, f32x2 sc, f32x2 sh) {
  const f32x2 z = {__uint_as_float(v << 16), __uint_as_float(v & 0xffff0000u)};
  const f32x2 r = __builtin_elementwise_fma(z, sc, sh);
  i16x2 b = __builtin_bit_cast(i16x2, __builtin_convertvector(r, bf16x2));  // one v_cvt_pk_bf16_f32
  b = __builtin_elementwise_max(b, (i16x2){0, 0});
  return __builtin_bit_cast(unsigned, b);
}

// LDS-DMA of 16 B per lane (64 lanes -> 1 KiB contiguous at lds_byte): issued in inline asm so
// hipcc neither tracks it (no conservative vmcnt(0) before every ds_read) nor reuses M0 (saved and
// restored inside the statement).  Completion is counted by the caller's explicit vmcnt.
// Every vector-memory instruction in these statements is preceded by s_nop 4 (with the s_movs: >= 5
// wait states): its descriptor / soffset SGPRs may have just been written by a VALU (readfirstlane in
// srd_u, or v_readlane restoring a spilled SGPR), and hipcc pads no hazard inside an asm string -- the
// persistent halo ring's partial stores went through a stale descriptor until this was added.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned lds_byte, unsigned voff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 4\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_byte), "v"(voff), "s"(r)
      : "memory");
}
// Two LDS-DMA rows of one wave (lds_byte and lds_byte + STRIDE) with one M0 save/restore; soff is
// a scalar byte offset added by the hardware to both.  Out-of-range rows must be expressed in voff
// (or a zero-extent SRD), never in soff.
// srd() of a wave-uniform (pointer, extent) chosen at run time: readfirstlane keeps the descriptor in
// SGPRs (an inline-asm "s" operand does not force that by itself)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd_u(const void* p, unsigned bytes) {
  const unsigned long long q = (unsigned long long)(size_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)q);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(q >> 32));
  return srd((const void*)(size_t)(((unsigned long long)hi << 32) | lo), __builtin_amdgcn_readfirstlane(bytes));
}
// one LDS-DMA row with a scalar offset (see dma16x2)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, unsigned lds_byte, unsigned voff, unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 4\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_byte), "v"(voff), "s"(r), "s"(soff)
      : "memory");
}
// (M0 is set with s_mov only: an s_add would clobber SCC behind the compiler's back)
template <int STRIDE>
__device__ __forceinline__ void dma16x2(__amdgpu_buffer_rsrc_t r, unsigned lds_byte, unsigned v0, unsigned v1,
                                        unsigned soff) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 4\n\t"
      "buffer_load_dwordx4 %3, %5, %6 offen lds\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %4, %5, %6 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_byte), "s"(lds_byte + STRIDE), "v"(v0), "v"(v1), "s"(r), "s"(soff)
      : "memory");
}
// buffer stores / an untracked load (inline asm: hipcc does not count them, the caller's explicit vmcnt does)
__device__ __forceinline__ void bstore64(__amdgpu_buffer_rsrc_t r, unsigned off, uint2 v) {
  asm volatile("s_nop 4\n\tbuffer_store_dwordx2 %0, %1, %2, 0 offen" ::"v"(v), "v"(off), "s"(r) : "memory");
}
// an 8-B buffer load the compiler does not track: the caller waits for it with an explicit vmcnt (so the
// wait can leave later LDS-DMAs in flight) and then ties the value with asm volatile("" : "+v"(v))
__device__ __forceinline__ uint2 bload64_asm(__amdgpu_buffer_rsrc_t r, unsigned off) {
  uint2 v;
  asm volatile("s_nop 4\n\tbuffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
  return v;
}
__device__ __forceinline__ void bstore32(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  asm volatile("s_nop 4\n\tbuffer_store_dword %0, %1, %2, 0 offen" ::"v"(v), "v"(off), "s"(r) : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ int swz_tr16(int row) { return ((row & 3) | ((row >> 1) & 4)) << 1; }
__device__ __forceinline__ int swz_tr8(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }

// Sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15), result in every lane of the row:
// four row rotations on the VALU.  __shfl_xor goes through ds_bpermute (an LDS round trip per
// step); in the conv epilogues that cost as much as the whole store phase.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x122, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x121, 0xF, 0xF, false));
  return v;
}

// row16_sum of N independent values, rotation-major: each value gets exactly row16_sum's additions,
// but the N chains interleave -- issued one chain at a time, every dependent DPP add waited out its
// VALU-to-DPP hazard (s_nop), and an epilogue with 32 of them spent more time there than on its stores
template <int N>
__device__ __forceinline__ void row16_sum_n(float (&v)[N]) {
#define ROW16_STEP(CTL)                                                                                      \
  _Pragma("unroll") for (int i = 0; i < N; ++i) v[i] +=                                                      \
      __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[i]), CTL, 0xF, 0xF, false));
  ROW16_STEP(0x128)
  ROW16_STEP(0x124)
  ROW16_STEP(0x122)
  ROW16_STEP(0x121)
#undef ROW16_STEP
}

}  // namespace
