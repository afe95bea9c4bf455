// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernel library.
//
// Every kernel in csrc/kernels is written for gfx950 only: 64-lane waves,
// MFMA 16x16x32 bf16 tiles, 160 KiB LDS per CU.  Host entry points are plain
// C ABI functions (`be_*`) that take raw device pointers and a hipStream_t so
// the Python layer (bioengine_worker_amd/ops/_native.py) can call them on
// PyTorch's current stream without pulling torch headers into the build.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(4))) float f32x4;    // MFMA 16x16 accumulator
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

#define BE_WAVE 64

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

// fp32 -> bf16 round-to-nearest-even (NaN stays NaN): one v_cvt_pk_bf16_f32 on gfx950 for a pair.
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

typedef __attribute__((ext_vector_type(2))) short s16x2_t;
// ReLU of two packed bf16 values as one v_pk_max_i16: a negative bf16 (sign bit set) is a negative
// int16, so max(.., 0) zeroes it and leaves non-negative values bit-exact.
__device__ __forceinline__ uint32_t relu_bf16x2(uint32_t w) {
  const s16x2_t z = {0, 0};
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s16x2_t, w), z));
}

__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that share an XCD (id % 8) get a contiguous range of logical tiles so that
// neighbouring tiles, which share halo rows and weight panels, hit the same private L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

#define BE_CHECK_LAUNCH() ((int)hipGetLastError())

// ---- per-device host state ---------------------------------------------------------------------
// A process may drive several GPUs (the 3-D EM slab path, multi-GPU replicas in one process): the
// one-time kernel attributes (hipFuncSetAttribute is per device) and the zero pages the implicit-GEMM
// loaders read for conv padding must be kept per device, never once per process.
#define BE_MAX_DEV 64
inline int be_cur_dev() {
  int d = 0;
  (void)hipGetDevice(&d);
  return (d < 0 || d >= BE_MAX_DEV) ? 0 : d;
}

// Zero-filled device buffer of `bytes` on the current device, allocated once per (device, slot).
inline const bf16_t* be_zero_page(int slot, size_t bytes) {
  static bf16_t* pages[4][BE_MAX_DEV] = {};
  bf16_t*& z = pages[slot & 3][be_cur_dev()];
  if (!z) {
    if (hipMalloc((void**)&z, bytes) != hipSuccess) { z = nullptr; return nullptr; }
    if (hipMemset(z, 0, bytes) != hipSuccess) return nullptr;
  }
  return z;
}
