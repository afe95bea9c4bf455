// Row-wise LayerNorm family for the ViT encoders (DINOv2 ViT-B/14, SAM ViT-L/8, SURVEY.md §2.5
// K8/K17), fused with the residual update that precedes every pre-norm transformer block:
//
//   x_new = x + gamma * y          (LayerScale residual; gamma optional, y optional)
//   out   = LN(x_new) * w + b      (fp32 statistics, bf16 out)
//
// One pass over HBM instead of three (residual add, LayerScale, norm).  One wave per row; the row
// (C <= 2048 channels) lives in registers between the statistics and the normalisation, so each
// element is read once and written at most twice (x_new and out).  Also LayerNorm2d over the
// channel axis of an NHWC map (SAM neck) — identical math on [pixels, C] rows.
#include "common.h"

namespace {

constexpr int MAXV = 4;  // 16-byte vectors per lane: C <= 64 lanes * 8 * MAXV = 2048

__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  const u32x4 r = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(r[j]); v[2 * j + 1] = hi_bf(r[j]); }
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = pack2bf(v[2 * j], v[2 * j + 1]);
  *reinterpret_cast<u32x4*>(p) = r;
}

// Q8: instead of bf16 `out`, write the normalised row as e4m3fn (q8) with its per-row dequantisation
// scale (qscale = amax / 448) — the input format of the fp8 GEMM (gemm_fp8.hip), so the GEMM's
// activation quantisation costs no extra pass over HBM.
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a, -448.f), 448.f), fminf(fmaxf(b, -448.f), 448.f), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c, -448.f), 448.f), fminf(fmaxf(d, -448.f), 448.f), w, true);
  return (uint32_t)w;
}

// MX: the normalised row as MX-fp8 -- e4m3fn q8 with one E8M0 power-of-two scale per 32 consecutive
// channels (uint8 [rows][C / 32], byte = e + 127, the smallest e with amax / 2^e <= 448): the A-operand
// format of the block-scaled GEMM (gemm_fp8.hip be_gemm_fp8_mx), so qkv / fc1 get MX activations
// straight from the LayerNorm.  A 32-channel block is 4 consecutive lanes' 8-channel vectors.
__device__ __forceinline__ int e8m0_exp(float amax) {
  if (!(amax > 0.f)) return -127;
  const float r = amax * (1.f / 448.f);
  const int bits = __float_as_int(r);
  int e = ((bits >> 23) & 0xff) - 127 + ((bits & 0x7fffff) ? 1 : 0);  // ceil(log2 r), normal r
  if (amax * __builtin_ldexpf(1.f, -e) > 448.f) ++e;
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

template <int NV, bool Q8 = false, bool MX = false>
__global__ __launch_bounds__(256) void add_ln_kernel(bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
                                                     const float* __restrict__ gamma, const float* __restrict__ w,
                                                     const float* __restrict__ bias, bf16_t* __restrict__ out,
                                                     float* __restrict__ stats, long long rows, int C, float eps,
                                                     int write_x, uint8_t* __restrict__ q8,
                                                     float* __restrict__ qscale, bf16_t* __restrict__ xo = nullptr,
                                                     const float* __restrict__ rs = nullptr, int rpn = 1) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  bf16_t* xr = x + row * C;
  bf16_t* xw = (xo ? xo : x) + row * C;  // where the updated residual goes (training keeps the input)
  const float rsc = rs ? rs[row / rpn] : 1.f;  // per-sample scale of y (stochastic depth keep mask)
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      load8(xr + c, v[k]);
      if (y) {
        float t[8];
        load8(y + row * C + c, t);
        if (gamma) {
          const float4 g0 = *reinterpret_cast<const float4*>(gamma + c);
          const float4 g1 = *reinterpret_cast<const float4*>(gamma + c + 4);
          const float g[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] += rsc * g[j] * t[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[k][j] += rsc * t[j];
        }
        // the residual stream is bf16: normalise exactly what the next block will read back
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = bf2f(f2bf(v[k][j]));
        if (write_x) store8(xw + c, v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[k][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  if (stats && lane == 0) { stats[2 * row] = mean; stats[2 * row + 1] = rstd; }
  if (!Q8 && !out) return;
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + c);
      const float4 w1 = *reinterpret_cast<const float4*>(w + c + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
      const float ww[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * ww[j] + bb[j];
      if (Q8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { v[k][j] = o[j]; amax = fmaxf(amax, fabsf(o[j])); }
      } else {
        store8(out + row * C + c, o);
      }
    }
  }
  if (Q8 && MX) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      float bm = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) bm = fmaxf(bm, fabsf(v[k][j]));
      bm = fmaxf(bm, __shfl_xor(bm, 1, 64));
      bm = fmaxf(bm, __shfl_xor(bm, 2, 64));
      if (c < C) {
        const int e = e8m0_exp(bm);
        const float inv = __builtin_ldexpf(1.f, -e);
        u32x2 o;
        o[0] = pack4_fp8(v[k][0] * inv, v[k][1] * inv, v[k][2] * inv, v[k][3] * inv);
        o[1] = pack4_fp8(v[k][4] * inv, v[k][5] * inv, v[k][6] * inv, v[k][7] * inv);
        *reinterpret_cast<u32x2*>(q8 + row * C + c) = o;
        if ((lane & 3) == 0) reinterpret_cast<uint8_t*>(qscale)[row * (C / 32) + c / 32] = (uint8_t)(e + 127);
      }
    }
    return;
  }
  if (Q8) {
    amax = fmaxf(wave_max(amax), 1e-12f);
    const float inv = 448.f / amax;
    if (lane == 0) qscale[row] = amax * (1.f / 448.f);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
        u32x2 o;
        o[0] = pack4_fp8(v[k][0] * inv, v[k][1] * inv, v[k][2] * inv, v[k][3] * inv);
        o[1] = pack4_fp8(v[k][4] * inv, v[k][5] * inv, v[k][6] * inv, v[k][7] * inv);
        *reinterpret_cast<u32x2*>(q8 + row * C + c) = o;
      }
    }
  }
}

// bias + exact (erf) GELU on a bf16 [rows, C] GEMM output, in place.
__global__ __launch_bounds__(256) void bias_gelu_kernel(bf16_t* __restrict__ h, const float* __restrict__ bias,
                                                        long long n8, int C) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const long long e = i * 8;
    const int c = (int)(e % C);
    float v[8];
    load8(h + e, v);
    const float4 b0 = *reinterpret_cast<const float4*>(bias + c);
    const float4 b1 = *reinterpret_cast<const float4*>(bias + c + 4);
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = v[j] + bb[j];
      v[j] = 0.5f * t * (1.f + erff(t * 0.70710678118654752f));
    }
    store8(h + e, v);
  }
}

}  // namespace

extern "C" {

// x: bf16 [rows, C] residual stream (updated in place to x + gamma*y when y != null and write_x);
// out: bf16 [rows, C] normalised (may be null); stats: optional float [rows, 2] (mean, rstd).
int be_add_layernorm(void* x, const void* y, const float* gamma, const float* w, const float* b, void* out,
                     float* stats, long long rows, int C, float eps, int write_x, hipStream_t s) {
  if (C % 8 != 0 || C > 64 * 8 * MAXV) return -1;
  if (out && (!w || !b)) return -2;
  const int nv = (C / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + 3) / 4));
  switch (nv) {
    case 1: hipLaunchKernelGGL(add_ln_kernel<1>, grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y, gamma, w, b,
                               (bf16_t*)out, stats, rows, C, eps, write_x, nullptr, nullptr); break;
    case 2: hipLaunchKernelGGL(add_ln_kernel<2>, grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y, gamma, w, b,
                               (bf16_t*)out, stats, rows, C, eps, write_x, nullptr, nullptr); break;
    case 3: hipLaunchKernelGGL(add_ln_kernel<3>, grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y, gamma, w, b,
                               (bf16_t*)out, stats, rows, C, eps, write_x, nullptr, nullptr); break;
    default: hipLaunchKernelGGL(add_ln_kernel<4>, grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y, gamma, w, b,
                                (bf16_t*)out, stats, rows, C, eps, write_x, nullptr, nullptr); break;
  }
  return BE_CHECK_LAUNCH();
}

// As be_add_layernorm, but the normalised output is e4m3fn q8 [rows, C] + qscale [rows] (fp8 GEMM input).
int be_add_layernorm_fp8(void* x, const void* y, const float* gamma, const float* w, const float* b, void* q8,
                         float* qscale, long long rows, int C, float eps, int write_x, hipStream_t s) {
  if (C % 8 != 0 || C > 64 * 8 * MAXV || !w || !b || !q8 || !qscale) return -1;
  const int nv = (C / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + 3) / 4));
#define LNQ(NV)                                                                                                \
  case NV:                                                                                                     \
    hipLaunchKernelGGL((add_ln_kernel<NV, true>), grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y, gamma, w, \
                       b, (bf16_t*)nullptr, (float*)nullptr, rows, C, eps, write_x, (uint8_t*)q8, qscale);       \
    break;
  switch (nv) {
    LNQ(1) LNQ(2) LNQ(3) LNQ(4)
    default: return -1;
  }
#undef LNQ
  return BE_CHECK_LAUNCH();
}

// As be_add_layernorm_fp8, with MX-fp8 output: q8 e4m3fn [rows, C] + E8M0 block scales (uint8
// [rows, C / 32]) in qscale.  C % 32 == 0.
int be_add_layernorm_mx(void* x, const void* y, const float* gamma, const float* w, const float* b, void* q8,
                        void* qscale, long long rows, int C, float eps, int write_x, hipStream_t s) {
  if (C % 32 != 0 || C > 64 * 8 * MAXV || !w || !b || !q8 || !qscale) return -1;
  const int nv = (C / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + 3) / 4));
#define LNM(NV)                                                                                                \
  case NV:                                                                                                     \
    hipLaunchKernelGGL((add_ln_kernel<NV, true, true>), grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y,  \
                       gamma, w, b, (bf16_t*)nullptr, (float*)nullptr, rows, C, eps, write_x, (uint8_t*)q8,    \
                       (float*)qscale);                                                                        \
    break;
  switch (nv) {
    LNM(1) LNM(2) LNM(3) LNM(4)
    default: return -1;
  }
#undef LNM
  return BE_CHECK_LAUNCH();
}

// Training variant: xo = x + rs[row / rpn] * y (x untouched; rs optional per-sample scale), out = LN(xo),
// stats = (mean, rstd) per row for the backward.  y == null: plain LN of x (xo ignored).
int be_add_layernorm_train(const void* x, const void* y, const float* rs, int rpn, void* xo, const float* w,
                           const float* b, void* out, float* stats, long long rows, int C, float eps, hipStream_t s) {
  if (C % 8 != 0 || C > 64 * 8 * MAXV || !w || !b || !out || !stats) return -1;
  if (y && !xo) return -2;
  const int nv = (C / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + 3) / 4));
#define LNT(NV)                                                                                                   \
  case NV:                                                                                                        \
    hipLaunchKernelGGL((add_ln_kernel<NV, false>), grid, dim3(256), 0, s, (bf16_t*)x, (const bf16_t*)y,            \
                       (const float*)nullptr, w, b, (bf16_t*)out, stats, rows, C, eps, y ? 1 : 0, (uint8_t*)nullptr, \
                       (float*)nullptr, (bf16_t*)xo, rs, rpn > 0 ? rpn : 1);                                      \
    break;
  switch (nv) {
    LNT(1) LNT(2) LNT(3) LNT(4)
    default: return -1;
  }
#undef LNT
  return BE_CHECK_LAUNCH();
}

int be_bias_gelu(void* h, const float* bias, long long rows, int C, hipStream_t s) {
  if (C % 8 != 0) return -1;
  const long long n8 = rows * C / 8;
  long long blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(bias_gelu_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (bf16_t*)h, bias, n8, C);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
