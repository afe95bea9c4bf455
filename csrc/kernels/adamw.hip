// Fused AdamW over one flat fp32 parameter buffer (all model parameters are views into it).
//
// Reference: AdamW(lr, weight_decay) created once per training run and stepped per batch at
// apps/cellpose-finetuning/main.py:1451-1453,1518 (torch.optim.AdamW, EXT).  SURVEY.md §2.5 K12.
//
// One launch updates every parameter: p, g, m, v are flat fp32 arrays, read/written with 16-byte
// vector accesses (memory-bound: 28 B/param moved, the minimum for fp32 master + 2 moments + grad
// read).  The data-parallel gradient mean (1/world) and an optional gradient-norm clip factor are
// folded in as `gscale`, so no separate scaling pass runs after the RCCL all-reduce.  An optional
// bf16 mirror of the updated weights is written in the same pass for the bf16 compute kernels.
#include <cstdlib>

#include "common.h"

namespace {

// hp (optional): device copy of {lr, wd, bc1, bc2, gscale} overriding the by-value scalars, so the
// update can live inside a captured HIP graph and still follow the host's LR schedule / step count.
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, bf16_t* __restrict__ pbf,
                                                    long long n, float lr, float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2, float gscale, const float* __restrict__ hp) {
  if (hp) {
    lr = hp[0]; wd = hp[1]; bc1 = hp[2]; bc2 = hp[3]; gscale = hp[4];
  }
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float step_size = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pa = &pp.x;
    const float* ga = &gg.x;
    float* ma = &mm.x;
    float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = ga[j] * gscale;
      pa[j] *= (1.f - lr * wd);
      ma[j] = b1 * ma[j] + (1.f - b1) * gj;
      va[j] = b2 * va[j] + (1.f - b2) * gj * gj;
      const float denom = sqrtf(va[j]) * rbc2 + eps;
      pa[j] -= step_size * ma[j] / denom;
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (pbf) {
      u32x2 o;
      o[0] = pack2bf(pp.x, pp.y);
      o[1] = pack2bf(pp.z, pp.w);
      reinterpret_cast<u32x2*>(pbf)[i] = o;
    }
  }
  // tail
  const long long t0 = n4 * 4;
  for (long long i = t0 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gj = g[i] * gscale;
    float pj = p[i] * (1.f - lr * wd);
    const float mj = b1 * m[i] + (1.f - b1) * gj;
    const float vj = b2 * v[i] + (1.f - b2) * gj * gj;
    pj -= step_size * mj / (sqrtf(vj) * rbc2 + eps);
    p[i] = pj; m[i] = mj; v[i] = vj;
    if (pbf) pbf[i] = f2bf(pj);
  }
}

// Same update, two float4 groups per thread per iteration with both groups' 4 loads issued before
// any use (8 x 16 B in flight per lane), and streaming (non-temporal) accesses: every byte is
// touched exactly once per step, so nothing is worth keeping in L2 / MALL.  A/B: be_adamw_set_variant.
__global__ __launch_bounds__(256) void adamw2_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ v,
                                                     bf16_t* __restrict__ pbf, long long n, float lr, float b1,
                                                     float b2, float eps, float wd, float bc1, float bc2, float gscale,
                                                     const float* __restrict__ hp) {
  if (hp) {
    lr = hp[0]; wd = hp[1]; bc1 = hp[2]; bc2 = hp[3]; gscale = hp[4];
  }
  typedef __attribute__((ext_vector_type(4))) float f4;
  const long long n4 = n / 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float step_size = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  const float decay = 1.f - lr * wd;
  f4* P = reinterpret_cast<f4*>(p);
  const f4* G = reinterpret_cast<const f4*>(g);
  f4* M = reinterpret_cast<f4*>(m);
  f4* V = reinterpret_cast<f4*>(v);
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const long long i2 = i + stride;
    f4 pp[2], gg[2], mm[2], vv[2];
    pp[0] = __builtin_nontemporal_load(P + i); pp[1] = __builtin_nontemporal_load(P + i2);
    gg[0] = __builtin_nontemporal_load(G + i); gg[1] = __builtin_nontemporal_load(G + i2);
    mm[0] = __builtin_nontemporal_load(M + i); mm[1] = __builtin_nontemporal_load(M + i2);
    vv[0] = __builtin_nontemporal_load(V + i); vv[1] = __builtin_nontemporal_load(V + i2);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gj = gg[u][j] * gscale;
        float pj = pp[u][j] * decay;
        const float mj = b1 * mm[u][j] + (1.f - b1) * gj;
        const float vj = b2 * vv[u][j] + (1.f - b2) * gj * gj;
        pj -= step_size * mj / (sqrtf(vj) * rbc2 + eps);
        pp[u][j] = pj; mm[u][j] = mj; vv[u][j] = vj;
      }
    }
    __builtin_nontemporal_store(pp[0], P + i); __builtin_nontemporal_store(pp[1], P + i2);
    __builtin_nontemporal_store(mm[0], M + i); __builtin_nontemporal_store(mm[1], M + i2);
    __builtin_nontemporal_store(vv[0], V + i); __builtin_nontemporal_store(vv[1], V + i2);
    if (pbf) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        u32x2 o;
        o[0] = pack2bf(pp[u][0], pp[u][1]);
        o[1] = pack2bf(pp[u][2], pp[u][3]);
        __builtin_nontemporal_store(o, reinterpret_cast<u32x2*>(pbf) + (u ? i2 : i));
      }
    }
  }
  for (; i < n4; i += stride) {  // the last partial round
    f4 pp = P[i], gg = G[i], mm = M[i], vv = V[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = gg[j] * gscale;
      float pj = pp[j] * decay;
      const float mj = b1 * mm[j] + (1.f - b1) * gj;
      const float vj = b2 * vv[j] + (1.f - b2) * gj * gj;
      pj -= step_size * mj / (sqrtf(vj) * rbc2 + eps);
      pp[j] = pj; mm[j] = mj; vv[j] = vj;
    }
    P[i] = pp; M[i] = mm; V[i] = vv;
    if (pbf) {
      u32x2 o;
      o[0] = pack2bf(pp[0], pp[1]);
      o[1] = pack2bf(pp[2], pp[3]);
      reinterpret_cast<u32x2*>(pbf)[i] = o;
    }
  }
  const long long t0 = n4 * 4;  // scalar tail
  for (long long k = t0 + (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
    const float gj = g[k] * gscale;
    float pj = p[k] * decay;
    const float mj = b1 * m[k] + (1.f - b1) * gj;
    const float vj = b2 * v[k] + (1.f - b2) * gj * gj;
    pj -= step_size * mj / (sqrtf(vj) * rbc2 + eps);
    p[k] = pj; m[k] = mj; v[k] = vj;
    if (pbf) pbf[k] = f2bf(pj);
  }
}

int g_adamw_variant = 1;  // 1: adamw2_kernel (1.916 vs 1.941 ms at ViT-L, profiles/r04/cpsam/adamw_ab.jsonl), 0: adamw_kernel

// sum of squares of a flat fp32 buffer (for gradient-norm clipping / logging); out must be zeroed.
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, long long n, float* __restrict__ out) {
  float s = 0.f;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) s += x[i] * x[i];
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

}  // namespace

extern "C" {

int be_adamw_flat(float* p, const float* g, float* m, float* v, void* pbf, long long n, float lr, float b1, float b2,
                  float eps, float wd, int step, float gscale, hipStream_t s) {
  if (n <= 0) return 0;
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  const long long n4 = (n + 3) / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (g_adamw_variant == 1)
    hipLaunchKernelGGL(adamw2_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, n, lr, b1, b2, eps, wd,
                       bc1, bc2, gscale, (const float*)nullptr);
  else
    hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, n, lr, b1, b2, eps, wd, bc1,
                       bc2, gscale, (const float*)nullptr);
  return BE_CHECK_LAUNCH();
}

// A/B switch of the flat update kernel: 1 = two float4 groups per lane + streaming accesses, 0 = one.
int be_adamw_set_variant(int variant) {
  g_adamw_variant = variant;
  return 0;
}

// Same update with {lr, wd, bc1, bc2, gscale} read from device memory (graph-capturable).  p/g/m/v/
// pbf point at the START of the range (16-byte aligned for the float4 path), n elements.
int be_adamw_flat_dev(float* p, const float* g, float* m, float* v, void* pbf, long long n, const float* hp, float b1,
                      float b2, float eps, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = (n + 3) / 4;
  int blocks = (int)((n4 + 255) / 256);
  // a background stream: at most one block per CU (BE_ADAMW_BG_BLOCKS caps it lower), leaving room
  // for the backward kernels it runs beside
  static const int cap = [] {
    const char* e = getenv("BE_ADAMW_BG_BLOCKS");
    const int c = e ? atoi(e) : 256;
    return c > 0 ? c : 256;
  }();
  if (blocks > cap) blocks = cap;
  if (g_adamw_variant == 1)
    hipLaunchKernelGGL(adamw2_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, n, 0.f, b1, b2, eps, 0.f,
                       1.f, 1.f, 1.f, hp);
  else
    hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, n, 0.f, b1, b2, eps, 0.f,
                       1.f, 1.f, 1.f, hp);
  return BE_CHECK_LAUNCH();
}

int be_sumsq(const float* x, long long n, float* out, hipStream_t s) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sumsq_kernel, dim3(blocks), dim3(256), 0, s, x, n, out);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
