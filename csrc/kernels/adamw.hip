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
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, s, p, g, m, v, (bf16_t*)pbf, n, lr, b1, b2, eps, wd, bc1, bc2,
                     gscale, (const float*)nullptr);
  return BE_CHECK_LAUNCH();
}

// Same update with {lr, wd, bc1, bc2, gscale} read from device memory (graph-capturable).  p/g/m/v/
// pbf point at the START of the range (16-byte aligned for the float4 path), n elements.
int be_adamw_flat_dev(float* p, const float* g, float* m, float* v, void* pbf, long long n, const float* hp, float b1,
                      float b2, float eps, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = (n + 3) / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks > 256) blocks = 256;  // a background stream: one block per CU, leave room for the backward
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
