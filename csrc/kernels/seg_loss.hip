// Fused Cellpose segmentation loss, forward and backward in ONE pass.
//
//   loss = MSE(y[:, 0:2], 5 * lbl[:, 1:3]) / 2 + BCEWithLogits(y[:, 2], lbl[:, 0] > 0.5)
//
// (cellpose ``_loss_fn_seg``, EXT; called per batch at apps/cellpose-finetuning/main.py:1514-1517
// and for validation at :1603-1608.  SURVEY.md §2.5 K11.)
//
// The loss is a plain mean, so dL/dy is pointwise: each lane computes its pixel's contribution to
// the loss AND writes the gradient (already scaled by 1/numel) while the operands are in registers.
// Autograd's backward then only multiplies by grad_output.  One block-level reduction + one atomic
// per block accumulates the loss.  y may be fp32 or bf16 (the network's dtype); lbl is fp32.
#include "common.h"

namespace {

template <bool YBF16>
__global__ __launch_bounds__(256) void seg_loss_kernel(const void* __restrict__ yv, const float* __restrict__ lbl, int B,
                                                       int HW, float* __restrict__ loss, void* __restrict__ gradv,
                                                       float inv_mse, float inv_bce) {
  const long long n = (long long)B * HW;
  const long long stride = (long long)gridDim.x * blockDim.x;
  float acc = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int b = (int)(i / HW), p = (int)(i % HW);
    const size_t base = (size_t)b * 3 * HW + p;
    float y0, y1, y2;
    if (YBF16) {
      const bf16_t* y = (const bf16_t*)yv;
      y0 = bf2f(y[base]); y1 = bf2f(y[base + HW]); y2 = bf2f(y[base + 2 * HW]);
    } else {
      const float* y = (const float*)yv;
      y0 = y[base]; y1 = y[base + HW]; y2 = y[base + 2 * HW];
    }
    const float t0 = 5.f * lbl[base + HW], t1 = 5.f * lbl[base + 2 * HW];
    const float tgt = lbl[base] > 0.5f ? 1.f : 0.f;
    const float d0 = y0 - t0, d1 = y1 - t1;
    // numerically stable BCE with logits: max(x,0) - x*t + log(1 + exp(-|x|))
    const float bce = fmaxf(y2, 0.f) - y2 * tgt + log1pf(__expf(-fabsf(y2)));
    acc += 0.5f * (d0 * d0 + d1 * d1) * inv_mse + bce * inv_bce;
    const float sig = 1.f / (1.f + __expf(-y2));
    const float g0 = d0 * inv_mse;  // d/dy of 0.5 * mean(d^2) over 2*n elements: d / (2n) * 2 * 0.5
    const float g1 = d1 * inv_mse;
    const float g2 = (sig - tgt) * inv_bce;
    if (YBF16) {
      bf16_t* g = (bf16_t*)gradv;
      g[base] = f2bf(g0); g[base + HW] = f2bf(g1); g[base + 2 * HW] = f2bf(g2);
    } else {
      float* g = (float*)gradv;
      g[base] = g0; g[base + HW] = g1; g[base + 2 * HW] = g2;
    }
  }
  acc = wave_sum(acc);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss, red[0] + red[1] + red[2] + red[3]);
}

}  // namespace

extern "C" int be_seg_loss(const void* y, int y_bf16, const float* lbl, int B, int HW, float* loss, void* grad,
                           hipStream_t s) {
  const long long n = (long long)B * HW;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  // MSELoss(mean) over 2*n flow elements, then /2; BCE mean over n
  const float inv_mse = 1.f / (float)(2 * n);
  const float inv_bce = 1.f / (float)n;
  if (y_bf16)
    hipLaunchKernelGGL((seg_loss_kernel<true>), dim3(blocks), dim3(256), 0, s, y, lbl, B, HW, loss, grad, inv_mse, inv_bce);
  else
    hipLaunchKernelGGL((seg_loss_kernel<false>), dim3(blocks), dim3(256), 0, s, y, lbl, B, HW, loss, grad, inv_mse, inv_bce);
  return BE_CHECK_LAUNCH();
}
