// Volume resampling for the BioImage.IO 3-D U-Net path (fibsem volume
// inference, reference apps/fibsem-mito-analysis/analysis_deployment.py:108-176):
//
//   be_maxpool3d_ndhwc    MaxPool3d(2) on NDHWC bf16 (floor mode, like nn.MaxPool3d(2))
//   be_depth2space3d      ConvTranspose3d(k=2, s=2) tail: the 1x1x1 MFMA conv to 8*Cout channels
//                         (channel (4 dz + 2 dy + dx) * Cout + c) scattered to the 2x-upsampled volume
//
// Both are pure HBM streams: one 16-byte load / store per 8 channels, coalesced along the
// contiguous channel axis (C % 8 == 0, host-checked), grid-stride loops sized for 256 CUs.
#include "common.h"

namespace {

__device__ __forceinline__ u32x4 max8(u32x4 a, u32x4 b) {
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // max of bf16 values is exact in bf16
    const float lo = fmaxf(lo_bf(a[j]), lo_bf(b[j]));
    const float hi = fmaxf(hi_bf(a[j]), hi_bf(b[j]));
    r[j] = (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
  }
  return r;
}

__global__ __launch_bounds__(256) void maxpool3d_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out, int N,
                                                        int D, int H, int W, int C) {
  const int Do = D / 2, Ho = H / 2, Wo = W / 2, C8 = C / 8;
  const long long total = (long long)N * Do * Ho * Wo * C8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % C8);
    long long v = i / C8;
    const int xo = (int)(v % Wo); v /= Wo;
    const int yo = (int)(v % Ho); v /= Ho;
    const int zo = (int)(v % Do);
    const int n = (int)(v / Do);
    const bf16_t* b = x + ((((long long)n * D + 2 * zo) * H + 2 * yo) * W + 2 * xo) * C + c8 * 8;
    const long long sy = (long long)W * C, sz = (long long)H * W * C;
    u32x4 m = *reinterpret_cast<const u32x4*>(b);
    m = max8(m, *reinterpret_cast<const u32x4*>(b + C));
    m = max8(m, *reinterpret_cast<const u32x4*>(b + sy));
    m = max8(m, *reinterpret_cast<const u32x4*>(b + sy + C));
    m = max8(m, *reinterpret_cast<const u32x4*>(b + sz));
    m = max8(m, *reinterpret_cast<const u32x4*>(b + sz + C));
    m = max8(m, *reinterpret_cast<const u32x4*>(b + sz + sy));
    m = max8(m, *reinterpret_cast<const u32x4*>(b + sz + sy + C));
    *reinterpret_cast<u32x4*>(out + i * 8) = m;
  }
}

// y [N, D, H, W, 8 C] -> out [N, 2D, 2H, 2W, C]; thread = one output voxel x 8 channels, so the
// stores are contiguous and each 16-byte load reads one sub-voxel's channel chunk
__global__ __launch_bounds__(256) void depth2space3d_kernel(const bf16_t* __restrict__ y, bf16_t* __restrict__ out,
                                                            int N, int D, int H, int W, int C) {
  const int D2 = 2 * D, H2 = 2 * H, W2 = 2 * W, C8 = C / 8;
  const long long total = (long long)N * D2 * H2 * W2 * C8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % C8);
    long long v = i / C8;
    const int xo = (int)(v % W2); v /= W2;
    const int yo = (int)(v % H2); v /= H2;
    const int zo = (int)(v % D2);
    const int n = (int)(v / D2);
    const int sub = (zo & 1) * 4 + (yo & 1) * 2 + (xo & 1);
    const bf16_t* src =
        y + ((((long long)n * D + (zo >> 1)) * H + (yo >> 1)) * W + (xo >> 1)) * (8LL * C) + sub * C + c8 * 8;
    *reinterpret_cast<u32x4*>(out + i * 8) = *reinterpret_cast<const u32x4*>(src);
  }
}

int grid_for(long long total) {
  long long g = (total + 255) / 256;
  return (int)(g < 256 * 16 ? (g < 1 ? 1 : g) : 256 * 16);
}

}  // namespace

extern "C" {

int be_maxpool3d_ndhwc(const void* x, void* out, int N, int D, int H, int W, int C, hipStream_t s) {
  if (C % 8 || N <= 0 || D < 2 || H < 2 || W < 2) return -10;
  const long long total = (long long)N * (D / 2) * (H / 2) * (W / 2) * (C / 8);
  hipLaunchKernelGGL(maxpool3d_kernel, dim3(grid_for(total)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)out, N, D, H,
                     W, C);
  return BE_CHECK_LAUNCH();
}

int be_depth2space3d(const void* y, void* out, int N, int D, int H, int W, int C, hipStream_t s) {
  if (C % 8 || N <= 0 || D <= 0 || H <= 0 || W <= 0) return -10;
  const long long total = (long long)N * 8 * D * H * W * (C / 8);
  hipLaunchKernelGGL(depth2space3d_kernel, dim3(grid_for(total)), dim3(256), 0, s, (const bf16_t*)y, (bf16_t*)out, N,
                     D, H, W, C);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
