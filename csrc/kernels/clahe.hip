// CLAHE (contrast-limited adaptive histogram equalisation) on 8-bit grayscale batches.
// the reference applies cv2.createCLAHE(clipLimit=3.0, tileGridSize=(16, 16))
// to brightfield images before Cellpose fine-tuning (apps/cellpose-finetuning/main.py:273-308).
// Semantics follow OpenCV's 8-bit CLAHE: the image is virtually extended with reflect-101 borders to
// a multiple of the tile grid, per-tile histograms are clipped at max(1, int(clip * tile_area / 256))
// with the excess redistributed evenly plus a strided residual, the LUT is
// round(cumsum * 255 / tile_area), and pixels blend the four nearest tile LUTs bilinearly in fp32
// (same operation order, no FMA contraction, round-half-even to uint8).
//
// MI355X mapping: kernel 1 = one workgroup per (image, tile): LDS histogram with atomics, the clip /
// redistribution / prefix scan in one wave; kernel 2 = one lane per pixel, the 4 LUT rows it
// needs come from L2 (a 16x16 grid of 256-byte LUTs is 64 KiB per image).
#include "common.h"

// HIP contracts a*b + c into FMAs by default and __fmul_rn / __fadd_rn are plain operators, so bit
// parity with OpenCV's separately rounded fp32 blend needs contraction off: tools/build_native.py
// compiles this file with -ffp-contract=off (the pragma alone is not honoured by hipcc's default).
#pragma clang fp contract(off)

namespace {

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

__global__ __launch_bounds__(256) void clahe_lut_kernel(const uint8_t* __restrict__ src, int H, int W, int tiles_x,
                                                        int tiles_y, int tile_h, int tile_w, float clip,
                                                        uint8_t* __restrict__ lut) {
  __shared__ int hist[256];
  const int b = blockIdx.z;
  const int ty = blockIdx.y, tx = blockIdx.x;
  const int tid = threadIdx.x;
  hist[tid] = 0;
  __syncthreads();
  const uint8_t* img = src + (size_t)b * H * W;
  const int area = tile_h * tile_w;
  for (int e = tid; e < area; e += 256) {
    const int y = reflect101(ty * tile_h + e / tile_w, H);
    const int x = reflect101(tx * tile_w + e % tile_w, W);
    atomicAdd(&hist[img[(size_t)y * W + x]], 1);
  }
  __syncthreads();
  if (tid < 64) {  // one wave: clip, redistribute, scan (256 bins = 4 per lane)
    int h[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = hist[tid * 4 + j];
    if (clip > 0.f) {
      int limit = (int)(clip * (float)area / 256.f);
      limit = limit < 1 ? 1 : limit;
      int clipped = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (h[j] > limit) { clipped += h[j] - limit; h[j] = limit; }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) clipped += __shfl_xor(clipped, o, 64);
      const int batch = clipped / 256;
      int residual = clipped - batch * 256;
      const int step = residual ? max(256 / residual, 1) : 1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = tid * 4 + j;
        h[j] += batch;
        // bins 0, step, 2*step, ... get one more while the residual lasts
        if (residual && i % step == 0 && i / step < residual) h[j] += 1;
      }
    }
    int s = h[0] + h[1] + h[2] + h[3];
    int incl = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (tid >= o) incl += v;
    }
    int run = incl - s;
    const float scale = 255.f / (float)area;
    uint8_t* L = lut + (((size_t)b * tiles_y + ty) * tiles_x + tx) * 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      run += h[j];
      float v = __fmul_rn((float)run, scale);
      v = fminf(fmaxf(rintf(v), 0.f), 255.f);
      L[tid * 4 + j] = (uint8_t)v;
    }
  }
}

__global__ __launch_bounds__(256) void clahe_apply_kernel(const uint8_t* __restrict__ src, int B, int H, int W,
                                                          int tiles_x, int tiles_y, int tile_h, int tile_w,
                                                          const uint8_t* __restrict__ lut, uint8_t* __restrict__ dst) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * H * W) return;
  const int b = (int)(gid / ((long long)H * W));
  const int p = (int)(gid % ((long long)H * W));
  const int y = p / W, x = p % W;
  const float inv_th = 1.f / (float)tile_h, inv_tw = 1.f / (float)tile_w;
  const float tyf = __fsub_rn(__fmul_rn((float)y, inv_th), 0.5f);
  int ty1 = (int)floorf(tyf);
  int ty2 = ty1 + 1;
  const float ya = __fsub_rn(tyf, (float)ty1);
  ty1 = max(ty1, 0);
  ty2 = min(ty2, tiles_y - 1);
  const float txf = __fsub_rn(__fmul_rn((float)x, inv_tw), 0.5f);
  int tx1 = (int)floorf(txf);
  int tx2 = tx1 + 1;
  const float xa = __fsub_rn(txf, (float)tx1);
  tx1 = max(tx1, 0);
  tx2 = min(tx2, tiles_x - 1);
  const int v = src[gid];
  const uint8_t* Lb = lut + (size_t)b * tiles_y * tiles_x * 256;
  const float l11 = Lb[(ty1 * tiles_x + tx1) * 256 + v], l12 = Lb[(ty1 * tiles_x + tx2) * 256 + v];
  const float l21 = Lb[(ty2 * tiles_x + tx1) * 256 + v], l22 = Lb[(ty2 * tiles_x + tx2) * 256 + v];
  const float xa1 = __fsub_rn(1.f, xa);
  const float top = __fadd_rn(__fmul_rn(l11, xa1), __fmul_rn(l12, xa));
  const float bot = __fadd_rn(__fmul_rn(l21, xa1), __fmul_rn(l22, xa));
  const float r = __fadd_rn(__fmul_rn(top, __fsub_rn(1.f, ya)), __fmul_rn(bot, ya));
  dst[gid] = (uint8_t)fminf(fmaxf(rintf(r), 0.f), 255.f);
}

}  // namespace

extern "C" {

// src/dst: uint8 [B, H, W]; lut: uint8 workspace [B, tiles_y, tiles_x, 256].
int be_clahe_u8(const void* src, void* dst, void* lut, int B, int H, int W, int tiles_x, int tiles_y, float clip,
                hipStream_t s) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  if (tiles_x <= 0 || tiles_y <= 0) return -1;
  const int He = H % tiles_y ? H + tiles_y - H % tiles_y : H;
  const int We = W % tiles_x ? W + tiles_x - W % tiles_x : W;
  const int th = He / tiles_y, tw = We / tiles_x;
  hipLaunchKernelGGL(clahe_lut_kernel, dim3(tiles_x, tiles_y, B), dim3(256), 0, s, (const uint8_t*)src, H, W, tiles_x,
                     tiles_y, th, tw, clip, (uint8_t*)lut);
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(clahe_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const uint8_t*)src, B, H,
                     W, tiles_x, tiles_y, th, tw, (const uint8_t*)lut, (uint8_t*)dst);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
