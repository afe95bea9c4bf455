// Batched random affine augmentation for Cellpose training (random_rotate_and_resize).
//
// Reference: cellpose ``transforms.random_rotate_and_resize`` (EXT, cv2 on the CPU), called per
// batch at apps/cellpose-finetuning/main.py:1501-1503 (train) and :1587-1593 (val).
// SURVEY.md §2.5 K9.
//
// For every output crop pixel the inverse affine gives the source position (per-image 2x3 matrix,
// flip folded in by the caller).  Image channels: bilinear, zero border (cv2.INTER_LINEAR,
// BORDER_CONSTANT).  Label channel 0 (cell probability / instance map): nearest.  Flow channels
// (dy, dx): bilinear, then rotated by -theta exactly as cellpose rotates the flow vectors.  One
// launch warps images and labels of the whole batch; outputs are NCHW fp32 (network input) and
// the label tensor the fused loss consumes.
#include "common.h"

namespace {

__device__ __forceinline__ float bil(const float* __restrict__ src, int H, int W, float sy, float sx) {
  const float fy = floorf(sy), fx = floorf(sx);
  const int y0 = (int)fy, x0 = (int)fx;
  const float wy = sy - fy, wx = sx - fx;
  float v = 0.f;
  if (y0 >= 0 && y0 < H && x0 >= 0 && x0 < W) v += (1.f - wy) * (1.f - wx) * src[y0 * W + x0];
  if (y0 >= 0 && y0 < H && x0 + 1 >= 0 && x0 + 1 < W) v += (1.f - wy) * wx * src[y0 * W + x0 + 1];
  if (y0 + 1 >= 0 && y0 + 1 < H && x0 >= 0 && x0 < W) v += wy * (1.f - wx) * src[(y0 + 1) * W + x0];
  if (y0 + 1 >= 0 && y0 + 1 < H && x0 + 1 >= 0 && x0 + 1 < W) v += wy * wx * src[(y0 + 1) * W + x0 + 1];
  return v;
}

// aff: [B, 8] = (a00, a01, a02, a10, a11, a12, cos(-theta), sin(-theta)) mapping OUTPUT (x, y) to
// SOURCE (x, y): xs = a00*x + a01*y + a02, ys = a10*x + a11*y + a12.  flip: [B] (x-flip of source).
__global__ __launch_bounds__(256) void affine_warp_kernel(const float* __restrict__ img, int C, const float* __restrict__ lbl,
                                                          int CL, int B, int H, int W, const float* __restrict__ aff,
                                                          const int* __restrict__ flip, int oh, int ow,
                                                          float* __restrict__ out_img, float* __restrict__ out_lbl) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)B * oh * ow;
  if (gid >= n) return;
  const int x = (int)(gid % ow);
  const int y = (int)((gid / ow) % oh);
  const int b = (int)(gid / ((long long)oh * ow));
  const float* A = aff + b * 8;
  float xs = A[0] * x + A[1] * y + A[2];
  const float ys = A[3] * x + A[4] * y + A[5];
  const bool fl = flip[b] != 0;
  if (fl) xs = (float)(W - 1) - xs;
  const size_t opix = (size_t)y * ow + x;
  for (int c = 0; c < C; ++c)
    out_img[((size_t)b * C + c) * oh * ow + opix] = bil(img + ((size_t)b * C + c) * H * W, H, W, ys, xs);
  if (lbl) {
    const float* L = lbl + (size_t)b * CL * H * W;
    // channel 0: nearest
    const int ny = (int)rintf(ys), nx = (int)rintf(xs);
    float l0 = 0.f;
    if (ny >= 0 && ny < H && nx >= 0 && nx < W) l0 = L[ny * W + nx];
    float* O = out_lbl + (size_t)b * CL * oh * ow;
    O[opix] = l0;
    if (CL >= 3) {
      const float v2 = bil(L + (size_t)H * W, H, W, ys, xs);        // flow y
      float v1 = bil(L + (size_t)2 * H * W, H, W, ys, xs);          // flow x
      if (fl) v1 = -v1;
      const float cs = A[6], sn = A[7];
      // cellpose: lbl[1] = -v1*sin(-t) + v2*cos(-t) ; lbl[2] = v1*cos(-t) + v2*sin(-t)
      O[(size_t)oh * ow + opix] = -v1 * sn + v2 * cs;
      O[(size_t)2 * oh * ow + opix] = v1 * cs + v2 * sn;
      for (int c = 3; c < CL; ++c) O[(size_t)c * oh * ow + opix] = bil(L + (size_t)c * H * W, H, W, ys, xs);
    }
  }
}

}  // namespace

extern "C" int be_affine_warp(const float* img, int C, const float* lbl, int CL, int B, int H, int W, const float* aff,
                              const int* flip, int oh, int ow, float* out_img, float* out_lbl, hipStream_t s) {
  const long long n = (long long)B * oh * ow;
  hipLaunchKernelGGL(affine_warp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, img, C, lbl, CL, B, H, W, aff,
                     flip, oh, ow, out_img, out_lbl);
  return BE_CHECK_LAUNCH();
}
