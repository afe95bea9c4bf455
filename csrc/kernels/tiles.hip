// Tile gather / tapered blend for tiled 2D inference (Cellpose run_net tiling, BioImage.IO blocked
// prediction, fibsem 2D tiles).  SURVEY.md §2.5 K2, K7, K14.
//
// be_tiles_gather: normalised image [B, C, H, W] fp32 (or bf16 when src_bf16) -> NHWC bf16 tiles
//   [B*nty*ntx, by, bx, cpad].  The image is implicitly zero-padded by (pad_y, pad_x) on the
//   top/left (cellpose pad_image_ND), so padding, channel padding, layout change and bf16 cast all
//   happen in one pass; tiles never exist in fp32 NCHW.
// be_tiles_blend: tile outputs [B*nt, nout, by, bx] fp32 -> [B, nout, H, W] fp32 by the separable
//   taper mask wy[ty] * wx[tx] (cellpose _taper_mask), normalised by the summed weights.  Output-
//   centric gather (each output pixel walks only the tiles that cover it), so there are no atomics
//   and the result is bit-deterministic.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void tiles_gather_kernel(const float* __restrict__ img, int B, int C, int H, int W,
                                                           int pad_y, int pad_x, const int* __restrict__ ys,
                                                           const int* __restrict__ xs, int nty, int ntx, int by, int bx,
                                                           int cpad, bf16_t* __restrict__ out) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long npix = (long long)B * nty * ntx * by * bx;
  if (gid >= npix) return;
  const int tx = (int)(gid % bx);
  long long r = gid / bx;
  const int ty = (int)(r % by);
  r /= by;
  const int t = (int)(r % (nty * ntx));
  const int b = (int)(r / (nty * ntx));
  const int yy = ys[t / ntx] + ty - pad_y;
  const int xx = xs[t % ntx] + tx - pad_x;
  const bool in = (yy >= 0 && yy < H && xx >= 0 && xx < W);
  bf16_t* o = out + gid * cpad;
  for (int c0 = 0; c0 < cpad; c0 += 8) {
    u32x4 v = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ca = c0 + 2 * j, cb = ca + 1;
      const float fa = (in && ca < C) ? img[(((size_t)b * C + ca) * H + yy) * W + xx] : 0.f;
      const float fb = (in && cb < C) ? img[(((size_t)b * C + cb) * H + yy) * W + xx] : 0.f;
      v[j] = pack2bf(fa, fb);
    }
    *reinterpret_cast<u32x4*>(o + c0) = v;
  }
}

__global__ __launch_bounds__(256) void tiles_blend_kernel(const float* __restrict__ yt, int B, int nout, int H, int W,
                                                          int pad_y, int pad_x, const int* __restrict__ ys,
                                                          const int* __restrict__ xs, int nty, int ntx, int by, int bx,
                                                          const float* __restrict__ wy, const float* __restrict__ wx,
                                                          float* __restrict__ out) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = (long long)B * H * W;
  if (gid >= n) return;
  const int x = (int)(gid % W);
  const int y = (int)((gid / W) % H);
  const int b = (int)(gid / ((long long)H * W));
  const int yp = y + pad_y, xp = x + pad_x;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float wsum = 0.f;
  for (int i = 0; i < nty; ++i) {
    const int ty = yp - ys[i];
    if (ty < 0 || ty >= by) continue;
    for (int j = 0; j < ntx; ++j) {
      const int tx = xp - xs[j];
      if (tx < 0 || tx >= bx) continue;
      const float w = wy[ty] * wx[tx];
      wsum += w;
      const float* src = yt + (((size_t)b * nty * ntx + i * ntx + j) * nout) * by * bx + (size_t)ty * bx + tx;
      for (int c = 0; c < nout && c < 4; ++c) acc[c] += w * src[(size_t)c * by * bx];
    }
  }
  const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
  for (int c = 0; c < nout && c < 4; ++c) out[(((size_t)b * nout + c) * H + y) * W + x] = acc[c] * inv;
}

}  // namespace

extern "C" {

int be_tiles_gather(const float* img, int B, int C, int H, int W, int pad_y, int pad_x, const int* ys, const int* xs,
                    int nty, int ntx, int by, int bx, int cpad, void* out, hipStream_t s) {
  if (cpad % 8) return -1;
  const long long n = (long long)B * nty * ntx * by * bx;
  hipLaunchKernelGGL(tiles_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, img, B, C, H, W, pad_y, pad_x, ys,
                     xs, nty, ntx, by, bx, cpad, (bf16_t*)out);
  return BE_CHECK_LAUNCH();
}

int be_tiles_blend(const float* yt, int B, int nout, int H, int W, int pad_y, int pad_x, const int* ys, const int* xs, int nty,
                   int ntx, int by, int bx, const float* wy, const float* wx, float* out, hipStream_t s) {
  if (nout > 4) return -1;
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(tiles_blend_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, yt, B, nout, H, W, pad_y, pad_x,
                     ys, xs, nty, ntx, by, bx, wy, wx, out);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
