// Image pre-processing for the cell-image-search pipeline:
//
//  * connected-component labelling (8-connectivity, skimage.measure.label semantics) by lock-free
//    union-find: init -> merge (each foreground pixel unites with its W/NW/N/NE neighbours, roots
//    linked larger->smaller index with atomicMin) -> path compression.  The root of a component is
//    its first pixel in raster order, which is exactly skimage's label order.
//  * per-component area and centroid sums (regionprops area / centroid) with 64-bit atomics.
//  * percentile-stretch to uint8 + PIL-style separable bicubic resample (a = -0.5, antialiased
//    support when downscaling, 8-bit rounding between passes) + ImageNet normalisation, writing the
//    bf16 NCHW batch the ViT engine consumes (reference normalizer.py:32-153: percentile_stretch,
//    to_rgb_uint8, to_dinov2_tensor).
#include "common.h"

namespace {

// Find with path halving.  Concurrent halving stores only ever replace a parent by one of its
// ancestors, and a link they overwrite (an atomicMin that landed on a node which had just stopped
// being a root) is re-established by uf_unite's retry on the returned old value, so the forest stays
// a valid union-find; without it, chains through one giant component (a noisy probability mask)
// make every find O(n) and the merge effectively quadratic.
__device__ __forceinline__ int uf_find_ro(const int* L, int x) {
  int p = L[x];
  while (p != x) {
    x = p;
    p = L[x];
  }
  return x;
}

// (merge phase only: the compress pass uses the read-only find, or its final root stores would
// race with other threads' halving stores)
__device__ __forceinline__ int uf_find(int* L, int x) {
  int p = L[x];
  while (p != x) {
    const int gp = L[p];
    if (gp != p) L[x] = gp;
    x = p;
    p = gp;
  }
  return x;
}

__device__ __forceinline__ void uf_unite(int* L, int a, int b) {
  for (;;) {
    a = uf_find(L, a);
    b = uf_find(L, b);
    if (a == b) return;
    if (a > b) { const int t = a; a = b; b = t; }
    const int old = atomicMin(&L[b], a);
    if (old == b) return;
    b = old;
  }
}

__global__ void ccl_init(const unsigned char* __restrict__ mask, int* __restrict__ L, long long n, long long HW) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) L[i] = mask[i] ? (int)(i % HW) : -1;
}

// images are stacked [B, H, W]; labels are linear indices within each image's slab
__global__ void ccl_merge(const unsigned char* __restrict__ mask, int* __restrict__ Lall, int B, int H, int W, int conn8) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (gid >= B * HW) return;
  if (!mask[gid]) return;
  const int b = (int)(gid / HW);
  const int p = (int)(gid % HW);
  const int y = p / W, x = p % W;
  int* L = Lall + b * HW;
  const unsigned char* m = mask + b * HW;
  if (x > 0 && m[p - 1]) uf_unite(L, p, p - 1);
  if (y > 0) {
    if (m[p - W]) uf_unite(L, p, p - W);
    if (conn8) {
      if (x > 0 && m[p - W - 1]) uf_unite(L, p, p - W - 1);
      if (x < W - 1 && m[p - W + 1]) uf_unite(L, p, p - W + 1);
    }
  }
}

__global__ void ccl_compress(int* __restrict__ Lall, int B, long long HW) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * HW) return;
  int* L = Lall + (gid / HW) * HW;
  const int p = (int)(gid % HW);
  if (L[p] >= 0) L[p] = uf_find_ro(L, p);
}

// 3-D, 6-connectivity (face neighbours); volume < 2^31 voxels (a z-slab per rank)
__global__ void ccl3d_merge(const unsigned char* __restrict__ m, int* __restrict__ L, int D, int H, int W) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (p >= D * HW || !m[p]) return;
  const int z = (int)(p / HW), y = (int)((p / W) % H), x = (int)(p % W);
  if (x > 0 && m[p - 1]) uf_unite(L, (int)p, (int)(p - 1));
  if (y > 0 && m[p - W]) uf_unite(L, (int)p, (int)(p - W));
  if (z > 0 && m[p - HW]) uf_unite(L, (int)p, (int)(p - HW));
}

// stats [B*HW, 3] int64: area, sum_y, sum_x indexed by root
__global__ void region_stats(const int* __restrict__ Lall, int B, int H, int W, unsigned long long* __restrict__ stats) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (gid >= B * HW) return;
  const int r = Lall[gid];
  if (r < 0) return;
  const int p = (int)(gid % HW);
  unsigned long long* s = stats + ((gid / HW) * HW + r) * 3;
  atomicAdd(s, 1ull);
  atomicAdd(s + 1, (unsigned long long)(p / W));
  atomicAdd(s + 2, (unsigned long long)(p % W));
}

// x: float [n, h, w, C] (channel-last), chan[3]: source channel per RGB output (-1 = mean of ch0/ch1),
// lo/hi: float [n, 3] percentiles; out: uint8 [n, 3, h, w]
__global__ void stretch_u8(const float* __restrict__ x, int n, int h, int w, int C, const int* __restrict__ chan,
                           const float* __restrict__ lo, const float* __restrict__ hi, unsigned char* __restrict__ out) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long hw = (long long)h * w;
  if (gid >= (long long)n * 3 * hw) return;
  const int i = (int)(gid / (3 * hw));
  const int c = (int)((gid / hw) % 3);
  const long long p = gid % hw;
  const float* px = x + ((long long)i * hw + p) * C;
  const int sc = chan[c];
  const float v = sc >= 0 ? px[sc] : (px[0] + px[1]) * 0.5f;
  const float l = lo[i * 3 + c];
  float hh = hi[i * 3 + c];
  if (hh <= l) hh = l + 1.0f;
  float t = (v - l) / (hh - l);
  t = fminf(fmaxf(t, 0.f), 1.f) * 255.f;
  out[gid] = (unsigned char)t;  // astype(uint8): truncation
}

// separable resample pass over uint8 planes: horizontal (along w) when horiz, else vertical.
// weights: [out_len, K] float (normalised), start: [out_len] int
__global__ void resample_u8(const unsigned char* __restrict__ in, int planes, int ih, int iw, int oh, int ow,
                            const float* __restrict__ wts, const int* __restrict__ start, int K, int horiz,
                            unsigned char* __restrict__ out) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long ohw = (long long)oh * ow;
  if (gid >= planes * ohw) return;
  const int pl = (int)(gid / ohw);
  const int oy = (int)((gid % ohw) / ow), ox = (int)(gid % ow);
  const unsigned char* src = in + (long long)pl * ih * iw;
  float acc = 0.f;
  if (horiz) {
    const int s0 = start[ox];
    for (int k = 0; k < K; ++k) {
      const float wk = wts[ox * K + k];
      if (wk != 0.f) acc += wk * (float)src[oy * iw + min(s0 + k, iw - 1)];
    }
  } else {
    const int s0 = start[oy];
    for (int k = 0; k < K; ++k) {
      const float wk = wts[oy * K + k];
      if (wk != 0.f) acc += wk * (float)src[min(s0 + k, ih - 1) * iw + ox];
    }
  }
  acc = fminf(fmaxf(rintf(acc), 0.f), 255.f);
  out[gid] = (unsigned char)acc;
}

// uint8 [n, 3, S, S] -> bf16 (v/255 - mean) / std
__global__ void imagenet_norm(const unsigned char* __restrict__ in, long long n3ss, long long ss, bf16_t* __restrict__ out) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n3ss) return;
  const int c = (int)((gid / ss) % 3);
  const float mean = c == 0 ? 0.485f : (c == 1 ? 0.456f : 0.406f);
  const float stdv = c == 0 ? 0.229f : (c == 1 ? 0.224f : 0.225f);
  out[gid] = f2bf(((float)in[gid] / 255.f - mean) / stdv);
}

inline unsigned nblk(long long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

// Bilinear resize of fp32 planes with torch's align_corners=False convention (cellpose resizes
// images to the model diameter and the flows back with cv2/torch bilinear; reference
// cellpose/transforms.py resize_image): src = max(0, (dst + 0.5) * in / out - 0.5), edge-clamped
// right/bottom neighbour.  One lane per output pixel; consecutive lanes along x read neighbouring
// source texels of one or two rows (L2 / L1 friendly).
__global__ void resize_bilinear_f32(const float* __restrict__ in, float* __restrict__ out, long long planes, int ih,
                                    int iw, int oh, int ow) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long n = planes * oh * ow;
  if (gid >= n) return;
  const int ox = (int)(gid % ow);
  const int oy = (int)((gid / ow) % oh);
  const long long pl = gid / ((long long)oh * ow);
  const float ry = (float)ih / (float)oh, rx = (float)iw / (float)ow;
  float sy = ry * ((float)oy + 0.5f) - 0.5f;
  float sx = rx * ((float)ox + 0.5f) - 0.5f;
  sy = sy < 0.f ? 0.f : sy;
  sx = sx < 0.f ? 0.f : sx;
  const int y0 = (int)sy, x0 = (int)sx;
  const int yp = y0 < ih - 1 ? 1 : 0, xp = x0 < iw - 1 ? 1 : 0;
  const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
  const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
  const float* p = in + pl * ih * iw;
  const float* r0 = p + (long long)y0 * iw + x0;
  const float* r1 = r0 + (long long)yp * iw;
  out[gid] = ly0 * (lx0 * r0[0] + lx1 * r0[xp]) + ly1 * (lx0 * r1[0] + lx1 * r1[xp]);
}

extern "C" {

// in [planes, ih, iw] fp32 -> out [planes, oh, ow] fp32.
int be_resize_bilinear(const float* in, float* out, long long planes, int ih, int iw, int oh, int ow, hipStream_t s) {
  const long long n = planes * oh * ow;
  if (n == 0) return 0;
  if (ih <= 0 || iw <= 0 || oh <= 0 || ow <= 0) return -1;
  hipLaunchKernelGGL(resize_bilinear_f32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, planes, ih, iw,
                     oh, ow);
  return BE_CHECK_LAUNCH();
}


// mask uint8 [B, H, W] -> labels int32 [B, H, W] (root linear index within the image, -1 background)
int be_ccl_conn(const void* mask, int B, int H, int W, int conn, int* labels, hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(ccl_init, dim3(nblk(n)), dim3(256), 0, s, (const unsigned char*)mask, labels, n, (long long)H * W);
  hipLaunchKernelGGL(ccl_merge, dim3(nblk(n)), dim3(256), 0, s, (const unsigned char*)mask, labels, B, H, W,
                     conn == 8 ? 1 : 0);
  hipLaunchKernelGGL(ccl_compress, dim3(nblk(n)), dim3(256), 0, s, labels, B, (long long)H * W);
  return BE_CHECK_LAUNCH();
}

int be_ccl3d(const void* mask, int D, int H, int W, int* labels, hipStream_t s) {
  const long long n = (long long)D * H * W;
  if (n == 0) return 0;
  if (n >= (1ll << 31)) return -1;
  hipLaunchKernelGGL(ccl_init, dim3(nblk(n)), dim3(256), 0, s, (const unsigned char*)mask, labels, n, n);
  hipLaunchKernelGGL(ccl3d_merge, dim3(nblk(n)), dim3(256), 0, s, (const unsigned char*)mask, labels, D, H, W);
  hipLaunchKernelGGL(ccl_compress, dim3(nblk(n)), dim3(256), 0, s, labels, 1, n);
  return BE_CHECK_LAUNCH();
}

int be_ccl(const void* mask, int B, int H, int W, int* labels, hipStream_t s) {
  return be_ccl_conn(mask, B, H, W, 8, labels, s);
}

int be_region_stats(const int* labels, int B, int H, int W, void* stats, hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(region_stats, dim3(nblk(n)), dim3(256), 0, s, labels, B, H, W, (unsigned long long*)stats);
  return BE_CHECK_LAUNCH();
}

int be_stretch_u8(const float* x, int n, int h, int w, int C, const int* chan, const float* lo, const float* hi,
                  void* out, hipStream_t s) {
  const long long tot = (long long)n * 3 * h * w;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(stretch_u8, dim3(nblk(tot)), dim3(256), 0, s, x, n, h, w, C, chan, lo, hi, (unsigned char*)out);
  return BE_CHECK_LAUNCH();
}

int be_resample_u8(const void* in, int planes, int ih, int iw, int oh, int ow, const float* wts, const int* start,
                   int K, int horiz, void* out, hipStream_t s) {
  const long long tot = (long long)planes * oh * ow;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(resample_u8, dim3(nblk(tot)), dim3(256), 0, s, (const unsigned char*)in, planes, ih, iw, oh, ow,
                     wts, start, K, horiz, (unsigned char*)out);
  return BE_CHECK_LAUNCH();
}

int be_imagenet_norm(const void* in, int n, int S, void* out, hipStream_t s) {
  const long long tot = (long long)n * 3 * S * S;
  if (tot == 0) return 0;
  hipLaunchKernelGGL(imagenet_norm, dim3(nblk(tot)), dim3(256), 0, s, (const unsigned char*)in, tot, (long long)S * S,
                     (bf16_t*)out);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
