// EM mitochondria post-processing and tiled-inference stitching (reference
// apps/fibsem-mito-analysis/analysis_deployment.py:108-176, 256-271):
//
//  * blend_gather   — Gaussian-window weighted stitching of overlapping tile predictions.  Gather
//                     form: each output pixel sums the (<= 2^d) tiles covering it in registers, so
//                     there are no atomics and the result is deterministic (the reference
//                     accumulates in float64 with scatter adds).  2-D and 3-D.
//  * morph_disk     — binary dilation / erosion with a disk footprint (scipy.ndimage semantics,
//                     out-of-image samples = border_value); closing = dilate then erode.
//  * edt            — exact Euclidean distance transform (scipy distance_transform_edt): a
//                     column pass (distance to the nearest background pixel along y) and a row pass
//                     computing the lower envelope of parabolas (Felzenszwalb-Huttenlocher), one
//                     thread per row/column.
//  * max_filter_1d  — separable square maximum filter (mode='nearest'), for peak_local_max.
//  * label_moments  — per-label area / first / second moments in fp64 (regionprops area,
//                     centroid, inertia tensor -> axis lengths, eccentricity).
#include "common.h"

namespace {

inline unsigned nblk(long long n) { return (unsigned)((n + 255) / 256); }

// probs [T, C, tile, tile(, tile)] tile t = (iz*ny + iy)*nx + ix at (iz, iy, ix) * stride; out [C, D, H, W]
__global__ void blend_gather(const float* __restrict__ probs, int C, int D, int H, int W, int nz, int ny, int nx,
                             int stride, int stride_z, int tz, int tile, const float* __restrict__ wz,
                             const float* __restrict__ wy, const float* __restrict__ wx, float* __restrict__ out) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long vox = (long long)D * H * W;
  if (gid >= vox) return;
  const int z = (int)(gid / ((long long)H * W));
  const int y = (int)((gid / W) % H);
  const int x = (int)(gid % W);
  const int sz = D > 1 ? stride_z : 1;  // z tiles (3-D models): own depth tz and z overlap
  const int iz1 = min(z / sz, nz - 1), iy1 = min(y / stride, ny - 1), ix1 = min(x / stride, nx - 1);
  // first tile whose extent [i*stride, i*stride + tile) still contains the pixel (floor division)
  const int iz0 = (D > 1 && z >= tz) ? (z - tz) / sz + 1 : 0;
  const int iy0 = y >= tile ? (y - tile) / stride + 1 : 0;
  const int ix0 = x >= tile ? (x - tile) / stride + 1 : 0;
  const long long tvol = (long long)(D > 1 ? tz : 1) * tile * tile;
  for (int c = 0; c < C; ++c) {
    float acc = 0.f, wacc = 0.f;
    for (int iz = iz0; iz <= iz1; ++iz) {
      const int lz = z - iz * sz;
      if (lz < 0 || lz >= (D > 1 ? tz : 1)) continue;
      const float fz = D > 1 ? wz[lz] : 1.f;
      for (int iy = iy0; iy <= iy1; ++iy) {
        const int ly = y - iy * stride;
        if (ly < 0 || ly >= tile) continue;
        for (int ix = ix0; ix <= ix1; ++ix) {
          const int lx = x - ix * stride;
          if (lx < 0 || lx >= tile) continue;
          const float w = fz * wy[ly] * wx[lx];
          const long long t = ((long long)iz * ny + iy) * nx + ix;
          acc += w * probs[(t * C + c) * tvol + ((long long)lz * tile + ly) * tile + lx];
          wacc += w;
        }
      }
    }
    out[c * vox + gid] = wacc > 0.f ? acc / wacc : 0.f;
  }
}

// op 0: dilation (any), op 1: erosion (all); footprint: |dy|^2 + |dx|^2 <= r^2
__global__ void morph_disk(const unsigned char* __restrict__ in, unsigned char* __restrict__ out, int B, int H, int W,
                           int r, int op, int border_value) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (gid >= B * HW) return;
  const int y = (int)((gid % HW) / W), x = (int)(gid % W);
  const unsigned char* m = in + (gid / HW) * HW;
  const int r2 = r * r;
  bool res = op == 1;
  for (int dy = -r; dy <= r; ++dy) {
    for (int dx = -r; dx <= r; ++dx) {
      if (dy * dy + dx * dx > r2) continue;
      const int yy = y + dy, xx = x + dx;
      const bool v = (yy >= 0 && yy < H && xx >= 0 && xx < W) ? (m[yy * W + xx] != 0) : (border_value != 0);
      if (op == 0 && v) { res = true; dy = r + 1; break; }
      if (op == 1 && !v) { res = false; dy = r + 1; break; }
    }
  }
  out[gid] = res ? 1 : 0;
}

// Bit-packed disk morphology: 64 pixels of a row per 64-bit word.  A footprint row dy covers
// dx in [-w, w], w = floor(sqrt(r^2 - dy^2)); its contribution to a word is the OR (dilation) /
// AND (erosion) of the word shifted by every dx, with the neighbouring words supplying the bits
// that cross the word edge.  Pixels outside the image read as border_value, exactly like
// morph_disk -- whose per-pixel loop over the (2r+1)^2 window took 0.13 s for the closing of a
// 256 x 2048^2 slab; this costs ~2 bit operations per pixel.
__device__ __forceinline__ unsigned long long mb_word(const unsigned long long* __restrict__ row, int k, int nwd, int W,
                                                      bool row_in, int border) {
  const unsigned long long bv = border ? ~0ull : 0ull;
  if (!row_in || k < 0 || k >= nwd) return bv;
  unsigned long long w = row[k];
  const int valid = W - 64 * k;  // pixels of this word inside the image
  if (valid < 64) {
    const unsigned long long m = (1ull << valid) - 1ull;
    w = (w & m) | (bv & ~m);
  }
  return w;
}

__global__ __launch_bounds__(256) void pack_bits_kernel(const unsigned char* __restrict__ in, unsigned long long* __restrict__ out,
                                                        long long rows, int W, int nwd) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= rows * nwd) return;
  const long long row = g / nwd;
  const int k = (int)(g % nwd);
  const unsigned char* p = in + row * W + 64 * k;
  const int n = min(64, W - 64 * k);
  unsigned long long w = 0;
  for (int i = 0; i < n; ++i) w |= (unsigned long long)(p[i] != 0) << i;
  out[g] = w;
}

__global__ __launch_bounds__(256) void unpack_bits_kernel(const unsigned long long* __restrict__ in, unsigned char* __restrict__ out,
                                                          long long rows, int W, int nwd) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= rows * W) return;
  const long long row = g / W;
  const int x = (int)(g % W);
  out[g] = (unsigned char)((in[row * nwd + (x >> 6)] >> (x & 63)) & 1ull);
}

__global__ __launch_bounds__(256) void morph_disk_bits_kernel(const unsigned long long* __restrict__ in,
                                                              unsigned long long* __restrict__ out, int B, int H, int W,
                                                              int nwd, int r, int op, int border) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)B * H * nwd) return;
  const int k = (int)(g % nwd);
  const long long by = g / nwd;
  const int y = (int)(by % H);
  const unsigned long long* base = in + (by - y) * nwd;  // slice start
  unsigned long long acc = op == 1 ? ~0ull : 0ull;
  for (int dy = -r; dy <= r; ++dy) {
    int w = 0;
    while ((w + 1) * (w + 1) + dy * dy <= r * r) ++w;
    const int yy = y + dy;
    const bool rin = yy >= 0 && yy < H;
    const unsigned long long* row = base + (long long)(rin ? yy : 0) * nwd;
    const unsigned long long p = mb_word(row, k - 1, nwd, W, rin, border);
    const unsigned long long c = mb_word(row, k, nwd, W, rin, border);
    const unsigned long long n = mb_word(row, k + 1, nwd, W, rin, border);
    unsigned long long v = c;
    for (int s = 1; s <= w; ++s) {
      // bit x of the result needs pixel x + s (from c, then n) and pixel x - s (from c, then p)
      const unsigned long long right = (c >> s) | (n << (64 - s));
      const unsigned long long left = (c << s) | (p >> (64 - s));
      v = op == 1 ? (v & right & left) : (v | right | left);
    }
    acc = op == 1 ? (acc & v) : (acc | v);
  }
  out[g] = acc;
}

// column pass: g[y, x] = (distance along y to the nearest background pixel)^2 (int), or -1 = none
__global__ void edt_cols(const unsigned char* __restrict__ fg, int* __restrict__ g, int B, int H, int W) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * W) return;
  const int b = (int)(gid / W), x = (int)(gid % W);
  const unsigned char* m = fg + (long long)b * H * W;
  int* gg = g + (long long)b * H * W;
  int last = -1;
  for (int y = 0; y < H; ++y) {
    if (!m[y * W + x]) last = y;
    gg[y * W + x] = last < 0 ? -1 : (y - last);
  }
  last = -1;
  for (int y = H - 1; y >= 0; --y) {
    if (!m[y * W + x]) last = y;
    int d = gg[y * W + x];
    if (last >= 0 && (d < 0 || last - y < d)) d = last - y;
    gg[y * W + x] = d < 0 ? -1 : d * d;
  }
}

// row pass: out[y, x] = sqrt(min_x' g[y, x'] + (x - x')^2) (lower envelope of parabolas, fp64
// intersections so 4k+ rows stay exact); v int / z double scratch [B*H, W] / [B*H, W+1]
// Row pass, one thread per PIXEL: d(q) = min_p (q - p)^2 + g(p), searched outwards from q until
// r^2 reaches the best value (every farther site is at least r^2): a few steps for thin EM
// foreground, neighbouring threads on neighbouring addresses.  A pixel whose search passes
// EDT2_RCAP flags its row, and edt_rows (the lower envelope) redoes exactly those rows -- as
// be_edt3d does; squared distances are exact integers, so the transform is unchanged.
constexpr int EDT2_RCAP = 64;
__global__ __launch_bounds__(256) void edt_rows_bf(const int* __restrict__ g, float* __restrict__ out, int B, int H, int W,
                                                   unsigned char* __restrict__ only) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * H * W) return;
  const long long row = gid / W;
  const int q = (int)(gid - row * W);
  const int* f = g + row * W;
  const int NONE = 0x7fffffff;
  int best = f[q] < 0 ? NONE : f[q];
  const int rmax = max(q, W - 1 - q);
  int r = 1;
  for (; r <= rmax && r <= EDT2_RCAP; ++r) {
    const int r2 = r * r;
    if (r2 >= best) break;
    if (q - r >= 0 && f[q - r] >= 0) best = min(best, r2 + f[q - r]);
    if (q + r < W && f[q + r] >= 0) best = min(best, r2 + f[q + r]);
  }
  if (r > EDT2_RCAP && r <= rmax && r * r < best) only[row] = 1;
  out[gid] = best == NONE ? 3.4e38f : (float)sqrt((double)best);
}

__global__ void edt_rows(const int* __restrict__ g, float* __restrict__ out, int* __restrict__ vbuf,
                         double* __restrict__ zbuf, int B, int H, int W, const unsigned char* __restrict__ only = nullptr) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * H) return;
  if (only && !only[gid]) return;
  const int* f = g + gid * W;
  float* o = out + gid * W;
  int* v = vbuf + gid * W;
  double* z = zbuf + gid * (W + 1);
  int k = -1;
  for (int q = 0; q < W; ++q) {
    if (f[q] < 0) continue;
    if (k < 0) {
      k = 0; v[0] = q; z[0] = -1e300; z[1] = 1e300;
      continue;
    }
    double s;
    for (;;) {
      const int p = v[k];
      s = ((double)f[q] + (double)q * q - ((double)f[p] + (double)p * p)) / (2.0 * (q - p));
      if (s <= z[k] && k > 0) { --k; continue; }
      break;
    }
    ++k; v[k] = q; z[k] = s; z[k + 1] = 1e300;
  }
  if (k < 0) {
    for (int q = 0; q < W; ++q) o[q] = 3.4e38f;
    return;
  }
  int j = 0;
  for (int q = 0; q < W; ++q) {
    while (z[j + 1] < (double)q) ++j;
    const double d = (double)(q - v[j]);
    o[q] = (float)sqrt(d * d + (double)f[v[j]]);
  }
}

// separable max filter, mode='nearest' (clamped indices); axis 0: along x, 1: along y
__global__ void max_filter_1d(const float* __restrict__ in, float* __restrict__ out, int B, int H, int W, int r, int axis) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (gid >= B * HW) return;
  const float* m = in + (gid / HW) * HW;
  const int y = (int)((gid % HW) / W), x = (int)(gid % W);
  float mx = -3.4e38f;
  if (axis == 0) {
    for (int d = -r; d <= r; ++d) mx = fmaxf(mx, m[y * W + min(max(x + d, 0), W - 1)]);
  } else {
    for (int d = -r; d <= r; ++d) mx = fmaxf(mx, m[min(max(y + d, 0), H - 1) * W + x]);
  }
  out[gid] = mx;
}

// mom [B, nlab, 6] fp64: n, sy, sx, syy, sxx, sxy (label 0 skipped)
__global__ void label_moments(const int* __restrict__ lab, int B, int H, int W, int nlab, double* __restrict__ mom) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long HW = (long long)H * W;
  if (gid >= B * HW) return;
  const int l = lab[gid];
  if (l <= 0 || l >= nlab) return;
  const double y = (double)((gid % HW) / W), x = (double)(gid % W);
  double* m = mom + ((gid / HW) * nlab + l) * 6;
  atomicAdd(m + 0, 1.0);
  atomicAdd(m + 1, y);
  atomicAdd(m + 2, x);
  atomicAdd(m + 3, y * y);
  atomicAdd(m + 4, x * x);
  atomicAdd(m + 5, x * y);
}

}  // namespace

extern "C" {

int be_blend_gather(const float* probs, int C, int D, int H, int W, int nz, int ny, int nx, int stride, int stride_z,
                    int tz, int tile, const float* wz, const float* wy, const float* wx, float* out, hipStream_t s) {
  const long long vox = (long long)D * H * W;
  if (vox == 0) return 0;
  hipLaunchKernelGGL(blend_gather, dim3(nblk(vox)), dim3(256), 0, s, probs, C, D, H, W, nz, ny, nx, stride, stride_z, tz,
                     tile, wz, wy, wx, out);
  return BE_CHECK_LAUNCH();
}

int be_morph_disk(const void* in, void* out, int B, int H, int W, int r, int op, int border_value, hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(morph_disk, dim3(nblk(n)), dim3(256), 0, s, (const unsigned char*)in, (unsigned char*)out, B, H, W,
                     r, op, border_value);
  return BE_CHECK_LAUNCH();
}

// Closing (dilation then erosion) of B slices [H, W] uint8 with a radius-r disk on the bit-packed
// form; bits: 2 * B * H * ceil(W / 64) uint64 of scratch.  Same result as two be_morph_disk calls.
// r < 64 (a shift never crosses more than one word).
int be_closing_disk_bits(const void* in, void* out, unsigned long long* bits, int B, int H, int W, int r, int border_value,
                         hipStream_t s) {
  const long long rows = (long long)B * H;
  if (rows * W == 0) return 0;
  if (r < 0 || r >= 64) return -1;
  const int nwd = (W + 63) / 64;
  const long long nw = rows * nwd;
  unsigned long long* a = bits;
  unsigned long long* b = bits + nw;
  hipLaunchKernelGGL(pack_bits_kernel, dim3(nblk(nw)), dim3(256), 0, s, (const unsigned char*)in, a, rows, W, nwd);
  hipLaunchKernelGGL(morph_disk_bits_kernel, dim3(nblk(nw)), dim3(256), 0, s, a, b, B, H, W, nwd, r, 0, border_value);
  hipLaunchKernelGGL(morph_disk_bits_kernel, dim3(nblk(nw)), dim3(256), 0, s, b, a, B, H, W, nwd, r, 1, border_value);
  hipLaunchKernelGGL(unpack_bits_kernel, dim3(nblk(rows * W)), dim3(256), 0, s, a, (unsigned char*)out, rows, W, nwd);
  return BE_CHECK_LAUNCH();
}

// fg uint8 [B, H, W] -> dist f32 [B, H, W]; scratch: g int [B*H*W], v int [B*H*W + B*H] (the
// tail holds the per-row fallback flags), z f64 [B*H*(W+1)]
int be_edt(const void* fg, float* dist, int* g, int* v, double* z, int B, int H, int W, hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  unsigned char* only = reinterpret_cast<unsigned char*>(v + n);
  hipLaunchKernelGGL(edt_cols, dim3(nblk((long long)B * W)), dim3(256), 0, s, (const unsigned char*)fg, g, B, H, W);
  (void)hipMemsetAsync(only, 0, (size_t)B * H, s);
  hipLaunchKernelGGL(edt_rows_bf, dim3(nblk(n)), dim3(256), 0, s, g, dist, B, H, W, only);
  hipLaunchKernelGGL(edt_rows, dim3(nblk((long long)B * H)), dim3(256), 0, s, g, dist, v, z, B, H, W, only);
  return BE_CHECK_LAUNCH();
}

int be_max_filter_1d(const float* in, float* out, int B, int H, int W, int r, int axis, hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(max_filter_1d, dim3(nblk(n)), dim3(256), 0, s, in, out, B, H, W, r, axis);
  return BE_CHECK_LAUNCH();
}

int be_label_moments(const int* lab, int B, int H, int W, int nlab, double* mom, hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(label_moments, dim3(nblk(n)), dim3(256), 0, s, lab, B, H, W, nlab, mom);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
