// Cellpose mask recovery on the GPU: flow following + histogram seeds + seed expansion + labels.
//
// Semantics follow the Cellpose algorithm (cellpose 3 dynamics.compute_masks / follow_flows /
// get_masks_torch, EXT; invoked by the reference through model.eval(..., niter, cellprob_threshold)
// at apps/cellpose-finetuning/main.py:3559-3567 and the model-runner cellpose pin), re-derived and
// checked against bioengine_worker_amd/cellpose/reference.py.  SURVEY.md §2.5 K3/K4.
//
// MI355X mapping:
//  * follow_flows: one lane per foreground pixel runs all `niter` Euler steps with its position in
//    registers; the (dy, dx) field is an interleaved float2 image (one 8-byte gather per bilinear
//    corner) that stays L2/MALL-resident across the steps.  The end point is binned straight into
//    the padded histogram with an integer atomic, so no point list round-trips through HBM.
//  * seeds: 5x5 local-max test on the histogram, compacted with one atomic per seed into a per-image
//    key list (count << 32 | raster index) that torch.sort orders exactly like cellpose's argsort.
//  * expansion: one wave per seed, its 11x11 window in LDS, 5 dilations, labels committed with
//    atomicMax (seeds are rank-ordered by count, so "last writer wins" == max rank).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int RPAD = 20;

__device__ __forceinline__ float2 ldflow(const float2* __restrict__ f, int H, int W, int y, int x) {
  if (y < 0 || y >= H || x < 0 || x >= W) return make_float2(0.f, 0.f);
  return f[y * W + x];
}

// flow2: [B, H, W] float2 (dy, dx) already masked by cellprob > thr and divided by 5.
// fg: [B, H, W] uint8.  hist: [B, H+2R, W+2R] int32 (zeroed).  pos: [B, H, W] int32 (-1 for bg).
__global__ __launch_bounds__(256) void follow_flows_kernel(const float2* __restrict__ flow2, const uint8_t* __restrict__ fg,
                                                           int* __restrict__ hist, int* __restrict__ pos, int B, int H,
                                                           int W, int niter) {
  const int HW = H * W;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * HW) return;
  const int b = (int)(gid / HW);
  const int pix = (int)(gid % HW);
  if (!fg[gid]) {
    pos[gid] = -1;
    return;
  }
  const float2* f = flow2 + (size_t)b * HW;
  float py = (float)(pix / W), px = (float)(pix % W);
  const float sy_scale = (H > 1) ? (float)H / (float)(H - 1) : 0.f;
  const float sx_scale = (W > 1) ? (float)W / (float)(W - 1) : 0.f;
  const float ymax = (float)(H - 1), xmax = (float)(W - 1);
  for (int t = 0; t < niter; ++t) {
    // grid_sample(align_corners=False) position for normalised coordinate 2p/(L-1)-1
    const float sy = py * sy_scale - 0.5f;
    const float sx = px * sx_scale - 0.5f;
    const float fy = floorf(sy), fx = floorf(sx);
    const int y0 = (int)fy, x0 = (int)fx;
    const float wy = sy - fy, wx = sx - fx;
    const float2 a = ldflow(f, H, W, y0, x0);
    const float2 bq = ldflow(f, H, W, y0, x0 + 1);
    const float2 c = ldflow(f, H, W, y0 + 1, x0);
    const float2 d = ldflow(f, H, W, y0 + 1, x0 + 1);
    const float w00 = (1.f - wy) * (1.f - wx), w01 = (1.f - wy) * wx, w10 = wy * (1.f - wx), w11 = wy * wx;
    const float dy = a.x * w00 + bq.x * w01 + c.x * w10 + d.x * w11;
    const float dx = a.y * w00 + bq.y * w01 + c.y * w10 + d.y * w11;
    py = fminf(fmaxf(py + dy, 0.f), ymax);
    px = fminf(fmaxf(px + dx, 0.f), xmax);
  }
  const int Wp = W + 2 * RPAD;
  int iy = (int)py + RPAD, ix = (int)px + RPAD;
  iy = min(max(iy, 0), H + RPAD - 1);
  ix = min(max(ix, 0), W + RPAD - 1);
  const int lin = iy * Wp + ix;
  pos[gid] = lin;
  atomicAdd(hist + (size_t)b * (H + 2 * RPAD) * Wp + lin, 1);
}

// follow_flows, MI355X layout: (1) XCD-aware block order — block ids are remapped so every XCD
// walks a contiguous range of images, one image's 2 MB flow field at a time in its private 4 MB
// L2 (round-robin dispatch would stream all B fields through every L2); (2) block-local
// foreground compaction — the block's 256 pixels are compacted in LDS so the Euler loop runs on
// full waves (at ~12 % foreground a pixel-per-lane launch runs 200 steps on mostly masked lanes).
__global__ __launch_bounds__(256) void follow_flows_xcd_kernel(const float2* __restrict__ flow2,
                                                               const uint8_t* __restrict__ fg, int* __restrict__ hist,
                                                               int* __restrict__ pos, int B, int H, int W, int niter) {
  __shared__ int list[256];
  __shared__ int wcount[4];
  const int HW = H * W;
  const long long n = (long long)B * HW;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const long long gid0 = (long long)blk * 256;
  const long long gid = gid0 + threadIdx.x;
  const bool in = gid < n;
  const bool f = in && fg[gid];
  if (in && !f) pos[gid] = -1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long m = __ballot(f);
  if (lane == 0) wcount[wv] = __popcll(m);
  __syncthreads();
  int base = 0;
  for (int i = 0; i < wv; ++i) base += wcount[i];
  const int total = wcount[0] + wcount[1] + wcount[2] + wcount[3];
  if (f) list[base + __popcll(m & ((1ull << lane) - 1ull))] = threadIdx.x;
  __syncthreads();
  if ((int)threadIdx.x >= total) return;
  const long long g = gid0 + list[threadIdx.x];
  const int b = (int)(g / HW);
  const int pix = (int)(g % HW);
  const float2* fl = flow2 + (size_t)b * HW;
  float py = (float)(pix / W), px = (float)(pix % W);
  const float sy_scale = (H > 1) ? (float)H / (float)(H - 1) : 0.f;
  const float sx_scale = (W > 1) ? (float)W / (float)(W - 1) : 0.f;
  const float ymax = (float)(H - 1), xmax = (float)(W - 1);
  for (int t = 0; t < niter; ++t) {
    const float sy = py * sy_scale - 0.5f;
    const float sx = px * sx_scale - 0.5f;
    const float fy = floorf(sy), fx = floorf(sx);
    const int y0 = (int)fy, x0 = (int)fx;
    const float wy = sy - fy, wx = sx - fx;
    const float2 a = ldflow(fl, H, W, y0, x0);
    const float2 bq = ldflow(fl, H, W, y0, x0 + 1);
    const float2 c = ldflow(fl, H, W, y0 + 1, x0);
    const float2 d = ldflow(fl, H, W, y0 + 1, x0 + 1);
    const float w00 = (1.f - wy) * (1.f - wx), w01 = (1.f - wy) * wx, w10 = wy * (1.f - wx), w11 = wy * wx;
    const float dy = a.x * w00 + bq.x * w01 + c.x * w10 + d.x * w11;
    const float dx = a.y * w00 + bq.y * w01 + c.y * w10 + d.y * w11;
    py = fminf(fmaxf(py + dy, 0.f), ymax);
    px = fminf(fmaxf(px + dx, 0.f), xmax);
  }
  const int Wp = W + 2 * RPAD;
  int iy = (int)py + RPAD, ix = (int)px + RPAD;
  iy = min(max(iy, 0), H + RPAD - 1);
  ix = min(max(ix, 0), W + RPAD - 1);
  const int lin = iy * Wp + ix;
  pos[g] = lin;
  atomicAdd(hist + (size_t)b * (H + 2 * RPAD) * Wp + lin, 1);
}

// Same, with PPT x 256 pixels per block compacted together: at the ~12 % foreground of a Cellpose
// batch a 256-pixel block leaves ~31 live lanes in one wave, so every Euler step issued its four
// float2 gathers for a half-empty wave (the loop is bound by gather issue, not by latency).  Pooling
// 1,024 pixels gives ~2 full waves per block.  Each pixel's result is independent of the order the
// list is walked in (integer histogram atomics), so the output equals the 256-pixel kernel's.
template <int PPT>
__global__ __launch_bounds__(256) void follow_flows_xcd_pool_kernel(const float2* __restrict__ flow2,
                                                                    const uint8_t* __restrict__ fg, int* __restrict__ hist,
                                                                    int* __restrict__ pos, int B, int H, int W, int niter) {
  __shared__ int list[256 * PPT];
  __shared__ int wcount[4 * PPT];
  const int HW = H * W;
  const long long n = (long long)B * HW;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const long long gid0 = (long long)blk * (256 * PPT);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long m[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {  // coalesced: pass k covers pixels gid0 + k*256 + [0, 256)
    const long long g = gid0 + k * 256 + threadIdx.x;
    const bool in = g < n;
    const bool f = in && fg[g];
    if (in && !f) pos[g] = -1;
    m[k] = __ballot(f);
    if (lane == 0) wcount[k * 4 + wv] = __popcll(m[k]);
  }
  __syncthreads();
  int total = 0;
#pragma unroll
  for (int i = 0; i < 4 * PPT; ++i) total += wcount[i];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    int base = 0;
    for (int i = 0; i < k * 4 + wv; ++i) base += wcount[i];
    if ((m[k] >> lane) & 1ull) list[base + __popcll(m[k] & ((1ull << lane) - 1ull))] = k * 256 + threadIdx.x;
  }
  __syncthreads();
  const float sy_scale = (H > 1) ? (float)H / (float)(H - 1) : 0.f;
  const float sx_scale = (W > 1) ? (float)W / (float)(W - 1) : 0.f;
  const float ymax = (float)(H - 1), xmax = (float)(W - 1);
  const int Wp = W + 2 * RPAD;
  for (int e = threadIdx.x; e < total; e += 256) {
    const long long g = gid0 + list[e];
    const int b = (int)(g / HW);
    const int pix = (int)(g % HW);
    const float2* fl = flow2 + (size_t)b * HW;
    float py = (float)(pix / W), px = (float)(pix % W);
    for (int t = 0; t < niter; ++t) {
      const float sy = py * sy_scale - 0.5f;
      const float sx = px * sx_scale - 0.5f;
      const float fy = floorf(sy), fx = floorf(sx);
      const int y0 = (int)fy, x0 = (int)fx;
      const float wy = sy - fy, wx = sx - fx;
      const float2 a = ldflow(fl, H, W, y0, x0);
      const float2 bq = ldflow(fl, H, W, y0, x0 + 1);
      const float2 c = ldflow(fl, H, W, y0 + 1, x0);
      const float2 d = ldflow(fl, H, W, y0 + 1, x0 + 1);
      const float w00 = (1.f - wy) * (1.f - wx), w01 = (1.f - wy) * wx, w10 = wy * (1.f - wx), w11 = wy * wx;
      const float dy = a.x * w00 + bq.x * w01 + c.x * w10 + d.x * w11;
      const float dx = a.y * w00 + bq.y * w01 + c.y * w10 + d.y * w11;
      py = fminf(fmaxf(py + dy, 0.f), ymax);
      px = fminf(fmaxf(px + dx, 0.f), xmax);
    }
    int iy = (int)py + RPAD, ix = (int)px + RPAD;
    iy = min(max(iy, 0), H + RPAD - 1);
    ix = min(max(ix, 0), W + RPAD - 1);
    const int lin = iy * Wp + ix;
    pos[g] = lin;
    atomicAdd(hist + (size_t)b * (H + 2 * RPAD) * Wp + lin, 1);
  }
}

// follow_flows with the flow field staged in LDS.  The XCD kernel above is bound by the latency
// of its dependent L2 gathers (position -> 4 bilinear corners -> next position, 200 times).  Here a
// workgroup owns a 32 x 32 pixel tile and stages the 64 x 64 window around it (16-pixel margin,
// zeros outside the image = ldflow's padding) in LDS once; a step whose 2 x 2 corner block lies in
// the window reads LDS (the (y, x) / (y + 1, x) pairs are one ds_read2_b64 each), a step outside it
// (a particle that travelled > 16 px past the tile) reads global memory as before.  Same float
// operations in the same order: results are bit-identical to follow_flows_kernel.
// FT = 16 (default: one pixel per thread, a 48 x 48 window) or 32 (1,024 pixels, up to four per
// thread, 64 x 64 window): at batch 1 the 32-pixel tiles ran each thread's pixels one after
// another (+0.3 ms latency), and at batch 32 their 37 KiB of LDS kept them off the CUs the convs
// of the next batch hold.
constexpr int FM = 16;

template <int FT>
__global__ __launch_bounds__(256) void follow_flows_lds_kernel(const float2* __restrict__ flow2,
                                                               const uint8_t* __restrict__ fg, int* __restrict__ hist,
                                                               int* __restrict__ pos, int B, int H, int W, int niter,
                                                               int tiles_x, int tiles_y) {
  constexpr int FWN = FT + 2 * FM, NP = FT * FT / 256;  // passes of 256 pixels
  // window row stride FWN + 1 float2 (odd in 8-byte units): with FWN, rows y and y + 2 (stride
  // 96 dwords = 32 mod 64 banks) or every row (FWN = 64: 128 dwords) shared their banks, and a
  // wave's corner reads -- lanes spread over the tile's rows -- measured 10 bank conflicts per LDS
  // instruction (profiles/r05/pmc/s35)
  constexpr int FWS = FWN + 1;
  constexpr int LG = FT == 32 ? 5 : 4;
  __shared__ float2 win[FWN * FWS];
  __shared__ short list[FT * FT];
  __shared__ int wcount[4 * NP];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);  // an XCD walks consecutive tiles of one image
  const int tpi = tiles_x * tiles_y;
  const int b = blk / tpi, q = blk - b * tpi;
  const int ty0 = (q / tiles_x) * FT, tx0 = (q % tiles_x) * FT;
  const size_t HW = (size_t)H * W;
  const uint8_t* fgb = fg + b * HW;
  int* posb = pos + b * HW;
  unsigned long long m[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {  // pass k: 256 pixels of whole tile rows (coalesced)
    const int p = k * 256 + tid;
    const int y = ty0 + (p >> LG), x = tx0 + (p & (FT - 1));
    const bool in = y < H && x < W;
    const bool f = in && fgb[(size_t)y * W + x];
    if (in && !f) posb[(size_t)y * W + x] = -1;
    m[k] = __ballot(f);
    if (lane == 0) wcount[k * 4 + wv] = __popcll(m[k]);
  }
  __syncthreads();
  int total = 0;
#pragma unroll
  for (int i = 0; i < 4 * NP; ++i) total += wcount[i];
  if (total == 0) return;  // workgroup-uniform
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    int base = 0;
    for (int i = 0; i < k * 4 + wv; ++i) base += wcount[i];
    if ((m[k] >> lane) & 1ull) list[base + __popcll(m[k] & ((1ull << lane) - 1ull))] = (short)(k * 256 + tid);
  }
  const float2* fl = flow2 + b * HW;
  const int wy0 = ty0 - FM, wx0 = tx0 - FM;
  for (int i = tid; i < FWN * FWN; i += 256) {
    const int wy = i / FWN, wx = i % FWN;
    const int gy = wy0 + wy, gx = wx0 + wx;
    win[wy * FWS + wx] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? fl[(size_t)gy * W + gx] : make_float2(0.f, 0.f);
  }
  __syncthreads();
  const float sy_scale = (H > 1) ? (float)H / (float)(H - 1) : 0.f;
  const float sx_scale = (W > 1) ? (float)W / (float)(W - 1) : 0.f;
  const float ymax = (float)(H - 1), xmax = (float)(W - 1);
  const int Wp = W + 2 * RPAD;
  for (int e = tid; e < total; e += 256) {
    const int p = list[e];
    const int y = ty0 + (p >> LG), x = tx0 + (p & (FT - 1));
    float py = (float)y, px = (float)x;
    for (int t = 0; t < niter; ++t) {
      const float sy = py * sy_scale - 0.5f;
      const float sx = px * sx_scale - 0.5f;
      const float fy = floorf(sy), fx = floorf(sx);
      const int y0 = (int)fy, x0 = (int)fx;
      const float wy = sy - fy, wx = sx - fx;
      const int ly = y0 - wy0, lx = x0 - wx0;
      float2 a, bq, c, d;
      if ((unsigned)ly < (unsigned)(FWN - 1) && (unsigned)lx < (unsigned)(FWN - 1)) {
        const float2* w = win + ly * FWS + lx;
        a = w[0];
        bq = w[1];
        c = w[FWS];
        d = w[FWS + 1];
      } else {
        a = ldflow(fl, H, W, y0, x0);
        bq = ldflow(fl, H, W, y0, x0 + 1);
        c = ldflow(fl, H, W, y0 + 1, x0);
        d = ldflow(fl, H, W, y0 + 1, x0 + 1);
      }
      const float w00 = (1.f - wy) * (1.f - wx), w01 = (1.f - wy) * wx, w10 = wy * (1.f - wx), w11 = wy * wx;
      const float dy = a.x * w00 + bq.x * w01 + c.x * w10 + d.x * w11;
      const float dx = a.y * w00 + bq.y * w01 + c.y * w10 + d.y * w11;
      py = fminf(fmaxf(py + dy, 0.f), ymax);
      px = fminf(fmaxf(px + dx, 0.f), xmax);
    }
    int iy = (int)py + RPAD, ix = (int)px + RPAD;
    iy = min(max(iy, 0), H + RPAD - 1);
    ix = min(max(ix, 0), W + RPAD - 1);
    const int lin = iy * Wp + ix;
    posb[(size_t)y * W + x] = lin;
    atomicAdd(hist + (size_t)b * (H + 2 * RPAD) * Wp + lin, 1);
  }
}

// Seeds: h > 10 and h == max over the 5x5 neighbourhood (zero outside).
__global__ __launch_bounds__(256) void seeds_kernel(const int* __restrict__ hist, int B, int Hp, int Wp,
                                                    long long* __restrict__ keys, int* __restrict__ nseeds, int cap) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int HWp = Hp * Wp;
  if (gid >= (long long)B * HWp) return;
  const int b = (int)(gid / HWp), lin = (int)(gid % HWp);
  const int* h = hist + (size_t)b * HWp;
  const int v = h[lin];
  if (v <= 10) return;
  const int y = lin / Wp, x = lin % Wp;
  int m = 0;
  for (int dy = -2; dy <= 2; ++dy) {
    const int yy = y + dy;
    if (yy < 0 || yy >= Hp) continue;
    for (int dx = -2; dx <= 2; ++dx) {
      const int xx = x + dx;
      if (xx < 0 || xx >= Wp) continue;
      m = max(m, h[yy * Wp + xx]);
    }
  }
  if (v < m) return;
  const int k = atomicAdd(nseeds + b, 1);
  if (k < cap) keys[(size_t)b * cap + k] = ((long long)v << 32) | (long long)lin;
}

// One wave per seed: 11x11 window of (hist > 2), 5 dilations from the centre, commit rank+1.
__global__ __launch_bounds__(256) void expand_kernel(const int* __restrict__ hist, const long long* __restrict__ keys_sorted,
                                                     const int* __restrict__ nseeds, int B, int Hp, int Wp, int cap,
                                                     int kmax, int* __restrict__ M1) {
  __shared__ uint8_t win[4][2][128];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long sid = (long long)blockIdx.x * 4 + wave;  // seed slot = b * kmax + k
  const int b = (int)(sid / kmax), k = (int)(sid % kmax);
  const bool active = (b < B) && (k < min(nseeds[b], cap));
  int sy = 0, sx = 0;
  const int* h = hist + (size_t)b * Hp * Wp;
  if (active) {
    const long long key = keys_sorted[(size_t)b * cap + k];
    const int lin = (int)(key & 0xffffffffLL);
    sy = lin / Wp;
    sx = lin % Wp;
  }
  uint8_t* cur = win[wave][0];
  uint8_t* nxt = win[wave][1];
  bool sup[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int c = lane + 64 * r;
    sup[r] = false;
    if (active && c < 121) {
      const int yy = sy - 5 + c / 11, xx = sx - 5 + c % 11;
      sup[r] = (yy >= 0 && yy < Hp && xx >= 0 && xx < Wp) && h[yy * Wp + xx] > 2;
    }
    if (c < 128) cur[c] = (c == 60) ? 1 : 0;  // centre (5,5)
  }
  __syncthreads();
  for (int it = 0; it < 5; ++it) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = lane + 64 * r;
      if (c < 121) {
        const int cy = c / 11, cx = c % 11;
        uint8_t any = 0;
        for (int dy = -1; dy <= 1; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            const int yy = cy + dy, xx = cx + dx;
            if (yy >= 0 && yy < 11 && xx >= 0 && xx < 11) any |= cur[yy * 11 + xx];
          }
        nxt[c] = (any && sup[r]) ? 1 : 0;
      }
    }
    __syncthreads();
    uint8_t* t = cur; cur = nxt; nxt = t;
  }
  if (active) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = lane + 64 * r;
      if (c < 121 && cur[c]) {
        const int yy = sy - 5 + c / 11, xx = sx - 5 + c % 11;
        atomicMax(M1 + (size_t)b * Hp * Wp + yy * Wp + xx, k + 1);
      }
    }
  }
}

// Per-pixel label from its end point; count pixels per label.  A thread takes LL consecutive pixels
// of one image row-major run and issues one counter atomic per run of equal labels (neighbouring
// pixels share their label: one atomic per pixel on a few hundred counters per image serialised
// in L2, 0.25 ms per batch of 32).
constexpr int LL = 8;
__global__ __launch_bounds__(256) void label_lookup_kernel(const int* __restrict__ pos, const int* __restrict__ M1, int B,
                                                           int HW, int HWp, int* __restrict__ M0, int* __restrict__ counts,
                                                           int nlab) {
  const int segs = (HW + LL - 1) / LL;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * segs) return;
  const int b = (int)(gid / segs);
  const int p0 = (int)(gid % segs) * LL, p1 = min(p0 + LL, HW);
  const int* pb = pos + (size_t)b * HW;
  const int* mb = M1 + (size_t)b * HWp;
  int* ob = M0 + (size_t)b * HW;
  int* cb = counts + (size_t)b * nlab;
  int cur = 0, run = 0;
  for (int q = p0; q < p1; ++q) {
    const int p = pb[q];
    const int lab = p >= 0 ? mb[p] : 0;
    ob[q] = lab;
    if (lab != cur) {
      if (cur > 0) atomicAdd(cb + cur, run);
      cur = lab;
      run = 0;
    }
    ++run;
  }
  if (cur > 0) atomicAdd(cb + cur, run);
}

// flow2 = (dY, dX) * (cellprob > thr) / 5 from a [B, 3, H, W] network output; fg mask.
__global__ __launch_bounds__(256) void prep_flow_kernel(const float* __restrict__ y, int B, int H, int W, float thr,
                                                        float2* __restrict__ flow2, uint8_t* __restrict__ fg) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int HW = H * W;
  if (gid >= (long long)B * HW) return;
  const int b = (int)(gid / HW), p = (int)(gid % HW);
  const float* yb = y + (size_t)b * 3 * HW;
  const bool f = yb[2 * HW + p] > thr;
  fg[gid] = f;
  flow2[gid] = f ? make_float2(yb[p] * 0.2f, yb[HW + p] * 0.2f) : make_float2(0.f, 0.f);
}

}  // namespace

extern "C" {

int be_cp_prep_flow(const float* y, int B, int H, int W, float thr, void* flow2, void* fg, hipStream_t s) {
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(prep_flow_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, y, B, H, W, thr, (float2*)flow2,
                     (uint8_t*)fg);
  return BE_CHECK_LAUNCH();
}

int be_cp_follow_flows(const void* flow2, const void* fg, int* hist, int* pos, int B, int H, int W, int niter,
                       hipStream_t s) {
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(follow_flows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float2*)flow2,
                     (const uint8_t*)fg, hist, pos, B, H, W, niter);
  return BE_CHECK_LAUNCH();
}

// Same result as be_cp_follow_flows (XCD-ordered, block-compacted launch).  BE_FOLLOW_POOL (A/B):
// pixels pooled per block for the compaction, 1 (256, the default) or 4 (1,024).  Pooling fills
// the waves but measured 1.52 vs 1.47 ms per batch of 32 (profiles/r04/headline/follow_pool_ab.txt):
// the Euler loop is bound by its dependent gather latency, and fewer waves hide less of it.
static int g_follow_pool = [] {
  const char* e = getenv("BE_FOLLOW_POOL");
  return e ? atoi(e) : 1;
}();

int be_cp_follow_flows_xcd(const void* flow2, const void* fg, int* hist, int* pos, int B, int H, int W, int niter,
                           hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  if (g_follow_pool == 4) {
    hipLaunchKernelGGL(follow_flows_xcd_pool_kernel<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s,
                       (const float2*)flow2, (const uint8_t*)fg, hist, pos, B, H, W, niter);
    return BE_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(follow_flows_xcd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const float2*)flow2,
                     (const uint8_t*)fg, hist, pos, B, H, W, niter);
  return BE_CHECK_LAUNCH();
}

// The pooled-compaction launch on its own entry (tests / A/B without the BE_FOLLOW_POOL switch).
int be_cp_follow_flows_xcd_pool(const void* flow2, const void* fg, int* hist, int* pos, int B, int H, int W, int niter,
                                hipStream_t s) {
  const long long n = (long long)B * H * W;
  if (n == 0) return 0;
  hipLaunchKernelGGL(follow_flows_xcd_pool_kernel<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, s,
                     (const float2*)flow2, (const uint8_t*)fg, hist, pos, B, H, W, niter);
  return BE_CHECK_LAUNCH();
}

// LDS-window launch (see follow_flows_lds_kernel): one 256-thread workgroup per 32 x 32 tile.
int be_cp_follow_flows_lds(const void* flow2, const void* fg, int* hist, int* pos, int B, int H, int W, int niter,
                           hipStream_t s) {
  if ((long long)B * H * W == 0) return 0;
  const long long t32 = (long long)B * ((W + 31) / 32) * ((H + 31) / 32);
  // 16-pixel tiles by default at every batch size: one pixel per thread and a 19 KiB workgroup
  // that fits beside the convs of the next batch (s29: compute_masks 3.17 vs 3.53 ms at batch 32,
  // headline +2 %); BE_FOLLOW_TILE=32 selects the 32-pixel tiles (64 x 64 window, 37 KiB)
  const char* ft = getenv("BE_FOLLOW_TILE");
  const int force = ft ? atoi(ft) : 16;
  (void)t32;
  if (force == 32) {
    const int tiles_x = (W + 31) / 32, tiles_y = (H + 31) / 32;
    hipLaunchKernelGGL(follow_flows_lds_kernel<32>, dim3((unsigned)t32), dim3(256), 0, s, (const float2*)flow2,
                       (const uint8_t*)fg, hist, pos, B, H, W, niter, tiles_x, tiles_y);
  } else {
    const int tiles_x = (W + 15) / 16, tiles_y = (H + 15) / 16;
    const long long nblk = (long long)B * tiles_x * tiles_y;
    hipLaunchKernelGGL(follow_flows_lds_kernel<16>, dim3((unsigned)nblk), dim3(256), 0, s, (const float2*)flow2,
                       (const uint8_t*)fg, hist, pos, B, H, W, niter, tiles_x, tiles_y);
  }
  return BE_CHECK_LAUNCH();
}

int be_cp_seeds(const int* hist, int B, int Hp, int Wp, long long* keys, int* nseeds, int cap, hipStream_t s) {
  const long long n = (long long)B * Hp * Wp;
  hipLaunchKernelGGL(seeds_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, hist, B, Hp, Wp, keys, nseeds, cap);
  return BE_CHECK_LAUNCH();
}

int be_cp_expand(const int* hist, const long long* keys_sorted, const int* nseeds, int B, int Hp, int Wp, int cap,
                 int kmax, int* M1, hipStream_t s) {
  const long long nslots = (long long)B * kmax;
  if (nslots == 0) return 0;
  hipLaunchKernelGGL(expand_kernel, dim3((unsigned)((nslots + 3) / 4)), dim3(256), 0, s, hist, keys_sorted, nseeds, B, Hp,
                     Wp, cap, kmax, M1);
  return BE_CHECK_LAUNCH();
}

int be_cp_label_lookup(const int* pos, const int* M1, int B, int HW, int HWp, int* M0, int* counts, int nlab,
                       hipStream_t s) {
  const long long n = (long long)B * ((HW + LL - 1) / LL);
  if (n == 0) return 0;
  hipLaunchKernelGGL(label_lookup_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pos, M1, B, HW, HWp, M0, counts,
                     nlab);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
