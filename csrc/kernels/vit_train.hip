// Row-wise backward kernels of the ViT training step (Cellpose-SAM fine-tuning, SURVEY.md §2.5 K8;
// reference training loop apps/cellpose-finetuning/main.py:1468-1546).  Everything between the
// hipBLASLt GEMMs and the flash-attention kernels is one fused pass each:
//
//  * be_ln_bwd        LayerNorm backward from the saved (mean, rstd) + the residual-stream
//                     gradient accumulation dx = LN'(dh) + s1[b] r1 + s2[b] r2 (fp32, optional bf16
//                     copy for the next GEMM) + per-block column partials of dw, db and sum(dx)
//                     (the following projection's bias gradient).
//  * be_gelu_fwd      g = gelu(f + bias) into a separate buffer (f is kept for the backward).
//  * be_gelu_bwd      df = dg * gelu'(f + bias) (bf16) + column partials of df (fc1 bias grad).
//  * be_scale_cast    y = s[b] * x (fp32 -> bf16) + column partials of y (bias grad of the GEMM that
//                     consumes it); s is the per-sample stochastic-depth keep factor.
//
// Column sums are never done with atomics: each block owns a row range and writes one partial row
// [nblocks, C]; the caller reduces the partials (deterministic, and tiny next to the GEMMs).
#include <cstdlib>

#include "common.h"

namespace {

constexpr int MAXV = 4;  // LN: C <= 64 lanes * 8 * MAXV

__device__ __forceinline__ void ld8(const bf16_t* p, float (&v)[8]) {
  const u32x4 r = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[2 * j] = lo_bf(r[j]); v[2 * j + 1] = hi_bf(r[j]); }
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&v)[8]) {
  u32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = pack2bf(v[2 * j], v[2 * j + 1]);
  *reinterpret_cast<u32x4*>(p) = r;
}
__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// one wave per row (4 rows in flight per block), `rpb` rows per block; column partials reduced over
// the block's waves through LDS and written as one row of each partial matrix.
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ stats, const float* __restrict__ w,
                                                     const float* __restrict__ r1, const float* __restrict__ s1,
                                                     const float* __restrict__ r2, const float* __restrict__ s2, int rpn,
                                                     float* __restrict__ dx, bf16_t* __restrict__ dxb,
                                                     float* __restrict__ pdw, float* __restrict__ pdb,
                                                     float* __restrict__ pcol, long long rows, int C, int rpb) {
  __shared__ float red[4][64 * 8 * MAXV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1e = min(r0 + rpb, rows);
  float aw[NV][8], ab[NV][8], ac[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) { aw[k][j] = 0.f; ab[k][j] = 0.f; ac[k][j] = 0.f; }
  // LN weight: loaded once, not per row
  float ww[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) ld8f(w + c, ww[k]);
  }
  for (long long row = r0 + wave; row < r1e; row += 4) {
    // every load of the row (incl. the residual-gradient terms) issued before its first store: a load
    // behind a store could only be waited for with vmcnt(0), which also waits for the store's ack
    const float mean = stats[2 * row], rstd = stats[2 * row + 1];
    const float sc1 = r1 ? (s1 ? s1[row / rpn] : 1.f) : 0.f;
    const float sc2 = r2 ? (s2 ? s2[row / rpn] : 1.f) : 0.f;
    float t1[NV][8], t2[NV][8];
    float g[NV][8], xh[NV][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
        if (r1) ld8f(r1 + row * C + c, t1[k]);
        if (r2) ld8f(r2 + row * C + c, t2[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
        float d[8], xv[8];
        ld8(dh + row * C + c, d);
        ld8(x + row * C + c, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xv[j] - mean) * rstd;
          g[k][j] = d[j] * ww[k][j];
          sg += g[k][j];
          sgx += g[k][j] * xh[k][j];
          aw[k][j] += d[j] * xh[k][j];
          ab[k][j] += d[j];
        }
      }
    }
    sg = wave_sum(sg) / C;
    sgx = wave_sum(sgx) / C;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[k][j] - sg - xh[k][j] * sgx);
        if (r1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += sc1 * t1[k][j];
        }
        if (r2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += sc2 * t2[k][j];
        }
        if (dx) st8f(dx + row * C + c, o);
        if (dxb) st8(dxb + row * C + c, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) ac[k][j] += o[j];
      }
    }
  }
  // block reduction of the three column partials (waves -> LDS -> one row each)
  auto flush = [&](float (&acc)[NV][8], float* out) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wave][c + j] = acc[k][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
      out[(long long)blockIdx.x * C + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    __syncthreads();
  };
  if (pdw) flush(aw, pdw);
  if (pdb) flush(ab, pdb);
  if (pcol) flush(ac, pcol);
}

// erf(x) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 outputs' 2^-9 step):
// one v_rcp, one v_exp and a few FMAs, branch-free, where the library erff takes range branches that
// diverge inside a wave (these passes stream [tokens, 4 * dim] activations and were VALU-heavy).
// e = exp(-x^2) is returned too: the GELU derivative reuses it.
__device__ __forceinline__ float erf_as(float x, float& e) {
  const float z = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  e = __expf(-z * z);
  return copysignf(1.f - p * e, x);
}
__device__ __forceinline__ float gelu_f(float t) {
  float e;
  return 0.5f * t * (1.f + erf_as(t * 0.70710678118654752f, e));
}
__device__ __forceinline__ float gelu_d(float t) {
  float e;  // exp(-t^2 / 2) from the erf evaluation
  const float er = erf_as(t * 0.70710678118654752f, e);
  return 0.5f * (1.f + er) + t * 0.3989422804014327f * e;
}

// elementwise kernels with column partials: a block owns `rpb` rows and all columns; thread t owns
// the 8-column chunks t, t + 256, ... (NC chunks), so the column sums stay in its registers.
template <int NC, int MODE>  // MODE 0: gelu fwd, 1: gelu bwd, 2: scale-cast
__global__ __launch_bounds__(256) void rowcol_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ f,
                                                     const float* __restrict__ xf, const float* __restrict__ bias,
                                                     const float* __restrict__ rs, int rpn, bf16_t* __restrict__ out,
                                                     float* __restrict__ pcol, long long rows, int C, int rpb) {
  const int C8 = C / 8;
  const long long r0 = (long long)blockIdx.x * rpb;
  const long long r1 = min(r0 + rpb, rows);
  float acc[NC][8];
  float bb[NC][8];
#pragma unroll
  for (int n = 0; n < NC; ++n) {
    const int ch = threadIdx.x + n * 256;
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc[n][j] = 0.f; bb[n][j] = 0.f; }
    if (bias && ch < C8) ld8f(bias + ch * 8, bb[n]);
  }
#pragma unroll 4  // several rows' 16-byte loads in flight per thread (the loop was latency-bound)
  for (long long row = r0; row < r1; ++row) {
    const float sc = rs ? rs[row / rpn] : 1.f;
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const int ch = threadIdx.x + n * 256;
      if (ch >= C8) continue;
      const long long e = row * C + ch * 8;
      float o[8];
      if (MODE == 0) {
        float t[8];
        ld8(f + e, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = gelu_f(t[j] + bb[n][j]);
      } else if (MODE == 1) {
        float d[8], t[8];
        ld8(a + e, d);
        ld8(f + e, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = d[j] * gelu_d(t[j] + bb[n][j]);
      } else {
        float t[8];
        ld8f(xf + e, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = sc * t[j];
      }
      st8(out + e, o);
      if (MODE != 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[n][j] += o[j];
      }
    }
  }
  if (MODE != 0 && pcol) {
#pragma unroll
    for (int n = 0; n < NC; ++n) {
      const int ch = threadIdx.x + n * 256;
      if (ch < C8) st8f(pcol + (long long)blockIdx.x * C + ch * 8, acc[n]);
    }
  }
}


// Column sums of the per-block partials [rows, C] fp32 -> out[C] (replaces a torch dim-0 reduction
// that cost ~9 us per call, 9 per transformer block).  Block = 8 columns x 32 row lanes: every lane
// issues its ~rows/32 loads back to back, one LDS step folds the 32 lanes.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ p0, float* __restrict__ out0,
                                                     const float* __restrict__ p1, float* __restrict__ out1, int rows,
                                                     int C) {
  __shared__ float red[32][9];
  const float* p = blockIdx.y ? p1 : p0;  // gridDim.y = 2: two partial matrices in one launch
  float* out = blockIdx.y ? out1 : out0;
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < C) {
    int r = rl;
    for (; r + 96 < rows; r += 128) {
      a0 += p[(long long)r * C + c];
      a1 += p[(long long)(r + 32) * C + c];
      a2 += p[(long long)(r + 64) * C + c];
      a3 += p[(long long)(r + 96) * C + c];
    }
    for (; r < rows; r += 32) a0 += p[(long long)r * C + c];
  }
  red[rl][cl] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) t += red[i][cl];
    out[c] = t;
  }
}

// Many small column reductions in one launch: the CPSAM backward produces ~120 fp32 partial
// matrices per step (LayerNorm dw/db, bias gradients); each reduced by its own launch costs a
// kernel boundary (~5 us at batch 1) for a few us of work.  The descriptors travel by value in the
// kernarg segment; blocks are laid out entry after entry (start[] prefix sums, scanned by the
// block's scalar unit); fixed summation order (deterministic).
constexpr int COLSUM_BATCH = 48;
struct ColsumBatch {
  int n;
  int start[COLSUM_BATCH + 1];
  int rows[COLSUM_BATCH];
  int C[COLSUM_BATCH];
  const float* p[COLSUM_BATCH];
  float* o[COLSUM_BATCH];
};

__global__ __launch_bounds__(256) void colsum_batched_kernel(const ColsumBatch b) {
  // block = 64 columns x 4 row-waves: every wave-load is one contiguous 256-byte row segment
  __shared__ float red[4][64];
  const int blk = blockIdx.x;
  int e = 0;
  while (e + 1 < b.n && blk >= b.start[e + 1]) ++e;
  const float* __restrict__ p = b.p[e];
  const int rows = b.rows[e], C = b.C[e];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blk - b.start[e]) * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < C) {
    int r = w;
    for (; r + 12 < rows; r += 16) {
      a0 += p[(long long)r * C + c];
      a1 += p[(long long)(r + 4) * C + c];
      a2 += p[(long long)(r + 8) * C + c];
      a3 += p[(long long)(r + 12) * C + c];
    }
    for (; r < rows; r += 4) a0 += p[(long long)r * C + c];
  }
  red[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && c < C) b.o[e][c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// Column partial sums of a bf16 [rows, C] matrix: block (x, y) sums rows [16 y, 16 y + 16) of columns
// [1024 x, +1024) (8 per thread, 16-byte loads, 8 rows in flight) into part[y, :] (fp32); the [ceil(rows/16), C]
// partials then go through a colsum (batched with the others).  Replaces torch's bf16 dim-0 reduction
// of the packed dqkv gradient (the qkv bias gradient), which ran at ~2.3 TB/s.
__global__ __launch_bounds__(128) void colpart_bf16_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                           int rows, int C) {
  const int c = (blockIdx.x * 128 + threadIdx.x) * 8;
  if (c >= C) return;
  const int r0 = blockIdx.y * 16, r1 = min(rows, r0 + 16);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int r = r0; r < r1; ++r) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(x + (long long)r * C + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[2 * j] += lo_bf(v[j]); a[2 * j + 1] += hi_bf(v[j]); }
  }
  float4* o = reinterpret_cast<float4*>(part + (long long)blockIdx.y * C + c);
  o[0] = make_float4(a[0], a[1], a[2], a[3]);
  o[1] = make_float4(a[4], a[5], a[6], a[7]);
}

// out[i] = sum_s ws[s, i] (split-K weight-gradient slabs), 4 floats per thread per slab
__global__ __launch_bounds__(256) void sum_slabs_kernel(const float* __restrict__ ws, float* __restrict__ out, int nslab,
                                                        long long n4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4* w = reinterpret_cast<const float4*>(ws);
  float4 t = w[i];
  for (int s = 1; s < nslab; ++s) {
    const float4 u = w[(long long)s * n4 + i];
    t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
  }
  reinterpret_cast<float4*>(out)[i] = t;
}

// g = gelu(f + bias) as a flat streaming pass (no column sums to keep): every thread converts U
// independent 8-element chunks, all U 16-byte loads issued before the first store; bias read per
// chunk (L2 / L1 resident).  The row-blocked rowcol form streamed at ~3.5 TB/s.
template <int U>
__global__ __launch_bounds__(256) void gelu_fwd_flat_kernel(const bf16_t* __restrict__ f, const float* __restrict__ bias,
                                                            bf16_t* __restrict__ g, long long n8, int C8) {
  const long long base = ((long long)blockIdx.x * U) * 256 + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * 256;
    if (i < n8) v[u] = *reinterpret_cast<const u32x4*>(f + i * 8);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * 256;
    if (i >= n8) continue;
    float bb[8];
    if (bias) ld8f(bias + (i % C8) * 8, bb);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) bb[j] = 0.f;
    }
    float o[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = gelu_f(lo_bf(v[u][j]) + bb[2 * j]);
      o[2 * j + 1] = gelu_f(hi_bf(v[u][j]) + bb[2 * j + 1]);
    }
    st8(g + i * 8, o);
  }
}

template <int MODE>
int launch_rowcol(const bf16_t* a, const bf16_t* f, const float* xf, const float* bias, const float* rs, int rpn,
                  bf16_t* out, float* pcol, long long rows, int C, int rpb, hipStream_t s) {
  if (C % 8 != 0 || rpb <= 0) return -1;
  const int nc = (C / 8 + 255) / 256;
  const dim3 grid((unsigned)((rows + rpb - 1) / rpb));
  if (rpn <= 0) rpn = 1;
  switch (nc) {
    case 1: hipLaunchKernelGGL((rowcol_kernel<1, MODE>), grid, dim3(256), 0, s, a, f, xf, bias, rs, rpn, out, pcol, rows, C, rpb); break;
    case 2: hipLaunchKernelGGL((rowcol_kernel<2, MODE>), grid, dim3(256), 0, s, a, f, xf, bias, rs, rpn, out, pcol, rows, C, rpb); break;
    case 3: hipLaunchKernelGGL((rowcol_kernel<3, MODE>), grid, dim3(256), 0, s, a, f, xf, bias, rs, rpn, out, pcol, rows, C, rpb); break;
    case 4: hipLaunchKernelGGL((rowcol_kernel<4, MODE>), grid, dim3(256), 0, s, a, f, xf, bias, rs, rpn, out, pcol, rows, C, rpb); break;
    default: return -2;
  }
  return BE_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

// dh: bf16 [rows, C] gradient of the LN output; x: bf16 LN input; stats: (mean, rstd) per row; w: LN
// weight.  dx (fp32, optional) / dxb (bf16, optional) = LN'(dh) + s1[row/rpn]*r1 + s2[row/rpn]*r2
// (r*, s* optional; s null = 1).  pdw / pdb / pcol: optional [ceil(rows/rpb), C] partials of
// sum(dh*xhat), sum(dh), sum(dx).
int be_ln_bwd(const void* dh, const void* x, const float* stats, const float* w, const float* r1, const float* s1,
              const float* r2, const float* s2, int rpn, float* dx, void* dxb, float* pdw, float* pdb, float* pcol,
              long long rows, int C, int rpb, hipStream_t s) {
  if (C % 8 != 0 || C > 64 * 8 * MAXV || rpb <= 0) return -1;
  const int nv = (C / 8 + 63) / 64;
  const dim3 grid((unsigned)((rows + rpb - 1) / rpb));
  if (rpn <= 0) rpn = 1;
#define LNB(NV)                                                                                                   \
  case NV:                                                                                                        \
    hipLaunchKernelGGL(ln_bwd_kernel<NV>, grid, dim3(256), 0, s, (const bf16_t*)dh, (const bf16_t*)x, stats, w, r1, \
                       s1, r2, s2, rpn, dx, (bf16_t*)dxb, pdw, pdb, pcol, rows, C, rpb);                            \
    break;
  switch (nv) {
    LNB(1) LNB(2) LNB(3) LNB(4)
    default: return -1;
  }
#undef LNB
  return BE_CHECK_LAUNCH();
}

// g = gelu(f + bias) (exact erf GELU), bf16 [rows, C].
int be_gelu_fwd(const void* f, const float* bias, void* g, long long rows, int C, int rpb, hipStream_t s) {
  static const int flat = [] {
    const char* e = getenv("BE_GELU_FWD_FLAT");
    return e ? atoi(e) : 1;
  }();
  if (flat && C % 8 == 0) {
    const long long n8 = rows * (C / 8);
    constexpr int U = 4;
    hipLaunchKernelGGL(gelu_fwd_flat_kernel<U>, dim3((unsigned)((n8 + 256 * U - 1) / (256 * U))), dim3(256), 0, s,
                       (const bf16_t*)f, bias, (bf16_t*)g, n8, C / 8);
    return BE_CHECK_LAUNCH();
  }
  return launch_rowcol<0>(nullptr, (const bf16_t*)f, nullptr, bias, nullptr, 1, (bf16_t*)g, nullptr, rows, C, rpb, s);
}

// df = dg * gelu'(f + bias) (bf16) + column partials of df [ceil(rows/rpb), C].
int be_gelu_bwd(const void* dg, const void* f, const float* bias, void* df, float* pcol, long long rows, int C, int rpb,
                hipStream_t s) {
  return launch_rowcol<1>((const bf16_t*)dg, (const bf16_t*)f, nullptr, bias, nullptr, 1, (bf16_t*)df, pcol, rows, C,
                          rpb, s);
}

// y = rs[row/rpn] * x (fp32 -> bf16; rs null = 1) + column partials of y.
int be_scale_cast(const float* x, const float* rs, int rpn, void* y, float* pcol, long long rows, int C, int rpb,
                  hipStream_t s) {
  return launch_rowcol<2>(nullptr, nullptr, x, nullptr, rs, rpn, (bf16_t*)y, pcol, rows, C, rpb, s);
}

// out[C] = sum over rows of p [rows, C] (fp32)
int be_colsum(const float* p, float* out, int rows, int C, hipStream_t s) {
  if (rows <= 0 || C <= 0) return -1;
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 7) / 8, 1), dim3(256), 0, s, p, out, p, out, rows, C);
  return BE_CHECK_LAUNCH();
}

// part [ceil(rows / 16), C] fp32 = per-16-row column sums of x bf16 [rows, C]; C % 8 == 0.
int be_colpart_bf16(const void* x, float* part, int rows, int C, hipStream_t s) {
  if (rows <= 0 || C <= 0 || C % 8 != 0) return -1;
  hipLaunchKernelGGL(colpart_bf16_kernel, dim3((unsigned)((C / 8 + 127) / 128), (unsigned)((rows + 15) / 16)), dim3(128),
                     0, s, (const bf16_t*)x, part, rows, C);
  return BE_CHECK_LAUNCH();
}

// out [n] = sum over nslab slabs of ws [nslab, n]; n % 4 == 0, 16-byte aligned.
int be_sum_slabs(const float* ws, float* out, int nslab, long long n, hipStream_t s) {
  if (nslab <= 0 || n <= 0 || n % 4 != 0) return -1;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(sum_slabs_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, ws, out, nslab, n4);
  return BE_CHECK_LAUNCH();
}

// n column reductions in ceil(n / 48) launches.  desc: host int64 array of n records
// {partial ptr, out ptr, rows, C}; partial [rows, C] fp32 contiguous, out [C] fp32.
int be_colsum_batched(const long long* desc, int n, hipStream_t s) {
  if (n < 0) return -1;
  for (int base = 0; base < n; base += COLSUM_BATCH) {
    ColsumBatch b{};
    b.n = n - base < COLSUM_BATCH ? n - base : COLSUM_BATCH;
    int blocks = 0;
    for (int i = 0; i < b.n; ++i) {
      const long long* d = desc + 4 * (long long)(base + i);
      b.p[i] = reinterpret_cast<const float*>(d[0]);
      b.o[i] = reinterpret_cast<float*>(d[1]);
      b.rows[i] = (int)d[2];
      b.C[i] = (int)d[3];
      if (!b.p[i] || !b.o[i] || b.rows[i] <= 0 || b.C[i] <= 0) return -2;
      b.start[i] = blocks;
      blocks += (b.C[i] + 63) / 64;
    }
    b.start[b.n] = blocks;
    hipLaunchKernelGGL(colsum_batched_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b);
    const int rc = BE_CHECK_LAUNCH();
    if (rc) return rc;
  }
  return 0;
}

// two [rows, C] partial matrices reduced in one launch (e.g. LayerNorm dw and db)
int be_colsum2(const float* p0, float* out0, const float* p1, float* out1, int rows, int C, hipStream_t s) {
  if (rows <= 0 || C <= 0) return -1;
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 7) / 8, 2), dim3(256), 0, s, p0, out0, p1, out1, rows, C);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
