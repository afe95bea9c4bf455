// SAM decomposed relative-position terms for the Cellpose-SAM training engine (SURVEY.md §2.5 K8;
// the reference fine-tunes Cellpose-SAM, apps/cellpose-finetuning/main.py:1278-1713), on MFMA.
//
// With a g x g token grid (g = 32: 256^2 crops, patch 8), per batch b / head h / token t = (y, x):
//   rel_h[b,h,t,k] = sum_c q[b,t,h,c] Rh[y,k,c]        rel_w[b,h,t,k] = sum_c q[b,t,h,c] Rw[x,k,c]
// and backward
//   dq[b,t,h,c]  += sum_k drh[b,h,t,k] Rh[y,k,c] + sum_k drw[b,h,t,k] Rw[x,k,c]
//   dRh[y,k,c]    = sum_{b,h,x} drh[b,h,(y,x),k] q[b,(y,x),h,c]   (dRw likewise over y)
//   rph.grad[y - k + g - 1] += dRh[y, k]                            (get_rel_pos gather, reversed)
//
// Every (b, h, grid line) is one 32 x 32 (or 32 x 64) MFMA tile: the "h" pass takes grid row y
// (tokens (y, 0..31), table Rh[y]), the "w" pass grid column x (tokens (0..31, x), table Rw[x]).
// These replace ~25 torch launches per block (fp32 copies of q, permutes, six batched fp32 GEMMs,
// index_add, adds) with 4.  fp32 operands (tables, gradients) are split hi + lo into two bf16 MFMA
// operands (error ~2^-16 relative); q is bf16 already and goes in exactly.
//
// MFMA v_mfma_f32_32x32x16_bf16 fragments (same convention as attention.hip / attention_bwd.hip):
// A lane = row (lane & 31), k = 8 (lane >> 5) .. +8 of the 16-step; B lane = column (lane & 31), same
// k; D register i of a lane = row 8 (i >> 2) + 4 (lane >> 5) + (i & 3), column lane & 31.
#include "common.h"

namespace {

constexpr int G = 32;   // grid side (tokens per line)
constexpr int C = 64;   // head dim
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ int tok_of(int pass, int line, int j) { return pass ? j * G + line : line * G + j; }

// 8 fp32 -> (hi, lo) bf16 fragments
__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint16_t h = f2bf(v[j]);
    hi[j] = (short)h;
    lo[j] = (short)f2bf(v[j] - bf2f(h));
  }
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ------------------------------------------------------------------ forward: rel_h, rel_w
__global__ __launch_bounds__(256) void relpos_fwd_kernel(const bf16_t* __restrict__ q, long long s_tok, long long s_head,
                                                         long long s_batch, const float* __restrict__ Rh,
                                                         const float* __restrict__ Rw, float* __restrict__ rel_h,
                                                         float* __restrict__ rel_w, int B, int H) {
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);  // (bh, line, pass)
  if (tile >= B * H * G * 2) return;
  const int pass = tile & 1, line = (tile >> 1) % G, bh = (tile >> 1) / G;
  const int b = bh / H, hh = bh % H;
  const bf16_t* qb = q + (long long)b * s_batch + (long long)hh * s_head;
  // R[line][k] = table[line - k + G - 1] (get_rel_pos at q == k size): read the table directly
  const float* T = (pass ? Rw : Rh) + (long long)(line - l32 + G - 1) * C;
  const int tokA = tok_of(pass, line, l32);
  f32x16 acc = zero16();
#pragma unroll
  for (int ks = 0; ks < C / 16; ++ks) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(qb + (long long)tokA * s_tok + ks * 16 + h * 8);
    float tv[8];
    const float4* tp = reinterpret_cast<const float4*>(T + ks * 16 + h * 8);
    const float4 t0 = tp[0], t1 = tp[1];
    tv[0] = t0.x; tv[1] = t0.y; tv[2] = t0.z; tv[3] = t0.w; tv[4] = t1.x; tv[5] = t1.y; tv[6] = t1.z; tv[7] = t1.w;
    bf16x8 bhi, blo;
    split8(tv, bhi, blo);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bhi, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, blo, acc, 0, 0, 0);
  }
  float* out = (pass ? rel_w : rel_h) + (long long)bh * G * G * G;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = 8 * (i >> 2) + 4 * h + (i & 3);
    out[(long long)tok_of(pass, line, r) * G + l32] = acc[i];
  }
}

// ------------------------------------------------------------------ backward: dq (one pass per launch)
// pass 0: dq += drh Rh (in place, fp32).  pass 1: out_bf16 = bf16(dq + drw Rw) (the q slot of the
// packed dqkv gradient) when out_bf16 is given, else dq += drw Rw.
__global__ __launch_bounds__(256) void relpos_bwd_dq_kernel(const float* __restrict__ drh, const float* __restrict__ drw,
                                                            const float* __restrict__ Rh, const float* __restrict__ Rw,
                                                            float* dq, long long q_tok, long long q_head,
                                                            long long q_batch, bf16_t* out_bf16, long long o_tok,
                                                            long long o_head, long long o_batch, int pass, int B, int H,
                                                            float* zero0, float* zero1) {
  // pass 0, block 0 zeroes the table gradients the later table kernel accumulates into (saves two
  // fill launches per transformer block)
  if (zero0 && blockIdx.x == 0)
    for (int i = threadIdx.x; i < (2 * G - 1) * C; i += blockDim.x) { zero0[i] = 0.f; zero1[i] = 0.f; }
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);  // (bh, line)
  if (tile >= B * H * G) return;
  const int line = tile % G, bh = tile / G;
  const int b = bh / H, hh = bh % H;
  const float* d = (pass ? drw : drh) + (long long)bh * G * G * G;
  const float* T = (pass ? Rw : Rh) + (long long)(line + G - 1) * C;  // row k: T - k * C
  const int tokA = tok_of(pass, line, l32);
  f32x16 acc[2] = {zero16(), zero16()};
#pragma unroll
  for (int ks = 0; ks < G / 16; ++ks) {
    float av[8];
    const float4* ap = reinterpret_cast<const float4*>(d + (long long)tokA * G + ks * 16 + h * 8);
    const float4 a0 = ap[0], a1 = ap[1];
    av[0] = a0.x; av[1] = a0.y; av[2] = a0.z; av[3] = a0.w; av[4] = a1.x; av[5] = a1.y; av[6] = a1.z; av[7] = a1.w;
    bf16x8 ahi, alo;
    split8(av, ahi, alo);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      float bv[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) bv[jj] = T[-(ks * 16 + h * 8 + jj) * C + cb * 32 + l32];
      bf16x8 bhi, blo;
      split8(bv, bhi, blo);
      acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, bhi, acc[cb], 0, 0, 0);
      acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, blo, acc[cb], 0, 0, 0);
      acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo, bhi, acc[cb], 0, 0, 0);
    }
  }
  // all 32 dq reads issued before any store: a read after a store would wait (vmcnt) for the
  // store's acknowledgement too, serialising 32 store + load round trips per lane
  float dqv[16][2];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int tok = tok_of(pass, line, 8 * (i >> 2) + 4 * h + (i & 3));
    const float* dr = dq + (long long)b * q_batch + (long long)tok * q_tok + (long long)hh * q_head;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) dqv[i][cb] = dr[cb * 32 + l32];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int tok = tok_of(pass, line, 8 * (i >> 2) + 4 * h + (i & 3));
    float* dr = dq + (long long)b * q_batch + (long long)tok * q_tok + (long long)hh * q_head;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int c = cb * 32 + l32;
      const float v = dqv[i][cb] + acc[cb][i];
      if (out_bf16)
        out_bf16[(long long)b * o_batch + (long long)tok * o_tok + (long long)hh * o_head + c] = f2bf(v);
      else
        dr[c] = v;
    }
  }
}

// ------------------------------------------------------------------ backward: rel-pos table gradients
// Block = (pass, line, split); its 4 waves take (b, h) pairs split*4 + wave, += nsplit*4, accumulate
// dT[line] [32 k x 64 c] in registers, reduce through LDS and add into the gathered table rows
// line - k + G - 1 with global fp32 atomics (tables zeroed by the pass-0 dq launch before it).
__global__ __launch_bounds__(256) void relpos_bwd_table_kernel(const float* __restrict__ drh,
                                                               const float* __restrict__ drw,
                                                               const bf16_t* __restrict__ q, long long s_tok,
                                                               long long s_head, long long s_batch, float* gRh,
                                                               float* gRw, int B, int H, int nsplit) {
  __shared__ float red[G * C];
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31, wave = threadIdx.x >> 6;
  const int blk = blockIdx.x;
  const int split = blk % nsplit, line = (blk / nsplit) % G, pass = blk / (nsplit * G);
  for (int i = threadIdx.x; i < G * C; i += 256) red[i] = 0.f;
  const float* dbase = pass ? drw : drh;
  f32x16 acc[2] = {zero16(), zero16()};
  for (int bh = split * 4 + wave; bh < B * H; bh += nsplit * 4) {
    const int b = bh / H, hh = bh % H;
    const float* d = dbase + (long long)bh * G * G * G;
    const bf16_t* qb = q + (long long)b * s_batch + (long long)hh * s_head;
#pragma unroll
    for (int ks = 0; ks < G / 16; ++ks) {
      // A[k = l32][j]: d[tok(j), k] for j = ks*16 + 8h .. +8
      float av[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) av[jj] = d[(long long)tok_of(pass, line, ks * 16 + h * 8 + jj) * G + l32];
      bf16x8 ahi, alo;
      split8(av, ahi, alo);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        bf16x8 bq;  // B[j][c = cb*32 + l32] = q[tok(j), c]
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          bq[jj] = (short)qb[(long long)tok_of(pass, line, ks * 16 + h * 8 + jj) * s_tok + cb * 32 + l32];
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ahi, bq, acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(alo, bq, acc[cb], 0, 0, 0);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = 8 * (i >> 2) + 4 * h + (i & 3);
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) atomicAdd(&red[k * C + cb * 32 + l32], acc[cb][i]);
  }
  __syncthreads();
  float* tab = pass ? gRw : gRh;
  for (int i = threadIdx.x; i < G * C; i += 256) {
    const int k = i / C, c = i % C;
    atomicAdd(&tab[(line - k + G - 1) * C + c], red[i]);
  }
}

}  // namespace

extern "C" {

// q: bf16 [B, N=1024, H, 64] view (element strides); Rh/Rw: the fp32 rel-pos TABLES [63, 64]
// (R[y][k] = table[y - k + 31], gathered in the kernels); rel_h/rel_w: fp32
// [B, H, 1024, 32].  Grid side must be 32 and head_dim 64.
int be_relpos_fwd(const void* q, long long s_tok, long long s_head, long long s_batch, const float* Rh, const float* Rw,
                  float* rel_h, float* rel_w, int B, int H, int g, int c, hipStream_t stream) {
  if (g != G || c != C) return -1;
  const int tiles = B * H * G * 2;
  hipLaunchKernelGGL(relpos_fwd_kernel, dim3((tiles + 3) / 4), dim3(256), 0, stream, (const bf16_t*)q, s_tok, s_head,
                     s_batch, Rh, Rw, rel_h, rel_w, B, H);
  return BE_CHECK_LAUNCH();
}

// drh/drw: fp32 [B, H, 1024, 32]; Rh/Rw: tables as above; dq: fp32 [B, N, H, 64] (strides), updated with the h term, then
// (pass 2) the w term is added and the sum written as bf16 into out (strides o_*) when out != null.
// q (for the table gradients): bf16 strides as in be_relpos_fwd; gRh / gRw: fp32 [2*32-1, 64]
// (overwritten: zeroed by the first dq launch, then accumulated by the table kernel).
int be_relpos_bwd(const float* drh, const float* drw, const float* Rh, const float* Rw, float* dq, long long q_tok,
                  long long q_head, long long q_batch, void* out, long long o_tok, long long o_head, long long o_batch,
                  const void* q, long long s_tok, long long s_head, long long s_batch, float* gRh, float* gRw, int B,
                  int H, int g, int c, hipStream_t stream) {
  if (g != G || c != C) return -1;
  const int tiles = B * H * G;
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(relpos_bwd_dq_kernel, dim3((tiles + 3) / 4), dim3(256), 0, stream, drh, drw, Rh, Rw, dq, q_tok,
                       q_head, q_batch, pass ? (bf16_t*)out : (bf16_t*)nullptr, o_tok, o_head, o_batch, pass, B, H,
                       pass ? (float*)nullptr : gRh, pass ? (float*)nullptr : gRw);
    const int rc = BE_CHECK_LAUNCH();
    if (rc) return rc;
  }
  const int nsplit = (B * H + 31) / 32 < 8 ? (B * H + 31) / 32 : 8;  // <= 8 (b, h) pairs per wave
  const int ns = nsplit < 1 ? 1 : nsplit;
  hipLaunchKernelGGL(relpos_bwd_table_kernel, dim3(2 * G * ns), dim3(256), 0, stream, drh, drw, (const bf16_t*)q,
                     s_tok, s_head, s_batch, gRh, gRw, B, H, ns);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
