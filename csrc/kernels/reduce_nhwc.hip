// Channel reductions over NHWC bf16 activations.
//
// be_nhwc_channel_sum: out[n, c] += sum_{hw} x[n, hw, c]   (fp32 accumulate)
//   Used for the Cellpose style vector (global average pool of the deepest encoder features,
//   cellpose ``make_style``) and for GroupNorm/BatchNorm statistics.
//   Grid = (N, SPLIT): each block streams HW/SPLIT pixels with 16-byte loads (8 channels per lane),
//   reduces across pixel groups through LDS, then one atomicAdd per (n, c) per block.
#include "common.h"

namespace {

template <int C8>  // channels / 8
__global__ __launch_bounds__(256) void nhwc_channel_sum_kernel(const bf16_t* __restrict__ x, float* __restrict__ out,
                                                               int HW, int C, int per_block, int square) {
  const int n = blockIdx.x;
  const int sb = blockIdx.y;
  const int tid = threadIdx.x;
  constexpr int PG = 256 / C8;  // pixel groups per block iteration
  const int cg = tid % C8;
  const int pg = tid / C8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int p0 = sb * per_block;
  const int p1 = min(HW, p0 + per_block);
  if (pg < PG) {
    for (int p = p0 + pg; p < p1; p += PG) {
      const u32x4 r = *reinterpret_cast<const u32x4*>(x + ((size_t)n * HW + p) * C + cg * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = lo_bf(r[j]), b = hi_bf(r[j]);
        if (square) { a *= a; b *= b; }
        acc[2 * j] += a;
        acc[2 * j + 1] += b;
      }
    }
  }
  __shared__ float red[256 * 8 / 8 * 8];  // PG * C8 * 8 <= 2048 floats
  float* myslot = red + (pg * C8 + cg) * 8;
  if (pg < PG) {
#pragma unroll
    for (int j = 0; j < 8; ++j) myslot[j] = acc[j];
  }
  __syncthreads();
  // reduce over pixel groups: thread t < C handles channel t
  for (int c = tid; c < C; c += 256) {
    const int g = c / 8, j = c % 8;
    float s = 0.f;
    for (int q = 0; q < PG; ++q) s += red[(q * C8 + g) * 8 + j];
    // one partial per (image, pixel split): out is [N, split, C], summed in a fixed order by the
    // caller -- float atomics here made the style vector (and, through bf16 rounding flips in the
    // decoder, the flows) differ run to run
    out[((size_t)n * gridDim.y + sb) * C + c] = s;
  }
}

}  // namespace

// out: [N, split, C] per-split partial sums (every element written; the caller reduces over split)
extern "C" int be_nhwc_channel_sum(const void* x, float* out, int N, int HW, int C, int split, int square,
                                   hipStream_t s) {
  if (C % 8 != 0 || C > 2048) return -1;
  const int per_block = (HW + split - 1) / split;
  dim3 grid(N, split);
  switch (C / 8) {
#define CASE(K) \
  case K:       \
    hipLaunchKernelGGL((nhwc_channel_sum_kernel<K>), grid, dim3(256), 0, s, (const bf16_t*)x, out, HW, C, per_block, square); break;
    CASE(1) CASE(2) CASE(4) CASE(8) CASE(16) CASE(32) CASE(64) CASE(128) CASE(256)
#undef CASE
    default: return -2;
  }
  return BE_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// Cellpose style vector + every decoder style shift in one launch (replaces ~8 small torch ops and
// an fp32 GEMM whose library call alone costs ~0.2 ms of host time per batch-1 request):
//   style[n, :]  = v / ||v||,  v = sums[n, :] * inv_hw                       (cellpose make_style)
//   shift[n, j]  = ((style_on ? style[n, :] . W[j, :] : 0) + b[j]) * s[j] + t[j]
// Grid (N, ceil(J / 64)): each block normalises its image's vector into LDS (recomputed per block,
// C <= 1024 values), then its 4 waves take 16 output rows each: lanes stream W[j, :] as float4
// (coalesced) against the LDS copy and a wave reduction finishes the dot product.
namespace {

__global__ __launch_bounds__(256) void style_shift_kernel(const float* __restrict__ sums, int C, float inv_hw,
                                                          const float* __restrict__ W, const float* __restrict__ b,
                                                          const float* __restrict__ s, const float* __restrict__ t,
                                                          int J, int style_on, float* __restrict__ style_out,
                                                          float* __restrict__ shifts) {
  __shared__ __attribute__((aligned(16))) float st[1024];
  __shared__ float red[4];
  const int n = blockIdx.x, jb = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float ss = 0.f;
  for (int c = tid; c < C; c += 256) {
    const float v = sums[(size_t)n * C + c] * inv_hw;
    st[c] = v;
    ss += v * v;
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wave] = ss;
  __syncthreads();
  const float nrm = sqrtf(red[0] + red[1] + red[2] + red[3]);
  for (int c = tid; c < C; c += 256) {
    const float v = st[c] / nrm;
    st[c] = v;
    if (jb == 0) style_out[(size_t)n * C + c] = v;
  }
  __syncthreads();
  for (int jj = wave; jj < 64; jj += 4) {
    const int j = jb * 64 + jj;
    if (j >= J) break;
    float acc = 0.f;
    if (style_on) {
      for (int k = lane * 4; k < C; k += 256) {
        const float4 w = *reinterpret_cast<const float4*>(W + (size_t)j * C + k);
        acc += w.x * st[k] + w.y * st[k + 1] + w.z * st[k + 2] + w.w * st[k + 3];
      }
      acc = wave_sum(acc);
    }
    if (lane == 0) shifts[(size_t)n * J + j] = (acc + b[j]) * s[j] + t[j];
  }
}

}  // namespace

// sums [N, C] fp32 (pooled channel sums) -> style [N, C], shifts [N, J]; W [J, C]; C % 4 == 0, C <= 1024.
extern "C" int be_style_shift(const float* sums, int N, int C, float inv_hw, const float* W, const float* b,
                              const float* s, const float* t, int J, int style_on, float* style_out, float* shifts,
                              hipStream_t st) {
  if (C % 4 != 0 || C > 1024 || N <= 0 || J <= 0) return -1;
  hipLaunchKernelGGL(style_shift_kernel, dim3(N, (J + 63) / 64), dim3(256), 0, st, sums, C, inv_hw, W, b, s, t, J,
                     style_on, style_out, shifts);
  return BE_CHECK_LAUNCH();
}
