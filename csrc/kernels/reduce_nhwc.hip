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
    atomicAdd(out + (size_t)n * C + c, s);
  }
}

}  // namespace

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
