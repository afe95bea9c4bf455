// IVF list scan with EXACT bf16 inner products (the high-recall cell-image-search tier).
//
// The reference ranks its >5 M-vector IVF-PQ candidates with 8-bit PQ codes on the CPU
// (FAISS IndexIVFPQ m=96, nprobe=64: /root/reference/apps/cell-image-search/index_manager.py:67-89).
// One MI355X holds 288 GB of HBM: 58 M x 768 bf16 vectors are 89 GB, so the full vectors stay
// resident, stored list-sorted (each IVF list one contiguous slab), and every candidate of the
// probed lists is scored exactly: recall is bounded only by the coarse probing, and the scan is a
// pure HBM stream (~190 MB per query at nprobe 64 / 58 M).
//
// One 256-thread workgroup per (query, probed list).  A row of D bf16 is read by 16 lanes, each
// owning D/16 dims as D/128 16-byte loads (16 lanes cover 256 contiguous bytes per load), the
// query's matching fp32 slice held in registers; four rows per wave in flight, a 16-lane shuffle
// reduction, the score written to the query's candidate row.  Top-k over the candidate rows is a
// separate selection; padding slots stay -inf.
#include "common.h"

namespace {

template <int CH>  // D = 128 * CH
__global__ __launch_bounds__(256) void ivf_scan_bf16_kernel(const float* __restrict__ q, const int* __restrict__ probes,
                                                           const long long* __restrict__ list_off,
                                                           const long long* __restrict__ cand_off,
                                                           const bf16_t* __restrict__ vecs, int nprobe,
                                                           long long cand_stride, float* __restrict__ out) {
  constexpr int D = 128 * CH;
  const int qi = blockIdx.y, p = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int sub = lane & 15, grp = lane >> 4;  // 16 lanes per row, 4 rows per wave
  float qv[CH][8];
  const float* qq = q + (size_t)qi * D;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const float4 a = *reinterpret_cast<const float4*>(qq + c * 128 + sub * 8);
    const float4 b = *reinterpret_cast<const float4*>(qq + c * 128 + sub * 8 + 4);
    qv[c][0] = a.x; qv[c][1] = a.y; qv[c][2] = a.z; qv[c][3] = a.w;
    qv[c][4] = b.x; qv[c][5] = b.y; qv[c][6] = b.z; qv[c][7] = b.w;
  }
  const int list = probes[qi * nprobe + p];
  const long long l0 = list_off[list], l1 = list_off[list + 1];
  float* o = out + (size_t)qi * cand_stride + cand_off[qi * nprobe + p];
  for (long long r0 = l0 + wave * 4 + grp; r0 < l1; r0 += 16 * 2) {
    // two rows per lane group in flight (r0 and r0 + 16)
    const long long r1 = r0 + 16;
    const bool has1 = r1 < l1;
    u32x4 v0[CH], v1[CH];
    const bf16_t* row0 = vecs + r0 * D + sub * 8;
    const bf16_t* row1 = vecs + (has1 ? r1 : r0) * D + sub * 8;
#pragma unroll
    for (int c = 0; c < CH; ++c) v0[c] = *reinterpret_cast<const u32x4*>(row0 + c * 128);
#pragma unroll
    for (int c = 0; c < CH; ++c) v1[c] = *reinterpret_cast<const u32x4*>(row1 + c * 128);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s0 = fmaf(lo_bf(v0[c][j]), qv[c][2 * j], s0);
        s0 = fmaf(hi_bf(v0[c][j]), qv[c][2 * j + 1], s0);
        s1 = fmaf(lo_bf(v1[c][j]), qv[c][2 * j], s1);
        s1 = fmaf(hi_bf(v1[c][j]), qv[c][2 * j + 1], s1);
      }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
      s0 += __shfl_xor(s0, off, 16);
      s1 += __shfl_xor(s1, off, 16);
    }
    if (sub == 0) {
      o[r0 - l0] = s0;
      if (has1) o[r1 - l0] = s1;
    }
  }
}

}  // namespace

extern "C" {

// q [Q, D] fp32; probes/cand_off [Q, nprobe]; list_off [nlist + 1]; vecs [N, D] bf16 list-sorted;
// out [Q, cand_stride] fp32 pre-filled with -inf.  D must be a multiple of 128, <= 1024.
int be_ivf_scan_bf16(const float* q, const int* probes, const long long* list_off, const long long* cand_off,
                     const void* vecs, int Q, int nprobe, int D, long long cand_stride, float* out, hipStream_t s) {
  if (Q == 0 || nprobe == 0) return 0;
  if (D % 128 || D > 1024) return -1;
  const dim3 grid(nprobe, Q);
  const bf16_t* v = reinterpret_cast<const bf16_t*>(vecs);
  switch (D / 128) {
    case 1: hipLaunchKernelGGL(ivf_scan_bf16_kernel<1>, grid, dim3(256), 0, s, q, probes, list_off, cand_off, v, nprobe, cand_stride, out); break;
    case 2: hipLaunchKernelGGL(ivf_scan_bf16_kernel<2>, grid, dim3(256), 0, s, q, probes, list_off, cand_off, v, nprobe, cand_stride, out); break;
    case 3: hipLaunchKernelGGL(ivf_scan_bf16_kernel<3>, grid, dim3(256), 0, s, q, probes, list_off, cand_off, v, nprobe, cand_stride, out); break;
    case 4: hipLaunchKernelGGL(ivf_scan_bf16_kernel<4>, grid, dim3(256), 0, s, q, probes, list_off, cand_off, v, nprobe, cand_stride, out); break;
    case 6: hipLaunchKernelGGL(ivf_scan_bf16_kernel<6>, grid, dim3(256), 0, s, q, probes, list_off, cand_off, v, nprobe, cand_stride, out); break;
    case 8: hipLaunchKernelGGL(ivf_scan_bf16_kernel<8>, grid, dim3(256), 0, s, q, probes, list_off, cand_off, v, nprobe, cand_stride, out); break;
    default: return -2;
  }
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
