// IVF-PQ list scan for inner-product search (reference FAISS IVFPQ m=96,
// 8-bit codes, nprobe=64, apps/cell-image-search/index_manager.py:67-89).
//
// score(q, x) = <q, c_list(x)> + sum_j LUT_q[j][code_j(x)],   LUT_q[j][k] = <q_j, codebook_j[k]>
//
// One workgroup per (query, probed list): the query's m x 256 lookup table (fp16) is staged in
// LDS once and every thread scans whole vectors of the list -- m code bytes read as 16-byte vector
// loads (codes are stored [N, m] row-major, sorted by list, so a list is one contiguous slab) and m
// LDS lookups accumulated in fp32 -- writing the approximate score into the query's candidate row.
// The top-k over the candidate row is a separate (library) selection; padding slots stay -inf.
#include <hip/hip_fp16.h>

#include "common.h"

namespace {

template <int M>
__global__ __launch_bounds__(256) void ivfpq_scan_kernel(const __half* __restrict__ lut, const float* __restrict__ base,
                                                         const int* __restrict__ probes,
                                                         const long long* __restrict__ list_off,
                                                         const long long* __restrict__ cand_off,
                                                         const unsigned char* __restrict__ codes, int nprobe,
                                                         long long cand_stride, float* __restrict__ out) {
  __shared__ __half t[M * 256];
  const int q = blockIdx.y, p = blockIdx.x;
  const __half* lq = lut + (size_t)q * M * 256;
  for (int e = threadIdx.x * 8; e < M * 256; e += 256 * 8)
    *reinterpret_cast<uint4*>(t + e) = *reinterpret_cast<const uint4*>(lq + e);
  __syncthreads();
  const int list = probes[q * nprobe + p];
  const long long l0 = list_off[list], l1 = list_off[list + 1];
  const float b = base[q * nprobe + p];
  float* o = out + (size_t)q * cand_stride + cand_off[q * nprobe + p];
  for (long long i = l0 + threadIdx.x; i < l1; i += 256) {
    const uint4* c = reinterpret_cast<const uint4*>(codes + i * M);
    float acc = b;
#pragma unroll
    for (int v = 0; v < M / 16; ++v) {
      const uint4 w = c[v];
      const unsigned ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int j = v * 16 + k;
        const unsigned code = (ww[k >> 2] >> ((k & 3) * 8)) & 0xffu;
        acc += __half2float(t[j * 256 + code]);
      }
    }
    o[i - l0] = acc;
  }
}

}  // namespace

extern "C" {

// lut [Q, m, 256] fp16; base/probes/cand_off [Q, nprobe]; list_off [nlist + 1]; codes [N, m] uint8
// (list-sorted, rows 16-byte aligned: m % 16 == 0); out [Q, cand_stride] fp32 pre-filled with -inf.
int be_ivfpq_scan(const void* lut, const float* base, const int* probes, const long long* list_off,
                  const long long* cand_off, const unsigned char* codes, int Q, int nprobe, int m,
                  long long cand_stride, float* out, hipStream_t s) {
  if (Q == 0 || nprobe == 0) return 0;
  const dim3 grid(nprobe, Q);
  const __half* l = reinterpret_cast<const __half*>(lut);
  switch (m) {
    case 16: hipLaunchKernelGGL(ivfpq_scan_kernel<16>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    case 32: hipLaunchKernelGGL(ivfpq_scan_kernel<32>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    case 48: hipLaunchKernelGGL(ivfpq_scan_kernel<48>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    case 64: hipLaunchKernelGGL(ivfpq_scan_kernel<64>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    case 96: hipLaunchKernelGGL(ivfpq_scan_kernel<96>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    // compressed tier (VectorIndex.compress): 4-dim sub-spaces; the 96 KB fp16 table still fits LDS
    case 128: hipLaunchKernelGGL(ivfpq_scan_kernel<128>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    case 192: hipLaunchKernelGGL(ivfpq_scan_kernel<192>, grid, dim3(256), 0, s, l, base, probes, list_off, cand_off, codes, nprobe, cand_stride, out); break;
    default: return -1;
  }
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
