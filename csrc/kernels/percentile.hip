// Exact per-row percentile normalisation (Cellpose normalize99, SURVEY.md §2.5 K7 / K18:
// x -> (x - p1) / (p99 - p1) with np.percentile 'linear' interpolation per image and channel).
//
// The PyTorch formulation sorts every row (64 rows x 262,144 px for a batch of 32 two-channel 512²
// images: a segmented radix sort with ~1 GB of key/index traffic and large temporaries) only to
// read six order statistics.  Here the six ranks (floor/ceil of each percentile's position, plus
// the min and max for the constant-image test) are found by an MSB-first radix SELECT on
// order-preserving uint32 keys: four passes of an 8-bit digit histogram + a per-row select step.
//
//  * pct_hist_kernel: grid (chunks, rows), 256 threads.  Pass 0 builds ONE 256-bin histogram of the
//    top digit (shared by all six targets); later passes count only the elements whose higher
//    digits equal a target's prefix, into that target's 256 bins.  Histograms live in LDS
//    (6 x 256 x 4 B), flushed once per block with global atomics (non-zero bins only).
//  * pct_select_kernel: one block per row: exclusive scan of each target's bins, pick the digit
//    holding the remaining rank, extend the prefix, clear the bins for the next pass.
//  * pct_apply_kernel: decode the six keys, interpolate p_lo / p_hi exactly like the oracle
//    (float32 a*(1-f) + b*f), write the normalised row (float4 vectorised).
//
// Traffic: 4 reads of the input + 1 read + 1 write — ~6 x 4 B per element instead of a full sort.
#include "common.h"

namespace {

constexpr int kT = 6;  // targets: lo(p_lower), hi(p_lower), lo(p_upper), hi(p_upper), min, max
constexpr int kThreads = 256;

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float kval(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

struct Ranks {
  uint32_t k[kT];
};

// state[r][t] = {prefix, remaining rank}
__global__ __launch_bounds__(kThreads) void pct_hist_kernel(const float* __restrict__ x, long long n, int chunk,
                                                            int pass, const uint32_t* __restrict__ state,
                                                            uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kT][256];
  const int r = blockIdx.y;
  const int ntg = pass == 0 ? 1 : kT;
  for (int i = threadIdx.x; i < ntg * 256; i += kThreads) (&h[0][0])[i] = 0;
  __syncthreads();
  const int shift = 24 - 8 * pass;
  const uint32_t hi_mask = pass == 0 ? 0u : (0xffffffffu << (shift + 8));
  uint32_t pre[kT];
#pragma unroll
  for (int t = 0; t < kT; ++t) pre[t] = state[((size_t)r * kT + t) * 2];
  const float* row = x + (size_t)r * n;
  const long long c0 = (long long)blockIdx.x * chunk;
  const long long c1 = c0 + chunk < n ? c0 + chunk : n;
  // Each thread counts runs of equal digits in registers and issues one LDS atomic per run: image
  // rows are smooth, so a thread's successive elements (256 apart) mostly share the top digit, and
  // one atomic per element serialised every wave on a handful of bins (0.22 ms per 32-image batch).
  if (pass == 0) {
    uint32_t cd = 0, cc = 0;
    for (long long i = c0 + threadIdx.x; i < c1; i += kThreads) {
      const uint32_t d = fkey(row[i]) >> 24;
      if (d != cd) {
        if (cc) atomicAdd(&h[0][cd], cc);
        cd = d;
        cc = 0;
      }
      ++cc;
    }
    if (cc) atomicAdd(&h[0][cd], cc);
  } else {
    uint32_t cd[kT], cc[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) { cd[t] = 0; cc[t] = 0; }
    for (long long i = c0 + threadIdx.x; i < c1; i += kThreads) {
      const uint32_t k = fkey(row[i]);
      const uint32_t d = (k >> shift) & 255u;
#pragma unroll
      for (int t = 0; t < kT; ++t) {
        if (((k ^ pre[t]) & hi_mask) == 0) {
          if (d != cd[t]) {
            if (cc[t]) atomicAdd(&h[t][cd[t]], cc[t]);
            cd[t] = d;
            cc[t] = 0;
          }
          ++cc[t];
        }
      }
    }
#pragma unroll
    for (int t = 0; t < kT; ++t)
      if (cc[t]) atomicAdd(&h[t][cd[t]], cc[t]);
  }
  __syncthreads();
  uint32_t* g = hist + (size_t)r * kT * 256;
  for (int i = threadIdx.x; i < ntg * 256; i += kThreads) {
    const uint32_t v = (&h[0][0])[i];
    if (v) atomicAdd(g + i, v);
  }
}

__global__ __launch_bounds__(kThreads) void pct_select_kernel(int pass, Ranks ranks, uint32_t* __restrict__ state,
                                                              uint32_t* __restrict__ hist) {
  __shared__ uint32_t scan[256];
  const int r = blockIdx.x, tid = threadIdx.x;
  const int shift = 24 - 8 * pass;
  uint32_t* g = hist + (size_t)r * kT * 256;
  for (int t = 0; t < kT; ++t) {
    const uint32_t c = g[(pass == 0 ? 0 : t) * 256 + tid];
    scan[tid] = c;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan
      const uint32_t v = tid >= o ? scan[tid - o] : 0u;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    uint32_t* st = state + ((size_t)r * kT + t) * 2;
    const uint32_t rank = pass == 0 ? ranks.k[t] : st[1];
    const uint32_t incl = scan[tid], excl = incl - c;
    __syncthreads();
    if (c > 0 && excl <= rank && rank < incl) {
      st[0] = (pass == 0 ? 0u : st[0]) | ((uint32_t)tid << shift);
      st[1] = rank - excl;
    }
    __syncthreads();
  }
  for (int t = 0; t < kT; ++t) g[t * 256 + tid] = 0;  // ready for the next pass / next call
}

__global__ __launch_bounds__(kThreads) void pct_apply_kernel(const float* __restrict__ x, long long n, int chunk,
                                                             float a_lo, float b_lo, float a_hi, float b_hi,
                                                             const uint32_t* __restrict__ state, float* __restrict__ out) {
  const int r = blockIdx.y;
  const uint32_t* st = state + (size_t)r * kT * 2;
  // same rounding as the oracle: weights (1 - f) and f rounded to fp32 on the host, fp32 math
  const float p1 = kval(st[0]) * a_lo + kval(st[2]) * b_lo;
  const float p99 = kval(st[4]) * a_hi + kval(st[6]) * b_hi;
  const float rng = p99 - p1;
  const float scale = rng > 1e-3f ? 1.0f / rng : 1.0f;
  const bool cst = kval(st[10]) - kval(st[8]) == 0.0f;
  const float* row = x + (size_t)r * n;
  float* orow = out + (size_t)r * n;
  const long long c0 = (long long)blockIdx.x * chunk;
  const long long c1 = c0 + chunk < n ? c0 + chunk : n;
  if ((n & 3) == 0) {
    for (long long i = c0 + 4 * threadIdx.x; i < c1; i += 4 * kThreads) {
      float4 v = *reinterpret_cast<const float4*>(row + i);
      v.x = cst ? 0.f : (v.x - p1) * scale;
      v.y = cst ? 0.f : (v.y - p1) * scale;
      v.z = cst ? 0.f : (v.z - p1) * scale;
      v.w = cst ? 0.f : (v.w - p1) * scale;
      *reinterpret_cast<float4*>(orow + i) = v;
    }
  } else {
    for (long long i = c0 + threadIdx.x; i < c1; i += kThreads) orow[i] = cst ? 0.f : (row[i] - p1) * scale;
  }
}

}  // namespace

extern "C" {

// Workspace bytes for `rows` rows (hist + state).  The workspace must be zero before its first use;
// histograms live at its start and are left zeroed by every call, the per-row state at its END, so
// calls with different row counts sharing one workspace never see each other's state as counts.
int be_pct_workspace_bytes(int rows, long long* out) {
  if (rows <= 0 || !out) return -1;
  *out = (long long)rows * kT * (256 + 2) * 4;
  return 0;
}

// x, out: [rows, n] float32 (out may alias x).  lower/upper in percent.
int be_pct_normalize(const float* x, int rows, long long n, float lower, float upper, float* out, void* ws,
                     long long ws_bytes, hipStream_t s) {
  if (rows <= 0 || n <= 0 || rows > 65535 || n > 0xffffffffLL) return -1;
  if (ws_bytes < (long long)rows * kT * (256 + 2) * 4) return -2;
  uint32_t* hist = static_cast<uint32_t*>(ws);
  uint32_t* state = hist + ws_bytes / 4 - (size_t)rows * kT * 2;
  const double pos_lo = lower / 100.0 * (double)(n - 1), pos_hi = upper / 100.0 * (double)(n - 1);
  const long long lo0 = (long long)pos_lo, lo1 = (long long)pos_hi;
  Ranks rk;
  rk.k[0] = (uint32_t)lo0;
  rk.k[1] = (uint32_t)(lo0 + 1 < n ? lo0 + 1 : n - 1);
  rk.k[2] = (uint32_t)lo1;
  rk.k[3] = (uint32_t)(lo1 + 1 < n ? lo1 + 1 : n - 1);
  rk.k[4] = 0;
  rk.k[5] = (uint32_t)(n - 1);
  const double f_lo = pos_lo - (double)lo0, f_hi = pos_hi - (double)lo1;
  // ~2 k-element chunks per block, at most 64 blocks per row (>= 256 CUs busy for batches >= 4 rows)
  int chunks = (int)((n + 4095) / 4096);
  if (chunks > 64) chunks = 64;
  int chunk = (int)((n + chunks - 1) / chunks);
  chunk = (chunk + 3) & ~3;
  chunks = (int)((n + chunk - 1) / chunk);
  const dim3 grid(chunks, rows);
  for (int pass = 0; pass < 4; ++pass) {
    hipLaunchKernelGGL(pct_hist_kernel, grid, dim3(kThreads), 0, s, x, n, chunk, pass, state, hist);
    hipLaunchKernelGGL(pct_select_kernel, dim3(rows), dim3(kThreads), 0, s, pass, rk, state, hist);
  }
  hipLaunchKernelGGL(pct_apply_kernel, grid, dim3(kThreads), 0, s, x, n, chunk, (float)(1.0 - f_lo), (float)f_lo,
                     (float)(1.0 - f_hi), (float)f_hi, state, out);
  return BE_CHECK_LAUNCH();
}

}  // extern "C"
